"""Validating / mutating admission webhook for kgwe custom resources
(reference: declared only — values.yaml:375-392 cert-manager webhook with
failurePolicy Fail, Makefile:111 controller-gen webhook).

`review()` takes an admission.k8s.io/v1 AdmissionReview and returns the
response AdmissionReview: the validating path rejects schema / semantic
errors (crds.validate); the mutating path returns a JSONPatch that applies
schema defaults and rewrites NVIDIA vocabulary (NVLink* preferences, `mig`,
backend NCCL) to the MI355X one (crds.default).

Pods for the kgwe scheduler get a microsecond creation stamp
(``kgwe.amd.com/created-at``, Unix seconds) on admission: the extender's bind
turns it into the pod-create -> bind latency sample of
``kgwe_scheduling_latency_ms`` (the apiserver's creationTimestamp has whole-
second resolution, useless for an 85 ms p99 target).
"""
from __future__ import annotations

import base64
import json
import time

from . import crds

ANN_CREATED = "kgwe.amd.com/created-at"
SCHEDULER_NAME = "kgwe-scheduler"


def _pod_patch(pod: dict) -> list | None:
    if (pod.get("spec") or {}).get("schedulerName") != SCHEDULER_NAME:
        return None
    ann = (pod.get("metadata") or {}).get("annotations")
    stamp = f"{time.time():.6f}"
    if ann is None:
        return [{"op": "add", "path": "/metadata/annotations", "value": {ANN_CREATED: stamp}}]
    if ANN_CREATED in ann:
        return None
    return [{"op": "add", "path": "/metadata/annotations/" + ANN_CREATED.replace("~", "~0").replace("/", "~1"),
             "value": stamp}]


def review(ar: dict, mutate: bool = False) -> dict:
    req = ar.get("request", {})
    uid = req.get("uid", "")
    obj = req.get("object") or {}
    resp: dict = {"uid": uid, "allowed": True}
    if req.get("operation") == "DELETE":
        return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}
    if (req.get("kind") or {}).get("kind") == "Pod" or obj.get("kind") == "Pod":
        patch = _pod_patch(obj) if mutate else None
        if patch:
            resp["patchType"] = "JSONPatch"
            resp["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
        return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}
    if mutate:
        new = crds.default(obj)
        if new != obj:
            patch = [{"op": "replace" if "spec" in obj else "add", "path": "/spec", "value": new["spec"]}]
            resp["patchType"] = "JSONPatch"
            resp["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
        obj = new
    errors = crds.validate(obj)
    if errors:
        resp["allowed"] = False
        resp["status"] = {"code": 422, "reason": "Invalid", "message": "; ".join(errors[:10])}
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}
