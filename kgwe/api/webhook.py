"""Validating / mutating admission webhook for kgwe custom resources
(reference: declared only — values.yaml:375-392 cert-manager webhook with
failurePolicy Fail, Makefile:111 controller-gen webhook).

`review()` takes an admission.k8s.io/v1 AdmissionReview and returns the
response AdmissionReview: the validating path rejects schema / semantic
errors (crds.validate); the mutating path returns a JSONPatch that applies
schema defaults and rewrites NVIDIA vocabulary (NVLink* preferences, `mig`,
backend NCCL) to the MI355X one (crds.default).
"""
from __future__ import annotations

import base64
import json

from . import crds


def review(ar: dict, mutate: bool = False) -> dict:
    req = ar.get("request", {})
    uid = req.get("uid", "")
    obj = req.get("object") or {}
    resp: dict = {"uid": uid, "allowed": True}
    if req.get("operation") == "DELETE":
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
