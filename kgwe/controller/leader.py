"""Lease-based leader election (coordination.k8s.io/v1 Lease).

Reference: leader-election settings only (values.yaml:65-71 lease 15 s /
renew 10 s / retry 2 s; scheduler-configmap.yaml:14-17) with 2 replicas and an
in-memory ledger that would diverge between them.  Here
only the lease holder runs the reconcilers and serves mutating extender
verbs; a follower that takes over rebuilds the ledger from pod annotations
(Reconciler.rebuild_ledger), so the apiserver stays the single source of
truth.  Acquire / renew use optimistic concurrency on resourceVersion.
"""
from __future__ import annotations

import threading
import time
from datetime import datetime, timezone

from .kube import ApiError, KubeClient


def _ts(t: float) -> str:
    return datetime.fromtimestamp(t, timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse(ts: str) -> float:
    return datetime.strptime(ts, "%Y-%m-%dT%H:%M:%S.%fZ").replace(tzinfo=timezone.utc).timestamp()


class LeaderElector:
    def __init__(self, kube: KubeClient, name: str, identity: str, namespace: str = "kube-system",
                 lease_s: float = 15.0, renew_s: float = 10.0, retry_s: float = 2.0,
                 on_started=None, on_stopped=None):
        self.kube, self.name, self.identity, self.ns = kube, name, identity, namespace
        self.lease_s, self.renew_s, self.retry_s = lease_s, renew_s, retry_s
        self.on_started, self.on_stopped = on_started, on_stopped
        self.is_leader = False
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    @property
    def path(self) -> str:
        return f"/apis/coordination.k8s.io/v1/namespaces/{self.ns}/leases"

    def try_acquire_or_renew(self, now: float | None = None) -> bool:
        now = time.time() if now is None else now
        spec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_s),
                "renewTime": _ts(now)}
        try:
            cur = self.kube.request("GET", f"{self.path}/{self.name}")
        except ApiError as e:
            if e.status != 404:
                return False
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.ns},
                    "spec": {**spec, "acquireTime": _ts(now)}}
            try:
                self.kube.request("POST", self.path, body)
                return True
            except ApiError:
                return False
        s = cur.get("spec", {})
        holder = s.get("holderIdentity")
        expired = now - _parse(s.get("renewTime", _ts(0))) > float(s.get("leaseDurationSeconds", self.lease_s))
        if holder != self.identity and not expired:
            return False
        new = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
               "metadata": {"name": self.name, "namespace": self.ns,
                            "resourceVersion": cur["metadata"]["resourceVersion"]},
               "spec": {**spec, "acquireTime": s.get("acquireTime") if holder == self.identity else _ts(now)}}
        try:
            self.kube.request("PUT", f"{self.path}/{self.name}", new)
            return True
        except ApiError:
            return False

    def _run(self):
        while not self._stop.is_set():
            ok = self.try_acquire_or_renew()
            if ok and not self.is_leader:
                self.is_leader = True
                if self.on_started:
                    self.on_started()
            elif not ok and self.is_leader:
                self.is_leader = False
                if self.on_stopped:
                    self.on_stopped()
            self._stop.wait(self.renew_s if self.is_leader else self.retry_s)

    def start(self) -> "LeaderElector":
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
