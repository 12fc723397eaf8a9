"""kube-scheduler stand-in that drives the extender over HTTP.

Runs the scheduling cycle kube-scheduler runs for a second-scheduler profile
(``schedulerName: kgwe-scheduler``, reference scheduler-configmap.yaml:18-60)
with the extender configured ``nodeCacheCapable: false`` (full Node objects in
ExtenderArgs): watch unscheduled pods -> POST /filter -> POST /prioritize ->
pick the highest score -> POST /bind.  Used by tests and by the latency
benchmark where no real kube-scheduler exists.
"""
from __future__ import annotations

import http.client
import json
import queue
import threading
import time
import urllib.parse

from .kube import KubeClient

SCHEDULER_NAME = "kgwe-scheduler"


class _Http:
    def __init__(self, base: str):
        u = urllib.parse.urlparse(base)
        self.host, self.port, self.prefix = u.hostname, u.port, u.path.rstrip("/")
        self.local = threading.local()

    def post(self, verb: str, obj) -> object:
        data = json.dumps(obj).encode()
        for attempt in range(2):
            c = getattr(self.local, "c", None)
            if c is None:
                c = self.local.c = http.client.HTTPConnection(self.host, self.port, timeout=30)
            try:
                c.request("POST", f"{self.prefix}/{verb}", body=data,
                          headers={"Content-Type": "application/json"})
                r = c.getresponse()
                return json.loads(r.read() or b"null")
            except (http.client.HTTPException, OSError):
                self.local.c = None
                if attempt:
                    raise
        return None


def _ready(node: dict) -> bool:
    conds = (node.get("status") or {}).get("conditions") or []
    return all(c.get("status") == "True" for c in conds if c.get("type") == "Ready")


class SchedulerSim:
    def __init__(self, kube: KubeClient, extender_url: str, bind_workers: int = 4,
                 on_bound=None, on_failed=None, retry_interval_s: float = 0.05):
        self.kube = kube
        self.ext = _Http(extender_url)
        self.on_bound = on_bound
        self.on_failed = on_failed
        self.retry = retry_interval_s
        self._q: queue.Queue = queue.Queue()
        self._bind_q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._nodes: list = []
        self._nodes_at = 0.0
        self._threads = [threading.Thread(target=self._watch, daemon=True),
                         threading.Thread(target=self._cycle, daemon=True)]
        self._threads += [threading.Thread(target=self._binder, daemon=True)
                          for _ in range(bind_workers)]
        self.stats = {"scheduled": 0, "unschedulable": 0, "bind_errors": 0}

    def start(self) -> "SchedulerSim":
        for t in self._threads:
            t.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _nodelist(self) -> list:
        if time.time() - self._nodes_at > 1.0 or not self._nodes:
            # kube-scheduler never offers a node that is not Ready (the
            # node.kubernetes.io/not-ready taint): neither does the stand-in.
            self._nodes = [n for n in self.kube.list_nodes() if _ready(n)]
            self._nodes_at = time.time()
        return self._nodes

    def invalidate_nodes(self) -> None:
        self._nodes_at = 0.0

    def _watch(self):
        rv = "0"
        while not self._stop.is_set():
            try:
                evs, rv = self.kube.watch("/api/v1/pods", rv, timeout_s=1)
            except Exception:  # noqa: BLE001
                time.sleep(0.05)
                continue
            for e in evs:
                pod = e["object"]
                spec = pod.get("spec", {})
                if e["type"] == "ADDED" and spec.get("schedulerName") == SCHEDULER_NAME \
                        and not spec.get("nodeName"):
                    self._q.put((pod, time.perf_counter()))

    def _cycle(self):
        while not self._stop.is_set():
            try:
                pod, seen = self._q.get(timeout=0.2)
            except queue.Empty:
                continue
            nodes = self._nodelist()
            try:
                fr = self.ext.post("filter", {"pod": pod, "nodes": {"items": nodes}})
            except Exception:  # noqa: BLE001
                self._requeue(pod, seen)
                continue
            passed = [n for n in (fr or {}).get("nodes", {}).get("items", [])]
            if not passed:
                self.stats["unschedulable"] += 1
                if self.on_failed:
                    self.on_failed(pod, fr)
                self._requeue(pod, seen)
                continue
            pr = self.ext.post("prioritize", {"pod": pod, "nodes": {"items": passed}}) or []
            scores = {h["host"]: h["score"] for h in pr}
            best = max((n["metadata"]["name"] for n in passed),
                       key=lambda nm: (scores.get(nm, 0), -hash(nm) % 1000, nm))
            self._bind_q.put((pod, best, seen))

    def _requeue(self, pod, seen):
        def later():
            time.sleep(self.retry)
            if not self._stop.is_set():
                self._q.put((pod, seen))
        threading.Thread(target=later, daemon=True).start()

    def _binder(self):
        while not self._stop.is_set():
            try:
                pod, node, seen = self._bind_q.get(timeout=0.2)
            except queue.Empty:
                continue
            md = pod["metadata"]
            try:
                res = self.ext.post("bind", {"podName": md["name"], "podNamespace": md.get("namespace", "default"),
                                             "podUID": md.get("uid", ""), "node": node}) or {}
            except Exception as e:  # noqa: BLE001
                res = {"error": str(e)}
            if res.get("error"):
                self.stats["bind_errors"] += 1
                if "waiting" in res["error"]:
                    self._requeue_bind(pod, node, seen)
                else:
                    self._requeue(pod, seen)
                continue
            self.stats["scheduled"] += 1
            if self.on_bound:
                self.on_bound(pod, node, time.perf_counter())

    def _requeue_bind(self, pod, node, seen):
        def later():
            time.sleep(self.retry)
            if not self._stop.is_set():
                self._bind_q.put((pod, node, seen))
        threading.Thread(target=later, daemon=True).start()
