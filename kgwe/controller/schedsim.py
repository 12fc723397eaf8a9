"""kube-scheduler stand-in that drives the extender over HTTP.

Runs the scheduling cycle kube-scheduler runs for a second-scheduler profile
(``schedulerName: kgwe-scheduler``, reference scheduler-configmap.yaml:18-60):
watch unscheduled pods -> POST /filter -> POST /prioritize -> pick the highest
score -> POST /bind.  ``node_cache_capable=False`` (the reference's setting)
sends full Node objects in every ExtenderArgs, True sends node names only.
When no node passes and the pod has a priority, it runs kube-scheduler's
PostFilter with the extender's ``preempt`` verb: the extender names the
victims per node, the stand-in evicts the cheapest node's victims (deletes
the pods) and retries the preemptor.  Unschedulable pods and failed binds
go back to the queue with kube-scheduler's pod backoff (podInitialBackoffSeconds
1 s, doubling to podMaxBackoffSeconds 10 s), and every bind runs in its own
thread as kube-scheduler runs each binding cycle in its own goroutine — a
gang member's bind is held by the extender until its gang is complete
(Permit), so binds must not queue behind one another.  Used by tests and by
the latency benchmark where no real kube-scheduler exists.  Node objects are serialised
once per node-list refresh (kube-scheduler keeps them encoded in its cache
too), so the stand-in's own cost stays out of the measured latency.
"""
from __future__ import annotations

import gc
import json
import queue
import threading
import time
import urllib.parse

from .kube import KubeClient

SCHEDULER_NAME = "kgwe-scheduler"


class _Http:
    """Extender client: one native keep-alive connection per calling thread
    (kgwe.core.native.HttpClient: gather-write of the body parts, GIL released
    for the round trip)."""

    def __init__(self, base: str):
        u = urllib.parse.urlparse(base)
        self.host, self.port, self.prefix = u.hostname, u.port, u.path.rstrip("/")
        self.local = threading.local()

    def _client(self):
        from ..core import native  # noqa: PLC0415

        c = getattr(self.local, "c", None)
        if c is None:
            c = self.local.c = native.HttpClient(self.host, self.port, 35.0)
        return c

    def post(self, verb: str, obj, raw: bool = False) -> object:
        parts = obj if isinstance(obj, list) else \
            [obj if isinstance(obj, (bytes, bytearray)) else json.dumps(obj).encode()]
        _, body = self._client().post(f"{self.prefix}/{verb}", parts)
        return body if raw else json.loads(body or b"null")

    def post_names(self, verb: str, parts: list) -> list:
        """POST and return only the node names of the reply (filter)."""
        return self._client().post_names(f"{self.prefix}/{verb}", parts)[1]


def _ready(node: dict) -> bool:
    conds = (node.get("status") or {}).get("conditions") or []
    return all(c.get("status") == "True" for c in conds if c.get("type") == "Ready")


class SchedulerSim:
    def __init__(self, kube: KubeClient, extender_url: str, bind_workers: int = 4,
                 on_bound=None, on_failed=None, initial_backoff_s: float = 1.0,
                 max_backoff_s: float = 10.0, node_cache_capable: bool = False, preempt: bool = True,
                 on_preempted=None, node_refresh_s: float = 1.0, percentage_of_nodes_to_score: float = 0.0,
                 max_bind_threads: int = 256):
        self.kube = kube
        self.ext = _Http(extender_url)
        self.on_bound = on_bound
        self.on_failed = on_failed
        self.on_preempted = on_preempted
        self.backoff0, self.backoff_max = initial_backoff_s, max_backoff_s
        self.max_bind_threads = max_bind_threads
        self._bind_idle = 0  # binder threads waiting for work
        self._bind_lock = threading.Lock()
        self.node_cache_capable = node_cache_capable
        self.node_refresh_s = node_refresh_s  # unused: the node cache follows a watch (see _informer)
        # the profile's percentageOfNodesToScore; 0 = kube-scheduler's adaptive default
        self.pct_to_score = float(percentage_of_nodes_to_score)
        self._start = 0  # kube-scheduler's rotating start index over the node list
        self.preempt = preempt
        self._node_json: dict[str, bytes] = {}
        self._node_rv: dict[str, str] = {}
        self._objs: dict = {}
        self._list_rv = None
        self._bound: dict[str, tuple] = {}  # pod uid -> (namespace, name) of bound pods
        self.retried: set = set()            # uids of pods that needed more than one cycle
        self._attempts: dict[str, int] = {}
        self._q: queue.Queue = queue.Queue()
        self._bind_q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._nodes: list = []
        self._nodes_at = 0.0
        self._nodes_lock = threading.Lock()
        self._threads = [threading.Thread(target=self._watch, daemon=True),
                         threading.Thread(target=self._cycle, daemon=True),
                         threading.Thread(target=self._informer, daemon=True)]
        self._bind_min = bind_workers
        self._threads += [threading.Thread(target=self._binder, args=(True,), daemon=True)
                          for _ in range(bind_workers)]
        self._n_binders = bind_workers
        self._rt = {"filter": [], "prioritize": [], "cycle": []}  # client-side round trips (s)
        self.stats = {"scheduled": 0, "unschedulable": 0, "bind_errors": 0, "preemptions": 0,
                      "preempt_calls": 0}

    def start(self) -> "SchedulerSim":
        try:  # WaitForCacheSync: the node cache is warm before the first cycle
            self._refresh_nodes()
        except Exception:  # noqa: BLE001
            pass
        # The cached fleet is long-lived: keep it out of CPython's cyclic GC,
        # whose full collections over ~10^6 Node-object dicts paused every
        # thread of the stand-in for ~100 ms (kube-scheduler has no such pause).
        gc.freeze()
        for t in self._threads:
            t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        for k, v in self._rt.items():  # client-observed round trips, ms
            if v:
                v = sorted(v)
                self.stats[f"{k}_rt_ms"] = {"p50": round(1000 * v[len(v) // 2], 3),
                                            "p99": round(1000 * v[min(len(v) - 1, int(len(v) * 0.99))], 3),
                                            "mean": round(1000 * sum(v) / len(v), 3)}

    def _refresh_nodes(self) -> None:
        """Full re-list (start-up, invalidate_nodes, watch failure)."""
        res = self.kube.request("GET", "/api/v1/nodes")
        objs = {n["metadata"]["name"]: n for n in res.get("items", [])}
        self._set_nodes(objs, str((res.get("metadata") or {}).get("resourceVersion", "0")))

    def _set_nodes(self, objs: dict, rv: str) -> None:
        # kube-scheduler never offers a node that is not Ready (the
        # node.kubernetes.io/not-ready taint): neither does the stand-in.
        # Re-serialise only nodes whose resourceVersion moved.
        old, old_rv = self._node_json, self._node_rv
        node_json, node_rv, nodes = {}, {}, []
        for name, n in objs.items():
            if not _ready(n):
                continue
            nodes.append(n)
            v = n["metadata"].get("resourceVersion")
            node_rv[name] = v
            node_json[name] = old[name] if v is not None and old_rv.get(name) == v and name in old \
                else json.dumps(n).encode()
        with self._nodes_lock:  # swap all at once: a cycle never sees a half-built cache
            self._objs, self._list_rv = objs, rv
            self._nodes, self._node_json, self._node_rv = nodes, node_json, node_rv
            self._nodes_at = time.time()

    def _informer(self):
        """kube-scheduler's node informer: list once, then apply watch events
        off the scheduling cycle.  (Re-listing 1,250 full Node objects parses
        ~9 MB under the GIL — ~0.2 s that stalled every pod queued behind it.)"""
        while not self._stop.is_set():
            with self._nodes_lock:
                rv, objs = self._list_rv, self._objs
            if rv is None:
                self._stop.wait(0.05)
                continue
            try:
                evs, new_rv = self.kube.watch("/api/v1/nodes", rv, timeout_s=1)
            except Exception:  # noqa: BLE001
                self._stop.wait(0.2)
                try:
                    self._refresh_nodes()
                except Exception:  # noqa: BLE001
                    pass
                continue
            if not evs:
                with self._nodes_lock:
                    if self._list_rv == rv:
                        self._list_rv = new_rv
                continue
            objs = dict(objs)
            for e in evs:
                o = e.get("object") or {}
                name = (o.get("metadata") or {}).get("name")
                if not name:
                    continue
                if e.get("type") == "DELETED":
                    objs.pop(name, None)
                else:
                    objs[name] = o
            self._set_nodes(objs, new_rv)

    def _nodelist(self) -> list:
        if not self._nodes:
            self._refresh_nodes()
        with self._nodes_lock:
            return self._nodes

    def _args(self, pod_json: bytes, names: list) -> list:
        """ExtenderArgs as a list of body parts (sent with one gather write:
        the cached Node objects are never joined into one buffer)."""
        if self.node_cache_capable:
            return [b'{"pod":', pod_json, b',"nodenames":', json.dumps(names).encode(), b"}"]
        with self._nodes_lock:
            nj = self._node_json
        parts = [b'{"pod":', pod_json, b',"nodes":{"items":[']
        first = True
        for n in names:
            j = nj.get(n)
            if j is None:
                continue
            if not first:
                parts.append(b",")
            parts.append(j)
            first = False
        parts.append(b"]}}")
        return parts

    def invalidate_nodes(self) -> None:
        self._refresh_nodes()

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
            t_cycle = time.perf_counter()
            pod.setdefault("_kgwe_t", {})["seen"] = seen
            pod["_kgwe_t"]["cycle"] = t_cycle
            nodes = self._nodelist()
            names = self._candidates([n["metadata"]["name"] for n in nodes])
            pod_json = json.dumps({k: v for k, v in pod.items() if k != "_kgwe_t"}).encode()
            try:
                t_f = time.perf_counter()
                passed = self.ext.post_names("filter", self._args(pod_json, names))
                self._rt["filter"].append(time.perf_counter() - t_f)
            except Exception as e:  # noqa: BLE001 - extender unreachable / bad reply: retry with backoff
                self.stats["cycle_errors"] = self.stats.get("cycle_errors", 0) + 1
                self.last_error = repr(e)
                self._requeue(pod, seen)
                continue
            if not passed:
                self.stats["unschedulable"] += 1
                if self.on_failed:
                    self.on_failed(pod, None)
                if self.preempt and int((pod.get("spec") or {}).get("priority") or 0) > 0:
                    self._post_filter(pod, names)
                self._requeue(pod, seen)
                continue
            t_p = time.perf_counter()
            pr = self.ext.post("prioritize", self._args(pod_json, passed)) or []
            self._rt["prioritize"].append(time.perf_counter() - t_p)
            scores = {h["host"]: h["score"] for h in pr}
            best = max(passed, key=lambda nm: (scores.get(nm, 0), -hash(nm) % 1000, nm))
            pod["_kgwe_t"]["bind_q"] = time.perf_counter()
            self._submit_bind(pod, best, seen)
            self._rt["cycle"].append(time.perf_counter() - t_cycle)

    def _candidates(self, names: list) -> list:
        """kube-scheduler's percentageOfNodesToScore: it stops searching after
        max(100, N * pct %) feasible nodes, starting where the previous cycle
        stopped, and only those reach the extender.  pct is the profile's
        setting, or with 0 the adaptive default max(5, 50 - N / 125); at 100
        every node is a candidate.  (Its own plugins would also drop full
        nodes; the extender filter covers that here.)"""
        n = len(names)
        if n <= 100 or self.pct_to_score >= 100.0:
            return names
        pct = self.pct_to_score if self.pct_to_score > 0 else max(5.0, 50.0 - n / 125.0)
        k = min(n, max(100, int(n * pct / 100.0)))
        start = self._start % n
        self._start = start + k
        return (names + names)[start:start + k]

    def _post_filter(self, pod: dict, names: list) -> None:
        """kube-scheduler PostFilter (DefaultPreemption) through the extender's
        preempt verb: pick the node needing the fewest evictions, evict them."""
        self.stats["preempt_calls"] += 1
        try:
            res = self.ext.post("preempt", {"pod": pod, "nodeNameToMetaVictims": {
                n: {"pods": [], "numPDBViolations": 0} for n in names}}) or {}
        except Exception:  # noqa: BLE001
            return
        plans = {n: [p["uid"] for p in (v or {}).get("pods") or []]
                 for n, v in (res.get("nodeNameToMetaVictims") or {}).items()}
        # kube-scheduler resolves every MetaPod against the node's own pods and
        # drops the whole extender result if one is not there
        # (convertPodUIDToPod): a victim on another node fails the preemption.
        for n, v in plans.items():
            for uid in v:
                on = self._bound.get(uid)
                if on is not None and on[2] != n:
                    self.stats["preempt_rejected"] = self.stats.get("preempt_rejected", 0) + 1
                    return
        plans = {n: v for n, v in plans.items() if v}
        if not plans:
            return
        node = min(plans, key=lambda n: (len(plans[n]), n))
        victims = plans[node]
        for uid in victims:
            ref = self._bound.pop(uid, None)
            if ref is not None:
                try:
                    self.kube.delete_pod(ref[0], ref[1])
                except Exception:  # noqa: BLE001
                    pass
        self.stats["preemptions"] += len(victims)
        if self.on_preempted:
            self.on_preempted(victims)

    def _requeue(self, pod, seen):
        uid = pod["metadata"].get("uid", "")
        self.retried.add(uid)
        # kube-scheduler's pod backoff: podInitialBackoffSeconds doubling per
        # attempt up to podMaxBackoffSeconds (defaults 1 s and 10 s)
        n = self._attempts[uid] = self._attempts.get(uid, 0) + 1
        delay = min(self.backoff_max, self.backoff0 * (2 ** min(n - 1, 10)))

        def later():
            time.sleep(delay)
            if not self._stop.is_set():
                self._q.put((pod, seen))
        threading.Thread(target=later, daemon=True).start()

    def _submit_bind(self, pod, node, seen):
        """One binding cycle per pod, concurrently (kube-scheduler: a goroutine
        each): a new binder thread is started whenever none is idle."""
        with self._bind_lock:
            spawn = self._bind_idle == 0 and self._n_binders < self.max_bind_threads
            if spawn:
                self._n_binders += 1
        self._bind_q.put((pod, node, seen))
        if spawn:
            threading.Thread(target=self._binder, args=(False,), daemon=True).start()

    def _binder(self, permanent: bool = True):
        while not self._stop.is_set():
            with self._bind_lock:
                self._bind_idle += 1
            try:
                pod, node, seen = self._bind_q.get(timeout=0.2 if permanent else 2.0)
            except queue.Empty:
                with self._bind_lock:
                    self._bind_idle -= 1
                    if not permanent:
                        self._n_binders -= 1
                        return
                continue
            with self._bind_lock:
                self._bind_idle -= 1
            md = pod["metadata"]
            pod.setdefault("_kgwe_t", {})["bind"] = time.perf_counter()
            try:
                res = self.ext.post("bind", {"podName": md["name"], "podNamespace": md.get("namespace", "default"),
                                             "podUID": md.get("uid", ""), "node": node}) or {}
            except Exception as e:  # noqa: BLE001
                res = {"error": str(e)}
            if res.get("error"):
                # a failed binding cycle (held gang bind timed out included):
                # the pod goes back to the scheduling queue with backoff
                self.stats["bind_errors"] += 1
                self._requeue(pod, seen)
                continue
            self.stats["scheduled"] += 1
            self._bound[md.get("uid", "")] = (md.get("namespace", "default"), md["name"], node)
            if self.on_bound:
                self.on_bound(pod, node, time.perf_counter())
