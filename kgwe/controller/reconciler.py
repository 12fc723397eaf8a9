"""Controller reconcile loops for GPUWorkload / GPUBudget / PartitionStrategy.

Reference: the designed flow (docs/architecture.md:139-168) —
"[controller] reconciles CR -> creates Pod(schedulerName=kgwe-scheduler,
podTemplate)", writes GPUWorkload.status, starts/stops cost tracking — none of
which exists in the reference (D1).  Here:

* GPUWorkload -> one Pod per workload (podTemplate + schedulerName
  ``kgwe-scheduler`` + amd.com/gpu or amd.com/gpu-<mode> limits + the spec as
  the ``kgwe.amd.com/workload`` annotation the extender parses) -> status
  (phase, node, GPUs / slices, score, estimated xGMI bandwidth, RCCL env,
  conditions, start/completion time, cost).
* Pod termination / deletion -> allocation release + cost finalisation.
* GPUBudget -> cost-engine budget; status (spend, utilisation, alerts).
* PartitionStrategy -> registered + rebalanced every rebalanceInterval.
* Failure detection / recovery (the reference only evicts a
  deleted node from its cache and leaves its allocations stale): a node that
  is deleted or stops being Ready, or a GPU of a running allocation that the
  amd-smi health policy marks Unhealthy, evicts the workloads on it — the
  allocation is released and, per ``spec.recovery`` (Reschedule, at most
  maxRestarts times), the GPUWorkload gets a fresh pod that the scheduler
  places elsewhere; status carries ``restarts`` / ``lastFailure``.
* Restart safety: on start the ledger is
  rebuilt from the full allocation annotation of already-bound pods
  (priority, preemptible, type, gang, share CU range included), so a
  controller restart or leader change neither leaks GPUs nor turns a
  non-preemptible job into a preemption victim; running cost records resume
  from the cost journal.
* Partition consolidation: under-used partitioned GPUs are emptied by
  evicting their preemptible inference pods (recreated and packed onto the
  fuller GPUs by best fit) and switched back to SPX.
* The optimizer loop (reference WorkloadOptimizer facade,
  src/optimizer/workload_optimizer.py:697-875, which nothing fed): per-
  allocation amd-smi telemetry -> IngestTelemetry every tick, completion ->
  the online model's training rows, PredictResources -> ``status.
  recommendation`` (rightsizing: GPUs, memory, partition mode), and
  GetPlacement with the ledger's busy GPUs over a bounded candidate set.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from datetime import datetime, timezone

from ..api import crds
from ..extender.server import ANN_ALLOC, ANN_BW, ANN_ENV, ANN_GPUS, ANN_NODE, ANN_PARTS, ANN_SCORE
from .kube import ApiError, KubeClient
from .schedsim import SCHEDULER_NAME

log = logging.getLogger("kgwe.controller")
HINT_CANDIDATE_NODES = 16  # nodes sent to GetPlacement (most free GPUs first)
RECOMMEND_EVERY_S = 30.0
ANN_WORKLOAD = "kgwe.amd.com/workload"
LABEL_WORKLOAD = "kgwe.amd.com/gpuworkload"


def _now_iso() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def pod_name(gw_name: str, restart: int = 0) -> str:
    """One pod per attempt: a lost node may keep the old pod Terminating."""
    return f"{gw_name}-gw" if restart == 0 else f"{gw_name}-gw-r{restart}"


def pod_for_workload(gw: dict, restart: int = 0) -> dict:
    md = gw["metadata"]
    spec = gw["spec"]
    req = spec["gpuRequirements"]
    tmpl = json.loads(json.dumps(spec.get("podTemplate") or {}))
    pod_spec = tmpl.get("spec") or {"containers": [{"name": "main", "image": "rocm/pytorch:latest"}]}
    pod_spec["schedulerName"] = SCHEDULER_NAME
    pod_spec.setdefault("restartPolicy", "Never")
    if "priority" in spec:
        pod_spec["priority"] = int(spec["priority"])
    if req.get("partition"):
        res = {f"amd.com/gpu-{req['partition']['mode'].lower()}": str(req["partition"].get("count", 1))}
    elif req.get("sharing"):
        res = {"amd.com/gpu-shared": "1"}
    else:
        res = {"amd.com/gpu": str(req.get("count", 1))}
    c0 = pod_spec["containers"][0]
    lim = c0.setdefault("resources", {}).setdefault("limits", {})
    lim.update(res)
    # Downward API: kgwe.launch reads the placement annotations at start.
    pod_spec.setdefault("volumes", []).append(
        {"name": "kgwe-podinfo", "downwardAPI": {"items": [
            {"path": "annotations", "fieldRef": {"fieldPath": "metadata.annotations"}}]}})
    c0.setdefault("volumeMounts", []).append({"name": "kgwe-podinfo", "mountPath": "/etc/kgwe"})
    labels = dict((tmpl.get("metadata") or {}).get("labels") or {})
    labels[LABEL_WORKLOAD] = md["name"]
    if spec.get("team"):
        labels["kgwe.amd.com/team"] = spec["team"]
    if spec.get("project"):
        labels["kgwe.amd.com/project"] = spec["project"]
    ann = dict((tmpl.get("metadata") or {}).get("annotations") or {})
    ann[ANN_WORKLOAD] = json.dumps({"metadata": {"name": md["name"], "namespace": md.get("namespace", "default"),
                                                 "labels": labels}, "spec": {k: v for k, v in spec.items()
                                                                             if k != "podTemplate"}})
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": pod_name(md["name"], restart), "namespace": md.get("namespace", "default"),
                         "labels": labels, "annotations": ann,
                         "ownerReferences": [{"apiVersion": f"{crds.GROUP}/{crds.VERSION}", "kind": "GPUWorkload",
                                              "name": md["name"], "uid": md.get("uid", ""),
                                              "controller": True}]},
            "spec": pod_spec}


class Reconciler:
    def __init__(self, platform, kube: KubeClient, optimizer=None, tick_s: float = 5.0,
                 consolidate: bool = True, recommend_every_s: float = RECOMMEND_EVERY_S):
        self.p = platform
        self.kube = kube
        self.optimizer = optimizer
        self.tick_s = tick_s
        self.consolidate = consolidate
        self.errors = 0                    # exceptions in the periodic loop (logged + counted)
        self.migrations = 0
        self._running: dict[str, tuple] = {}  # pod uid -> (ns, gpuworkload, bound at)
        self._next_recommend = 0.0
        self.recommend_every_s = recommend_every_s
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._strategy_next: dict[str, float] = {}
        self._evicting: set[str] = set()  # pod uids being evicted by the controller
        self._lost_nodes: set[str] = set()
        self.restored = 0

    # ------------------------------------------------------------- lifecycle
    def start(self) -> "Reconciler":
        """(Re)start — also called by the leader elector on every takeover: the
        new leader first rebuilds the ledger from the apiserver."""
        self._stop.clear()
        self._threads = []
        self.restored = self.rebuild_ledger()
        for fn in (self._watch_workloads, self._watch_pods, self._watch_budgets, self._watch_strategies,
                   self._watch_nodes, self._periodic):
            t = threading.Thread(target=fn, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self) -> None:
        self._stop.set()

    def rebuild_ledger(self) -> int:
        """Restore allocations from bound pods' annotations (restart safety)."""
        n = 0
        try:
            pods = self.kube.list_pods()
        except Exception:  # noqa: BLE001
            return 0
        for pod in pods:
            md = pod.get("metadata", {})
            ann = md.get("annotations") or {}
            node = pod.get("spec", {}).get("nodeName")
            if not node or ANN_GPUS not in ann:
                continue
            if pod.get("status", {}).get("phase") in ("Succeeded", "Failed"):
                continue
            uid = md.get("uid") or f"{md.get('namespace')}/{md.get('name')}"
            try:
                alloc = json.loads(ann[ANN_ALLOC]) if ANN_ALLOC in ann else None
            except ValueError:
                alloc = None
            if alloc is None:  # pods bound by an older controller: placement only
                alloc = {"node": node, "namespace": md.get("namespace", "default"),
                         "team": (md.get("labels") or {}).get("kgwe.amd.com/team", ""),
                         "gpus": [g for g in ann.get(ANN_GPUS, "").split(",") if g],
                         "partitions": [p for p in ann.get(ANN_PARTS, "").split(",") if p],
                         "priority": pod.get("spec", {}).get("priority", 0)}
            alloc["uid"] = uid
            alloc["node"] = node
            if self.p.restore_allocation(alloc):
                n += 1
                wl = (md.get("labels") or {}).get(LABEL_WORKLOAD)
                if wl:
                    self._running[uid] = (md.get("namespace", "default"), wl, time.time())
        return n

    def _loop(self, path: str, handler):
        rv = "0"
        while not self._stop.is_set():
            try:
                evs, rv = self.kube.watch(path, rv, timeout_s=2)
            except Exception:  # noqa: BLE001
                time.sleep(0.2)
                continue
            for e in evs:
                try:
                    handler(e["type"], e["object"])
                except Exception as ex:  # noqa: BLE001 - keep the loop alive, surface in status
                    self._record_error(e.get("object", {}), ex)

    def _record_error(self, obj: dict, ex: Exception):
        md = obj.get("metadata", {})
        if obj.get("kind") == "GPUWorkload":
            try:
                self.kube.patch_cr_status("GPUWorkload", md.get("namespace"), md.get("name"),
                                          {"message": f"reconcile error: {ex}"})
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------- GPUWorkload
    def _watch_workloads(self):
        self._loop(f"/apis/{crds.GROUP}/{crds.VERSION}/gpuworkloads", self.on_workload)

    def on_workload(self, typ: str, gw: dict):
        md = gw["metadata"]
        ns, name = md.get("namespace", "default"), md["name"]
        if typ == "DELETED":
            self.kube.delete_pod(ns, (gw.get("status") or {}).get("podName") or pod_name(name))
            return
        if gw.get("status", {}).get("phase") in ("Scheduling", "Scheduled", "Running", "Succeeded", "Failed"):
            return
        restart = int((gw.get("status") or {}).get("restarts") or 0)
        gw = crds.default(gw)
        errs = crds.validate(gw)
        if errs:
            self.kube.patch_cr_status("GPUWorkload", ns, name, {
                "phase": "Failed", "message": "; ".join(errs),
                "conditions": [{"type": "Valid", "status": "False", "reason": "Invalid",
                                "message": "; ".join(errs), "lastTransitionTime": _now_iso()}]})
            return
        rec = None
        if self.optimizer is not None:
            try:  # optimizer hint -> +10 preferred-node bonus
                req = gw["spec"]["gpuRequirements"]
                busy, cand = self._hint_view(int(req.get("count", 1) or 1))
                hint = self.optimizer.GetPlacement({"workload_id": f"{ns}/{name}",
                                                    "cluster_topology": cand,
                                                    "requirements": {"gpu_count": req.get("count", 1),
                                                                     "prefer_xgmi": True,
                                                                     "busy_gpus": busy}})
                if hint.get("preferred_nodes"):
                    gw["spec"]["preferredNodes"] = hint["preferred_nodes"]
            except Exception as e:  # noqa: BLE001 - the hint is optional
                log.warning("GetPlacement for %s/%s failed: %s", ns, name, e)
            rec = self._recommend(ns, name, gw["spec"])
        pod = pod_for_workload(gw, restart)
        try:
            self.kube.create_pod(pod)
        except ApiError as e:
            if e.status != 409:
                raise
        st = {"phase": "Scheduling", "podName": pod["metadata"]["name"],
              "conditions": [{"type": "PodCreated", "status": "True", "reason": "Created",
                              "lastTransitionTime": _now_iso()}]}
        if rec:
            st["recommendation"] = rec
        self.kube.patch_cr_status("GPUWorkload", ns, name, st)

    # ------------------------------------------------------------- Pods
    def _watch_pods(self):
        self._loop("/api/v1/pods", self.on_pod)

    def on_pod(self, typ: str, pod: dict):
        md = pod.get("metadata", {})
        wl = (md.get("labels") or {}).get(LABEL_WORKLOAD)
        ns = md.get("namespace", "default")
        uid = md.get("uid") or f"{ns}/{md.get('name')}"
        phase = pod.get("status", {}).get("phase")
        ann = md.get("annotations") or {}
        if typ == "DELETED" or phase in ("Succeeded", "Failed"):
            rel = self.p.release(uid)
            # a preempted gang member: the gang goes as a unit (the extender's
            # preempt verb can only name the victims on the preemptor's node)
            peers = set(rel.get("evict_gang_peers") or [])
            # a share group's leader: its members connected to the serving process that
            # just went away; evicted, they reschedule and the first becomes the new leader
            orphans = set(rel.get("orphaned_share_members") or [])
            if peers or orphans:
                for a in self.p.allocations():
                    if a["uid"] in peers:
                        self.evict(a, f"gang member {uid} preempted")
                    elif a["uid"] in orphans:
                        self.evict(a, f"share group leader {uid} is gone")
            run = self._running.pop(uid, None)
            if run and self.optimizer is not None and uid not in self._evicting:
                try:  # a finished run -> a training row of the online model
                    self.optimizer.IngestTelemetry({"workload_id": f"{run[0]}/{run[1]}", "completed": True,
                                                    "duration_seconds": time.time() - run[2]})
                except Exception as e:  # noqa: BLE001
                    log.warning("optimizer completion for %s failed: %s", uid, e)
            if uid in self._evicting:  # the eviction path owns the workload's status
                if typ == "DELETED":
                    self._evicting.discard(uid)
                return
            if wl and not self._is_current_pod(ns, wl, md.get("name", "")):
                return  # an earlier attempt's pod going away
            if wl:
                st = {"phase": "Failed" if phase == "Failed" else "Succeeded", "completionTime": _now_iso()}
                cost = rel.get("cost")
                if cost:
                    st["cost"] = cost["adjusted_cost"]
                try:
                    self.kube.patch_cr_status("GPUWorkload", ns, wl, st)
                except ApiError:
                    pass
            return
        if wl and pod.get("spec", {}).get("nodeName") and ANN_GPUS in ann:
            self._running.setdefault(uid, (ns, wl, time.time()))
            st = {"phase": "Running" if phase == "Running" else "Scheduled",
                  "scheduledNode": ann.get(ANN_NODE) or pod["spec"]["nodeName"],
                  "allocatedGPUs": [g for g in ann.get(ANN_GPUS, "").split(",") if g],
                  "partitionSlices": [g for g in ann.get(ANN_PARTS, "").split(",") if g],
                  "schedulingScore": int(ann.get(ANN_SCORE, "0") or 0),
                  "estimatedBandwidth": float(ann.get(ANN_BW, "0") or 0),
                  "rcclEnv": json.loads(ann.get(ANN_ENV, "{}")),
                  "startTime": _now_iso(),
                  "conditions": [{"type": "Scheduled", "status": "True", "reason": "Bound",
                                  "lastTransitionTime": _now_iso()}]}
            self.kube.patch_cr_status("GPUWorkload", ns, wl, st)

    def _is_current_pod(self, ns: str, wl: str, name: str) -> bool:
        try:
            st = self.kube.get_cr("GPUWorkload", ns, wl).get("status") or {}
        except ApiError:
            return True
        return st.get("podName", name) == name

    # ------------------------------------------------------------- failures
    def _watch_nodes(self):
        self._loop("/api/v1/nodes", self.on_node)

    def on_node(self, typ: str, node: dict):
        name = node.get("metadata", {}).get("name", "")
        if typ == "DELETED":
            self.evict_node(name, "node deleted")
            self.p.remove_node(name)
            return
        ready = next((c.get("status") for c in (node.get("status") or {}).get("conditions") or []
                      if c.get("type") == "Ready"), "True")
        if ready != "True":
            if name not in self._lost_nodes:
                self._lost_nodes.add(name)
                self.p.set_cordon(name, True)  # before eviction: replacements go elsewhere
                self.evict_node(name, f"node NotReady (Ready={ready})")
        elif name in self._lost_nodes:
            self._lost_nodes.discard(name)
            self.p.set_cordon(name, False)

    def evict_node(self, node: str, reason: str) -> int:
        n = 0
        for a in self.p.allocations():
            if a.get("node") == node:
                self.evict(a, reason)
                n += 1
        return n

    def health_sweep(self) -> int:
        """Evict allocations holding a GPU (or a slice of one) that the health
        policy marks Unhealthy."""
        snap = self.p.snapshot().get("nodes", {})
        n = 0
        for a in self.p.allocations():
            gpus = {g["uuid"]: g for g in (snap.get(a.get("node")) or {}).get("gpus", [])}
            held = list(a.get("gpus", [])) + [p.rsplit("/p", 1)[0] for p in a.get("partitions", [])]
            bad = [u for u in held if gpus.get(u, {}).get("health", {}).get("status") == "Unhealthy"]
            if bad:
                why = "; ".join(gpus[bad[0]]["health"].get("reasons") or ["unhealthy"])
                self.evict(a, f"GPU {bad[0]} Unhealthy: {why}")
                n += 1
        return n

    def evict(self, alloc: dict, reason: str, migration: bool = False) -> None:
        """Release an allocation whose node or GPU failed; reschedule or fail
        its GPUWorkload per spec.recovery.  migration=True (partition
        consolidation): always reschedule, without using the recovery budget."""
        uid = alloc["uid"]
        self._running.pop(uid, None)
        pod = next((p for p in self.kube.list_pods(alloc.get("namespace"))
                    if (p["metadata"].get("uid") or "") == uid), None)
        self._evicting.add(uid)
        self.p.release(uid)
        if pod is None:
            self._evicting.discard(uid)
            return
        md = pod["metadata"]
        ns = md.get("namespace", "default")
        wl = (md.get("labels") or {}).get(LABEL_WORKLOAD)
        self.kube.delete_pod(ns, md["name"])
        if not wl:
            return
        try:
            gw = self.kube.get_cr("GPUWorkload", ns, wl)
        except ApiError:
            return
        gw = crds.default(gw)
        rec = gw["spec"].get("recovery") or {}
        restarts = int((gw.get("status") or {}).get("restarts") or 0)
        if migration:
            st = gw.get("status") or {}
            self.kube.patch_cr_status("GPUWorkload", ns, wl, {
                "phase": "Pending", "migrations": int(st.get("migrations") or 0) + 1,
                "restarts": restarts + 1,  # pod name generation; recovery budget below is separate
                "recoveryRestarts": int(st.get("recoveryRestarts", restarts) or 0),
                "scheduledNode": "", "allocatedGPUs": [], "partitionSlices": [],
                "conditions": [{"type": "Migrated", "status": "True", "reason": "PartitionConsolidation",
                                "message": reason, "lastTransitionTime": _now_iso()}]})
            return
        gen = restarts
        restarts = int((gw.get("status") or {}).get("recoveryRestarts", restarts) or 0)
        cond = {"type": "Evicted", "status": "True", "reason": "NodeOrGPUFailure", "message": reason,
                "lastTransitionTime": _now_iso()}
        if rec.get("policy", "Reschedule") == "Reschedule" and restarts < int(rec.get("maxRestarts", 3)):
            self.kube.patch_cr_status("GPUWorkload", ns, wl, {
                "phase": "Pending", "restarts": gen + 1, "recoveryRestarts": restarts + 1,
                "lastFailure": reason,
                "scheduledNode": "", "allocatedGPUs": [], "partitionSlices": [], "conditions": [cond]})
            # The status watch event (phase Pending) drives on_workload: a fresh
            # pod, which the scheduler places away from the failure.
        else:
            self.kube.patch_cr_status("GPUWorkload", ns, wl, {
                "phase": "Failed", "lastFailure": reason, "restarts": gen, "recoveryRestarts": restarts,
                "message": f"evicted: {reason}", "completionTime": _now_iso(), "conditions": [cond]})

    # ------------------------------------------------------------- GPUBudget
    def _watch_budgets(self):
        self._loop(f"/apis/{crds.GROUP}/{crds.VERSION}/gpubudgets", self.on_budget)

    def on_budget(self, typ: str, b: dict):
        if typ == "DELETED":
            return
        b = crds.default(b)
        errs = crds.validate(b)
        md = b["metadata"]
        if errs:
            self.kube.patch_cr_status("GPUBudget", md.get("namespace"), md["name"],
                                      {"conditions": [{"type": "Valid", "status": "False",
                                                       "message": "; ".join(errs)}]})
            return
        if typ == "ADDED" or "currentSpend" not in (b.get("status") or {}):
            spec = dict(b["spec"])
            if spec.get("scope", "Namespace") == "Namespace":
                spec.setdefault("scopeId", md.get("namespace", "default"))
            elif spec.get("scope") == "Team":
                spec.setdefault("scopeId", spec.get("teamId", ""))
            self.p.create_budget({"metadata": md, "spec": spec})

    def _budget_status(self):
        for b in self.p.budgets():
            ns, _, name = b["id"].rpartition("/")
            alerts = [a for a in self.p.alerts() if a["budget_id"] == b["id"]]
            try:
                self.kube.patch_cr_status("GPUBudget", ns or None, name, {
                    "currentSpend": f"{b['spend']:.2f}", "utilizationPercent": round(b["utilization_percent"], 2),
                    "periodStart": datetime.fromtimestamp(b["period_start_s"], timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
                    "periodEnd": datetime.fromtimestamp(b["period_end_s"], timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
                    "alerts": [{"severity": a["severity"], "threshold": a["threshold"], "message": a["message"]}
                               for a in alerts[-10:]]})
            except ApiError:
                pass

    # ------------------------------------------------------------- PartitionStrategy
    def _watch_strategies(self):
        self._loop(f"/apis/{crds.GROUP}/{crds.VERSION}/partitionstrategies", self.on_strategy)

    def on_strategy(self, typ: str, s: dict):
        name = s["metadata"]["name"]
        if typ == "DELETED":
            self._strategy_next.pop(name, None)
            return
        s = crds.default(s)
        err = "; ".join(crds.validate(s)) or self.p.register_strategy(s)
        if err:
            self.kube.patch_cr_status("PartitionStrategy", None, name, {
                "conditions": [{"type": "Valid", "status": "False", "message": err}]})
            return
        self._strategy_next[name] = 0.0  # rebalance at next tick

    def _rebalance_due(self, now: float):
        for st in self.p.strategies():
            name = st["name"]
            if name not in self._strategy_next or now < self._strategy_next[name]:
                continue
            ops = self.p.rebalance(name)
            self._strategy_next[name] = now + max(1, st.get("rebalanceIntervalSeconds", 300))
            dist: dict = {}
            for g in (n for nd in self.p.snapshot()["nodes"].values() for n in nd["gpus"]):
                dist[g["partition"]["compute"]] = dist.get(g["partition"]["compute"], 0) + 1
            try:
                self.kube.patch_cr_status("PartitionStrategy", None, name, {
                    "lastRebalanceTime": _now_iso(), "currentDistribution": dist,
                    "appliedNodes": sorted({o["node"] for o in ops}),
                    "conditions": [{"type": "Rebalanced", "status": "True",
                                    "message": f"{len(ops)} reconfiguration(s)"}]})
            except ApiError:
                pass

    # ------------------------------------------------------------- periodic
    def _periodic(self):
        while not self._stop.wait(self.tick_s):
            self.tick_once(time.time())

    def tick_once(self, now: float) -> None:
        # Each step fails on its own: one broken step neither hides the error
        # nor starves the others.  Errors are logged and counted
        # (kgwe_controller_errors_total on /metrics via the platform).
        for name, step in (("telemetry", self.p.refresh_telemetry), ("health", self.health_sweep),
                           ("tick", lambda: self.p.tick(now)), ("rebalance", lambda: self._rebalance_due(now)),
                           ("consolidate", lambda: self._consolidate(now)),
                           ("optimizer", lambda: self._feed_optimizer(now)),
                           ("budgets", self._budget_status)):
            try:
                step()
            except Exception as e:  # noqa: BLE001
                self.errors += 1
                log.exception("controller %s step failed: %s", name, e)
                try:
                    self.p.count_error(name)
                except Exception:  # noqa: BLE001
                    pass

    # ------------------------------------------------------------- consolidation
    def _consolidate(self, now: float) -> None:
        if not self.consolidate:
            return
        for m in self.p.consolidate_partitions(now, plan_only=True):
            alloc = next((a for a in self.p.allocations() if a["uid"] == m["uid"]), None)
            if alloc is None:
                continue
            self.migrations += 1
            self.evict(alloc, f"partition consolidation: {m['from']} -> a fuller GPU", migration=True)

    # ------------------------------------------------------------- optimizer loop
    def _hint_view(self, k: int) -> tuple[list, dict]:
        """(busy GPU uuids, snapshot restricted to the nodes with the most free
        GPUs) — GetPlacement sees the ledger and a bounded candidate set, not
        the whole fleet per workload."""
        snap = self.p.snapshot()
        busy = set()
        for a in self.p.allocations():
            busy.update(a.get("gpus", []))
            if a.get("shared_gpu"):
                busy.add(a["shared_gpu"])
            busy.update(p.rsplit("/p", 1)[0] for p in a.get("partitions", []))
        nodes = snap.get("nodes", {})
        free = {n: sum(1 for g in v["gpus"] if g["uuid"] not in busy) for n, v in nodes.items()}
        keep = sorted((n for n in nodes if free[n] >= k), key=lambda n: (-free[n], n))[:HINT_CANDIDATE_NODES]
        return sorted(busy), {"nodes": {n: nodes[n] for n in keep}}

    def _recommend(self, ns: str, name: str, spec: dict) -> dict | None:
        try:
            hints = {"workload_type": spec.get("workloadType", "Training"),
                     "framework": spec.get("framework"),
                     "strategy": (spec.get("distributedConfig") or {}).get("strategy")}
            if spec.get("modelParamsBillions") is not None:
                hints["model_params_billions"] = float(spec["modelParamsBillions"])
            pr = self.optimizer.PredictResources({"workload_id": f"{ns}/{name}", "hints": hints})
        except Exception as e:  # noqa: BLE001
            log.warning("PredictResources for %s/%s failed: %s", ns, name, e)
            return None
        if not pr or pr.get("error"):
            return None
        return {"gpus": pr.get("recommended_gpus"), "memoryGB": pr.get("recommended_memory_gb"),
                "partition": pr.get("recommended_partition"),
                "expectedUtilization": round(float(pr.get("expected_utilization") or 0.0), 1),
                "confidence": round(float(pr.get("confidence") or 0.0), 3),
                "costPerHour": round(float(pr.get("estimated_cost_per_hour") or 0.0), 3),
                "reasoning": pr.get("reasoning", [])[-3:], "updated": _now_iso()}

    def _feed_optimizer(self, now: float) -> None:
        if self.optimizer is None or not self._running:
            return
        gpus = {g["uuid"]: g for n in self.p.snapshot().get("nodes", {}).values() for g in n["gpus"]}
        for a in self.p.allocations():
            run = self._running.get(a["uid"])
            if run is None:
                continue
            held = list(a.get("gpus", [])) + ([a["shared_gpu"]] if a.get("shared_gpu") else []) + \
                [p.rsplit("/p", 1)[0] for p in a.get("partitions", [])]
            samples = []
            for u in held:
                g = gpus.get(u)
                if g is None:
                    continue
                samples.append({"timestamp": now, "gpu_uuid": u,
                                "gpu_utilization": float(g["util"]["gfx_activity"]),
                                "memory_used_bytes": int(g["memory_used_gb"] * 2**30),
                                "memory_total_bytes": int(max(1.0, g["memory_total_gb"]) * 2**30),
                                "power_watts": float(g["util"]["power_w"]),
                                "temperature_celsius": float(g["util"]["temperature_c"])})
            if samples:
                # one sample per allocation per tick: the mean over its GPUs
                n = len(samples)
                agg = dict(samples[0])
                for k in ("gpu_utilization", "power_watts", "temperature_celsius"):
                    agg[k] = sum(x[k] for x in samples) / n
                agg["memory_used_bytes"] = sum(x["memory_used_bytes"] for x in samples) // n
                self.optimizer.IngestTelemetry({"workload_id": f"{run[0]}/{run[1]}", "samples": [agg]})
        if now >= self._next_recommend:
            self._next_recommend = now + self.recommend_every_s
            for uid, (ns, wl, _) in list(self._running.items()):
                try:
                    gw = self.kube.get_cr("GPUWorkload", ns, wl)
                except ApiError:
                    continue
                rec = self._recommend(ns, wl, gw.get("spec") or {})
                if rec:
                    self.kube.patch_cr_status("GPUWorkload", ns, wl, {"recommendation": rec})
