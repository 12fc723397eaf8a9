"""Scheduling-latency benchmark: pod create -> bind p99 through the full stack.

Four OS processes, like a real control plane (all traffic is real HTTP):
  * apiserver  — FakeApiServer (nodes, pods, bindings, watch);
  * scheduler  — SchedulerSim, the kube-scheduler cycle for the
                 ``kgwe-scheduler`` profile (watch -> filter -> prioritize ->
                 bind against the extender, nodeCacheCapable=false);
  * controller — the ExtenderServer on top of the C++ core (discovery
                 snapshot of a mocked fleet of 8xMI355X nodes, scheduler,
                 partition controller, cost engine) and its housekeeping;
  * load driver — this process: pod creation, the pod reaper (delete, then
                 the controller releases) and the latency bookkeeping.

Workload mix (Poisson arrivals at `rate` pods/s; every pod is deleted and its
allocation released after a random lifetime, so the fleet stays busy but not
full): 8-GPU FSDP training (the flagship job shape), 4/2/1-GPU jobs and
CPX-slice inference pods (which drive partition auto-provisioning).

Latency = CLOCK_MONOTONIC (perf_counter, shared by all processes) from just
before the pod POST to the moment the bind verb returned success — the KPI's
definition, "time from pod creation to GPU binding" (reference
docs/PRD.md:440).  Quantiles come from the native log-linear histogram,
never a running max (the reference's "P99", scheduler.go:818).  The
product's own ``kgwe_scheduling_latency_ms`` histogram (fed by the
extender's bind from the pods' admission stamps) is reported beside it.

Scale / pressure knobs:
  --full-nodes    kube-like Node objects (~7 KB: labels, conditions, images,
                  nodeInfo) in the apiserver, so nodeCacheCapable=false
                  ExtenderArgs carry ~9 MB at 1,250 nodes;
  --node-cache    nodeCacheCapable=true (node names only);
  --nodes-to-score  the profile's percentageOfNodesToScore.  The chart sets 100:
                  the extender's verbs cost ~1 us per node, and a sampled
                  window (kube's adaptive default: 40 % of 1,250 nodes) hides
                  free partition slices and xGMI groups on the nodes outside
                  it, so slice pods provision fresh partitioned GPUs instead
                  of filling existing ones;
  --lifetime      pod lifetimes; long lifetimes fill the fleet, so pods queue
                  and high-priority pods preempt through the extender's
                  preempt verb.  Then ``sched_p99_ms`` (pods bound on their
                  first cycle) and ``p99_ms`` (every pod, queue wait
                  included) differ, and queue depth / preemption rate are
                  real.
"""
from __future__ import annotations

import argparse
import gc
import heapq
import json
import multiprocessing as mp
import os
import queue
import random
import sys
import threading
import time

MIX = [  # (weight, kind, gpus)
    (0.10, "fsdp", 8), (0.15, "train", 4), (0.20, "train", 2), (0.35, "train", 1),
    (0.20, "cpx", 1),
]


def _pod(name: str, kind: str, gpus: int, priority: int, preemptible: bool = True) -> dict:
    from ..controller.schedsim import SCHEDULER_NAME

    ann = {"kgwe.amd.com/topology": "xGMIOptimal" if gpus > 1 else "None",
           "kgwe.amd.com/workload-type": "Inference" if kind == "cpx" else "Training",
           # what kgwe's mutating webhook stamps at admission (kgwe.api.webhook)
           "kgwe.amd.com/created-at": f"{time.time():.6f}"}
    if kind == "fsdp":
        ann["kgwe.amd.com/strategy"] = "FSDP"
    if not preemptible:
        ann["kgwe.amd.com/preemptible"] = "false"
    res = {"amd.com/gpu-cpx": "1"} if kind == "cpx" else {"amd.com/gpu": str(gpus)}
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "bench", "annotations": ann,
                         "labels": {"kgwe.amd.com/team": "team-" + kind}},
            "spec": {"schedulerName": SCHEDULER_NAME, "priority": priority,
                     "containers": [{"name": "main", "image": "rocm/pytorch",
                                     "resources": {"limits": res}}]}}


def full_node(name: str, i: int, gpus: int = 8) -> dict:
    """A Node object of kube-typical size (~7 KB)."""
    labels = {"kubernetes.io/hostname": name, "kubernetes.io/os": "linux", "kubernetes.io/arch": "amd64",
              "node.kubernetes.io/instance-type": "mi355x-8gpu", "topology.kubernetes.io/zone": f"zone-{i % 4}",
              "topology.kubernetes.io/region": "region-1", "amd.com/gpu.product": "MI355X",
              "amd.com/gpu.count": str(gpus), "amd.com/gpu.family": "CDNA4", "amd.com/gpu.vram": "288G",
              "feature.node.kubernetes.io/cpu-model.vendor_id": "AMD", "beta.kubernetes.io/os": "linux",
              "feature.node.kubernetes.io/kernel-version.full": "6.8.0-45-generic",
              "node-role.kubernetes.io/gpu": "", "pool": f"pool-{i % 8}"}
    images = [{"names": [f"registry.example.com/team/image-{k}@sha256:{(i * 131 + k):064x}",
                         f"registry.example.com/team/image-{k}:v1.{k}"], "sizeBytes": 1_000_000_000 + k}
              for k in range(20)]
    conds = [{"type": t, "status": "True" if t == "Ready" else "False",
              "lastHeartbeatTime": "2026-10-16T00:00:00Z", "lastTransitionTime": "2026-10-01T00:00:00Z",
              "reason": f"Kubelet{t}", "message": f"kubelet reports {t}"}
             for t in ("MemoryPressure", "DiskPressure", "PIDPressure", "NetworkUnavailable", "Ready")]
    alloc = {"cpu": "191", "memory": "2100000000Ki", "pods": "110", "amd.com/gpu": str(gpus),
             "ephemeral-storage": "3450000000Ki", "hugepages-1Gi": "0"}
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "uid": f"{i:08x}-aaaa-bbbb-cccc-{i:012x}", "resourceVersion": str(100000 + i),
                         "creationTimestamp": "2026-01-01T00:00:00Z", "labels": labels,
                         "annotations": {"node.alpha.kubernetes.io/ttl": "0",
                                         "volumes.kubernetes.io/controller-managed-attach-detach": "true"}},
            "spec": {"podCIDR": f"10.{i // 256}.{i % 256}.0/24", "providerID": f"provider://zone/{name}",
                     "taints": []},
            "status": {"capacity": dict(alloc, cpu="192"), "allocatable": alloc, "conditions": conds,
                       "addresses": [{"type": "InternalIP", "address": f"10.128.{i // 256}.{i % 256}"},
                                     {"type": "Hostname", "address": name}],
                       "daemonEndpoints": {"kubeletEndpoint": {"Port": 10250}},
                       "nodeInfo": {"machineID": f"{i:032x}", "systemUUID": f"{i * 7:032x}", "bootID": f"{i * 3:032x}",
                                    "kernelVersion": "6.8.0-45-generic", "osImage": "Ubuntu 22.04.4 LTS",
                                    "containerRuntimeVersion": "containerd://1.7.12", "kubeletVersion": "v1.30.4",
                                    "kubeProxyVersion": "v1.30.4", "operatingSystem": "linux",
                                    "architecture": "amd64"},
                       "images": images}}


def _apiserver_proc(conn):
    from ..controller.apiserver import FakeApiServer

    sys.setswitchinterval(0.0005)  # threaded stand-in for a Go apiserver
    api = FakeApiServer().start()
    conn.send(api.url)
    while conn.recv() != "stop":  # "freeze": the fleet is loaded
        gc.freeze()
    api.stop()


def _scheduler_proc(api_url: str, ext_url: str, bound_q, stop_ev, ready_ev, node_cache: bool,
                    nodes_to_score: float = 100.0):
    from ..controller.kube import KubeClient
    from ..controller.schedsim import SchedulerSim

    def on_bound(pod, node, t):
        uid = pod["metadata"].get("uid", "")
        bound_q.put((pod["metadata"]["name"], uid, t, uid in sim.retried, pod.get("_kgwe_t") or {}))

    def on_preempted(victims):
        bound_q.put(("__preempted__", json.dumps(victims), 0.0, False))

    # The stand-in is a threaded CPython process (watch, cycle, informer, 4
    # binders): hand the GIL over at 0.5 ms instead of 5 ms, so the cycle
    # thread is not parked behind a binder's JSON work (Go has no such lock).
    sys.setswitchinterval(0.0005)
    # static fleet: the node list is cached like kube-scheduler's informer
    sim = SchedulerSim(KubeClient(api_url), ext_url, on_bound=on_bound, on_preempted=on_preempted,
                       node_cache_capable=node_cache, node_refresh_s=60.0,
                       percentage_of_nodes_to_score=nodes_to_score).start()
    ready_ev.set()
    stop_ev.wait()
    sim.stop()
    bound_q.put(("__stats__", json.dumps(sim.stats), 0.0, False))


def _controller_proc(conn, api_url: str, n_nodes: int, full_nodes: bool, tick_s: float,
                     reclaim_idle_s: float, parent_api=None, mean_lifetime_s: float = 0.0):
    """The kgwe controller: ExtenderServer on the C++ core plus its periodic
    housekeeping, alone in its process as in production (the load driver's
    threads must not share its GIL).  Commands over `conn`:
    ("release", [uids]) — pods deleted (the controller's pod watch);
    ("preempted", [uids]) — victims evicted by kube-scheduler;
    ("stop", None) — reply with the controller-side results."""
    from ..controller.kube import KubeClient
    from ..core import Platform, make_fixture
    from ..extender.server import ExtenderServer

    sys.setswitchinterval(0.001)  # as kgwe.controller.main sets it for the extender's threads
    kube = KubeClient(api_url)
    # Housekeeping as the controller runs it (tick: gang expiry, cost sampling,
    # idle-partition reclaim).  Pod lifetimes here are seconds, not hours, so
    # the reclaim hysteresis is scaled down with them (production default 60 s).
    # Likewise the preemption policy's clocks: production waits for jobs within
    # 30 s of their expected end (of hours); here within a fifth of the mean
    # lifetime, for at most one mean lifetime.  Lifetimes are not declared by
    # the pods: the scheduler learns them per workload type from releases.
    sched_cfg = ({"preemptionWaitWindowSeconds": 0.2 * mean_lifetime_s,
                  "preemptionMaxWaitSeconds": mean_lifetime_s} if mean_lifetime_s > 0 else {})
    plat = Platform({"enforceBudgets": True, "partitionReclaimIdleSeconds": reclaim_idle_s,
                     # consolidation's hysteresis and per-pod cooldown, scaled the same way
                     # (production: 120 s below 75 % occupancy, one move per pod per hour)
                     "partitionConsolidateAfterSeconds": reclaim_idle_s,
                     "migrationCooldownSeconds": 4.0 * reclaim_idle_s,
                     "scheduler": sched_cfg})
    for i in range(n_nodes):
        name = f"mi355x-{i:03d}"
        plat.add_fake_node(make_fixture(name, 8, 2))
        kube.create_node(full_node(name, i) if full_nodes else
                         {"apiVersion": "v1", "kind": "Node",
                          "metadata": {"name": name, "labels": {"kubernetes.io/hostname": name,
                                                                "amd.com/gpu.product": "MI355X"}},
                          "status": {"allocatable": {"amd.com/gpu": "8"}}})
    ext = ExtenderServer(plat, kube=kube, host="127.0.0.1", port=0).start()
    if parent_api is not None:
        parent_api.send("freeze")  # every Node object is in the apiserver now
    gc.freeze()
    done = threading.Event()
    slice_util: list[float] = []
    queue_depth: list[int] = []

    def partition_sampler():  # time-average of CPX/QPX/DPX slice occupancy
        while not done.is_set():
            m = plat.partition_metrics()
            if any(k != "SPX" and v.get("gpus", 0) for k, v in m.get("modes", {}).items()):
                slice_util.append(m.get("slice_utilization", 0.0))
            time.sleep(0.1)

    def housekeeping():
        while not done.is_set():
            plat.tick()
            plat.consolidate_partitions(plan_only=False)  # the controller's consolidation (ledger move)
            queue_depth.append(plat.queue_depth())
            time.sleep(tick_s)

    threading.Thread(target=partition_sampler, daemon=True).start()
    threading.Thread(target=housekeeping, daemon=True).start()
    conn.send(ext.url)
    while True:
        cmd, arg = conn.recv()
        if cmd == "release":
            for uid in arg:
                plat.release(uid)
        elif cmd == "preempted":
            for uid in arg:
                plat.release(uid)
            plat.count_preemptions(len(arg))
        elif cmd == "stop":
            done.set()
            sm = plat.scheduler_metrics()
            pm = plat.partition_metrics()
            conn.send({
                "queue_depth_max": max(queue_depth) if queue_depth else 0,
                "queue_depth_mean": round(sum(queue_depth) / len(queue_depth), 2) if queue_depth else 0.0,
                "core_schedule_p99_ms": round(sm.get("p99_ms", 0.0), 3),
                # the product's own kgwe_scheduling_latency_ms histogram, fed by the
                # extender's bind from the pods' admission stamps (not by this harness)
                "extender_histogram_p99_ms": round(plat.pod_latency_quantile_ms(0.99), 3),
                "extender_histogram_count": plat.pod_latency_count(),
                "partition_reconfigs": pm.get("ops_total", 0),
                # reference "MIG instance utilization 92 %" (README.md:160): share of
                # partition slices in use on partitioned GPUs, time-averaged over the run
                "partition_slice_utilization_pct": (round(100.0 * sum(slice_util) / len(slice_util), 2)
                                                    if slice_util else None),
                "partition_slice_samples": len(slice_util),
                "topology_optimal_placements": sm.get("topology_optimal", 0),
                "preemptions_deferred_wait": sm.get("preemptions_deferred_wait", 0),
                "preemptions_rate_limited": sm.get("preemptions_rate_limited", 0),
                "extender_phases_ms": ext.phase_summary(),
                "extender_server": {k: v for k, v in ext.stats().items() if k != "verbs"},
            })
            ext.stop()
            return


def run(n_pods: int = 2000, job_gpus: int = 8, n_nodes: int = 64, rate: float = 50.0,
        lifetime_s: tuple = (0.5, 3.0), seed: int = 7, timeout_s: float = 300.0,
        tick_s: float = 1.0, reclaim_idle_s: float = 2.0, full_nodes: bool = False,
        node_cache: bool = False, nodes_to_score: float = 100.0) -> dict:
    from ..controller.kube import KubeClient
    from ..core import LatencyHistogram

    ctx = mp.get_context("fork")
    rnd = random.Random(seed)
    parent, child = ctx.Pipe()
    api_p = ctx.Process(target=_apiserver_proc, args=(child,), daemon=True)
    api_p.start()
    api_url = parent.recv()
    kube = KubeClient(api_url)
    ctl, ctl_child = ctx.Pipe()
    ctl_p = ctx.Process(target=_controller_proc, args=(ctl_child, api_url, n_nodes, full_nodes, tick_s,
                                                       reclaim_idle_s, parent, 0.5 * sum(lifetime_s)),
                        daemon=True)
    ctl_p.start()
    ext_url = ctl.recv()
    ctl_lock = threading.Lock()

    def ctl_send(cmd, arg):
        with ctl_lock:
            ctl.send((cmd, arg))

    bound_q = ctx.Queue()
    stop_ev, ready_ev = ctx.Event(), ctx.Event()
    sch_p = ctx.Process(target=_scheduler_proc, args=(api_url, ext_url, bound_q, stop_ev, ready_ev, node_cache,
                              nodes_to_score),
                        daemon=True)
    sch_p.start()
    ready_ev.wait(timeout=120)  # node cache synced

    hist, job_hist, first_hist = LatencyHistogram(), LatencyHistogram(), LatencyHistogram()
    created: dict[str, float] = {}
    preempted: list[str] = []
    phase: dict = {}
    sim_stats: dict = {}
    lock = threading.Lock()
    n_bound = [0]
    all_done = threading.Event()
    reaper_kube = KubeClient(api_url)

    def consumer():
        while not all_done.is_set():
            try:
                name, uid, t, was_retried, *tt = bound_q.get(timeout=0.2)
            except queue.Empty:
                continue
            if name == "__stats__":
                sim_stats.update(json.loads(uid))
                continue
            if name == "__preempted__":  # kube-scheduler evicted them: the controller releases
                victims = json.loads(uid)
                ctl_send("preempted", victims)
                preempted.extend(victims)
                continue
            with lock:
                t0 = created.pop(name, None)
                name_of[uid] = name
                n_bound[0] += 1
                finished = n_bound[0] >= n_pods + 1
            if t0 is not None:  # the harness's own clock; bind() feeds the product's histogram
                ms = (t - t0) * 1000.0
                (job_hist if name.startswith("job-") else hist).record_ms(ms)
                if not was_retried:
                    first_hist.record_ms(ms)
                    tt = tt[0] if tt else {}
                    if tt.get("seen") and tt.get("bind"):  # where the time went (one clock: CLOCK_MONOTONIC)
                        for k, a, b in (("apiserver_watch", t0, tt["seen"]), ("sched_queue", tt["seen"], tt["cycle"]),
                                        ("filter_prioritize", tt["cycle"], tt["bind_q"]),
                                        ("bind_queue", tt["bind_q"], tt["bind"]), ("bind", tt["bind"], t)):
                            phase.setdefault(k, LatencyHistogram()).record_ms(max(0.0, (b - a) * 1000.0))
            with lock:
                heapq.heappush(expiry, (time.perf_counter() + rnd.uniform(*lifetime_s), name, uid))
            if finished:
                all_done.set()

    def reaper():  # one thread, one keep-alive connection: delete, then the controller releases
        while not all_done.is_set():
            now = time.perf_counter()
            due = []
            with lock:
                while expiry and expiry[0][0] <= now:
                    due.append(heapq.heappop(expiry))
            for _, name, uid in due:
                reaper_kube.delete_pod("bench", name)
            if due:
                ctl_send("release", [uid for _, _, uid in due])
            time.sleep(0.01)

    expiry: list = []
    protected: set[str] = set()
    name_of: dict[str, str] = {}
    threading.Thread(target=consumer, daemon=True).start()
    threading.Thread(target=reaper, daemon=True).start()
    time.sleep(0.3)  # scheduler process: first watch established
    t_start = time.perf_counter()
    with lock:
        created["job-fsdp"] = time.perf_counter()
    kube.create_pod(_pod("job-fsdp", "fsdp", job_gpus, 1000))
    weights = [m[0] for m in MIX]
    next_t = time.perf_counter()
    for i in range(n_pods):
        _, kind, g = rnd.choices(MIX, weights)[0]
        name = f"p{i:05d}"
        next_t += rnd.expovariate(rate)
        delay = next_t - time.perf_counter()
        if delay > 0:
            time.sleep(delay)
        with lock:
            created[name] = time.perf_counter()
        # priority classes: 90 % best effort (0), 8 % production (100), 2 % critical (1000);
        # a fifth of the best-effort pods declare themselves non-preemptible
        pr = rnd.random()
        keep = pr < 0.90 and rnd.random() < 0.2
        if keep:
            protected.add(name)
        kube.create_pod(_pod(name, kind, g, 0 if pr < 0.90 else 100 if pr < 0.98 else 1000, not keep))
    all_done.wait(timeout=timeout_s)
    wall = time.perf_counter() - t_start
    stop_ev.set()
    sch_p.join(timeout=5)
    try:  # the simulator's final stats message (the consumer has stopped by now)
        while True:
            m = bound_q.get(timeout=2.0)
            if m[0] == "__stats__":
                sim_stats.update(json.loads(m[1]))
                break
    except queue.Empty:
        pass
    ctl_send("stop", None)
    ctl_res = ctl.recv()
    ctl_p.join(timeout=5)
    parent.send("stop")
    api_p.join(timeout=5)
    out = {
        "pods": n_pods + 1, "bound": n_bound[0], "nodes": n_nodes, "gpus": n_nodes * 8,
        "arrival_rate_per_s": rate, "lifetime_s": list(lifetime_s),
        "node_objects": "full (~7 KB each)" if full_nodes else "minimal",
        "node_cache_capable": node_cache,
        # the kgwe-scheduler profile's percentageOfNodesToScore (0: kube's adaptive default)
        "percentage_of_nodes_to_score": nodes_to_score,
        # pods bound on their FIRST scheduling cycle: the scheduler's own latency
        "sched_p50_ms": round(first_hist.quantile_ms(0.50), 3),
        "sched_p99_ms": round(first_hist.quantile_ms(0.99), 3),
        "sched_count": first_hist.count(),
        "queued_pods": n_bound[0] - first_hist.count(),
        "p50_ms": round(hist.quantile_ms(0.50), 3), "p90_ms": round(hist.quantile_ms(0.90), 3),
        "p99_ms": round(hist.quantile_ms(0.99), 3), "max_ms": round(hist.max_ms(), 3),
        "mean_ms": round(hist.mean_ms(), 3),
        "fsdp_job_latency_ms": round(job_hist.max_ms(), 3),
        "throughput_pods_per_s": round(n_bound[0] / wall, 1),
        # PRD KPI "preemption rate < 5 %" (docs/PRD.md:444): preemptions per bound pod
        "preemptions": len(preempted),
        "preemption_rate_pct": round(100.0 * len(preempted) / max(1, n_bound[0]), 3),
        "preempt_verb_calls": sim_stats.get("preempt_calls"),
        "non_preemptible_pods": len(protected),
        "non_preemptible_evicted": sum(1 for v in preempted if name_of.get(v, v) in protected),
        "first_cycle_breakdown_ms": {k: {"p50": round(h.quantile_ms(0.5), 3), "p99": round(h.quantile_ms(0.99), 3)}
                                     for k, h in phase.items()},
        "scheduler_round_trips_ms": {k[:-6]: v for k, v in sim_stats.items() if k.endswith("_rt_ms")},
        "processes": "apiserver | kube-scheduler sim | controller (extender+core) | load driver",
    }
    out.update(ctl_res)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--rate", type=float, default=50.0)
    ap.add_argument("--job-gpus", type=int, default=8)
    ap.add_argument("--lifetime", default="0.5,3.0", help="min,max pod lifetime seconds")
    ap.add_argument("--full-nodes", action="store_true")
    ap.add_argument("--node-cache", action="store_true", help="nodeCacheCapable=true (names only)")
    ap.add_argument("--nodes-to-score", type=float, default=100.0,
                    help="the profile's percentageOfNodesToScore (chart default 100; 0 = kube-scheduler's "
                         "adaptive default, 40 %% of 1,250 nodes)")
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--then-nodes", type=int, default=0,
                    help="afterwards run the same load on a fleet of this many nodes "
                         "(reported under 'fleet_<n>_nodes')")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    lo, hi = (float(x) for x in a.lifetime.split(","))
    res = run(n_pods=a.pods, job_gpus=a.job_gpus, n_nodes=a.nodes, rate=a.rate, lifetime_s=(lo, hi),
              full_nodes=a.full_nodes, node_cache=a.node_cache, timeout_s=a.timeout,
              nodes_to_score=a.nodes_to_score)
    if a.then_nodes:
        res[f"fleet_{a.then_nodes}_nodes"] = run(
            n_pods=a.pods, job_gpus=a.job_gpus, n_nodes=a.then_nodes, rate=a.rate, lifetime_s=(lo, hi),
            full_nodes=a.full_nodes, node_cache=a.node_cache, timeout_s=a.timeout,
            nodes_to_score=a.nodes_to_score)
    print(json.dumps(res) if a.json else json.dumps(res, indent=1), flush=True)
    os._exit(0)  # reaper timers / daemon threads: do not wait for them


if __name__ == "__main__":
    main()
