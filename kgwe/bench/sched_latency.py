"""Scheduling-latency benchmark: pod create -> bind p99 through the full stack.

Three OS processes, like a real control plane (all traffic is real HTTP):
  * apiserver  — FakeApiServer (nodes, pods, bindings, watch);
  * scheduler  — SchedulerSim, the kube-scheduler cycle for the
                 ``kgwe-scheduler`` profile (watch -> filter -> prioritize ->
                 bind against the extender, nodeCacheCapable=false);
  * controller — this process: the ExtenderServer on top of the C++ core
                 (discovery snapshot of a mocked fleet of 8xMI355X nodes,
                 scheduler, partition controller, cost engine) plus the load
                 driver and the pod reaper.

Workload mix (Poisson arrivals at `rate` pods/s; every pod is deleted and its
allocation released after a random lifetime, so the fleet stays busy but not
full): 8-GPU FSDP training (the flagship job shape), 4/2/1-GPU jobs and
CPX-slice inference pods (which drive partition auto-provisioning).

Latency = CLOCK_MONOTONIC (perf_counter, shared by all processes) from just
before the pod POST to the moment the bind verb returned success — the KPI's
definition, "time from pod creation to GPU binding" (reference
docs/PRD.md:440).  Quantiles come from the native log-linear histogram,
never a running max (the reference's "P99", scheduler.go:818).
"""
from __future__ import annotations

import argparse
import heapq
import json
import multiprocessing as mp
import os
import queue
import random
import threading
import time

MIX = [  # (weight, kind, gpus)
    (0.10, "fsdp", 8), (0.15, "train", 4), (0.20, "train", 2), (0.35, "train", 1),
    (0.20, "cpx", 1),
]


def _pod(name: str, kind: str, gpus: int, priority: int) -> dict:
    from ..controller.schedsim import SCHEDULER_NAME

    ann = {"kgwe.amd.com/topology": "xGMIOptimal" if gpus > 1 else "None",
           "kgwe.amd.com/workload-type": "Inference" if kind == "cpx" else "Training",
           # what kgwe's mutating webhook stamps at admission (kgwe.api.webhook)
           "kgwe.amd.com/created-at": f"{time.time():.6f}"}
    if kind == "fsdp":
        ann["kgwe.amd.com/strategy"] = "FSDP"
    res = {"amd.com/gpu-cpx": "1"} if kind == "cpx" else {"amd.com/gpu": str(gpus)}
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "bench", "annotations": ann,
                         "labels": {"kgwe.amd.com/team": "team-" + kind}},
            "spec": {"schedulerName": SCHEDULER_NAME, "priority": priority,
                     "containers": [{"name": "main", "image": "rocm/pytorch",
                                     "resources": {"limits": res}}]}}


def _apiserver_proc(conn):
    from ..controller.apiserver import FakeApiServer

    api = FakeApiServer().start()
    conn.send(api.url)
    conn.recv()  # block until told to stop
    api.stop()


def _scheduler_proc(api_url: str, ext_url: str, bound_q, stop_ev):
    from ..controller.kube import KubeClient
    from ..controller.schedsim import SchedulerSim

    def on_bound(pod, node, t):
        bound_q.put((pod["metadata"]["name"], pod["metadata"].get("uid", ""), t))

    sim = SchedulerSim(KubeClient(api_url), ext_url, on_bound=on_bound).start()
    stop_ev.wait()
    sim.stop()
    bound_q.put(("__stats__", json.dumps(sim.stats), 0.0))


def run(n_pods: int = 2000, job_gpus: int = 8, n_nodes: int = 64, rate: float = 50.0,
        lifetime_s: tuple = (0.5, 3.0), seed: int = 7, timeout_s: float = 300.0,
        tick_s: float = 1.0, reclaim_idle_s: float = 2.0) -> dict:
    from ..controller.kube import KubeClient
    from ..core import LatencyHistogram, Platform, make_fixture
    from ..extender.server import ExtenderServer

    ctx = mp.get_context("fork")
    rnd = random.Random(seed)
    parent, child = ctx.Pipe()
    api_p = ctx.Process(target=_apiserver_proc, args=(child,), daemon=True)
    api_p.start()
    api_url = parent.recv()
    kube = KubeClient(api_url)
    # Housekeeping as the controller runs it (tick: gang expiry, cost sampling,
    # idle-partition reclaim).  Pod lifetimes here are seconds, not hours, so
    # the reclaim hysteresis is scaled down with them (production default 60 s).
    plat = Platform({"enforceBudgets": True, "partitionReclaimIdleSeconds": reclaim_idle_s})
    for i in range(n_nodes):
        name = f"mi355x-{i:03d}"
        plat.add_fake_node(make_fixture(name, 8, 2))
        kube.create_node({"apiVersion": "v1", "kind": "Node",
                          "metadata": {"name": name, "labels": {"kubernetes.io/hostname": name,
                                                                "amd.com/gpu.product": "MI355X"}},
                          "status": {"allocatable": {"amd.com/gpu": "8"}}})
    ext = ExtenderServer(plat, kube=kube, host="127.0.0.1", port=0).start()
    bound_q = ctx.Queue()
    stop_ev = ctx.Event()
    sch_p = ctx.Process(target=_scheduler_proc, args=(api_url, ext.url, bound_q, stop_ev), daemon=True)
    sch_p.start()

    hist, job_hist = LatencyHistogram(), LatencyHistogram()
    created: dict[str, float] = {}
    lock = threading.Lock()
    n_bound = [0]
    all_done = threading.Event()
    reaper_kube = KubeClient(api_url)

    def consumer():
        while not all_done.is_set():
            try:
                name, uid, t = bound_q.get(timeout=0.2)
            except queue.Empty:
                continue
            if name == "__stats__":
                continue
            with lock:
                t0 = created.pop(name, None)
                n_bound[0] += 1
                finished = n_bound[0] >= n_pods + 1
            if t0 is not None:  # the harness's own clock; bind() feeds the product's histogram
                ms = (t - t0) * 1000.0
                (job_hist if name.startswith("job-") else hist).record_ms(ms)
            with lock:
                heapq.heappush(expiry, (time.perf_counter() + rnd.uniform(*lifetime_s), name, uid))
            if finished:
                all_done.set()

    def reaper():  # one thread, one keep-alive connection: delete + release
        while not all_done.is_set():
            now = time.perf_counter()
            due = []
            with lock:
                while expiry and expiry[0][0] <= now:
                    due.append(heapq.heappop(expiry))
            for _, name, uid in due:
                reaper_kube.delete_pod("bench", name)
                plat.release(uid)
            time.sleep(0.01)

    slice_util: list[float] = []

    def partition_sampler():  # time-average of CPX/QPX/DPX slice occupancy
        while not all_done.is_set():
            m = plat.partition_metrics()
            if any(k != "SPX" and v.get("gpus", 0) for k, v in m.get("modes", {}).items()):
                slice_util.append(m.get("slice_utilization", 0.0))
            time.sleep(0.1)

    def housekeeping():
        while not all_done.is_set():
            plat.tick()
            time.sleep(tick_s)

    expiry: list = []
    threading.Thread(target=consumer, daemon=True).start()
    threading.Thread(target=reaper, daemon=True).start()
    threading.Thread(target=partition_sampler, daemon=True).start()
    threading.Thread(target=housekeeping, daemon=True).start()
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
        kube.create_pod(_pod(name, kind, g, rnd.randint(0, 100)))
    all_done.wait(timeout=timeout_s)
    wall = time.perf_counter() - t_start
    stop_ev.set()
    sch_p.join(timeout=5)
    parent.send("stop")
    api_p.join(timeout=5)
    sm = plat.scheduler_metrics()
    pm = plat.partition_metrics()
    out = {
        "pods": n_pods + 1, "bound": n_bound[0], "nodes": n_nodes, "gpus": n_nodes * 8,
        "arrival_rate_per_s": rate,
        "p50_ms": round(hist.quantile_ms(0.50), 3), "p90_ms": round(hist.quantile_ms(0.90), 3),
        "p99_ms": round(hist.quantile_ms(0.99), 3), "max_ms": round(hist.max_ms(), 3),
        "mean_ms": round(hist.mean_ms(), 3),
        "fsdp_job_latency_ms": round(job_hist.max_ms(), 3),
        "throughput_pods_per_s": round(n_bound[0] / wall, 1),
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
        # PRD KPI "preemption rate < 5 %" (docs/PRD.md:444): preemptions per bound pod
        "preemptions": sm.get("preemptions", 0),
        "preemption_rate_pct": round(100.0 * sm.get("preemptions", 0) / max(1, n_bound[0]), 3),
        "extender_phases_ms": ext.tracer.summary(),
        "processes": "apiserver | kube-scheduler sim | extender+core",
    }
    ext.stop()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--rate", type=float, default=50.0)
    ap.add_argument("--job-gpus", type=int, default=8)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    res = run(n_pods=a.pods, job_gpus=a.job_gpus, n_nodes=a.nodes, rate=a.rate)
    print(json.dumps(res) if a.json else json.dumps(res, indent=1), flush=True)
    os._exit(0)  # reaper timers / daemon threads: do not wait for them


if __name__ == "__main__":
    main()
