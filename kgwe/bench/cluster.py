"""Stock-kube vs kgwe on ONE arrival trace: the cluster-level A/B behind the
reference's relative claims (README.md:157-161: utilisation 35 -> 87 %,
cost per training run $1,000 -> $620, "MIG" utilisation 92 %;
docs/PRD.md:117-124: all-reduce 142 -> 228 GB/s random vs topology-aware).
The reference ships no simulator, trace or method for any of them.

A discrete-event simulation in simulated time over a fleet of 8xMI355X nodes.
Both columns replay the SAME seeded trace of arrivals and durations:

* **stock** — what kube-scheduler does with the AMD device plugin alone:
  whole GPUs only (an inference pod holds a full GPU), NodeResourcesFit
  LeastAllocated (spread, random tie-break), no topology or partition
  awareness, no gang scheduling (the pods of a multi-pod job are bound one
  by one and hold their GPUs idle until the last one binds, possibly on
  different nodes).
* **kgwe** — the real C++ core (``kgwe.core.Platform``): xGMI-aware best-fit
  packing, all-or-nothing gangs kept on one xGMI island, CPX partition
  slices auto-provisioned for inference pods and reclaimed when idle,
  partition consolidation (``Platform.consolidate_partitions``), metering by
  the C++ cost engine.

Queueing is identical for both: FIFO with backfill (a job that does not fit
waits; later jobs that fit start), no preemption.

Model (stated, not measured):
* a running pod keeps its GPU (slice) busy at ``demand`` of a full GPU —
  0.95 for training, 0.11 for a CPX-sized inference server (one XCD's worth
  of work) — the gfx_activity analogue of the reference's "SM utilisation";
* a multi-GPU job's all-reduce runs at the ring's slowest hop: an xGMI link
  inside a node (153.6 GB/s x 0.85) or the node NIC across nodes
  (400 GbE = 50 GB/s x 0.9); its run time stretches by
  ``(1 - f) + f * bw_best / bw_actual`` with ``f`` its communication share
  at the best placement.
"""
from __future__ import annotations

import argparse
import heapq
import json
import math
import random
from dataclasses import dataclass, field

XGMI_HOP_GBPS = 153.6 * 0.85
NIC_HOP_GBPS = 50.0 * 0.9

# name, arrivals/h, pods, gpus per pod (1/8 = CPX slice), mean hours, comm share f, demand
CLASSES = [
    ("fsdp8", 0.9, 1, 8, 6.0, 0.12, 0.95),
    ("train4", 1.6, 1, 4, 3.0, 0.10, 0.95),
    ("ddp4x1", 1.2, 4, 1, 3.0, 0.15, 0.95),
    ("train2", 3.0, 1, 2, 2.0, 0.08, 0.95),
    ("train1", 9.0, 1, 1, 1.0, 0.0, 0.90),
    ("infer", 4.0, 1, 0.125, 8.0, 0.0, 0.11),
]
PRICE_GPU_H = None  # taken from the cost engine's MI355X table at run time


@dataclass
class Job:
    jid: int
    cls: str
    arrive: float
    pods: int
    gpus: float
    hours: float
    f: float
    demand: float
    start: float = -1.0
    end: float = -1.0
    placed: list = field(default_factory=list)  # per pod: (node, n_gpus or slice id)
    bound_at: list = field(default_factory=list)
    bw: float = 0.0
    stretch: float = 1.0

    @property
    def is_train(self) -> bool:
        return self.cls != "infer"


def make_trace(hours: float, seed: int, scale: float = 1.0) -> list[Job]:
    rnd = random.Random(seed)
    jobs: list[Job] = []
    for name, rate, pods, gpus, mean_h, f, demand in CLASSES:
        t = 0.0
        while True:
            t += rnd.expovariate(rate * scale)
            if t >= hours:
                break
            # lognormal durations (sigma 0.6) with the class mean
            dur = mean_h * math.exp(rnd.gauss(0.0, 0.6) - 0.18)
            jobs.append(Job(0, name, t * 3600.0, pods, gpus, dur, f, demand))
    jobs.sort(key=lambda j: j.arrive)
    for i, j in enumerate(jobs):
        j.jid = i
    return jobs


# --------------------------------------------------------------------------- policies
class Stock:
    """kube-scheduler + device plugin: whole GPUs, LeastAllocated, no gangs."""

    name = "stock"

    def __init__(self, nodes: int, seed: int):
        self.free = [8] * nodes
        self.rnd = random.Random(seed ^ 0x5EED)
        self.n = nodes

    def place_pod(self, gpus: float) -> int | None:
        need = max(1, int(math.ceil(gpus)))
        best, cands = -1, []
        for i, f in enumerate(self.free):
            if f >= need:
                if f > best:
                    best, cands = f, [i]
                elif f == best:
                    cands.append(i)
        if not cands:
            return None
        i = self.rnd.choice(cands)
        self.free[i] -= need
        return i

    def release_pod(self, node: int, gpus: float) -> None:
        self.free[node] += max(1, int(math.ceil(gpus)))

    def allocated(self) -> float:
        return float(8 * self.n - sum(self.free))

    def islands(self) -> int:
        return sum(1 for f in self.free if f == 8)

    def slice_util(self):
        return None


class Kgwe:
    """The C++ platform core, driven in simulated time."""

    name = "kgwe"

    def __init__(self, nodes: int, reclaim_idle_s: float, consolidate: bool):
        from ..core import Platform, make_fixture

        self.p = Platform({"enforceBudgets": False, "partitionReclaimIdleSeconds": -1,
                           "scheduler": {"enablePreemption": False}})
        for i in range(nodes):
            self.p.add_fake_node(make_fixture(f"n{i:03d}", 8, 2))
        self.n = nodes
        self.reclaim_idle_s = reclaim_idle_s
        self.consolidate = consolidate
        self.used_gpus = 0
        self.used_slices = 0
        self.migrations = 0

    @staticmethod
    def _wl(uid: str, gpus: float, cls: str, gang: str = "", size: int = 0) -> dict:
        if gpus < 1:
            return {"uid": uid, "workloadType": "Inference", "preemptible": True,
                    "gpuRequirements": {"partition": {"mode": "CPX", "count": 1}}}
        w = {"uid": uid, "workloadType": "Training", "preemptible": False,
             "gpuRequirements": {"count": int(gpus),
                                 "topology": {"preference": "xGMIOptimal" if gpus > 1 or gang
                                              else "None"}},
             "distributedConfig": {"strategy": "FSDP" if cls == "fsdp8" else "DataParallel"}}
        if gang:
            w["gang"] = {"name": gang, "size": size}
        return w

    def place_job(self, job: Job) -> list | None:
        if job.pods == 1:
            d = self.p.schedule(self._wl(f"j{job.jid}", job.gpus, job.cls))
            if not d.get("ok"):
                return None
            placed = [(d["node"], d["gpus"] or d["partitions"])]
        else:
            members = [self._wl(f"j{job.jid}-{k}", job.gpus, job.cls, gang=f"g{job.jid}",
                                size=job.pods) for k in range(job.pods)]
            ds = self.p.schedule_gang(members)
            if not ds or not all(d.get("ok") for d in ds):
                return None
            placed = [(d["node"], d["gpus"]) for d in ds]
        if job.gpus < 1:
            self.used_slices += 1
        else:
            self.used_gpus += int(job.gpus) * job.pods
        return placed

    def release_job(self, job: Job, now: float) -> None:
        uids = [f"j{job.jid}"] if job.pods == 1 else [f"j{job.jid}-{k}" for k in range(job.pods)]
        for u in uids:
            self.p.release(u, now)
        if job.gpus < 1:
            self.used_slices -= 1
        else:
            self.used_gpus -= int(job.gpus) * job.pods

    def housekeeping(self, now: float) -> list:
        moves = []
        if self.consolidate:
            moves = self.p.consolidate_partitions(now, plan_only=False)
            self.migrations += len(moves)
        self.p.reclaim_idle_after(now, self.reclaim_idle_s)
        return moves

    def allocated(self) -> float:
        return self.used_gpus + self.used_slices / 8.0

    def islands(self) -> int:
        snap = self.p.snapshot()
        busy = {g for a in self.p.allocations() for g in a["gpus"]}
        out = 0
        for n in snap["nodes"].values():
            gs = n["gpus"]
            if len(gs) == 8 and all(g["partition"]["compute"] == "SPX" and g["uuid"] not in busy
                                    for g in gs):
                out += 1
        return out

    def slice_util(self):
        m = self.p.partition_metrics()
        tot = sum(v.get("slices", 0) for k, v in m.get("modes", {}).items() if k != "SPX")
        return (self.used_slices / tot) if tot else None


# --------------------------------------------------------------------------- engine
def _pct(xs: list[float], q: float) -> float | None:
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))]


def simulate(policy, jobs: list[Job], nodes: int, horizon_s: float, warmup_s: float,
             tick_s: float = 300.0) -> dict:
    import copy

    jobs = [copy.copy(j) for j in jobs]
    for j in jobs:
        j.placed, j.bound_at = [], []
    from ..core import Platform

    meter = Platform({"enforceBudgets": False})  # the C++ cost engine, sim clock
    ev: list = []
    for j in jobs:
        heapq.heappush(ev, (j.arrive, 1, j.jid, "arrive"))
    t = 0.0
    while t < horizon_s:
        t += tick_s
        heapq.heappush(ev, (t, 0, -1, "tick"))
    queue: list[Job] = []          # jobs waiting (kgwe: whole job; stock: job with unbound pods)
    running: dict[int, Job] = {}
    pending_pods: dict[int, int] = {}  # stock: pods still unbound per job
    stats = {"busy": 0.0, "alloc": 0.0, "islands": 0.0, "slice": 0.0, "slice_t": 0.0, "t": 0.0}
    now = 0.0
    busy_now = 0.0
    waits8, waits_all, costs, bws = [], [], {}, []
    done_work_h = 0.0
    metered = 0.0
    train_usd = train_work_h = infer_usd = infer_pod_h = 0.0

    # fleet-shape gauges are sampled on the housekeeping tick (they need a
    # topology snapshot); busy / allocated GPUs are exact at every event
    shape = {"islands": float(policy.islands()), "slice": policy.slice_util()}

    def integrate(t1: float) -> None:
        nonlocal now
        lo, hi = max(now, warmup_s), min(t1, horizon_s)
        if hi > lo:
            dt = hi - lo
            stats["t"] += dt
            stats["busy"] += busy_now * dt
            stats["alloc"] += policy.allocated() * dt
            stats["islands"] += shape["islands"] * dt
            if shape["slice"] is not None:
                stats["slice"] += shape["slice"] * dt
                stats["slice_t"] += dt
        now = t1

    def start(job: Job) -> None:
        nonlocal busy_now
        job.start = now
        nodes_used = {p[0] for p in job.placed}
        if job.pods > 1 or job.gpus > 1:
            job.bw = XGMI_HOP_GBPS if len(nodes_used) == 1 else NIC_HOP_GBPS
            job.stretch = (1 - job.f) + job.f * XGMI_HOP_GBPS / job.bw
            if job.pods > 1:  # one pod is always one node: only multi-pod jobs can differ
                bws.append(job.bw)
        run_s = job.hours * 3600.0 * job.stretch
        job.end = now + run_s
        busy_now += job.demand * job.gpus * job.pods if job.gpus >= 1 else job.demand
        running[job.jid] = job
        heapq.heappush(ev, (job.end, 2, job.jid, "finish"))
        for k in range(job.pods):  # metering starts when each pod was bound
            t0 = job.bound_at[k] if k < len(job.bound_at) else now
            meter.cost_start({"uid": f"{policy.name}-{job.jid}-{k}", "namespace": "sim",
                              "team": job.cls, "gpu_count": max(1, int(job.gpus)),
                              "partition_mode": "CPX" if job.gpus < 1 and policy.name == "kgwe"
                              else "", "tier": "OnDemand"}, t0)
            if t0 < now:  # held idle while waiting for its gang
                meter.cost_sample(f"{policy.name}-{job.jid}-{k}", 0.0, 0.0, t0)
                meter.cost_sample(f"{policy.name}-{job.jid}-{k}", 0.0, 0.0, now)
            util = 100.0 * min(1.0, job.demand / (job.gpus if job.gpus < 1 else 1.0)) \
                if policy.name == "kgwe" or job.gpus >= 1 else 100.0 * job.demand
            meter.cost_sample(f"{policy.name}-{job.jid}-{k}", util, util, now)
        if job.arrive >= warmup_s:
            w = (now - job.arrive) / 60.0
            waits_all.append(w)
            if job.cls == "fsdp8":
                waits8.append(w)

    def try_schedule() -> None:
        i = 0
        while i < len(queue):
            job = queue[i]
            if isinstance(policy, Stock):
                while pending_pods[job.jid] > 0:
                    node = policy.place_pod(job.gpus)
                    if node is None:
                        break
                    job.placed.append((node, job.gpus))
                    job.bound_at.append(now)
                    pending_pods[job.jid] -= 1
                if pending_pods[job.jid] == 0:
                    queue.pop(i)
                    start(job)
                    continue
            else:
                placed = policy.place_job(job)
                if placed is not None:
                    job.placed = placed
                    job.bound_at = [now] * job.pods
                    queue.pop(i)
                    start(job)
                    continue
            i += 1

    while ev:
        t, _, jid, kind = heapq.heappop(ev)
        if t > horizon_s:
            break
        integrate(t)
        if kind == "arrive":
            job = jobs[jid]
            queue.append(job)
            pending_pods[jid] = job.pods
            try_schedule()
        elif kind == "finish":
            job = running.pop(jid)
            busy_now -= job.demand * job.gpus * job.pods if job.gpus >= 1 else job.demand
            if isinstance(policy, Stock):
                for node, g in job.placed:
                    policy.release_pod(node, g)
            else:
                policy.release_job(job, now)
            cost = 0.0
            for k in range(job.pods):
                rec = meter.cost_finalize(f"{policy.name}-{job.jid}-{k}", now)
                cost += rec["adjusted_cost"] if rec else 0.0
            metered += cost
            if job.arrive >= warmup_s:
                costs.setdefault(job.cls, []).append(cost)
                work = job.hours * (job.gpus * job.pods if job.gpus >= 1 else job.gpus)
                done_work_h += work
                if job.is_train:
                    train_usd += cost
                    train_work_h += work
                else:
                    infer_usd += cost
                    infer_pod_h += job.hours
            try_schedule()
        else:  # housekeeping tick
            if isinstance(policy, Kgwe):
                policy.housekeeping(now)
            try_schedule()
            shape["islands"] = float(policy.islands())
            shape["slice"] = policy.slice_util()
    integrate(horizon_s)
    T = stats["t"] or 1.0
    total = 8.0 * nodes
    usd_train_h = train_usd / train_work_h if train_work_h else None
    return {
        "cluster_busy_util_pct": round(100.0 * stats["busy"] / T / total, 2),
        "cluster_alloc_util_pct": round(100.0 * stats["alloc"] / T / total, 2),
        "free_8gpu_islands_avg": round(stats["islands"] / T, 2),
        "slice_util_pct": (round(100.0 * stats["slice"] / stats["slice_t"], 2)
                           if stats["slice_t"] else None),
        "fsdp8_wait_min_p50": _r(_pct(waits8, 0.5)), "fsdp8_wait_min_p99": _r(_pct(waits8, 0.99)),
        "wait_min_p50": _r(_pct(waits_all, 0.5)), "wait_min_p99": _r(_pct(waits_all, 0.99)),
        "jobs_completed": sum(len(v) for v in costs.values()),
        "jobs_queued_at_end": len(queue),
        "completed_gpu_hours_of_work": round(done_work_h, 1),
        "cost_per_job_usd": {k: round(sum(v) / len(v), 2) for k, v in sorted(costs.items())},
        # metered $ per GPU-hour of training WORK (held-idle gang time and
        # cross-node slow-down included), and the same for a reference run of
        # 8 GPUs x 6 h of work (the flagship FSDP job)
        "usd_per_training_work_gpu_hour": round(usd_train_h, 3) if usd_train_h else None,
        "cost_per_training_run_usd": round(usd_train_h * 48.0, 2) if usd_train_h else None,
        "usd_per_inference_pod_hour": round(infer_usd / infer_pod_h, 3) if infer_pod_h else None,
        "usd_per_work_gpu_hour": round(metered / done_work_h, 3) if done_work_h else None,
        "multi_pod_allreduce_busbw_gbps_mean": round(sum(bws) / len(bws), 1) if bws else None,
        "multi_pod_jobs_on_one_node_pct": (round(100.0 * sum(1 for b in bws if b == XGMI_HOP_GBPS)
                                                 / len(bws), 1) if bws else None),
        "migrations": getattr(policy, "migrations", 0),
    }


def _r(x):
    return None if x is None else round(x, 1)


def run(nodes: int = 16, days: float = 5.0, warmup_days: float = 1.0, seed: int = 11,
        load: float = 1.0, consolidate: bool = True) -> dict:
    horizon = (days + warmup_days) * 86400.0
    jobs = make_trace(horizon / 3600.0, seed, scale=load * nodes / 16.0)
    stock = simulate(Stock(nodes, seed), jobs, nodes, horizon, warmup_days * 86400.0)
    kg = simulate(Kgwe(nodes, reclaim_idle_s=1800.0, consolidate=consolidate), jobs, nodes,
                  horizon, warmup_days * 86400.0)

    def ratio(a, b):
        return round(a / b, 3) if a and b else None

    return {
        "fleet": f"{nodes} x 8 MI355X", "simulated_days": days, "warmup_days": warmup_days,
        "jobs_in_trace": len(jobs), "seed": seed, "load_scale": load,
        "classes": [{"name": c[0], "per_hour": round(c[1] * load * nodes / 16.0, 2), "pods": c[2],
                     "gpus_per_pod": c[3], "mean_hours": c[4], "comm_share": c[5],
                     "demand": c[6]} for c in CLASSES],
        "stock": stock, "kgwe": kg,
        "ratios": {
            "busy_util": ratio(kg["cluster_busy_util_pct"], stock["cluster_busy_util_pct"]),
            "cost_per_training_run": ratio(kg["cost_per_training_run_usd"],
                                           stock["cost_per_training_run_usd"]),
            "cost_per_inference_pod_hour": ratio(kg["usd_per_inference_pod_hour"],
                                                 stock["usd_per_inference_pod_hour"]),
            "fsdp8_wait_p99": ratio(kg["fsdp8_wait_min_p99"], stock["fsdp8_wait_min_p99"]),
            "usd_per_work_gpu_hour": ratio(kg["usd_per_work_gpu_hour"], stock["usd_per_work_gpu_hour"]),
            "allreduce_busbw": ratio(kg["multi_pod_allreduce_busbw_gbps_mean"],
                                     stock["multi_pod_allreduce_busbw_gbps_mean"]),
            "completed_work": ratio(kg["completed_gpu_hours_of_work"],
                                    stock["completed_gpu_hours_of_work"]),
        },
        "model": "simulated time; demand 0.95 training / 0.11 CPX-sized inference; ring busBW "
                 f"xGMI hop {XGMI_HOP_GBPS:.0f} GB/s vs NIC hop {NIC_HOP_GBPS:.0f} GB/s",
    }


_T95 = {2: 12.706, 3: 4.303, 4: 3.182, 5: 2.776, 6: 2.571, 7: 2.447, 8: 2.365, 9: 2.306, 10: 2.262}


def _mean_ci(xs: list) -> dict | None:
    """Mean and the half-width of its 95 % confidence interval (Student t)."""
    xs = [x for x in xs if x is not None]
    if not xs:
        return None
    n = len(xs)
    m = sum(xs) / n
    if n < 2:
        return {"mean": round(m, 3), "ci95": None, "n": n}
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (n - 1))
    return {"mean": round(m, 3), "ci95": round(_T95.get(n, 1.96) * sd / math.sqrt(n), 3), "n": n,
            "min": round(min(xs), 3), "max": round(max(xs), 3)}


def _one(args) -> dict:
    nodes, days, warmup, seed, load = args
    return run(nodes, days, warmup, seed, load)


SWEEP_KEYS = ("cluster_busy_util_pct", "cluster_alloc_util_pct", "cost_per_training_run_usd",
              "usd_per_inference_pod_hour", "usd_per_work_gpu_hour", "fsdp8_wait_min_p99", "wait_min_p99",
              "multi_pod_allreduce_busbw_gbps_mean", "completed_gpu_hours_of_work", "slice_util_pct",
              "free_8gpu_islands_avg")


def sweep(nodes: int, days: float, warmup_days: float, seeds: list, loads: list, workers: int = 4) -> dict:
    """The A/B over arrival-rate multipliers and trace seeds: per load, the
    mean and 95 % CI over seeds of each column's metrics and of the
    kgwe / stock ratios (each ratio taken per seed, on the same trace)."""
    import multiprocessing as mp

    todo = [(nodes, days, warmup_days, s, ld) for ld in loads for s in seeds]
    with mp.get_context("fork").Pool(max(1, workers)) as pool:
        res = pool.map(_one, todo, chunksize=1)
    out = {"fleet": f"{nodes} x 8 MI355X", "simulated_days": days, "warmup_days": warmup_days,
           "seeds": seeds, "loads": loads, "by_load": {}, "model": res[0]["model"]}
    for ld in loads:
        rs = [r for r, t in zip(res, todo) if t[4] == ld]
        row = {"jobs_in_trace": _mean_ci([r["jobs_in_trace"] for r in rs]),
               "stock": {k: _mean_ci([r["stock"].get(k) for r in rs]) for k in SWEEP_KEYS},
               "kgwe": {k: _mean_ci([r["kgwe"].get(k) for r in rs]) for k in SWEEP_KEYS},
               "ratios": {k: _mean_ci([r["ratios"].get(k) for r in rs]) for k in rs[0]["ratios"]},
               "kgwe_wins_busy_util_in_seeds": sum(1 for r in rs if (r["ratios"]["busy_util"] or 0) > 1.0)}
        out["by_load"][str(ld)] = row
    return out


def sweep_markdown(sw: dict) -> str:
    def f(c, unit="", nd=1):
        if not c:
            return "n/a"
        ci = f" ± {c['ci95']:.{nd}f}" if c.get("ci95") is not None else ""
        return f"{c['mean']:.{nd}f}{ci}{unit}"

    lines = [f"Fleet {sw['fleet']}, {sw['simulated_days']} simulated days after {sw['warmup_days']} warm-up, "
             f"seeds {sw['seeds']} (mean ± 95 % CI over seeds; ratios are kgwe / stock per seed).", "",
             "| load | jobs | busy util stock | busy util kgwe | **ratio** | cost / training run ratio | "
             "$ / inference pod-hour ratio | fsdp8 wait p99 stock → kgwe (min) | all-reduce busBW ratio | "
             "completed work ratio |", "|---|---|---|---|---|---|---|---|---|---|"]
    for ld, row in sw["by_load"].items():
        st, kg, ra = row["stock"], row["kgwe"], row["ratios"]
        lines.append(
            f"| {ld}x | {f(row['jobs_in_trace'], nd=0)} | {f(st['cluster_busy_util_pct'], ' %')} | "
            f"{f(kg['cluster_busy_util_pct'], ' %')} | **{f(ra['busy_util'], 'x', 3)}** | "
            f"{f(ra['cost_per_training_run'], 'x', 3)} | {f(ra['cost_per_inference_pod_hour'], 'x', 3)} | "
            f"{f(st['fsdp8_wait_min_p99'], nd=0)} → {f(kg['fsdp8_wait_min_p99'], nd=0)} | "
            f"{f(ra['allreduce_busbw'], 'x', 2)} | {f(ra['completed_work'], 'x', 3)} |")
    return "\n".join(lines) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe bench-cluster")
    ap.add_argument("--sweep", action="store_true", help="loads x seeds, with confidence intervals")
    ap.add_argument("--loads", default="0.5,0.75,1.0,1.5,2.0")
    ap.add_argument("--seeds", default="11,12,13,14,15")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--markdown", default="", help="with --sweep: also write the table to this file")
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--days", type=float, default=5.0)
    ap.add_argument("--warmup-days", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--load", type=float, default=1.0, help="arrival-rate multiplier")
    ap.add_argument("--no-consolidate", action="store_true")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    if a.sweep:
        out = sweep(a.nodes, a.days, a.warmup_days, [int(x) for x in a.seeds.split(",")],
                    [float(x) for x in a.loads.split(",")], a.workers)
        if a.markdown:
            with open(a.markdown, "w") as fh:
                fh.write(sweep_markdown(out))
        print(json.dumps(out) if a.json else json.dumps(out, indent=1), flush=True)
        return 0
    out = run(a.nodes, a.days, a.warmup_days, a.seed, a.load, consolidate=not a.no_consolidate)
    print(json.dumps(out) if a.json else json.dumps(out, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
