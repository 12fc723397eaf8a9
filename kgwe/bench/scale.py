"""Control-plane scale benchmark: the C++ scheduling core on a fleet of the
PRD's target size (docs/PRD.md:449-450: 10,000+ GPUs, topology queries
< 10 ms), in process, no HTTP.

A churn of 1/2/4/8-GPU xGMI workloads keeps ~2,000 allocations live; every
Schedule() call (filter + score of every node + reserve) and every topology
hint query is timed into the native histogram.

    python -m kgwe bench-scale [--nodes 1250] [--ops 3000] [--json]
"""
from __future__ import annotations

import argparse
import json
import random
import time


def run(nodes: int = 1250, ops: int = 3000, live_max: int = 2000, seed: int = 1) -> dict:
    from ..core import LatencyHistogram, Platform, make_fixture

    p = Platform({})
    t0 = time.perf_counter()
    for i in range(nodes):
        p.add_fake_node(make_fixture(f"mi355x-{i:05d}", 8, 2))
    build_s = time.perf_counter() - t0
    rnd = random.Random(seed)
    hs, hh = LatencyHistogram(), LatencyHistogram()
    live: list[str] = []
    ok = 0
    for i in range(ops):
        g = rnd.choice([1, 1, 2, 4, 8])
        w = {"metadata": {"name": f"w{i}", "uid": f"w{i}"},
             "spec": {"gpuRequirements": {"count": g, "topology": {
                 "preference": "xGMIOptimal" if g > 1 else "None"}}}}
        t = time.perf_counter()
        d = p.schedule(w)
        hs.record_ms((time.perf_counter() - t) * 1000)
        if d["ok"]:
            ok += 1
            live.append(f"w{i}")
        if len(live) > live_max:
            p.release(live.pop(rnd.randrange(len(live))))
        if i % 10 == 0:
            t = time.perf_counter()
            p.hints(rnd.choice([2, 4, 8]))
            hh.record_ms((time.perf_counter() - t) * 1000)
    m = p.scheduler_metrics()
    return {"nodes": nodes, "gpus": nodes * 8, "ops": ops, "scheduled": ok,
            "live_allocations": len(live), "fleet_build_s": round(build_s, 2),
            "schedule_ms": {"p50": hs.quantile_ms(0.5), "p99": hs.quantile_ms(0.99), "max": hs.max_ms()},
            "core_schedule_p99_ms": m.get("p99_ms"),
            "topology_query_ms": {"p50": hh.quantile_ms(0.5), "p99": hh.quantile_ms(0.99),
                                  "max": hh.max_ms()}}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe bench-scale")
    ap.add_argument("--nodes", type=int, default=1250)
    ap.add_argument("--ops", type=int, default=3000)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    r = run(a.nodes, a.ops)
    print(json.dumps(r) if a.json else json.dumps(r, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
