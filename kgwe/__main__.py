"""`python -m kgwe <component> [...]` — one entry point for every binary the
reference's Makefile / Dockerfiles declare (Makefile:44-70: controller,
scheduler, discovery, mig-controller, cost-engine, exporter, agent; all
absent there)."""
from __future__ import annotations

import sys

COMMANDS = {
    "controller": "kgwe.controller.main",      # extender + webhook + reconcilers (+ cost/partition/exporter)
    "agent": "kgwe.agent.agent",               # node discovery + probes + telemetry exporter (:9400)
    "optimizer": "kgwe.optimizer.server",      # gRPC :50051
    "bench-sched": "kgwe.bench.sched_latency",  # pod-create -> bind latency benchmark
    "bench-scale": "kgwe.bench.scale",  # scheduling core on a 10k-GPU fleet
    "bench-cluster": "kgwe.bench.cluster",  # stock kube vs kgwe on one trace (simulated)
    "bench-scaling": "kgwe.bench.scaling",  # bench.py at 1/2/4/8 GPUs -> scaling curve
    "bench-infer": "kgwe.bench.infer",  # bf16 decode server / co-located servers on one GPU
    "serve-batch": "kgwe.serving.batch_server",  # one continuous-batching server per share group
    "busbw": "kgwe.parallel.busbw",            # RCCL all-reduce bus bandwidth sweep
    "crds": "kgwe.api.crds",                   # render CRD YAML
    "launch": "kgwe.launch",                   # container entrypoint (placement env)
    "build": "kgwe._build",                    # compile native artefacts (gfx950)
}


def main() -> int:
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        print("usage: python -m kgwe {" + ",".join(COMMANDS) + "} [args]", file=sys.stderr)
        return 2
    import importlib
    import runpy

    name = COMMANDS[sys.argv[1]]
    sys.argv = [f"kgwe {sys.argv[1]}"] + sys.argv[2:]
    mod = importlib.import_module(name)
    if hasattr(mod, "main"):
        r = mod.main()
        return int(r or 0)
    runpy.run_module(name, run_name="__main__")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
