"""``python -m kgwe bench-scaling``: the headline job at 1 / 2 / 4 / 8 GPUs of
one node, back to back, as the BASELINE asks ("measured at 1, 2, 4 and 8 GPUs
with the scaling curve reported").

Each point is a fresh ``python bench.py --gpus N`` (which spawns its own N
ranks under torch.distributed.run); this process never touches the GPU —
it only counts devices (``torch.cuda.device_count`` does not initialise HIP
on this image) and skips the points the node cannot host.  Prints one JSON
object: per N the tokens/s (whole job and per GPU), weak-scaling efficiency
against N=1, avg gfx_activity, RCCL all-reduce busBW and the FSDP2 row.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def run_point(n: int, extra: list[str], timeout: int) -> dict:
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    if r.returncode != 0 or not lines:
        return {"n_gpus": n, "error": f"rc={r.returncode}: {r.stderr[-600:]}"}
    return json.loads(lines[-1])


def curve(points: list[dict]) -> list[dict]:
    base = next((p for p in points if p.get("n_gpus") == 1 and "error" not in p), None)
    rows = []
    for p in points:
        if "error" in p:
            rows.append(p)
            continue
        n = p["n_gpus"]
        per = p["tokens_per_s_per_gpu"]
        rows.append({
            "n_gpus": n, "tokens_per_s": p["tokens_per_s"], "tokens_per_s_per_gpu": per,
            "weak_scaling_efficiency": round(per / base["tokens_per_s_per_gpu"], 4) if base else None,
            "ms_per_step": p["ms_per_step"], "util_pct": p["value"],
            "util_whole_process_pct": p.get("util_whole_process_pct"),
            "mfu_bf16_dense": p.get("mfu_bf16_dense"), "parallelism": p["config"]["parallelism"],
            "allreduce_busbw_gbps": p.get("allreduce_busbw_gbps"),
            "fsdp_row_tokens_per_s": (p.get("fsdp_row") or {}).get("tokens_per_s"),
            "p99_sched_latency_ms": p.get("p99_sched_latency_ms"),
        })
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe bench-scaling")
    ap.add_argument("--gpus-list", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=1200, help="seconds per point")
    ap.add_argument("--json", action="store_true")
    a, extra = ap.parse_known_args(argv)
    have = gpu_count()
    want = [int(x) for x in a.gpus_list.split(",") if x.strip()]
    points, skipped = [], []
    for n in want:
        if n > max(have, 0):
            skipped.append({"n_gpus": n, "skipped": f"node has {have} GPU(s)"})
            continue
        # scheduling / cluster rows are GPU-count independent: measure them once
        args = ["--steps", str(a.steps), "--warmup", str(a.warmup), *extra]
        if points:
            args += ["--no-sched", "--no-cluster"]
        points.append(run_point(n, args, a.timeout))
        print(f"[bench-scaling] N={n}: " + json.dumps(curve(points)[-1]), file=sys.stderr, flush=True)
    out = {"curve": curve(points), "skipped": skipped, "gpus_on_node": have}
    print(json.dumps(out) if a.json else json.dumps(out, indent=1), flush=True)
    return 0 if points and all("error" not in p for p in points) else 1


if __name__ == "__main__":
    raise SystemExit(main())
