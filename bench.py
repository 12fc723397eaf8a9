#!/usr/bin/env python3
"""Headline benchmark: avg GPU utilisation + p99 scheduling latency of an FSDP
Llama-3-8B job on MI355X (BASELINE.json metric/config).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line.  Two ways in, one code path per rank:

* launched by torchrun (``WORLD_SIZE`` set): this process IS a rank;
* launched bare (no ``WORLD_SIZE``; the usual ``python bench.py --gpus N``):
  this process is only a launcher.  It never touches the GPU (no HIP call, no
  ``import torch``): it starts ``torch.distributed.run`` with N ranks as a
  CHILD process (one rank per GPU, RCCL over xGMI, rendezvous on 127.0.0.1),
  forwards the ranks' logs, re-emits rank 0's JSON line and exits non-zero
  if any rank failed.  N=1 goes through the same launcher.

What each rank measures
-----------------------
1. Scheduling (rank 0, CPU only): the job's GPUWorkload and a stream of
   background workloads go through the real extender HTTP server (filter ->
   prioritize -> bind, the kube-scheduler extender contract) over a fake
   apiserver holding a mocked fleet of 8xMI355X nodes; pod-create -> bind
   latencies feed a histogram whose p99 is reported (reference KPI:
   docs/PRD.md:440; its in-process "P99" was a running max).  It runs in a
   child process started BEFORE the rank touches the GPU and overlaps the
   model build / training, so the GPU does not idle behind it.
2. Training: W untimed warmup steps, then exactly K timed steps bracketed by
   barrier + synchronize; the max wall time over ranks is used.  Each rank
   samples amd-smi gfx_activity of its GPU (a) during the K timed steps ->
   ``value`` (mean over ranks) and (b) over the rank's whole life (model
   build, warmup, timed steps, extra rows) -> ``util_whole_process_pct``.
3. At N > 1 an FSDP2 row (PyTorch ``fully_shard``) is timed on the same
   shape after the headline row (``--fsdp-row``), and the RCCL all-reduce
   bus bandwidth over the job's own ranks is swept first.  On RCCL the
   sharded-DP path is also timed for a few steps with the other gradient
   reduce-scatter dtype (``--reduce-row``: fp32 vs bf16 bytes over xGMI).
   Before the ranks start, the launcher runs the HIP xGMI peer-pull probe
   over the N GPUs in a child process of its own (``xgmi_probe``: each link
   alone, then all links at once).
Synthetic tokens (a fresh uniform batch every step), random-init weights of
the Llama-3-8B architecture, bf16 compute, fp32 master weights + AdamW step
inside every timed step.  Headline data parallelism is kgwe's sharded DP
(ZeRO-2 = FSDP SHARD_GRAD_OP: fp32 master weights, Adam moments and reduced
gradients sharded over ranks; the 16 GB of bf16 weights stay replicated
because 288 GB of HBM3E has room).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

BASELINE_UTIL = 87.0      # reference README.md:157-160: KGWE avg GPU utilisation (H100 DGX)
BASELINE_P99_MS = 85.0    # reference docs/PRD.md:440: KGWE p99 scheduling latency
MI355X_BF16_DENSE = 2.5e15
METRIC = ("p99 scheduling latency (ms) + avg GPU-util %, 8-GPU FSDP job on one "
          "MI355X node")
HERE = os.path.dirname(os.path.abspath(__file__))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=4,
                    help="sequences per GPU per step (4 x 4096 tokens: +7%% tok/s over 2 on "
                         "MI355X, 181 GB peak at 1 GPU; 288 GB of HBM3E has the room)")
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing")
    ap.add_argument("--sched-pods", type=int, default=1500,
                    help="workloads pushed through the extender for the latency p99")
    ap.add_argument("--sched-rate", type=float, default=75.0, help="pod arrivals per second")
    ap.add_argument("--sched-nodes", type=int, default=1250,
                    help="fleet of the scheduling-latency row (8 MI355X each; 1250 = 10,000 GPUs)")
    ap.add_argument("--no-sched", action="store_true")
    ap.add_argument("--no-cluster", action="store_true",
                    help="skip the stock-kube vs kgwe cluster simulation row")
    ap.add_argument("--no-busbw", action="store_true", help="skip the RCCL all-reduce busBW probe")
    ap.add_argument("--no-xgmi-probe", action="store_true",
                    help="skip the per-link xGMI bandwidth probe the launcher runs at N > 1")
    ap.add_argument("--sdpa", action="store_true", help="force PyTorch SDPA attention")
    ap.add_argument("--parallel", default="zero", choices=["zero", "fsdp"],
                    help="headline row. zero: replicated bf16 weights + sharded fp32 "
                         "optimizer/gradients (kgwe.parallel.zero, default); fsdp: PyTorch FSDP2")
    ap.add_argument("--fsdp-row", default="auto", choices=["auto", "on", "off"],
                    help="also time an FSDP2 row after the headline (auto: when N > 1)")
    ap.add_argument("--reduce-dtype", default="bf16", choices=["fp32", "bf16"],
                    help="gradient reduce-scatter dtype of the sharded-DP path at N > 1.  bf16 (default): "
                         "half the bytes over xGMI, and the weight-gradient GEMMs write straight into the "
                         "reduce-scatter buckets (no gradient copy); against fp32 it moves the weights by "
                         "no more than the bf16 rounding of the gradients themselves does "
                         "(tests/test_parallel_cpu.py, worlds 4 and 8)")
    ap.add_argument("--reduce-row", default="auto", choices=["auto", "on", "off"],
                    help="also time the sharded-DP path with the OTHER reduce dtype for a few "
                         "steps (auto: at N > 1 on RCCL) — what halving the reduce-scatter "
                         "bytes over xGMI buys")
    ap.add_argument("--extra-rows-timeout", type=float, default=420.0,
                    help="N > 1: seconds the rows after the headline (busBW sweep, other reduce dtype, "
                         "FSDP2) may take before rank 0 prints the line without them (0: no limit)")
    ap.add_argument("--in-process", action="store_true",
                    help="run as a single rank in this process (no launcher)")
    return ap.parse_args(argv)


# --------------------------------------------------------------------------- launcher
def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def xgmi_probe(n: int, env: dict) -> dict | None:
    """Per-link xGMI bandwidth of the GPUs the job runs on (N1: the HIP
    LDS-staged peer-pull probe), in a child process that finishes before any
    rank starts, so it never shares the GPUs with training."""
    import subprocess

    try:
        r = subprocess.run([sys.executable, "-m", "kgwe.agent.probes", "--xgmi", str(n)], cwd=HERE,
                           env=env, capture_output=True, text=True, timeout=180)
        js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not js:
            raise RuntimeError(f"rc={r.returncode}: {r.stderr[-300:]}")
        return json.loads(js[-1]).get("xgmi")
    except Exception as e:  # noqa: BLE001 - optional row, reported, never faked
        print(f"[bench] xGMI probe failed: {e}", file=sys.stderr, flush=True)
        return {"error": str(e)[:300]}


def launch(args, argv: list[str]) -> int:
    """Parent: spawn N ranks under torch.distributed.run, never touch the GPU."""
    import subprocess
    import threading

    n = max(1, args.gpus)
    probe = None
    if n > 1 and not args.no_xgmi_probe:
        env0 = dict(os.environ)
        env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        probe = xgmi_probe(n, env0)
    port = _free_port()
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["KGWE_BENCH_LAUNCHER"] = "1"
    env.setdefault("OMP_NUM_THREADS", "4")
    env.setdefault("PYTHONUNBUFFERED", "1")
    print(f"[bench] launching {n} rank(s): {' '.join(cmd[2:7])} ...", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, cwd=HERE, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    lines: list[str] = []

    def pump():
        for ln in proc.stdout:
            if ln.startswith('{"metric"'):
                lines.append(ln.strip())
            else:
                sys.stderr.write(ln)
                sys.stderr.flush()

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    rc = proc.wait()
    t.join(timeout=10)
    if rc != 0 or not lines:
        print(f"[bench] rank launcher failed: rc={rc}, result lines={len(lines)}", file=sys.stderr)
        return rc or 1
    out = json.loads(lines[-1])
    if out.get("n_gpus") != n:
        print(f"[bench] rank 0 reported n_gpus={out.get('n_gpus')} for --gpus {n}", file=sys.stderr)
        return 1
    out["launcher"] = f"bench.py -> torch.distributed.run --nproc-per-node {n} (child process)"
    if probe is not None:
        out["xgmi_probe"] = probe
    print(json.dumps(out), flush=True)
    return 0


# --------------------------------------------------------------------------- rank
def start_scheduling_bench(args, world: int):
    """Child process tree (apiserver / scheduler sim / extender), CPU only."""
    import subprocess

    # The reference's scale target: 10,000+ GPUs (docs/PRD.md:449) = 1,250
    # 8-GPU nodes, node names only on the wire (nodeCacheCapable: true, the
    # chart's default); the same load on a 64-node fleet is reported beside it.
    cmd = [sys.executable, "-m", "kgwe.bench.sched_latency", "--json", "--pods",
           str(args.sched_pods), "--rate", str(args.sched_rate), "--job-gpus", str(max(1, world)),
           "--nodes", str(args.sched_nodes), "--node-cache", "--then-nodes", "64"]
    return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=HERE,
                            preexec_fn=_side_bench_affinity(world))


def _side_bench_affinity(world: int, count: int = 8, skip: int = 0):
    """preexec_fn pinning a CPU-side benchmark's process tree to `count` of the
    LAST cores this process may use (after skipping `skip` of them), when there
    are enough cores to leave the training ranks (Python launch threads, RCCL
    proxies) cores of their own: the side benchmarks must not skew an 8-rank
    step time, nor the ranks (or each other) their latency tails."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    if len(allowed) < 10 + 4 * max(1, world):
        return None
    cores = set(allowed[len(allowed) - skip - count:len(allowed) - skip])

    def pin():
        try:
            os.sched_setaffinity(0, cores)
        except OSError:
            pass
    return pin


def start_cluster_sim():
    import subprocess

    cmd = [sys.executable, "-m", "kgwe.bench.cluster", "--json"]
    return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=HERE,
                            preexec_fn=_side_bench_affinity(int(os.environ.get("WORLD_SIZE", "1")), count=2, skip=8))


def collect(proc, what: str, timeout: float = 400.0) -> dict | None:
    if proc is None:
        return None
    try:
        out, err = proc.communicate(timeout=timeout)
        js = [ln for ln in out.splitlines() if ln.startswith("{")]
        if proc.returncode != 0 or not js:
            raise RuntimeError(f"rc={proc.returncode}: {err[-400:]}")
        return json.loads(js[-1])
    except Exception as e:  # noqa: BLE001 - report, never fake a number
        proc.kill()
        print(f"[bench] {what} failed: {e}", file=sys.stderr)
        return None


def meter_cost(world: int, tps: float, util: float | None) -> dict | None:
    """Reference row "cost per training run" (README.md:161): a 1B-token run of
    this job at the measured throughput and utilisation, metered by the C++
    cost engine (MI355X on-demand price, utilisation-adjusted)."""
    try:
        from kgwe.core import Platform

        p = Platform({})
        t0, dur = 1.0e9, 1e9 / tps  # seconds for 1B tokens
        p.cost_start({"uid": "bench-run", "namespace": "bench", "team": "bench",
                      "gpu_count": world, "tier": "on_demand"}, t0)
        u = util if util is not None else 0.0
        for i in range(1, 11):
            p.cost_sample("bench-run", u, u, t0 + dur * i / 10)
        rec = p.cost_finalize("bench-run", t0 + dur)
        return {"run_tokens": int(1e9), "run_hours": round(dur / 3600, 3), "gpus": world,
                "raw_cost_usd": round(rec["raw_cost"], 2),
                "adjusted_cost_usd": round(rec["adjusted_cost"], 2),
                "usd_per_gpu_hour": round(rec["raw_cost"] / (world * dur / 3600), 3)}
    except Exception as e:  # noqa: BLE001 - optional row, never fake it
        print(f"[bench] cost metering failed: {e}", file=sys.stderr)
        return None


def _row(tr, res, args, info, kdist) -> dict:
    """Aggregate one timed run over ranks."""
    world = info.world_size
    t_max = kdist.all_reduce_max(res.seconds, info)
    got = kdist.all_gather_floats([res.util_mean if res.util_mean is not None else -1.0,
                                   res.loss], info)
    utils = [u[0] for u in got]
    losses = [u[1] for u in got]
    valid = [u for u in utils if u >= 0]
    tps = tr.tokens_per_step * args.steps * world / t_max
    return {"parallelism": tr.parallelism, "seconds": t_max,
            "ms_per_step": round(1000 * t_max / args.steps, 2),
            "util": sum(valid) / len(valid) if valid else None,
            "util_per_rank": [round(u, 2) if u >= 0 else None for u in utils], "losses": losses,
            "tokens_per_s": tps,
            "mfu": tr.cfg.flops_per_token(args.seq_len) * tps / (MI355X_BF16_DENSE * world),
            "peak_mem_gb": res.peak_mem_gb, "util_samples": res.util_samples}


def _release_memory() -> None:
    import gc

    import torch

    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def rank_main(args) -> int:
    import faulthandler
    import threading
    import time

    faulthandler.dump_traceback_later(900, exit=False)  # stack dump if a phase hangs
    rank = int(os.environ.get("RANK", "0"))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    # CPU-side benchmarks first: child processes forked before any GPU call.
    sched_p = start_scheduling_bench(args, world_env) if rank == 0 and not args.no_sched else None
    cluster_p = start_cluster_sim() if rank == 0 and not args.no_cluster else None

    import torch

    from kgwe.bench.train import TrainConfig, Trainer, timed_run
    from kgwe.ops import attn as attn_ops
    from kgwe.parallel import dist as kdist
    from kgwe.utils.amdsmi_util import UtilSampler

    if args.sdpa:
        attn_ops.set_force_sdpa(True)
    info = kdist.init(force_group=True)
    world = info.world_size
    if args.gpus != world:
        if info.is_main:
            print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        kdist.shutdown()
        return 2
    life = UtilSampler(info.local_rank, interval_s=0.1)
    if info.device.type == "cuda":
        life.start()

    reduce_dtype = torch.bfloat16 if args.reduce_dtype == "bf16" else torch.float32
    tc = TrainConfig(model=args.model, seq_len=args.seq_len, micro_batch=args.micro_batch,
                     activation_checkpointing=args.ckpt, parallel=args.parallel,
                     reduce_dtype=reduce_dtype)
    tr = Trainer(tc, info)
    head = _row(tr, timed_run(tr, args.steps, args.warmup), args, info, kdist)
    attention = ("sdpa" if (args.sdpa or not attn_ops.hip_flash_available()) else "kgwe_flash_attn")
    tuned = tr.tuned_gemms

    # Everything below the headline is secondary (bus-bandwidth sweep, the other
    # reduce dtype, the FSDP2 row).  At N > 1 a watchdog bounds it: if the rows
    # are not done in --extra-rows-timeout seconds, rank 0 prints the line with
    # what it has and every rank exits, so a stuck secondary row can never cost
    # the headline that was already measured.
    extras = {"busbw": None, "reduce_row": None, "fsdp": None}
    emit_lock = threading.Lock()
    emitted = [False]

    def bail():
        with emit_lock:
            if emitted[0]:
                return
            emitted[0] = True
        why = {"error": f"not finished within {args.extra_rows_timeout:.0f} s (watchdog)"}
        print(f"[bench] rank {info.rank}: secondary rows timed out, emitting the headline", file=sys.stderr,
              flush=True)
        if info.is_main:
            life.stop()
            own = [life.mean] if life.mean is not None else []
            emit({k: (v if v is not None or k == "busbw" else why) for k, v in extras.items()}, own)
        else:
            time.sleep(15.0)  # rank 0 prints first
        os._exit(0)

    watchdog = None
    if world > 1 and args.extra_rows_timeout > 0:
        watchdog = threading.Timer(args.extra_rows_timeout, bail)
        watchdog.daemon = True
        watchdog.start()

    # Reference row "142 -> 228 GB/s" (all-reduce bus bandwidth, docs/PRD.md:117-124):
    # RCCL over xGMI on this job's own ranks.
    if world > 1 and not args.no_busbw:
        from kgwe.parallel import busbw as kbus

        try:
            extras["busbw"] = kbus.torch_sweep(sizes=[1 << 26, 1 << 28, 1 << 30], iters=10, info=info)
        except Exception as e:  # noqa: BLE001 - reported, never faked
            print(f"[bench] rank {info.rank}: busBW sweep failed: {e!r}", file=sys.stderr, flush=True)

    # Reduce-dtype row: the sharded-DP path again with the other gradient
    # reduce-scatter dtype (fp32 <-> bf16), a few steps, reported beside the
    # headline.  A failure is reported in the row, never faked.
    reduce_row = None
    fsdp = None

    def emit(rows: dict, life_valid: list) -> None:
        busbw, reduce_row, fsdp = rows["busbw"], rows["reduce_row"], rows["fsdp"]
        sched = collect(sched_p, "scheduling benchmark")
        cluster = collect(cluster_p, "cluster simulation", timeout=120)
        p99 = sched["p99_ms"] if sched else None
        util = head["util"]
        tps = head["tokens_per_s"]
        out = {
            "metric": METRIC,
            "value": round(util, 2) if util is not None else None,
            "unit": "% avg amd-smi gfx_activity over the K timed training steps (mean over ranks)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(util / BASELINE_UTIL, 4) if util is not None else None,
            "dtype": "bf16",
            "data": "synthetic tokens, random-init weights",
            "config": {"model": args.model, "global_batch": args.micro_batch * world,
                       "seq_len": args.seq_len, "parallelism": head["parallelism"],
                       "micro_batch_per_gpu": args.micro_batch,
                       "activation_checkpointing": args.ckpt,
                       "grad_reduce_dtype": args.reduce_dtype if world > 1 else None},
            "p99_sched_latency_ms": round(p99, 3) if p99 is not None else None,
            "vs_baseline_p99": round(BASELINE_P99_MS / p99, 2) if p99 else None,
            "util_whole_process_pct": (round(sum(life_valid) / len(life_valid), 2)
                                       if life_valid else None),
            "util_whole_process_note": "gfx_activity from rank start (after import) to the end "
                                       "of the last timed row: model build, warmup, busBW sweep "
                                       "and the FSDP row included",
            "tokens_per_s": round(tps, 1),
            "tokens_per_s_per_gpu": round(tps / world, 1),
            "mfu_bf16_dense": round(head["mfu"], 4),
            "util_per_rank": head["util_per_rank"],
            "util_samples_rank0": head["util_samples"],
            "loss_per_rank": [round(x, 4) for x in head["losses"]],
            "peak_mem_gb_rank0": round(head["peak_mem_gb"], 1),
            "attention": attention,
            "gemm_solutions": "tuned (kgwe/tuning)" if tuned else "library default",
            "fsdp_row": fsdp,
            "reduce_dtype_row": reduce_row,
            "allreduce_busbw_gbps": (round(busbw["peak_busbw_gbps"], 1) if busbw else None),
            "allreduce_sweep": busbw["rows"] if busbw else None,
            "sched": sched,
            "cluster_sim": cluster,
            "cost": meter_cost(world, tps, util),
        }
        print(json.dumps(out), flush=True)

    want_reduce = args.reduce_row == "on" or (args.reduce_row == "auto" and world > 1
                                              and info.backend == "nccl")
    if want_reduce and args.parallel == "zero":
        other = torch.float32 if reduce_dtype == torch.bfloat16 else torch.bfloat16
        if tr.dp is not None:
            tr.dp.close()
        tr = None
        _release_memory()
        k2, w2 = min(args.steps, 5), min(args.warmup, 2)
        try:
            tr3 = Trainer(TrainConfig(model=args.model, seq_len=args.seq_len,
                                      micro_batch=args.micro_batch,
                                      activation_checkpointing=args.ckpt, parallel="zero",
                                      reduce_dtype=other), info)
            a3 = argparse.Namespace(**{**vars(args), "steps": k2})
            r3 = _row(tr3, timed_run(tr3, k2, w2), a3, info, kdist)
            reduce_row = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r3.items()
                          if k not in ("losses", "seconds")}
            reduce_row.update({"grad_reduce_dtype": "bf16" if other == torch.bfloat16 else "fp32",
                               "steps": k2, "warmup": w2})
            tr3.dp.close()
            del tr3
        except Exception as e:  # noqa: BLE001 - reported, never faked
            print(f"[bench] rank {info.rank}: reduce-dtype row failed: {e!r}", file=sys.stderr, flush=True)
            reduce_row = {"error": repr(e)[:300]}
            tr3 = None
        extras["reduce_row"] = reduce_row
        _release_memory()

    want_fsdp = args.fsdp_row == "on" or (args.fsdp_row == "auto" and world > 1)
    if want_fsdp and args.parallel != "fsdp":
        if tr is not None and tr.dp is not None:
            tr.dp.close()
        tr = None
        _release_memory()
        tc2 = TrainConfig(model=args.model, seq_len=args.seq_len, micro_batch=args.micro_batch,
                          activation_checkpointing=args.ckpt, parallel="fsdp")
        # A secondary row: a failure on every rank alike (out of memory, an
        # unsupported op) is reported in the row instead of losing the
        # headline that was already measured.
        try:
            tr2 = Trainer(tc2, info)
            r2 = _row(tr2, timed_run(tr2, args.steps, min(args.warmup, 3)), args, info, kdist)
            fsdp = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r2.items()
                    if k not in ("losses", "seconds")}
            del tr2
        except Exception as e:  # noqa: BLE001 - reported, never faked
            print(f"[bench] rank {info.rank}: FSDP row failed: {e!r}", file=sys.stderr, flush=True)
            fsdp = {"parallelism": f"fsdp{world}", "error": repr(e)[:300]}
            tr2 = None
            _release_memory()
        extras["fsdp"] = fsdp
    with emit_lock:  # from here on the normal path owns the line
        if emitted[0]:
            time.sleep(3600)  # the watchdog is emitting and will end the process
        emitted[0] = True
    if watchdog is not None:
        watchdog.cancel()
    life.stop()
    life_util = [u[0] for u in kdist.all_gather_floats(
        [life.mean if life.mean is not None else -1.0], info)]
    life_valid = [u for u in life_util if u >= 0]

    if info.is_main:
        emit(extras, life_valid)
    kdist.barrier(info)
    kdist.shutdown()
    return 0


def main(argv=None) -> int:
    raw = list(sys.argv[1:] if argv is None else argv)
    args = parse(raw)
    if "WORLD_SIZE" not in os.environ and not args.in_process:
        return launch(args, raw)
    return rank_main(args)


if __name__ == "__main__":
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(main())
