"""Per-call GEMM times inside one Llama-3-8B training step (torch.profiler),
split into forward / backward, so each in-step GEMM can be compared with its
standalone time (tools/gemm_layouts.py).  GPU only.

    PYTHONPATH=. python tools/gemm_instep.py [--no-overlap] [--warmup 2]

--no-overlap builds the sharded-DP wrapper with overlap_step=False (AdamW and
the W^T refresh after backward instead of beside it) to show what the
side-stream work costs the GEMMs it runs next to.  KGWE_GEMM_TUNING=0 turns the
committed TunableOp table off.
"""
from __future__ import annotations

import argparse
import collections
import functools

import torch
from torch.profiler import ProfilerActivity, profile


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-overlap", action="store_true")
    a = ap.parse_args()
    from kgwe.bench import train as T
    from kgwe.parallel import dist as kdist

    if a.no_overlap:
        T.ShardedDataParallel = functools.partial(T.ShardedDataParallel, overlap_step=False)
    info = kdist.init()
    tr = T.Trainer(T.TrainConfig(model=a.model), info)
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    tr.step()
    ev1.record()
    torch.cuda.synchronize()
    print(f"step (unprofiled) {ev0.elapsed_time(ev1):.1f} ms", flush=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.step()
        torch.cuda.synchronize()
    mms = sorted((e for e in prof.events() if e.name == "aten::mm"), key=lambda e: e.time_range.start)
    first_lm = next((i for i, e in enumerate(mms) if 128256 in e.input_shapes[0] + e.input_shapes[1]), None)
    rows = collections.OrderedDict()
    for i, e in enumerate(mms):
        phase = "fwd" if first_lm is not None and i <= first_lm else "bwd"
        key = (phase, str(e.input_shapes[:2]))
        r = rows.setdefault(key, [0, 0.0, []])
        r[0] += 1
        r[1] += e.device_time_total
        r[2].append(e.device_time_total)
    tot = 0.0
    for (phase, shp), (n, us, xs) in rows.items():
        a_, b_ = eval(shp)  # noqa: S307 - our own shape list
        m, k, nn = a_[0], a_[1], b_[1]
        tf = 2.0 * m * k * nn * n / (us * 1e-6) / 1e12
        xs = sorted(xs)
        print(f"{phase} {shp:<40} calls {n:3d}  avg {us / n:8.1f} us  min {xs[0]:8.1f}  max {xs[-1]:8.1f}"
              f"  {tf:6.0f} TF/s", flush=True)
        tot += us
    print(f"GEMM total {tot / 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
