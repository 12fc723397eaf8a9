"""RCCL all-reduce bus-bandwidth sweep (the reference's "142 -> 228 GB/s"
all-reduce metric, docs/PRD.md:119-124, measured here over xGMI).

Two drivers for the same measurement:
  * ``native``: one process, ncclCommInitAll over the visible GPUs
    (``kgwe_rccl_allreduce_sweep`` in libkgwe_probes.so, C++ over librccl);
  * ``torch``: one process per GPU (torchrun), torch.distributed "nccl" =
    RCCL, the same rank layout training uses.
busBW = algBW * 2(n-1)/n.  The reference's claim is 142 -> 228 GB/s
(random vs topology-aware placement, docs/PRD.md:117-124).  On one GPU a
sweep still runs and reports busBW 0 (nothing crosses a link): numbers on
xGMI need >= 2 GPUs.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import time

SIZES = [1 << p for p in range(20, 31, 2)]  # 1 MiB .. 1 GiB


def native_sweep(ndev: int = 0, sizes=SIZES, iters: int = 20) -> dict:
    from ..agent import probes  # noqa: PLC0415

    L = probes.lib()
    fn = L.kgwe_rccl_allreduce_sweep
    fn.restype = ctypes.c_int
    n = len(sizes)
    arr = (ctypes.c_int64 * n)(*sizes)
    us, alg, bus = (ctypes.c_double * n)(), (ctypes.c_double * n)(), (ctypes.c_double * n)()
    rc = fn(ndev, arr, n, iters, us, alg, bus)
    if rc < 0:
        raise RuntimeError(f"kgwe_rccl_allreduce_sweep failed rc={rc}")
    return {"driver": "native", "ndev": rc,
            "rows": [{"bytes": sizes[i], "us": us[i], "algbw_gbps": alg[i], "busbw_gbps": bus[i]}
                     for i in range(n)]}


def torch_sweep(sizes=SIZES, iters: int = 20, info=None) -> dict:
    """All-reduce sweep over the default process group.  With ``info`` given
    the caller owns the group (it is neither created nor destroyed here)."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    from . import dist as kdist  # noqa: PLC0415

    own = info is None
    if own:
        info = kdist.init(force_group=True)
    n = info.world_size
    rows = []
    sync = torch.cuda.synchronize if info.device.type == "cuda" else (lambda: None)
    buf = torch.zeros(max(sizes) // 2, dtype=torch.bfloat16, device=info.device)
    for s in sizes:
        x = buf[: s // 2]
        for _ in range(3):
            dist.all_reduce(x)
        sync()
        kdist.barrier(info)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        sync()
        t = kdist.all_reduce_max((time.perf_counter() - t0) / iters, info)
        alg = s / t / 1e9
        rows.append({"bytes": s, "us": t * 1e6, "algbw_gbps": alg,
                     "busbw_gbps": alg * 2 * (n - 1) / n if n > 1 else 0.0})
    del buf
    out = {"driver": "torch", "ndev": n, "rows": rows,
           "peak_busbw_gbps": max(r["busbw_gbps"] for r in rows)}
    if own:
        kdist.shutdown()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe busbw")
    ap.add_argument("--driver", choices=["native", "torch"], default="native")
    ap.add_argument("--ndev", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args(argv)
    res = native_sweep(a.ndev, iters=a.iters) if a.driver == "native" else torch_sweep(iters=a.iters)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
