"""Micro-benchmark of the memory-bound HIP ops at Llama-3-8B step shapes:
time per call and effective HBM bandwidth (bytes the op must move / time).

    python tools/ops_bench.py [--tokens 16384]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kgwe.ops import functional as K  # noqa: E402


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def report(name, ms, nbytes):
    print(f"{name:<34} {ms * 1000:8.1f} us  {nbytes / ms / 1e9:6.2f} TB/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    T = ap.parse_args().tokens
    dev = "cuda"
    H, F = 4096, 14336
    bf = torch.bfloat16
    x = torch.randn(T, H, device=dev, dtype=bf)
    r = torch.randn(T, H, device=dev, dtype=bf)
    w = torch.ones(H, device=dev, dtype=bf)
    eb = T * H * 2
    report("rmsnorm fwd (+residual)", bench(lambda: K.rmsnorm(x, w, 1e-5, residual=r)), 4 * eb)
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    y, hres = K.rmsnorm(xr, wr, 1e-5, residual=r.clone().requires_grad_())
    g1, g2 = torch.randn_like(y), torch.randn_like(hres)
    report("rmsnorm bwd (+residual grad)",
           bench(lambda: torch.autograd.grad((y, hres), (xr, wr), (g1, g2), retain_graph=True)),
           4 * eb)
    gu = torch.randn(T, 2 * F, device=dev, dtype=bf).requires_grad_()
    o = K.swiglu(gu)
    go = torch.randn_like(o)
    report("swiglu fwd", bench(lambda: K.swiglu(gu)), 3 * T * F * 2)
    report("swiglu bwd", bench(lambda: torch.autograd.grad(o, gu, go, retain_graph=True)),
           5 * T * F * 2)
    report("transpose [T, 4096]", bench(lambda: K.transpose(x)), 2 * eb)
    big = torch.randn(T, F, device=dev, dtype=bf)
    report("transpose [T, 14336]", bench(lambda: K.transpose(big)), 2 * T * F * 2)
    report("torch copy [T, 4096] (reference)", bench(lambda: x.clone()), 2 * eb)


if __name__ == "__main__":
    main()
