"""Weight-gradient GEMM options at the Llama-3-8B step's shapes (T = 16,384
tokens): dW[N, K] = dY[T, N]^T X[T, K], both operands stored token-major.
GPU only.

    PYTHONPATH=. python tools/wgrad_bench.py [--tokens 16384]

Arms per shape:
  raw     torch.mm(dy.t(), x)                       (library picks the layout)
  cur     kgwe.ops.functional._Linear's choice      (transpose the smaller operand)
  both    transpose both, then the forward-style "x @ W^T" GEMM
  gemm_*  the GEMM alone of each arm (operands pre-transposed)
"""
from __future__ import annotations

import argparse

import torch

from kgwe.ops import functional as F


def bench(fn, iters=20):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    a = ap.parse_args()
    T = a.tokens
    d, f, qkv, V = 4096, 14336, 6144, 128256
    for name, N, K in (("wqkv", qkv, d), ("wo", d, d), ("w13", 2 * f, d), ("w2", d, f), ("lm_head", V, d)):
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * N * K * T
        dyT, xT = F.transpose(dy), F.transpose(x)
        arms = {
            "raw": lambda: torch.mm(dy.t(), x),
            "cur": (lambda: torch.mm(dy.t(), F.transpose(x).t())) if N >= K
                   else (lambda: torch.mm(F.transpose(dy), x)),
            "both": lambda: torch.mm(F.transpose(dy), F.transpose(x).t()),
            "gemm_tt": lambda: torch.mm(dy.t(), xT.t()),
            "gemm_nn": lambda: torch.mm(dyT, x),
            "gemm_nt": lambda: torch.mm(dyT, xT.t()),
            # dW^T = X^T dY (the other output orientation; same operands)
            "rawT": lambda: torch.mm(x.t(), dy),
            "T_tt": lambda: torch.mm(x.t(), dyT.t()),
            "T_nn": lambda: torch.mm(xT, dy),
            "T_nt": lambda: torch.mm(xT, dyT.t()),
            "tr_dy": lambda: F.transpose(dy),
            "tr_x": lambda: F.transpose(x),
        }
        cells = []
        for k, fn in arms.items():
            ms = bench(fn)
            tf = "" if k.startswith("tr_") else f" {flop / ms / 1e9:5.0f}TF"
            cells.append(f"{k}:{ms:6.3f}ms{tf}")
        print(f"{name:<8} N={N:<6} K={K:<6} " + "  ".join(cells), flush=True)
        del dy, x, dyT, xT
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
