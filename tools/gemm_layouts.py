"""hipBLASLt bf16 GEMM throughput on MI355X for the Llama-3-8B step's shapes in
every operand layout (which storage order of weights / activations gives the
library's fastest kernel), plus a square 8192^3 reference.  GPU only.

    python tools/gemm_layouts.py [--tokens 8192]
"""
from __future__ import annotations

import argparse

import torch


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


def run(M, N, K, label):
    """C[M,N] = A[M,K] @ B[K,N]; A / B stored row-major ('n') or as the
    transpose of a row-major tensor ('t')."""
    dev = "cuda"
    out = []
    for la in "nt":
        for lb in "nt":
            a = (torch.randn(M, K, device=dev, dtype=torch.bfloat16) if la == "n"
                 else torch.randn(K, M, device=dev, dtype=torch.bfloat16).t())
            b = (torch.randn(K, N, device=dev, dtype=torch.bfloat16) if lb == "n"
                 else torch.randn(N, K, device=dev, dtype=torch.bfloat16).t())
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ms = bench(lambda: torch.mm(a, b, out=c))
            out.append((la + lb, ms, 2.0 * M * N * K / ms / 1e9))
            del a, b, c
    best = max(out, key=lambda r: r[2])
    cells = "  ".join(f"{l}:{ms:7.3f}ms {tf:6.0f}TF" for l, ms, tf in out)
    print(f"{label:<28} M={M:<6} N={N:<6} K={K:<6} {cells}   best {best[0]}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    a = ap.parse_args()
    T = a.tokens
    torch.backends.cuda.matmul.allow_bf16_reduced_precision_reduction = True
    run(8192, 8192, 8192, "square reference")
    d, f, qkv, V = 4096, 14336, 6144, 128256
    for name, n_out, k_in in (("wqkv", qkv, d), ("wo", d, d), ("w13", 2 * f, d), ("w2", d, f),
                              ("lm_head", V, d)):
        run(T, n_out, k_in, f"{name} fwd   y=xW^T")
        run(T, k_in, n_out, f"{name} dgrad dx=dyW")
        run(n_out, k_in, T, f"{name} wgrad dW=dy^Tx")


if __name__ == "__main__":
    main()
