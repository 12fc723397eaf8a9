"""Weight-gradient GEMM variants for the Llama-3-8B projections at T tokens:
dW[N, K] = dY[T, N]^T X[T, K] computed (a) as the trainer does now
(transpose the smaller operand -> "nn"/"tt"), (b) transposed problem
dW^T = X^T dY in hipBLASLt's "nt" layout (both operands K-contiguous) + a
transpose of the result.  GPU only.   python tools/wgrad_variants.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kgwe.ops.functional import transpose  # noqa: E402


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
    T = int(os.environ.get("TOKENS", "16384"))
    for name, N, K in (("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w13", 28672, 4096),
                       ("w2", 4096, 14336)):
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        ref = (dy.float().t() @ x.float())
        cur = (lambda: torch.mm(dy.t(), transpose(x).t())) if N >= K else (lambda: torch.mm(transpose(dy), x))
        def swapped():
            wt = torch.mm(transpose(x), transpose(dy).t())  # [K, N], "nt"
            return transpose(wt)
        def nt_direct():  # dW = dY^T X as "nt": A = dY^T [N,T] row-major, B = X^T [K,T] row-major
            return torch.mm(transpose(dy), transpose(x).t())
        flops = 2.0 * T * N * K
        for label, fn in (("current", cur), ("swapped-nt", swapped), ("nt-direct", nt_direct)):
            out = fn()
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            ms = bench(fn)
            print(f"{name:5} N={N:6} K={K:6} {label:11} {ms:7.3f} ms {flops / ms / 1e9:7.0f} TF/s  rel err {err:.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
