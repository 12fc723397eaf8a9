"""Weight-gradient GEMM: the hand-written kernel (kgwe.ops.gemm.wgrad) against
the library in every layout, on the Llama-3-8B shapes at T tokens.  Random
operands; interleaved rounds in one process; median of the rounds."""
import argparse
import statistics
import sys

import torch

sys.path.insert(0, ".")
from kgwe.ops import functional as F  # noqa: E402
from kgwe.ops.gemm import wgrad  # noqa: E402

SHAPES = {"wo/wq": (4096, 4096), "wqkv": (6144, 4096), "w13": (28672, 4096), "w2": (4096, 14336),
          "lm_head": (128256, 4096)}


def timed(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--splits", default="0")
    a = ap.parse_args()
    T = a.tokens
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        flops = 2.0 * T * N * K
        variants = {"lib tn (dy.t() @ x)": lambda: torch.mm(dy.t(), x)}
        if N >= K:
            variants["lib + transpose(x) [in-step today]"] = lambda: torch.mm(dy.t(), F.transpose(x).t())
        else:
            variants["lib + transpose(dy) [in-step today]"] = lambda: torch.mm(F.transpose(dy), x)
        # both operands transposed: the library's fastest ("nt") layout, at the price of two transposes
        variants["lib nt + transpose(dy) + transpose(x)"] = lambda: torch.mm(F.transpose(dy), F.transpose(x).t())
        dyt, xt = F.transpose(dy), F.transpose(x)
        variants["lib nt alone (operands pre-transposed)"] = lambda: torch.mm(dyt, xt.t())
        for s in [int(v) for v in a.splits.split(",")]:
            variants[f"kgwe wgrad splits={s or 'auto'}"] = (lambda s=s: wgrad(dy, x, splits=s))
        ref = torch.mm(dy.t(), x).float()
        got = wgrad(dy, x).float()
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        for fn in variants.values():
            fn()
        torch.cuda.synchronize()
        res = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                res[k].append(timed(fn, a.iters))
        print(f"{name}: dW[{N},{K}] over {T} tokens, rel err vs library {err:.2e}", flush=True)
        for k, v in res.items():
            ms = statistics.median(v)
            print(f"   {k:42s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s  (min {min(v):.3f})", flush=True)


if __name__ == "__main__":
    main()
