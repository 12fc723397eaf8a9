"""Training-stack sanity at full scale: Llama-3-8B on ONE fixed synthetic
batch for N steps (the model must memorise it, so the loss has to fall fast
from ln(vocab) ~ 11.8).  Exercises every HIP kernel, the sharded-DP AdamW and
the transposed-weight refresh together at the bench shape.  GPU only.

    python tools/convergence.py [--steps 30] [--micro-batch 4] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from kgwe.bench.train import TrainConfig, Trainer
    from kgwe.parallel import dist as kdist

    info = kdist.init(force_group=True)
    tr = Trainer(TrainConfig(model=a.model, micro_batch=a.micro_batch, seq_len=a.seq_len, lr=a.lr,
                             data="fixed"), info)
    losses, t0 = [], time.perf_counter()
    for i in range(a.steps):
        loss = float(tr.step().float().item())
        losses.append(round(loss, 4))
        print(f"step {i + 1:3d} loss {loss:.4f}", flush=True)
    res = {"model": a.model, "tokens_per_step": tr.tokens_per_step, "lr": a.lr, "steps": a.steps,
           "data": "one fixed synthetic batch (memorisation)", "ln_vocab": round(math.log(tr.cfg.vocab_size), 4),
           "losses": losses, "wall_s": round(time.perf_counter() - t0, 1),
           "finite": all(math.isfinite(x) for x in losses)}
    if info.is_main:
        print(json.dumps(res), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
    kdist.shutdown()
    return 0 if res["finite"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
