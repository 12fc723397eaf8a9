"""Tune the GEMMs of the Llama training step on MI355X and write the results
file that ``kgwe.utils.gemm_tuning.enable()`` loads.

    python tools/tune_gemm.py [--model llama3-8b] [--seq-len 4096] [--micro-batch 2]

Runs one training step with TunableOp tuning ON: every new GEMM shape is timed
over the hipBLASLt candidate solutions.  A heartbeat thread prints progress
and rewrites the results file every 30 s, so a run cut short still leaves the
shapes it finished; a re-run loads them and only tunes what is missing.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_results(path: str) -> int:
    """The results-file format TunableOp reads back: validator lines, then one
    "op_signature,params_signature,solution,time_ms" line per tuned shape."""
    import torch.cuda.tunable as tunable

    results = tunable.get_results()
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        for k, v in tunable.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for op_sig, param_sig, kernel, ms in results:
            f.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
    os.replace(tmp, path)
    return len(results)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from kgwe.bench.train import TrainConfig, Trainer
    from kgwe.parallel import dist as kdist
    from kgwe.utils import gemm_tuning

    out = a.out or str(gemm_tuning.RESULTS)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    os.environ["KGWE_GEMM_TUNING"] = "0"  # the Trainer must not enable TunableOp itself
    info = kdist.init(force_group=True)
    tr = Trainer(TrainConfig(model=a.model, seq_len=a.seq_len, micro_batch=a.micro_batch), info)
    t0 = time.time()
    tr.step()  # allocator warm, kernels loaded, before tuning starts
    torch.cuda.synchronize()
    print(f"[tune] untuned step {time.time() - t0:.1f}s", flush=True)
    os.environ["KGWE_GEMM_TUNING"] = "1"
    gemm_tuning.enable(out, tune=True)
    stop = threading.Event()

    def heartbeat():
        while not stop.wait(30):
            n = write_results(out)
            print(f"[tune] {time.time() - t0:.0f}s: {n} shapes tuned so far", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    tr.step()
    torch.cuda.synchronize()
    stop.set()
    n = write_results(out)
    print(f"[tune] done in {time.time() - t0:.0f}s: {n} GEMM shapes -> {out}", flush=True)
    import torch.cuda.tunable as tunable

    for r in tunable.get_results():
        print("[tune]", *r, flush=True)
    kdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
