"""Op-level attribution of one Llama-3-8B training step (torch.profiler):
which aten ops own the device time, grouped by input shapes — used to find
stray copies / fills around the HIP kernels.  GPU only.

    python tools/torch_prof.py [--micro-batch 2] [--steps 1]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--rows", type=int, default=45)
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from kgwe.bench.train import TrainConfig, Trainer
    from kgwe.parallel import dist as kdist

    info = kdist.init(force_group=True)
    tr = Trainer(TrainConfig(model=args.model, micro_batch=args.micro_batch,
                             seq_len=args.seq_len), info)
    for _ in range(2):
        tr.step()
    tr.sync()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        for _ in range(args.steps):
            tr.step()
        tr.sync()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_device_time_total", row_limit=args.rows, max_name_column_width=60,
                   max_shapes_column_width=90))
    kdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
