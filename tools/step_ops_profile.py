"""Which framework ops launch the small kernels of one Llama-3-8B training
step (copies, fills, casts): torch.profiler over one step after warmup, aten
ops ranked by device time with call counts.  GPU only.

    PYTHONPATH=. python tools/step_ops_profile.py [--model llama3-8b] [--warmup 2]
"""
from __future__ import annotations

import argparse

import torch
from torch.profiler import ProfilerActivity, profile

from kgwe.bench.train import TrainConfig, Trainer
from kgwe.parallel import dist as kdist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=40)
    a = ap.parse_args()
    info = kdist.init()
    tr = Trainer(TrainConfig(model=a.model), info)
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_device_time_total", row_limit=a.rows, max_name_column_width=40,
                   max_shapes_column_width=60), flush=True)
    ka = prof.key_averages()
    print(ka.table(sort_by="device_time_total", row_limit=a.rows, max_name_column_width=60), flush=True)


if __name__ == "__main__":
    main()
