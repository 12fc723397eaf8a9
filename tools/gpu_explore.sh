#!/bin/bash
# Op-level profile of one 8B step + micro-batch 4 throughput check.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/torch_prof.py > gpurun_out/torch_prof.log 2>&1; rc=$?; echo "torch_prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --no-sched --micro-batch 4 > gpurun_out/bench_mb4.log 2>&1; rc=$?; echo "mb4 rc=$rc"; tail -1 gpurun_out/bench_mb4.log | cut -c1-900
