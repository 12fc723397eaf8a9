#!/bin/bash
# Throughput at micro-batch 4 (16k tokens / GPU / step) + op-level profile.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-sched --micro-batch 4 > gpurun_out/bench_mb4.log 2>&1; rc=$?; echo "mb4 rc=$rc"; tail -1 gpurun_out/bench_mb4.log | cut -c1-800; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/torch_prof.py --micro-batch 4 --rows 30 > gpurun_out/torch_prof_mb4.log 2>&1; rc=$?; echo "prof rc=$rc"
