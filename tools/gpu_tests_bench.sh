#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests -m gpu -q -rs > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-sched ${BENCH_ARGS} > gpurun_out/bench_quick.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_quick.log | cut -c1-1200
