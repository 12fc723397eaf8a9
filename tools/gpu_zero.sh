#!/bin/bash
# GPU tests, then sharded-DP vs FSDP2 bench, then a kernel profile of the default path.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -m pytest tests -m gpu -q -rs > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-sched --parallel zero > gpurun_out/bench_zero.log 2>&1; rc=$?; echo "zero rc=$rc"; tail -1 gpurun_out/bench_zero.log | cut -c1-900; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-sched --parallel fsdp > gpurun_out/bench_fsdp.log 2>&1; rc=$?; echo "fsdp rc=$rc"; tail -1 gpurun_out/bench_fsdp.log | cut -c1-900; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_zero
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-sched > gpurun_out/prof_zero.log 2>&1; rc=$?; echo "prof rc=$rc"
