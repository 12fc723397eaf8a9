#!/bin/bash
# Full bench (sched latency + 8B FSDP training) + rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.log | cut -c1-1500
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --in-process --steps 2 --warmup 1 --no-sched --no-cluster ${BENCH_ARGS} > gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
