#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -m pytest tests/test_ops_gpu.py -q -x -k "fsdp2 or rope_rejects or tiny" > gpurun_out/pytest_fsdp.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_fsdp.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; rc=$?; echo "probe rc=$rc"; grep -v "amdgpu.ids" gpurun_out/rccl_probe.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-sched > gpurun_out/bench_8b.log 2>&1; echo "bench8b rc=$?"; tail -12 gpurun_out/bench_8b.log
