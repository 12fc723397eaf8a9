#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests -m gpu -q -rs -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; echo "attn rc=$rc"; grep -v amdgpu.ids gpurun_out/attn_bench.log | tail -5
