#!/bin/bash
# Attention microbench + per-kernel times + stall counters.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_flash_attn_gpu.py -q -x > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/attn_bench.log | tail -3; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/attn_stats gpurun_out/attn_pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_stats -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/attn_stats.log 2>&1; rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -h "fa_" gpurun_out/attn_stats/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/attn_pmc -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/attn_pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"
