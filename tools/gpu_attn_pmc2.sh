#!/bin/bash
# Attention microbench + 3 counter passes (kernel-trace only, no sys/runtime trace).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/attn_bench.log | tail -3; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/pmc1 -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/pmc1.log 2>&1; rc=$?; echo "pmc1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/pmc2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d gpurun_out/pmc3 -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/pmc3.log 2>&1; rc=$?; echo "pmc3 rc=$rc"
for i in 1 2 3; do f=$(find gpurun_out/pmc$i -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 tools/pmc_dump.py "$f"; done
