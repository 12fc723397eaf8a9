#!/bin/bash
# Hardware counters for the flash-attention kernels (counters only with --kernel-trace; no sys/runtime trace).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc1 -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/pmc1.log 2>&1; rc=$?; echo "pmc1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM -d gpurun_out/pmc2 -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/pmc2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmc3 -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/pmc3.log 2>&1; rc=$?; echo "pmc3 rc=$rc"
find gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 -name "*.csv" | head
