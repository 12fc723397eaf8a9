#!/bin/bash
# PMC counters of the flash-attention kernels at the training batch (B=4):
# MFMA busy, wave occupancy, waits, instruction mix.  One --pmc pass.
set -o pipefail
mkdir -p gpurun_out/fa_pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/fa_pmc/run
FA_B=4 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS \
  -d gpurun_out/fa_pmc/run -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/fa_pmc/pmc.log 2>&1 || { tail -5 gpurun_out/fa_pmc/pmc.log; exit 1; }
f=$(find gpurun_out/fa_pmc/run -name "*counter_collection.csv" | head -1)
python3 tools/pmc_dump.py "$f" > gpurun_out/fa_pmc/pmc_per_kernel.txt
cat gpurun_out/fa_pmc/pmc_per_kernel.txt
