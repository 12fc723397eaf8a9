#!/bin/bash
# Forward-kernel PMC passes for both forward variants (ping-pong, classic).
set -o pipefail
mkdir -p gpurun_out/fa_pmc
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for variant in pp classic; do
  for pass in 1 2; do
    eval "C=\$P$pass"
    d=gpurun_out/fa_pmc/${variant}_$pass; rm -rf $d
    if [ $variant = classic ]; then export KGWE_FA_FWD=classic; else unset KGWE_FA_FWD; fi
    ITERS=3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $d -o run --output-format csv -- python3 tools/attn_bwd_only.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    f=$(find $d -name "*counter_collection.csv" | head -1)
    echo "== $variant pass $pass"; python3 tools/pmc_dump.py "$f" fa_fwd
  done
done
