#!/bin/bash
# In-step per-shape GEMM times with a candidate TunableOp table vs the default.
set -o pipefail
mkdir -p gpurun_out/tune_check
export PYTHONUNBUFFERED=1 PYTHONPATH=.
F=${TUNE_FILE:?candidate TunableOp csv}
KGWE_GEMM_TUNING_FILE=$F timeout -k 10 300 python tools/gemm_instep.py --no-overlap > gpurun_out/tune_check/cand_noov.log 2>&1 || { tail gpurun_out/tune_check/cand_noov.log; exit 1; }
timeout -k 10 300 python tools/gemm_instep.py --no-overlap > gpurun_out/tune_check/base_noov.log 2>&1 || exit 1
KGWE_GEMM_TUNING_FILE=$F timeout -k 10 300 python tools/gemm_instep.py > gpurun_out/tune_check/cand.log 2>&1 || exit 1
for f in cand_noov base_noov cand; do echo "== $f"; grep -v "amdgpu.ids\|Warn\|warn\|^\[kgwe" gpurun_out/tune_check/$f.log; done
