#!/bin/bash
# Step time vs the workgroup cap of the background (beside-backward) AdamW
# launches (KGWE_ADAMW_BG_GRID), Llama-3-8B on one MI355X.
set -o pipefail
mkdir -p gpurun_out/adamw_grid
export PYTHONUNBUFFERED=1
for g in ${GRIDS:-0 1024 256 128 64}; do
  KGWE_ADAMW_BG_GRID=$g timeout -k 10 300 python bench.py --in-process --no-sched --no-cluster \
    --steps 10 --warmup 3 > gpurun_out/adamw_grid/g$g.log 2>&1 || { tail -20 gpurun_out/adamw_grid/g$g.log; exit 1; }
  python -c "
import json,sys
l=[x for x in open('gpurun_out/adamw_grid/g$g.log') if x.startswith('{')][-1]
d=json.loads(l); print('grid $g', d['ms_per_step'], 'ms/step', d['mfu_bf16_dense'])"
done
KGWE_ADAMW_BG_GRID=${GI_GRID:-256} PYTHONPATH=. timeout -k 10 300 python tools/gemm_instep.py > gpurun_out/adamw_grid/gi.log 2>&1
grep -v amdgpu.ids gpurun_out/adamw_grid/gi.log | grep -v Warn
