#!/bin/bash
# Step time vs WHERE the side-stream optimizer update of a completed gradient
# bucket is issued (KGWE_ZERO_UPDATE_AT=bucket|attn), Llama-3-8B, one MI355X.
set -o pipefail
mkdir -p gpurun_out/zero_sched
export PYTHONUNBUFFERED=1
for m in ${MODES:-bucket attn}; do
  KGWE_ZERO_UPDATE_AT=$m timeout -k 10 300 python bench.py --in-process --no-sched --no-cluster \
    --steps 10 --warmup 3 > gpurun_out/zero_sched/$m.log 2>&1 || { tail -20 gpurun_out/zero_sched/$m.log; exit 1; }
  python -c "
import json
l=[x for x in open('gpurun_out/zero_sched/$m.log') if x.startswith('{')][-1]
d=json.loads(l); print('$m', d['ms_per_step'], 'ms/step', d['mfu_bf16_dense'], 'loss', d['loss_per_rank'])"
done
KGWE_ZERO_UPDATE_AT=${GI_MODE:-attn} PYTHONPATH=. timeout -k 10 300 python tools/gemm_instep.py > gpurun_out/zero_sched/gi.log 2>&1
grep -v amdgpu.ids gpurun_out/zero_sched/gi.log | grep -v Warn
