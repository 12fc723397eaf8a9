#!/bin/bash
# Step time and in-step GEMM times with the AdamW state streamed nontemporally
# (default) vs plain cached accesses (KGWE_ADAMW_NT=0), Llama-3-8B, one MI355X.
set -o pipefail
mkdir -p gpurun_out/adamw_nt
export PYTHONUNBUFFERED=1 PYTHONPATH=.
for nt in 1 0 1 0; do
  KGWE_ADAMW_NT=$nt timeout -k 10 300 python bench.py --in-process --no-sched --no-cluster \
    --steps 10 --warmup 3 > gpurun_out/adamw_nt/b$nt.log 2>&1 || { tail -20 gpurun_out/adamw_nt/b$nt.log; exit 1; }
  python -c "
import json
l=[x for x in open('gpurun_out/adamw_nt/b$nt.log') if x.startswith('{')][-1]
d=json.loads(l); print('nt=$nt', d['ms_per_step'], 'ms/step', d['mfu_bf16_dense'], 'loss', d['loss_per_rank'])"
done
KGWE_ADAMW_NT=1 timeout -k 10 300 python tools/gemm_instep.py > gpurun_out/adamw_nt/gi.log 2>&1
grep -v "amdgpu.ids\|Warn\|warn\|^\[kgwe" gpurun_out/adamw_nt/gi.log
