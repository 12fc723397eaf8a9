#!/bin/bash
# Step time vs gradient-bucket size (KGWE_BUCKET_MELEMS, 2^20 elements), one MI355X.
set -o pipefail
mkdir -p gpurun_out/bucket
export PYTHONUNBUFFERED=1 PYTHONPATH=.
for m in ${SIZES:-100 50 200 400 100}; do
  KGWE_BUCKET_MELEMS=$m timeout -k 10 300 python bench.py --in-process --no-sched --no-cluster \
    --steps 10 --warmup 3 > gpurun_out/bucket/m$m.log 2>&1 || { tail -20 gpurun_out/bucket/m$m.log; exit 1; }
  python -c "
import json
l=[x for x in open('gpurun_out/bucket/m$m.log') if x.startswith('{')][-1]
d=json.loads(l); print('bucket ${m}M', d['ms_per_step'], 'ms/step', d['mfu_bf16_dense'], d['peak_mem_gb_rank0'], 'GB')"
done
