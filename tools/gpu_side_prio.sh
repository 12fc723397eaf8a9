#!/bin/bash
# Step time vs the HIP stream priority of the side stream that runs the
# optimizer update beside backward (KGWE_SIDE_PRIORITY), Llama-3-8B, one MI355X.
set -o pipefail
mkdir -p gpurun_out/side_prio
export PYTHONUNBUFFERED=1 PYTHONPATH=.
python -c "import torch; print('stream priority range', torch.cuda.Stream.priority_range())"
for p in ${PRIOS:-0 1 -1 0 1}; do
  KGWE_SIDE_PRIORITY=$p timeout -k 10 300 python bench.py --in-process --no-sched --no-cluster \
    --steps 10 --warmup 3 > gpurun_out/side_prio/p$p.log 2>&1 || { tail -20 gpurun_out/side_prio/p$p.log; exit 1; }
  python -c "
import json
l=[x for x in open('gpurun_out/side_prio/p$p.log') if x.startswith('{')][-1]
d=json.loads(l); print('prio=$p', d['ms_per_step'], 'ms/step', d['mfu_bf16_dense'])"
done
