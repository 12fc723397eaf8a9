#!/bin/bash
# Co-location vs hardware queue count: GPU_MAX_HW_QUEUES per client process.
set -o pipefail
mkdir -p gpurun_out/infer_diag2
export PYTHONUNBUFFERED=1
for q in 1 2; do
for style in strided ledger; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -m kgwe.bench.infer colocate --clients 8 --batch 4 --prompt 512 --new 257 --mask-style $style --json \
    > gpurun_out/infer_diag2/coloc_q${q}_$style.json 2> gpurun_out/infer_diag2/coloc_q${q}_$style.err || { tail -20 gpurun_out/infer_diag2/coloc_q${q}_$style.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/infer_diag2/coloc_q${q}_$style.json'));print('q$q $style', {k:d[k] for k in ('aggregate_tokens_per_s','alone_tokens_per_s','combined_batch_tokens_per_s','per_client_step_ms')})"
done
done
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -m kgwe.bench.infer colocate --clients 4 --batch 4 --prompt 512 --new 257 --cu-percent 25 --mask-style strided --json \
    > gpurun_out/infer_diag2/coloc4_q1.json 2> gpurun_out/infer_diag2/coloc4_q1.err || { tail -20 gpurun_out/infer_diag2/coloc4_q1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/infer_diag2/coloc4_q1.json'));print('4 clients q1', {k:d[k] for k in ('aggregate_tokens_per_s','alone_tokens_per_s','per_client_step_ms')})"
