#!/bin/bash
# Co-location throughput vs clients x hardware queues per client (ledger CU masks).
set -o pipefail
mkdir -p gpurun_out/infer_sweep
export PYTHONUNBUFFERED=1
for n in 8 4 2; do
  for q in 1 2 3 4 6; do
    timeout -k 10 200 python -m kgwe.bench.infer colocate --clients $n --cu-percent $((100 / n)) --batch 4 --prompt 512 --new 257 \
      --hw-queues $q --skip-baselines --json > gpurun_out/infer_sweep/c${n}_q${q}.json 2> gpurun_out/infer_sweep/c${n}_q${q}.err \
      || { tail -20 gpurun_out/infer_sweep/c${n}_q${q}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/infer_sweep/c${n}_q${q}.json'));print('clients=$n q=$q agg', d['aggregate_tokens_per_s'], 'step_ms', d['per_client_step_ms'][0], d['cu_masks'][:2])"
  done
done
