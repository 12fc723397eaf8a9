#!/bin/bash
# Co-location with the platform's share env (XCD-aligned CU masks, 2 HW queues
# per client), 8 and 4 clients, plus a rocprofv3 kernel profile of one client.
set -o pipefail
mkdir -p gpurun_out/infer_final
export PYTHONUNBUFFERED=1
for n in 8 4; do
  pct=$(python -c "print(100 / $n)")
  timeout -k 10 300 python -m kgwe.bench.infer colocate --clients $n --cu-percent $pct --batch 4 --prompt 512 --new 257 --json \
    > gpurun_out/infer_final/coloc_$n.json 2> gpurun_out/infer_final/coloc_$n.err || { tail -20 gpurun_out/infer_final/coloc_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/infer_final/coloc_$n.json'));print($n, {k:d[k] for k in ('aggregate_tokens_per_s','alone_tokens_per_s','combined_batch_tokens_per_s','density_vs_alone','per_client_step_ms','hw_queues_per_client','cu_masks')})"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/infer_final/prof -o run --output-format csv -- python -m kgwe.bench.infer run --batch 4 --prompt 512 --new 257 --json > gpurun_out/infer_final/prof_run.json 2> gpurun_out/infer_final/prof.err || { tail -20 gpurun_out/infer_final/prof.err; exit 1; }
find gpurun_out/infer_final/prof -name "*kernel_stats.csv" | head -3
