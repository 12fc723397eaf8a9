#!/bin/bash
# Co-location diagnosis: one decode client alone (whole GPU / 32-CU masks of two
# shapes), then 8 clients with ledger / strided / no masks.
set -o pipefail
mkdir -p gpurun_out/infer_diag
export PYTHONUNBUFFERED=1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -m kgwe.bench.infer run --batch 4 --prompt 512 --new 257 --json \
    > gpurun_out/infer_diag/$name.json 2> gpurun_out/infer_diag/$name.err || { tail -5 gpurun_out/infer_diag/$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/infer_diag/$name.json'));print('$name', round(d['tokens_per_s'],1), 'tok/s', round(d['step_ms'],3), 'ms/step')"
}
run alone_full || exit 1
run alone_mask_contig HSA_CU_MASK=0:0-31 || exit 1
run alone_mask_strided HSA_CU_MASK=0:$(python -c "print(','.join(str(8*j) for j in range(32)))") || exit 1
run alone_mask_contig64 HSA_CU_MASK=0:0-63 || exit 1
run alone_nograph --no-graph 2>/dev/null || true
for style in ledger strided none; do
  timeout -k 10 300 python -m kgwe.bench.infer colocate --clients 8 --batch 4 --prompt 512 --new 257 --mask-style $style --json \
    > gpurun_out/infer_diag/coloc_$style.json 2> gpurun_out/infer_diag/coloc_$style.err || { tail -20 gpurun_out/infer_diag/coloc_$style.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/infer_diag/coloc_$style.json'));print('$style', {k:d[k] for k in ('aggregate_tokens_per_s','alone_tokens_per_s','combined_batch_tokens_per_s','per_client_step_ms','start_skew_ms')})"
done
