#!/bin/bash
# Inference harness on one MI355X: decode-kernel numerics, hipGraph decode vs
# full forward, then the co-located serving runs (ledger masks, strided masks).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_infer_gpu.py -x -v -rs --timeout 400 --timeout-method thread \
  > gpurun_out/pytest_infer.log 2>&1 || { tail -40 gpurun_out/pytest_infer.log; exit 1; }
tail -12 gpurun_out/pytest_infer.log
timeout -k 10 400 python -m kgwe.bench.infer colocate --clients 8 --batch 4 --prompt 512 --new 257 --json \
  > gpurun_out/coloc_ledger.json 2> gpurun_out/coloc_ledger.err || { tail -20 gpurun_out/coloc_ledger.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/coloc_ledger.json'));print({k:d[k] for k in ('aggregate_tokens_per_s','alone_tokens_per_s','combined_batch_tokens_per_s','density_vs_alone','vs_one_process_combined_batch','per_client_tokens_per_s','start_skew_ms')})"
timeout -k 10 400 python -m kgwe.bench.infer colocate --clients 8 --batch 4 --prompt 512 --new 257 --mask-style strided --json \
  > gpurun_out/coloc_strided.json 2> gpurun_out/coloc_strided.err || { tail -20 gpurun_out/coloc_strided.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/coloc_strided.json'));print({k:d[k] for k in ('aggregate_tokens_per_s','alone_tokens_per_s','density_vs_alone','per_client_tokens_per_s')})"
