#!/bin/bash
# Fused decode projections: numerics + graph decode tests, tok/s fused vs
# unfused (one client, whole GPU), kernel profile of the fused step.
set -o pipefail
mkdir -p gpurun_out/decode
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_infer_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "not colocated" > gpurun_out/decode/pytest.log 2>&1 || { tail -40 gpurun_out/decode/pytest.log; exit 1; }
tail -2 gpurun_out/decode/pytest.log
for f in 1 0; do
  KGWE_DECODE_FUSED=$f timeout -k 10 200 python -m kgwe.bench.infer run --batch 4 --prompt 512 --new 257 --json \
    > gpurun_out/decode/run_fused$f.json 2> gpurun_out/decode/run_fused$f.err || { tail -20 gpurun_out/decode/run_fused$f.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/decode/run_fused$f.json').read().strip().splitlines()[-1]);print('fused=$f', round(d['tokens_per_s'],1), 'tok/s', round(d['step_ms'],3), 'ms/step')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/decode/prof -o run --output-format csv \
  -- python -m kgwe.bench.infer run --batch 4 --prompt 512 --new 257 --json > gpurun_out/decode/prof.log 2>&1 || { tail -20 gpurun_out/decode/prof.log; exit 1; }
python -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/decode/prof/run_kernel_stats.csv')))
for r in rows[:14]: print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Percentage'][:5], '%')"
