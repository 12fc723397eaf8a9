#!/bin/bash
# A/B of the dK/dV kernels: numerics under each, timing + kernel trace.
set -o pipefail
mkdir -p gpurun_out/fa_ab
export PYTHONUNBUFFERED=1
for kv in 64 32; do
  KGWE_FA_DKDV=$kv timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/fa_ab/pytest_$kv.log 2>&1 || { echo "tests failed for $kv"; tail -30 gpurun_out/fa_ab/pytest_$kv.log; exit 1; }
  echo "dkdv$kv: $(tail -1 gpurun_out/fa_ab/pytest_$kv.log)"
  KGWE_FA_DKDV=$kv timeout -k 10 200 python tools/attn_bench.py > gpurun_out/fa_ab/bench_$kv.log 2>&1 || { tail -20 gpurun_out/fa_ab/bench_$kv.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/fa_ab/bench_$kv.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KGWE_FA_DKDV=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fa_ab/prof -o run --output-format csv \
  -- python tools/attn_bench.py > gpurun_out/fa_ab/prof.log 2>&1 || { tail -20 gpurun_out/fa_ab/prof.log; exit 1; }
grep -E "fa_bwd|fa_fwd" gpurun_out/fa_ab/prof/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
