#!/bin/bash
# Flash-attention iteration on one MI355X: numerics tests, timing at the bench
# shape, and a per-kernel rocprofv3 profile of the same run.
set -o pipefail
mkdir -p gpurun_out/fa_iter
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/fa_iter/pytest.log 2>&1 || { tail -30 gpurun_out/fa_iter/pytest.log; exit 1; }
tail -2 gpurun_out/fa_iter/pytest.log
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/fa_iter/attn_bench.log 2>&1 \
  || { tail -20 gpurun_out/fa_iter/attn_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_iter/attn_bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fa_iter/prof -o run --output-format csv \
  -- python tools/attn_bench.py > gpurun_out/fa_iter/prof.log 2>&1 || { tail -20 gpurun_out/fa_iter/prof.log; exit 1; }
f=$(find gpurun_out/fa_iter/prof -name "*kernel_stats.csv" | head -1)
python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]:
    print(r['Name'][:70].ljust(70), r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Percentage'][:5], '%')"
rm -rf gpurun_out/fa_iter/pmc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS \
  -d gpurun_out/fa_iter/pmc -o run --output-format csv -- python3 tools/attn_bwd_only.py > gpurun_out/fa_iter/pmc.log 2>&1 || { tail -5 gpurun_out/fa_iter/pmc.log; exit 1; }
f=$(find gpurun_out/fa_iter/pmc -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 tools/pmc_dump.py "$f"
