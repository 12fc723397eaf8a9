#!/bin/bash
# Round check on one MI355X: GPU test suite, driver smoke(), default bench line.
# A test failure does not stop the later steps (the bench line is still
# wanted); a timeout / abort / crash does.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "
from kgwe.agent import probes
for gb in (1, 4):
    print(gb, 'GiB', probes.probe_hbm(0, gb << 30, 10))" > gpurun_out/probe_hbm.log 2>&1 || { tail -20 gpurun_out/probe_hbm.log; exit 1; }
cat gpurun_out/probe_hbm.log
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rs --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 500 python bench.py ${BENCH_ARGS} > gpurun_out/bench_default.log 2>&1 \
  || { tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-1500
exit $rc
