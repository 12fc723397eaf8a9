#!/bin/bash
# One gpurun call: GPU tests, bench, rocprofv3 kernel stats.  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
python -c "import kgwe.utils.amdsmi_util as a; print('amdsmi', a.available()); import torch; print(torch.cuda.get_device_name(0)); h=a.handle_for_torch_device(0); print(a.snapshot(h))" > gpurun_out/env.log 2>&1 || true
timeout -k 10 400 python -m pytest tests -m gpu -q -rs > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 420 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROFILE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 2 --no-sched ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
  echo "prof rc=$?"
fi
