#!/bin/bash
# Same-box A/B of the whole training step: this tree vs the round-2
# session-2 starting point (its flash-attention + SwiGLU kernels, GEMM table,
# normal-priority update stream), alternating, Llama-3-8B, one MI355X.
set -o pipefail
mkdir -p gpurun_out/session_ab
export PYTHONUNBUFFERED=1 PYTHONPATH=.
run() {
  timeout -k 10 300 env "$@" python bench.py --in-process --no-sched --no-cluster --steps 10 --warmup 3 \
    > gpurun_out/session_ab/$tag.log 2>&1 || { tail -20 gpurun_out/session_ab/$tag.log; exit 1; }
  python -c "
import json
l=[x for x in open('gpurun_out/session_ab/$tag.log') if x.startswith('{')][-1]
d=json.loads(l); print('$tag', d['ms_per_step'], 'ms/step', d['tokens_per_s'], 'tok/s', d['mfu_bf16_dense'])"
}
for i in 1 2; do
  tag=now$i run KGWE_QUIET=1
  tag=start$i run KGWE_OPS_LIB=$PWD/fa_var_bin/libkgwe_ops_sessionstart.so KGWE_SIDE_PRIORITY=0 \
      KGWE_GEMM_TUNING_FILE=$PWD/fa_var_bin/tunable_sessionstart.csv
done
