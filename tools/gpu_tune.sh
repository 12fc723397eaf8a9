#!/bin/bash
# Tune the Llama-3-8B step's GEMMs (TunableOp over hipBLASLt), then bench with the results.
# Results go to gpurun_out/ (merged back even when the tuning run is cut short).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OUT=gpurun_out/tunableop_mi355x.csv
[ -f kgwe/tuning/tunableop_mi355x.csv ] && cp kgwe/tuning/tunableop_mi355x.csv $OUT
export PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 KGWE_TUNE_MS_PER_SOLUTION=${KGWE_TUNE_MS_PER_SOLUTION:-4} KGWE_TUNE_ITERS=${KGWE_TUNE_ITERS:-4}
timeout -k 10 ${TUNE_SECONDS:-840} python tools/tune_gemm.py --micro-batch ${MB:-2} --out $OUT > gpurun_out/tune.log 2>&1; rc=$?; echo "tune rc=$rc"; grep "\[tune\]" gpurun_out/tune.log | tail -25 | cut -c1-250; [ $rc -ne 0 ] && exit $rc
KGWE_GEMM_TUNING_FILE=$OUT timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-sched --micro-batch ${MB:-2} > gpurun_out/bench_tuned.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_tuned.log | cut -c1-700
