#!/bin/bash
# TunableOp GEMM tuning of the bench step at micro-batch 4 (16,384-token GEMMs);
# the existing micro-batch-2 entries are kept (the tuner only tunes new shapes).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cp kgwe/tuning/tunableop_mi355x.csv gpurun_out/tunableop_mi355x.csv
timeout -k 10 1080 python tools/tune_gemm.py --micro-batch 4 --out gpurun_out/tunableop_mi355x.csv \
  2>&1 | tee gpurun_out/tune_mb4.log | grep -E "tune|rror"
