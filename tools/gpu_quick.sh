#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 180 python tools/attn_probe.py > gpurun_out/attn_probe.log 2>&1; echo "attn rc=$?"; cat gpurun_out/attn_probe.log | grep -v amdgpu.ids
timeout -k 10 240 python bench.py --model llama3.2-1b --seq-len 4096 --micro-batch 2 --steps 5 --warmup 2 --no-sched > gpurun_out/bench_1b.log 2>&1; echo "bench1b rc=$?"; tail -12 gpurun_out/bench_1b.log
timeout -k 10 500 python bench.py --steps 3 --warmup 2 --no-sched > gpurun_out/bench_8b.log 2>&1; echo "bench8b rc=$?"; tail -12 gpurun_out/bench_8b.log
