#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NCCL_DEBUG=INFO timeout -k 10 150 python tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "probe rc=$?"
grep -v "amdgpu.ids" gpurun_out/rccl_probe.log | grep -vE "^\s*$" | tail -60
