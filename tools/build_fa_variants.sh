#!/bin/bash
# Build one timing binary per flash-attention compile-time variant into
# fa_var_bin/ (git-ignored, travels with gpurun); run with `tools/gpu.sh fa-variants`.
# "base" is the shipped configuration; every other binary is compared to it.
# Variants here: the AMDGPU machine-scheduler strategies (same source, another
# instruction order) — extend with -D flags of native/ops/flash_attn.hip as needed.
set -e
cd "$(dirname "$0")/.."
mkdir -p fa_var_bin
rm -f fa_var_bin/fa_*
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Xclang -target-feature -Xclang -packed-fp32-ops"
b() { /opt/rocm/bin/hipcc $FLAGS "${@:2}" tools/fa_variants.hip -o fa_var_bin/fa_$1 2> fa_var_bin/build_$1.log || echo "variant $1 failed to build"; }
b base &
b maxilp -mllvm -amdgpu-sched-strategy=max-ilp &
b maxmem -mllvm -amdgpu-sched-strategy=max-memory-clause &
b iterilp -mllvm -amdgpu-sched-strategy=iterative-ilp &
wait
ls -la fa_var_bin/
