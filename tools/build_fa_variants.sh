#!/bin/bash
# Build one timing binary per flash-attention compile-time variant into
# fa_var_bin/ (git-ignored, travels with gpurun); run with `tools/gpu.sh fa-variants`.
# "base" is the shipped configuration; every other binary is compared to it.
set -e
cd "$(dirname "$0")/.."
mkdir -p fa_var_bin
rm -f fa_var_bin/fa_*
b() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "${@:2}" tools/fa_variants.hip -o fa_var_bin/fa_$1; }
b base -fno-slp-vectorize &
b nofuse -fno-slp-vectorize -DFA_DQ_DELTA=0 &
wait
