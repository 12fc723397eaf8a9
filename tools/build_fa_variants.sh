#!/bin/bash
# Build one timing binary per flash-attention compile-time variant into
# fa_var_bin/ (git-ignored, travels with gpurun); run with tools/gpu_fa_variants.sh.
# "base" is the 8-wave x 1 sub-block forward (the previous default).
set -e
cd "$(dirname "$0")/.."
mkdir -p fa_var_bin
rm -f fa_var_bin/fa_*
b() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "${@:2}" tools/fa_variants.hip -o fa_var_bin/fa_$1; }
b base -DFA_FWD_WAVES=8 -DFA_FWD_QPW=1 &
b w4 -DFA_FWD_WAVES=4 -DFA_FWD_QPW=1 &
b base2 -DFA_FWD_WAVES=8 -DFA_FWD_QPW=1 &
b w2q2v -DFA_FWD_WAVES=2 -DFA_FWD_QPW=2 -mllvm -amdgpu-mfma-vgpr-form=1 &
wait
