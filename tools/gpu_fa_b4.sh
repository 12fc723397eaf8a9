#!/bin/bash
# Flash-attention variants at the training step's batch (B=4), causal, each twice.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/fa_b4.log
: > $out
export FA_B=4
timeout -k 10 60 fa_var_bin/fa_base base >> $out 2>&1 || exit $?
for b in fa_var_bin/fa_*; do t=${b##*/fa_}; [ "$t" = base ] && continue
  timeout -k 10 60 $b $t /tmp/fa_base.bin >> $out 2>&1 || exit $?; done
for b in $(ls -r fa_var_bin/fa_*); do t=${b##*/fa_}
  timeout -k 10 60 $b ${t}_2 /tmp/fa_base.bin >> $out 2>&1 || exit $?; done
cat $out
