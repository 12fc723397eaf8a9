#!/bin/bash
# Run the flash-attention variant binaries built by tools/build_fa_variants.sh
# (fa_var_bin/fa_*), base first; every variant is compared to base's dump.
# Each binary runs causal (the training shape) and, with FA_CAUSAL=0, full.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/fa_variants.log
: > $out
timeout -k 10 60 fa_var_bin/fa_base base >> $out 2>&1 || exit $?
for b in fa_var_bin/fa_*; do
  t=${b##*/fa_}
  [ "$t" = base ] && continue
  timeout -k 10 60 $b $t /tmp/fa_base.bin >> $out 2>&1 || exit $?
done
for b in fa_var_bin/fa_*; do
  t=${b##*/fa_}
  FA_CAUSAL=0 timeout -k 10 60 $b ${t}_full /tmp/none.bin >> $out 2>&1 || exit $?
done
# second pass, reverse order (clock drift / box noise)
for b in $(ls -r fa_var_bin/fa_*); do
  t=${b##*/fa_}
  timeout -k 10 60 $b ${t}_2 /tmp/fa_base.bin >> $out 2>&1 || exit $?
done
cat $out
