#!/bin/bash
# One runner for everything this repository does on an MI355X box:
#
#   gpurun --timeout 1100 -- 'bash tools/gpu.sh <task> [args...]'
#
# Tasks (each GPU step runs under its own time limit; the first step that
# times out, aborts or crashes ends the script):
#   check                 GPU test suite, __graft_entry__.smoke(), default bench line
#   tests [pytest args]   GPU tests only (default: the whole suite)
#   bench [bench args]    python bench.py ...
#   prof  [bench args]    rocprofv3 kernel trace + stats of two in-process training steps
#   pmc OUT C1,C2,.. -- prog.py [args]
#                         one rocprofv3 --pmc pass (kernel trace only) of a python program;
#                         per-kernel table in gpurun_out/OUT/pmc_per_kernel.txt
#                         (PMC_KERNELS="substr ..." restricts it to matching kernel names)
#   trace OUT -- prog.py [args]
#                         rocprofv3 kernel trace + stats of a python program
#   wgrad [bench args]    weight-gradient GEMM: numerics, then tools/wgrad_kernel_bench.py
#   attn                  attention numerics, then tools/attn_bench.py
#   decode-bench [M]      decode projections (batch M, default 32) and decode attention, kernel by kernel
#   fa-variants           time / compare the flash-attention compile-time variants in fa_var_bin/
#   attn-modes M...       forward attention: numerics tests + timing at B = 2 / 4, once per KGWE_FA_FWD value
#                         (selects a kernel only with profiles/r03_attn/skew_kernel.patch applied; plain: attn-modes 0)
#   ops                   tools/ops_bench.py (every hand-written op against its roofline)
#   infer N [args]        co-location bench with N clients (kgwe.bench.infer colocate)
#   sched [args]          extender latency bench (kgwe.bench.sched_latency)
#   sched-suite           the eight latency / pressure runs reported under profiles/*_sched/
#   probe-pmc             counter validation of the HBM / LDS probe kernels
#   ab VAR=VALUE [bench args]
#                         the training bench with VAR=VALUE set, then without, twice over, on
#                         the same box (KGWE_OPS_LIB=path/of/another/libkgwe_ops.so compares
#                         two builds of the kernels; KGWE_WGRAD=library two dW paths)
# Output goes to gpurun_out/<task>*; summaries worth keeping are copied by hand
# into profiles/.
set -o pipefail
task=${1:?task}; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PYTEST="python -u -m pytest -v -rs --timeout 120 --timeout-method thread"

rocprof_env() { cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; }

# run LIMIT LOG cmd...: one GPU step; on failure prints the log's tail and ends the script.
run() {
  local limit=$1 log=$2; shift 2
  echo "== $* (limit ${limit}s) -> $log"
  timeout -k 10 "$limit" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -40 "$log"; echo "step failed rc=$rc"; exit $rc; fi
}

case "$task" in
check)
  run 120 gpurun_out/probe_hbm.log python -c "
from kgwe.agent import probes
for gb in (1, 4):
    print(gb, 'GiB', probes.probe_hbm(0, gb << 30, 10))"
  cat gpurun_out/probe_hbm.log
  # a failing test (rc 1) does not stop the later steps: the bench line is still wanted
  echo "== pytest -m gpu"
  timeout -k 10 800 $PYTEST tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_gpu.log
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  run 200 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
  tail -2 gpurun_out/smoke.log
  run 600 gpurun_out/bench_default.log python bench.py "$@"
  tail -1 gpurun_out/bench_default.log | cut -c1-2000
  exit $rc ;;
tests)
  [ $# -eq 0 ] && set -- tests -m gpu
  run 800 gpurun_out/pytest_gpu.log $PYTEST "$@"
  tail -5 gpurun_out/pytest_gpu.log ;;
bench)
  run 700 gpurun_out/bench.log python bench.py "$@"
  tail -1 gpurun_out/bench.log | cut -c1-2000 ;;
prof)
  rocprof_env; rm -rf gpurun_out/prof
  run 400 gpurun_out/prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --in-process --steps 2 --warmup 1 --no-sched --no-cluster "$@"
  f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  python3 tools/prof_summary.py "$f" gpurun_out/prof/summary --title "bench.py training step (2 steps)" --steps 2 \
    && head -45 gpurun_out/prof/summary/SUMMARY.md
  t=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
  python3 tools/step_table.py "$t" > gpurun_out/prof/summary/step_table.md && cat gpurun_out/prof/summary/step_table.md ;;
pmc)
  out=gpurun_out/${1:?out dir}; counters=${2:?counters}; shift 2; [ "$1" = "--" ] && shift
  rocprof_env; rm -rf "$out"; mkdir -p "$out"
  echo "== pmc ${counters} -- $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${counters//,/ } -d "$out/run" -o run --output-format csv -- \
    python3 "$@" > "$out/pmc.log" 2>&1 || { tail -5 "$out/pmc.log"; exit 1; }
  f=$(find "$out/run" -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_dump.py "$f" ${PMC_KERNELS} > "$out/pmc_per_kernel.txt" && cat "$out/pmc_per_kernel.txt" ;;
trace)
  out=gpurun_out/${1:?out dir}; shift; [ "$1" = "--" ] && shift
  rocprof_env; rm -rf "$out"; mkdir -p "$out"
  run 300 "$out/trace.log" rocprofv3 --kernel-trace --stats -d "$out/run" -o run --output-format csv -- python3 "$@"
  f=$(find "$out/run" -name "*kernel_stats.csv" | head -1)
  python3 tools/prof_summary.py "$f" "$out/summary" --title "$*" && head -35 "$out/summary/SUMMARY.md" ;;
wgrad)
  run 300 gpurun_out/wgrad_test.log $PYTEST tests/test_wgrad_gpu.py -x
  tail -3 gpurun_out/wgrad_test.log
  run 400 gpurun_out/wgrad_bench.log python -u tools/wgrad_kernel_bench.py "$@"
  cat gpurun_out/wgrad_bench.log ;;
attn)
  run 300 gpurun_out/attn_test.log $PYTEST tests/test_flash_attn_gpu.py -x
  tail -3 gpurun_out/attn_test.log
  run 200 gpurun_out/attn_bench.log python tools/attn_bench.py
  grep -v amdgpu.ids gpurun_out/attn_bench.log | tail -8 ;;
decode-bench)
  # serving-batch decode kernels one by one: projections against the library GEMM, attention split sweep
  run 300 gpurun_out/decode_bench.log python tools/skinny_bench.py "$@"
  grep "^M=" gpurun_out/decode_bench.log ;;
fa-variants)
  # compile-time variants of native/ops/flash_attn.hip built by tools/build_fa_variants.sh into
  # fa_var_bin/: "base" first (it dumps its outputs), every other binary is compared with it;
  # FA_B / FA_CAUSAL in the environment choose batch and masking
  [ -x fa_var_bin/fa_base ] || { echo "run tools/build_fa_variants.sh first"; exit 1; }
  run 120 gpurun_out/fa_var_base.log fa_var_bin/fa_base base
  tail -1 gpurun_out/fa_var_base.log
  for b in fa_var_bin/fa_*; do
    tag=${b#fa_var_bin/fa_}; [ "$tag" = base ] && continue
    run 120 "gpurun_out/fa_var_$tag.log" "$b" "$tag" /tmp/fa_base.bin
    tail -1 "gpurun_out/fa_var_$tag.log"
  done ;;
attn-modes)
  # forward kernel variants (KGWE_FA_FWD, read once per process): numerics, then timing
  for mode in "$@"; do
    export KGWE_FA_FWD=$mode
    echo "== KGWE_FA_FWD=$mode"
    run 300 "gpurun_out/attn_test_m$mode.log" $PYTEST tests/test_flash_attn_gpu.py -x
    tail -1 "gpurun_out/attn_test_m$mode.log"
    run 200 "gpurun_out/attn_modes_m$mode.log" python tools/attn_fwd_modes.py
    grep "^mode" "gpurun_out/attn_modes_m$mode.log"
  done ;;
ops)
  run 400 gpurun_out/ops_bench.log python tools/ops_bench.py "$@"
  cat gpurun_out/ops_bench.log ;;
infer)
  n=${1:?clients}; shift
  mkdir -p gpurun_out/infer
  pct=$(python -c "print(100 / $n)")
  echo "== colocate $n clients"
  timeout -k 10 400 python -m kgwe.bench.infer colocate --clients "$n" --cu-percent "$pct" --batch 4 --prompt 512 --new 257 --json "$@" \
    > "gpurun_out/infer/coloc_$n.json" 2> "gpurun_out/infer/coloc_$n.err" || { tail -20 "gpurun_out/infer/coloc_$n.err"; exit 1; }
  python - "gpurun_out/infer/coloc_$n.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ("aggregate_tokens_per_s", "alone_tokens_per_s", "combined_batch_tokens_per_s", "density_vs_alone",
        "per_client_step_ms", "hw_queues_per_client", "cu_masks", "mode", "hbm_cap")
print({k: d[k] for k in keys if k in d})
EOF
  ;;
sched)
  run 900 gpurun_out/sched.log python -m kgwe.bench.sched_latency "$@"
  tail -1 gpurun_out/sched.log | cut -c1-3000 ;;
sched-suite)
  # The extender latency runs that profiles/*_sched/ reports (CPU only; run on the
  # GPU box because its cores are the ones the driver's bench runs on).
  mkdir -p gpurun_out/sched
  one() { # name args...
    local name=$1; shift
    echo "== $name: $*"
    timeout -k 10 900 python -m kgwe.bench.sched_latency --json --timeout 700 "$@" \
      > "gpurun_out/sched/$name.json" 2> "gpurun_out/sched/$name.err" || { tail -5 "gpurun_out/sched/$name.err"; exit 1; }
    python tools/sched_brief.py "gpurun_out/sched/$name.json"
  }
  one scale_1250n_names_50pps   --pods 3000 --nodes 1250 --rate 50 --node-cache
  one scale_1250n_names_50pps_sampled --pods 3000 --nodes 1250 --rate 50 --node-cache --nodes-to-score 0
  one scale_1250n_names_100pps  --pods 5000 --nodes 1250 --rate 100 --node-cache
  one scale_1250n_full_10pps    --pods 600 --nodes 1250 --rate 10 --full-nodes
  one scale_64n_names_50pps     --pods 2000 --nodes 64 --rate 50 --node-cache
  one pressure_64n              --pods 2000 --nodes 64 --rate 50 --lifetime 5,15 --node-cache
  one pressure_1250n            --pods 10000 --nodes 1250 --rate 100 --lifetime 32,64 --node-cache
  one pressure_1250n_2x         --pods 8000 --nodes 1250 --rate 100 --lifetime 60,120 --node-cache
  ;;
probe-pmc)
  rocprof_env
  run 120 gpurun_out/probe_plain.log python3 tools/probe_pmc.py run
  tail -1 gpurun_out/probe_plain.log
  declare -A pass=( [f]="FETCH_SIZE" [w]="WRITE_SIZE"
                    [s]="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
                    [r]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_BUBBLE_sum" )
  for k in f w s r; do
    rm -rf "gpurun_out/ppmc_$k"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc ${pass[$k]} -d "gpurun_out/ppmc_$k" -o run --output-format csv -- \
      python3 tools/probe_pmc.py run > "gpurun_out/ppmc_$k.log" 2>&1 || { echo "pass $k failed"; tail -5 "gpurun_out/ppmc_$k.log"; exit 1; }
  done
  csv() { find "gpurun_out/ppmc_$1" -name "*counter_collection.csv" | head -1; }
  python3 tools/probe_pmc.py summarize "$(csv f)" "$(csv w)" "$(csv s)" "$(csv r)" > gpurun_out/probe_pmc_summary.md
  cat gpurun_out/probe_pmc_summary.md ;;
ab)
  setting=${1:?VAR=VALUE}; shift
  for pass in 1 2; do
    env "$setting" true || exit 2
    export "$setting"
    run 500 "gpurun_out/ab_other_$pass.log" python bench.py --no-sched --no-cluster "$@"
    echo "$setting: $(tail -1 "gpurun_out/ab_other_$pass.log" | cut -c1-300)"
    unset "${setting%%=*}"
    run 500 "gpurun_out/ab_tree_$pass.log" python bench.py --no-sched --no-cluster "$@"
    echo "default: $(tail -1 "gpurun_out/ab_tree_$pass.log" | cut -c1-300)"
  done ;;
*)
  echo "unknown task $task"; exit 2 ;;
esac
