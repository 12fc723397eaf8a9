#!/bin/bash
# rocprofv3 counter validation of the HBM / LDS-staged probe kernels: one
# --pmc pass per counter group (TCC FETCH_SIZE uses 3 TCC counters, WRITE_SIZE
# 2: separate passes), each under its own hard time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ppmc_f gpurun_out/ppmc_w gpurun_out/ppmc_s
timeout -k 10 120 python3 tools/probe_pmc.py run > gpurun_out/probe_plain.log 2>&1 || { tail -5 gpurun_out/probe_plain.log; exit 1; }
tail -1 gpurun_out/probe_plain.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/ppmc_f -o run --output-format csv -- python3 tools/probe_pmc.py run > gpurun_out/ppmc_f.log 2>&1 || { echo "fetch pass failed"; tail -5 gpurun_out/ppmc_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/ppmc_w -o run --output-format csv -- python3 tools/probe_pmc.py run > gpurun_out/ppmc_w.log 2>&1 || { echo "write pass failed"; tail -5 gpurun_out/ppmc_w.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES -d gpurun_out/ppmc_s -o run --output-format csv -- python3 tools/probe_pmc.py run > gpurun_out/ppmc_s.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/ppmc_s.log; exit 1; }
F=$(find gpurun_out/ppmc_f -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/ppmc_w -name "*counter_collection.csv" | head -1)
S=$(find gpurun_out/ppmc_s -name "*counter_collection.csv" | head -1)
rm -rf gpurun_out/ppmc_r
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_BUBBLE_sum -d gpurun_out/ppmc_r -o run --output-format csv -- python3 tools/probe_pmc.py run > gpurun_out/ppmc_r.log 2>&1 || { echo "raw pass failed"; tail -5 gpurun_out/ppmc_r.log; exit 1; }
R=$(find gpurun_out/ppmc_r -name "*counter_collection.csv" | head -1)
python3 tools/probe_pmc.py summarize "$F" "$W" "$S" "$R" > gpurun_out/probe_pmc_summary.md && cat gpurun_out/probe_pmc_summary.md
