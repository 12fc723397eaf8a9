mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python tools/gemm_instep.py > gpurun_out/gi_default.log 2>&1 && \
timeout -k 10 300 python tools/gemm_instep.py --no-overlap > gpurun_out/gi_nooverlap.log 2>&1 && \
KGWE_GEMM_TUNING=0 timeout -k 10 300 python tools/gemm_instep.py > gpurun_out/gi_notune.log 2>&1
