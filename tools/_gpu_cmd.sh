set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_s7.log 2>&1 || { tail -20 gpurun_out/gpu_tests_s7.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s7.log
timeout -k 10 900 python tools/ablate.py --variants "jit,jit:-DPCN_STAGE_FAST=0,jit,jit:-DPCN_STAGE_FAST=0,jit" --hits 0.5 --iters 40 > gpurun_out/ab_stage.log 2>&1
cat gpurun_out/ab_stage.log
