set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 900 python tools/ablate.py --variants "jit,jit:-DPCN_FASTPATH=0,jit:-DPCN_PF_FAST=0,jit:-DPCN_FASTPATH=0+-DPCN_PF_FAST=0,jit,jit:-DPCN_FASTPATH=0" --hits 0.5 --iters 40 > gpurun_out/ab_fast.log 2>&1
cat gpurun_out/ab_fast.log | cut -c1-200
