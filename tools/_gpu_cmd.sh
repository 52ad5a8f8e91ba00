set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "config_parity or fuzz_parity or counters" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python tools/ablate.py --variants "jit,jit:-DPCN_FLUSH_ROT=0,jit,jit:-DPCN_FLUSH_ROT=0,jit,jit:-DPCN_FLUSH_ROT=0" --hits 0.5 --iters 40 > gpurun_out/ab_rot.log 2>&1
cut -c1-150 gpurun_out/ab_rot.log
