set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dense.log 2>&1; rc=$?
tail -3 gpurun_out/t_dense.log
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/ablate.py --cfg 5 --log2n 22 --variants "jit,jit4,jit" --hits 0.5 > gpurun_out/ab_dense.log 2>&1
CFG5_HOOK=tc timeout -k 10 600 python tools/ablate.py --cfg 5 --log2n 22 --variants "jit" --hits 0.5 >> gpurun_out/ab_dense.log 2>&1
cut -c1-170 gpurun_out/ab_dense.log
