set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_cfg5.log 2>&1; rc=$?
tail -3 gpurun_out/t_cfg5.log
[ $rc = 0 ] || exit $rc
TAG=r02_c5 bash tools/bench_configs.sh
