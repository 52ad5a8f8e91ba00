set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_horus.py > gpurun_out/t_horus.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/t_horus.log | head -40
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -5 gpurun_out/t_all.log
exit $rc
