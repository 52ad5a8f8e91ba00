set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_firewall.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_fw_tests.log 2>&1
rc=$?; tail -25 gpurun_out/gpu_fw_tests.log; exit $rc
