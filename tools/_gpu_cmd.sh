set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conntrack.py tests/test_gpu_firewall.py -x -q --timeout 120 --timeout-method thread -k "not fuzz_parity" > gpurun_out/gpu_ct_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_ct_tests.log; [ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/gpu_ct_tests.log | head; exit $rc; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-e2e --no-fw > gpurun_out/bench_ct.json 2> gpurun_out/bench_ct.err
rc=$?; python -c "import json; d=json.load(open('gpurun_out/bench_ct.json')); print(d['value'], d['stateful_conntrack'])"; exit $rc
