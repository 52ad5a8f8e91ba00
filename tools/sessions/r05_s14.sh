#!/bin/bash
# Round 5, session 14: the adaptive deal window for stage A (the stateful
# traffic is mostly rule hits) against none (PCN_IPT_DEBUG_DEAL_ADAPT=0).
TAG=r05_s14
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py tests/test_gpu_firewall.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_DEAL_ADAPT=0 run ct_probe_noadapt_$r 300 python tools/ct_probe.py --steps 6
done
run bench_ct 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-fw --no-hits --no-update
exit 0
