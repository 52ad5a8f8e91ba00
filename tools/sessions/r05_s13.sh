#!/bin/bash
# Round 5, session 13: stage A without its discarded counters (A/B against
# PCN_IPT_DEBUG_STAGE_A_COUNTS=1), with the stateful GPU tests on it.
TAG=r05_s13
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py tests/test_gpu_horus.py tests/test_gpu_sweep.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_STAGE_A_COUNTS=1 run ct_probe_sacount_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
