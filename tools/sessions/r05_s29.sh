#!/bin/bash
# Round 5, session 29: key buckets of 2^kbits >= n (24 bits at 2^24: three 8-bit
# sort passes) against 2^kbits >= 2n (25 bits, a 9-bit first pass); the stateful
# tests on the new rule (the colliding-connections test restates it).
TAG=r05_s29
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
run ab_lib 600 env NAMES="k25" bash tools/ab.sh lib
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_fw 600 tests/test_gpu_firewall.py
pytest_gpu tests_split 600 tests/test_gpu_flow_split.py
exit 0
