#!/bin/bash
# Round 4, session 14: 14-bit digits in the LRU radix-select passes (six launches a
# batch instead of seven, one digit pass fewer on a batch's stamps) -- stateful tests
# on the product build, then ct_probe against 11-bit digits
# (build/ab/libpcn_ipt_ct_ev11.so) at the bench's 2^20-slot table and at 2^18.
# (Session 13 measured a one-workgroup LRU cut: 234 us a batch at 2^18 slots against
# ~140 for the passes; removed.)
TAG=r04_s14
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_stateful 600 tests/test_gpu_conntrack.py tests/test_gpu_firewall.py
KEEP_GOING=1
NAMES="ev11" run ct_ab_ev 400 bash tools/ab.sh lib
NAMES="ev11" PROBE_ARGS="--cap-log2 18" run ct_ab_ev_c18 400 bash tools/ab.sh lib
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_ct" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_ct.log" 2>&1 )
echo "== prof_ct rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
