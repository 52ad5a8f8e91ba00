#!/bin/bash
# Round 4, session 12: the LRU cut of a table of <= 2^18 slots in one workgroup and
# one launch (ct_lru_small_kernel) -- the stateful GPU tests on it, then ct_probe
# against the multi-workgroup passes (build/ab/libpcn_ipt_ct_lrupass.so) at 2^16 and
# 2^18 flows, and a kernel trace of the probe.
TAG=r04_s12
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_stateful 600 tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py
KEEP_GOING=1
NAMES="lrupass" run ct_ab_lru 400 bash tools/ab.sh lib
NAMES="lrupass" PROBE_ARGS="--flows 262144" run ct_ab_lru_f18 400 bash tools/ab.sh lib
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_ct" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_ct.log" 2>&1 )
echo "== prof_ct rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
