#!/bin/bash
# Round 5, session 26: ct_count with 16 packets' loads in flight per thread (was 4:
# 16 dependent round trips a thread at 2^24), ct_heads in 1024-thread workgroups
# (its per-workgroup reservation atomics land on five addresses); A/B of each.
TAG=r05_s26
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
run ab_lib 900 env NAMES="u4 h256 old" bash tools/ab.sh lib
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
