#!/bin/bash
# Round 4, session 13: the one-workgroup LRU cut against the multi-workgroup passes
# on tables it takes (2^18 slots, the pcn_ipt_ct_enable default, and 2^16), 2^16 flows.
TAG=r04_s13
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
NAMES="lrupass" PROBE_ARGS="--cap-log2 18" run ct_ab_lru_c18 400 bash tools/ab.sh lib
NAMES="lrupass" PROBE_ARGS="--cap-log2 17 --flows 32768" run ct_ab_lru_c17 400 bash tools/ab.sh lib
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_ct18" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 --cap-log2 18 > "$O/prof_ct18.log" 2>&1 )
echo "== prof_ct18 rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
