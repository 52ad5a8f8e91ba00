#!/bin/bash
# Round 5, session 16: the LRU cut with its stamp loads in flight together (16 a thread
# in each radix-select pass, 4 in the eviction).
TAG=r05_s16
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
