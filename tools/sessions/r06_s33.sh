#!/bin/bash
# Round 6, session 33: the LRU digit passes adding the first two digits once, then lane by lane or by bit ballots:
# conntrack suite, probe, kernel trace.
TAG=${TAG:-r06_s33}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py tests/test_gpu_flow_split.py
for r in 1 2; do run ct_probe_$r 300 python tools/ct_probe.py --steps 6; done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
python3 tools/ktsum.py "$O/ct_prof" > "$O/ct_prof.txt" 2>&1 || true
python3 tools/trace_seq.py "$O/ct_prof" > "$O/ct_prof_seq.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
exit 0
