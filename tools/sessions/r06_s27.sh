#!/bin/bash
# Round 6, session 27: the flow split's owner words without scratch: flow-split and
# conntrack suites, kernel trace of the split, the bench line.
TAG=${TAG:-r06_s27}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_fs 900 tests/test_gpu_flow_split.py tests/test_gpu_conntrack.py
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-e2e > "$O/prof.log" 2>&1 )
echo "== prof rc=$?"
python3 tools/ktsum.py "$O/prof" > "$O/prof.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
run bench 500 python bench.py --steps 50 --warmup 10
exit 0
