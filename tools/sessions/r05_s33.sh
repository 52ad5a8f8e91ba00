#!/bin/bash
# Round 5, session 33: the radix up-sweep adds the first lane's digit group with one
# atomic (the last pass's input holds each connection's packets as one run of equal
# keys: 45 us against 21-24); one batch's kernel sequence; the sort and stateful tests.
TAG=r05_s33
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 3 > "$O/tr.log" 2>&1 )
echo "== tr rc=$?"
python3 tools/trace_seq.py "$O/tr" > "$O/sequence.txt"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
