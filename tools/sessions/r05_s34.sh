#!/bin/bash
# Round 5, session 34: the radix up-sweep's digit grouping in the last pass only;
# the segment waves' count (64 default, against 8 and 1,024: ct_seg_fix took 21 us
# with 1,024 waves and nothing to fix); one batch's kernel sequence; tests.
TAG=r05_s34
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
run ab_lib 600 env NAMES="w8 w1024" bash tools/ab.sh lib
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 3 > "$O/tr.log" 2>&1 )
echo "== tr rc=$?"
python3 tools/trace_seq.py "$O/tr" > "$O/sequence.txt"
( cd /tmp && PCN_IPT_LIBRARY=$R/polycube_amd/build/ab/libpcn_ipt_ct_w8.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr8" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 3 > "$O/tr8.log" 2>&1 )
echo "== tr8 rc=$?"
python3 tools/trace_seq.py "$O/tr8" > "$O/sequence_w8.txt"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
