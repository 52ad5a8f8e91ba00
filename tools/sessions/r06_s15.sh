#!/bin/bash
# Round 6, session 15: ct_count's bins as a row per workgroup plus one reduction
# kernel (against the per-workgroup device atomics), the next round's loads issued
# before the atomics: conntrack suite, timing A/B, kernel trace, stateful sweep.
TAG=${TAG:-r06_s15}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py tests/test_gpu_flow_split.py
for r in 1 2; do
  run ct_rows_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_CT_COUNT_ATOMIC=1 run ct_atomic_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
python3 tools/ktsum.py "$O/ct_prof" > "$O/ct_prof.txt" 2>&1 || true
python3 tools/trace_seq.py "$O/ct_prof" > "$O/ct_prof_seq.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_sweep 900 tests/test_gpu_sweep.py -k stateful
exit 0
