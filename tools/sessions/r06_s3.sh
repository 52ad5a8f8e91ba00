#!/bin/bash
# Round 6, session 3: the stateful stage A that builds the walk records itself (ct_prep
# skipped, frames read once): conntrack / firewall / sweep suites, timing A/B against
# ct_prep, kernel statistics.
TAG=r06_s3
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
for r in 1 2; do
  run ct_probe_fused_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_CT_FUSED=0 run ct_probe_prep_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
python3 tools/ktsum.py "$O/ct_prof" > "$O/ct_prof.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_fw 900 tests/test_gpu_firewall.py tests/test_gpu_horus.py tests/test_gpu_flow_split.py
pytest_gpu tests_sweep 900 tests/test_gpu_sweep.py
exit 0
