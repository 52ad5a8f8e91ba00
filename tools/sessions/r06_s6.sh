#!/bin/bash
# Round 6, session 6: the fused stage A without cross-workgroup waits (each group
# publishes its ports word and the lanes to complete; ct_stale_agg / ct_stale_fix
# complete them after the launch): conntrack / firewall / sweep suites, timing against
# ct_prep, kernel statistics.
TAG=r06_s6
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
for r in 1 2; do
  run ct_fused_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_CT_FUSED=0 run ct_prep_$r 300 python tools/ct_probe.py --steps 6
done
run ct_fused_1flow 300 python tools/ct_probe.py --steps 3 --flows 1 --p-noise 0 --p-err 0 --p-icmp 0
run ct_fused_noicmp 300 python tools/ct_probe.py --steps 6 --p-icmp 0 --p-err 0
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
python3 tools/ktsum.py "$O/ct_prof" > "$O/ct_prof.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_fw 900 tests/test_gpu_firewall.py tests/test_gpu_horus.py tests/test_gpu_flow_split.py
pytest_gpu tests_sweep 900 tests/test_gpu_sweep.py
exit 0
