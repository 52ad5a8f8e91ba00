#!/bin/bash
# Round 5, session 40: ct_heads clears the long echo replies' key-bucket bitmap after a
# batch that set bits (ct_hbits_clear was a launch a batch); the stateful suites.
TAG=r05_s40
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_fw 600 tests/test_gpu_firewall.py
pytest_gpu tests_sweep 900 tests/test_gpu_sweep.py
exit 0
