#!/bin/bash
# Round 5, session 8: reduce-then-scan radix passes (PCN_IPT_DEBUG_RADIX=rts)
# against the onesweep look-back: sort tests in both modes, stateful batch
# timings and kernel traces of both.
TAG=r05_s8
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_RADIX=rts run ct_probe_rts_$r 300 python tools/ct_probe.py --steps 6
done
export PCN_IPT_DEBUG_RADIX=rts
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof_rts" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof_rts.log" 2>&1 )
echo "== ct_prof_rts rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_ct_rts 600 tests/test_gpu_conntrack.py
exit 0
