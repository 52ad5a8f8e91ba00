#!/bin/bash
# Round 5, session 11: radix seg pass with buffer loads, values loaded with the ranking, one write-out loop.

TAG=r05_s11
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
KEEP_GOING=1
for r in 1 2; do
  PCN_IPT_DEBUG_RADIX=rts run ct_probe_rts_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_RADIX=rts512 run ct_probe_rts512_$r 300 python tools/ct_probe.py --steps 6
done
for m in rts rts512; do
  export PCN_IPT_DEBUG_RADIX=$m
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof_$m" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof_$m.log" 2>&1 )
  echo "== ct_prof_$m rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
exit 0
