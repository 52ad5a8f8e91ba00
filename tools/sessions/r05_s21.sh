#!/bin/bash
# Round 5, session 21: (a) the radix pass kernel with the first sub-tile's keys
# waited for before the loop, so the loop head no longer waits for the previous
# sub-tile's stores; (b) a layout experiment for the walk's record fills: the
# same stateful batch with the frames of every 64-frame group ordered by key
# bucket (ct_probe --group-sort), so each 128-byte line of walk records holds
# records of nearby keys, walked by waves in flight together.
TAG=r05_s21
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_plain_$r 300 python tools/ct_probe.py --steps 6
  run ct_probe_gsort_$r 300 python tools/ct_probe.py --steps 6 --group-sort
done
for v in plain gsort; do
  a=""; [ $v = gsort ] && a="--group-sort"
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof_$v" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 $a > "$O/ct_prof_$v.log" 2>&1 )
  echo "== ct_prof_$v rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
exit 0
