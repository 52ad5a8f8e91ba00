#!/bin/bash
# Round 6, session 29: radix passes in 512-thread workgroups, two per CU (super-tiles
# half as long): radix and conntrack suites, kernel traces with 512 / 1024, probes.
TAG=${TAG:-r06_s29}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_rx 600 tests/test_gpu_radix.py
for w in 512 1024; do
  ( cd /tmp && PCN_IPT_DEBUG_RADIX_PB=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$w" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$w.log" 2>&1 )
  echo "== prof_$w rc=$?"
  python3 tools/ktsum.py "$O/prof_$w" > "$O/prof_$w.txt" 2>&1 || true
  python3 tools/trace_seq.py "$O/prof_$w" > "$O/prof_${w}_seq.txt" 2>&1 || true
  find "$O" -name "*kernel_trace.csv" -delete
done
for r in 1 2; do
  run probe512_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_RADIX_PB=1024 run probe1024_$r 300 python tools/ct_probe.py --steps 6
done
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
exit 0
