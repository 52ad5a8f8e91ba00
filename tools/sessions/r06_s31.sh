#!/bin/bash
# Round 6, session 31: the up-sweep's last pass with equal-digit vectors aggregated:
# radix and conntrack suites, kernel traces against a build without (uni0), probes.
TAG=${TAG:-r06_s31}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_rx 600 tests/test_gpu_radix.py
for v in new uni0; do
  lib=$R/polycube_amd/libpcn_ipt.so
  [ $v = uni0 ] && lib=$R/polycube_amd/build/ab/libpcn_ipt_uni0.so
  ( cd /tmp && PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$v.log" 2>&1 )
  echo "== prof_$v rc=$?"
  python3 tools/trace_seq.py "$O/prof_$v" > "$O/prof_${v}_seq.txt" 2>&1 || true
  python3 tools/ktsum.py "$O/prof_$v" > "$O/prof_$v.txt" 2>&1 || true
  find "$O" -name "*kernel_trace.csv" -delete
done
for r in 1 2; do
  run probe_new_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_LIBRARY=$R/polycube_amd/build/ab/libpcn_ipt_uni0.so run probe_uni0_$r 300 python tools/ct_probe.py --steps 6
done
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
exit 0
