#!/bin/bash
# Round 6, session 19: ct_count by selects with 16-byte loads and rows + reduction:
# conntrack suite (counters against the oracle), then kernel traces of the builds
# (prefetch on / off, 8 / 16 packets a thread, one / two workgroups per CU).
TAG=${TAG:-r06_s19}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py tests/test_gpu_flow_split.py
for spec in "base 1" "base 2" "pf1 1" "pf1u8 1" "u8 1" "u8 2"; do
  set -- $spec
  v=$1 w=$2
  lib=$R/polycube_amd/build/ab/libpcn_ipt_ct_$v.so
  [ $v = base ] && lib=$R/polycube_amd/libpcn_ipt.so
  ( cd /tmp && PCN_IPT_DEBUG_CT_COUNT_WPC=$w PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${v}_$w" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_${v}_$w.log" 2>&1 )
  echo "== prof_${v}_$w rc=$?"
  python3 tools/ktsum.py "$O/prof_${v}_$w" > "$O/prof_${v}_$w.txt" 2>&1 || true
  find "$O" -name "*kernel_trace.csv" -delete
done
exit 0
