#!/bin/bash
# Round 6, session 18 (measurement builds): ct_count's time with and without its
# LDS atomics, loads only, 8 / 32 packets in flight a thread; kernel trace each.
TAG=${TAG:-r06_s18}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
for v in base ab1 ab2 u8 u32; do
  lib=$R/polycube_amd/build/ab/libpcn_ipt_ct_$v.so
  [ $v = base ] && lib=$R/polycube_amd/libpcn_ipt.so
  ( cd /tmp && PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$v.log" 2>&1 )
  echo "== prof_$v rc=$?"
  python3 tools/ktsum.py "$O/prof_$v" > "$O/prof_$v.txt" 2>&1 || true
  find "$O" -name "*kernel_trace.csv" -delete
done
exit 0
