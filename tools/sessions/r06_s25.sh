#!/bin/bash
# Round 6, session 25: the bench line after ct_count and the radix up-sweep /
# column scan; measurement builds of the LRU deletion (no slot store / no stores)
# under a kernel trace.
TAG=${TAG:-r06_s25}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run bench 500 python bench.py --steps 50 --warmup 10
for v in ev1 ev2; do
  ( cd /tmp && PCN_IPT_LIBRARY=$R/polycube_amd/build/ab/libpcn_ipt_ct_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$v.log" 2>&1 )
  echo "== prof_$v rc=$?"
  python3 tools/ktsum.py "$O/prof_$v" > "$O/prof_$v.txt" 2>&1 || true
  find "$O" -name "*kernel_trace.csv" -delete
done
exit 0
