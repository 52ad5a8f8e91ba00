#!/bin/bash
# Round 5, session 42: speculative segment length 512 (default) against 1024 and 2048
# records now that only the active cuts get waves (fewer cuts: less for ct_seg_fix
# to chain on traffic whose flows open and close inside the batch).
TAG=r05_s42
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run ab_lib 600 env NAMES="seg1024 seg2048" bash tools/ab.sh lib
for L in default seg1024; do
  lib=$R/polycube_amd/libpcn_ipt.so; [ $L != default ] && lib=$R/polycube_amd/build/ab/libpcn_ipt_ct_$L.so
  ( cd /tmp && PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$L" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$L.log" 2>&1 )
  echo "== prof_$L rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
exit 0
