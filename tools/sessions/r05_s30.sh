#!/bin/bash
# Round 5, session 30: what the speculative-segment machinery costs on the bench
# traffic, which has no run long enough to cut (PCN_CT_SEG=0 build: no cut waves in
# the walk, no ct_seg_fix), under a kernel trace of both libraries.
TAG=r05_s30
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run ab_lib 600 env NAMES="noseg" bash tools/ab.sh lib
for L in default noseg; do
  lib=$R/polycube_amd/libpcn_ipt.so; [ $L = noseg ] && lib=$R/polycube_amd/build/ab/libpcn_ipt_ct_noseg.so
  ( cd /tmp && PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$L" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$L.log" 2>&1 )
  echo "== prof_$L rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
exit 0
