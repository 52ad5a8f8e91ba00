#!/bin/bash
# Round 5, session 28: what ct_count's counter flush costs (a measurement build
# that skips it: timing only), under a kernel trace of both libraries.
TAG=r05_s28
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run ab_lib 600 env NAMES="noflush" bash tools/ab.sh lib
for L in default noflush; do
  lib=$R/polycube_amd/libpcn_ipt.so; [ $L = noflush ] && lib=$R/polycube_amd/build/ab/libpcn_ipt_ct_noflush.so
  ( cd /tmp && PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$L" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$L.log" 2>&1 )
  echo "== prof_$L rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
exit 0
