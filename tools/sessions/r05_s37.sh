#!/bin/bash
# Round 5, session 37: ct_heads keys per thread, 16 (default) against 32 and 8 (fewer,
# larger workgroups: fewer reservation atomics on the five class counters); kernel
# statistics of each.
TAG=r05_s37
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run ab_lib 600 env NAMES="hp32 hp8" bash tools/ab.sh lib
for L in default hp32 hp8; do
  lib=$R/polycube_amd/libpcn_ipt.so; [ $L != default ] && lib=$R/polycube_amd/build/ab/libpcn_ipt_ct_$L.so
  ( cd /tmp && PCN_IPT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$L" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$L.log" 2>&1 )
  echo "== prof_$L rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
exit 0
