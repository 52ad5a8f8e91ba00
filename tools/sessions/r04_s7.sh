#!/bin/bash
# Round 4, session 7: narrower conntrack key buckets (PCN_IPT_DEBUG_CT_KBITS): two
# sort passes instead of three against more bucket collisions in the walk.  The
# conntrack tests with 18-bit buckets (collisions everywhere), then ct_probe at
# 2^24 frames with 65536 and 262144 flows, radix 9 (default) and 10
# (build/ab/libpcn_ipt_ct_r10.so), and a kernel trace of each.
TAG=r04_s7
source "$(dirname "$0")/../gpu_lib.sh"
PCN_IPT_DEBUG_CT_KBITS=18 pytest_gpu tests_kbits18 400 tests/test_gpu_conntrack.py
KEEP_GOING=1
probe() {   # probe <name> <lib> <kbits|-> [ct_probe args]
  local name=$1 lib=$2 kb=$3
  shift 3
  for r in 1 2; do
    if [ "$kb" = - ]; then
      PCN_IPT_LIBRARY=$lib run "${name}_$r" 200 python tools/ct_probe.py --steps 6 "$@"
    else
      PCN_IPT_DEBUG_CT_KBITS=$kb PCN_IPT_LIBRARY=$lib run "${name}_$r" 200 python tools/ct_probe.py --steps 6 "$@"
    fi
  done
}
D=$R/polycube_amd/libpcn_ipt.so
R10=$R/polycube_amd/build/ab/libpcn_ipt_ct_r10.so
for flows in 65536 262144; do
  probe "f${flows}_k25" "$D" - --flows $flows
  probe "f${flows}_k18" "$D" 18 --flows $flows
  probe "f${flows}_k20" "$D" 20 --flows $flows
  probe "f${flows}_r10_k20" "$R10" 20 --flows $flows
  probe "f${flows}_r10_k25" "$R10" - --flows $flows
done
for kb in 25 18; do
  ( cd /tmp && PCN_IPT_DEBUG_CT_KBITS=$kb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_k$kb" -o run \
      --output-format csv -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_k$kb.log" 2>&1 )
  echo "== prof_k$kb rc=$?"
  find "$O/prof_k$kb" -name "*kernel_trace.csv" -delete
done
exit 0
