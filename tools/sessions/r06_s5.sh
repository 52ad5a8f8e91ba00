#!/bin/bash
# Round 6, session 5: where the fused stage A's extra 420 us go (measurement builds of the
# chain program: no stale-port tracking / records built but not stored / no records), and
# the traffic without ICMP (no stale-port look-backs), fused against ct_prep.
TAG=r06_s5
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
for r in 1 2; do
  run fused_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_DBG_HZ=1" run nostale_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_DBG_CTREC=1" run nostore_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_DBG_CTREC=2" run norec_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_DBG_CTREC=2 -DPCN_DBG_HZ=1" run norec_nostale_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_CT_FUSED=0 run prep_$r 300 python tools/ct_probe.py --steps 6
  run fused_noicmp_$r 300 python tools/ct_probe.py --steps 6 --p-icmp 0 --p-err 0
  PCN_IPT_DEBUG_CT_FUSED=0 run prep_noicmp_$r 300 python tools/ct_probe.py --steps 6 --p-icmp 0 --p-err 0
done
exit 0
