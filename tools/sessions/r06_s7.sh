#!/bin/bash
# Round 6, session 7: key buckets by Mersenne folding (no 64-bit division), the stale
# fix kernel over 1024-group runs with its masks loaded at once, and the LDS-coalesced
# record stores (PCN_CTREC_LDS) as an A/B.
TAG=r06_s7
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
PCN_IPT_JIT_DEFS="-DPCN_CTREC_LDS=1" pytest_gpu tests_ct_lds 600 tests/test_gpu_conntrack.py -k "stage_a or headline_size or icmp_only or long_runs"
for r in 1 2; do
  run ct_fused_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_CTREC_LDS=1" run ct_lds_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
( cd /tmp && PCN_IPT_JIT_DEFS="-DPCN_CTREC_LDS=1" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof_lds" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof_lds.log" 2>&1 )
echo "== ct_prof_lds rc=$?"
python3 tools/ktsum.py "$O/ct_prof" > "$O/ct_prof.txt" 2>&1 || true
python3 tools/ktsum.py "$O/ct_prof_lds" > "$O/ct_prof_lds.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_sweep 900 tests/test_gpu_sweep.py -k stateful
exit 0
