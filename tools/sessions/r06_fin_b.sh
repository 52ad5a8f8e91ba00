#!/bin/bash
# Round 6, final evidence (part b): every GPU test, the smoke, the stateful probe and its
# kernel statistics, kernel traces of every config's classify launches (rocprofv3 --stats),
# and the walk's / stage A's fetch and L2 -> memory read requests.
TAG=${TAG:-r06_fin_b}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
python3 tools/ktsum.py "$O/ct_prof" > "$O/ct_prof.txt" 2>&1 || true
python3 tools/trace_seq.py "$O/ct_prof" > "$O/ct_prof_seq.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
ktrace ktrace_cfg3_24 3 24 50
ktrace ktrace_cfg2_20 2 20 50
ktrace ktrace_cfg5_22 5 22 50
ktrace ktrace_cfg5_22_tc 5 22 50 tc
for k in ktrace_cfg3_24 ktrace_cfg2_20 ktrace_cfg5_22 ktrace_cfg5_22_tc; do
  python3 tools/ktsum.py "$O/$k" > "$O/$k.txt" 2>&1 || true
done
find "$O" -name "*kernel_trace.csv" -delete
K="ct_walk ct_heads ct_count radix_pass radix_up classify ct_stale"
pmcct ct_fetch "FETCH_SIZE" "$K"
pmcct ct_rdreq "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "$K"
exit 0
