#!/bin/bash
# Round 5, final evidence (part g) on the final tree: part f plus sessions 39-40
# (the walk plan in the walk and ct_tail; ct_heads clears the echo-reply bitmap):
# every GPU test, the smoke, the headline bench line (every leg), the stateful
# kernel statistics and the walk's fetch and L2 -> memory read requests.
TAG=r05_final_g
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 50 --warmup 10
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_bench" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/prof_bench.log" 2>&1 )
echo "== prof_bench rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
K="ct_prep ct_walk ct_heads ct_count radix_pass radix_up"
pmcct ct_fetch "FETCH_SIZE" "$K"
pmcct ct_rdreq "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "$K"
exit 0
