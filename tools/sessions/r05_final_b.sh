#!/bin/bash
# Round 5, final evidence (part b), after the flow split's count kernel with its
# frame loads issued together: its tests and the stateful bench leg; kernel-trace statistics of each config and of
# the headline bench; per-kernel counters of the stateful pipeline (ct_prep,
# ct_walk, ct_heads, ct_count and the radix sort's kernels): fetch, write, SQ
# cycles and the L2 -> memory read requests.
TAG=r05_final_b
source "$(dirname "$0")/../gpu_lib.sh"
# first the flow split with every item's frame words loaded together
pytest_gpu tests_flow 300 tests/test_gpu_flow_split.py tests/test_gpu_multirank.py
KEEP_GOING=1
run bench_ct 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-fw --no-hits --no-update
ktrace ktrace_cfg3_24 3 24 30
ktrace ktrace_cfg2_20 2 20 100
ktrace ktrace_cfg5_22 5 22 30 xdp
ktrace ktrace_cfg5_22_tc 5 22 30 tc
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_bench" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/prof_bench.log" 2>&1 )
echo "== prof_bench rc=$?"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
K="ct_prep ct_walk ct_heads ct_count radix_pass radix_up pcn_classify_jit"
pmcct ct_fetch "FETCH_SIZE" "$K"
pmcct ct_write "WRITE_SIZE" "$K"
pmcct ct_sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU" "$K"
pmcct ct_rdreq "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "$K"
pmcct ct_lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "$K"
exit 0
