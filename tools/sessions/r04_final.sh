#!/bin/bash
# Round 4, final evidence on the committed tree, one call: every GPU test and the
# smoke; HBM traffic of the HEAD chain programs (configs 3, 2, 5 XDP / TC) into
# profiles/pmc_traffic.json; the bench lines that report it (config 3 headline with
# every leg, config 2 at 2^20, config 5 XDP and TC at 2^22) and the 2-rank
# self-launch; kernel-trace statistics of each config and of the headline bench.
TAG=r04_final
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# the two-item deal for chains of 2+ summary blocks (config 5) against the build
# without it (build/ab/libpcn_ipt_base.so); config 3 (one block) as a control
run ab_deal2_cfg5 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5,1 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
CFG5_HOOK=tc run ab_deal2_cfg5_tc 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
run ab_deal2_cfg3 300 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5 --iters 30 --variants "jit,lib:base"
KEEP_GOING=0
pmct config3 3 24
pmct config2 2 20
pmct config5 5 22 xdp
pmct config5_tc 5 22 tc
KEEP_GOING=1
run bench 400 python bench.py --steps 50 --warmup 10
run bench_cfg2 200 python bench.py --config 2 --log2n 20 --steps 100 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5 200 python bench.py --config 5 --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5_tc 200 python bench.py --config 5 --hook tc --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
PCN_BENCH_DEVICE=0 run bench_2rank 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw \
  --no-hits --no-update
ktrace ktrace_cfg3_24 3 24 30
ktrace ktrace_cfg2_20 2 20 100
ktrace ktrace_cfg5_22 5 22 30 xdp
ktrace ktrace_cfg5_22_tc 5 22 30 tc
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_bench" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/prof_bench.log" 2>&1 )
echo "== prof_bench rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
# per-kernel counters of the stateful pipeline (ct_prep, ct_walk, ct_heads, ct_count)
K="ct_prep ct_walk ct_heads ct_count"
pmcct ct_fetch "FETCH_SIZE" "$K"
pmcct ct_write "WRITE_SIZE" "$K"
pmcct ct_sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU" "$K"
exit 0
