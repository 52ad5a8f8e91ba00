#!/bin/bash
# Round 4, session 1: HEAD checks of the new hooks, the bench line with its new legs,
# the 2-rank self-launch, config-2 fixed-cost ablations at 2^20 and 2^24, PMC traffic
# for configs 2/3/5, and the queued long-run threshold A/B of the stateful walk.
TAG=r04_s1
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_new 300 tests/test_gpu_horus.py::test_stale_groups_stay_inside_their_words \
  tests/test_gpu_conntrack.py::test_long_runs_of_colliding_connections tests/test_gpu_parity.py -k "not ragged"
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 50 --warmup 10
cp "$O/bench.log" "$O/bench_full.log"
PCN_BENCH_DEVICE=0 run bench_2rank 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw \
  --no-hits --no-update
# config 2: where the fixed cost of a 2^20 launch goes
for n in 20 24; do
  run ablate_cfg2_$n 600 python -u tools/ablate.py --cfg 2 --log2n $n --hits 0.5 --iters 30 \
    --variants "jit,jit1,jit4,jit5,jit,jit@GRID_CUS=128,jit@GRID_CUS=512"
done
ktrace ktrace_cfg2_20 2 20 100
ktrace ktrace_cfg3_24 3 24 30
# PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE) on the HEAD chain programs
( cd /tmp && timeout -k 10 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1 ) || true
pmc pmc_cfg3 3 24
pmc pmc_cfg2 2 20
pmc pmc_cfg5 5 22 xdp
pmc pmc_cfg5_tc 5 22 tc
# stateful walk: long-run threshold 64 / 96 against 128
NAMES="lr64 lr96" run ct_ab_lr 600 bash tools/ab.sh lib
exit 0
