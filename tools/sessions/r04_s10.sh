#!/bin/bash
# Round 4, session 10: a pack event after every launch (host only) -- every GPU test,
# the smoke and the bench lines again on it; ct_prep at 5 waves per SIMD
# (build/ab/libpcn_ipt_ct_prepw5.so, 2 VGPRs spilled) against the default on ct_probe.
TAG=r04_final2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 50 --warmup 10
run bench_cfg2 200 python bench.py --config 2 --log2n 20 --steps 100 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5 200 python bench.py --config 5 --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5_tc 200 python bench.py --config 5 --hook tc --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
PCN_BENCH_DEVICE=0 run bench_2rank 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw \
  --no-hits --no-update
NAMES="prepw5" run ct_ab_prepw5 400 bash tools/ab.sh lib
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_bench" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/prof_bench.log" 2>&1 )
echo "== prof_bench rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
