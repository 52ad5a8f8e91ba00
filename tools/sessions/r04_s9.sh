#!/bin/bash
# Round 4, session 9 + final evidence in one call (GPU boxes are scarce): IP bucket
# entries that hold the class of a bucket without a boundary -- every GPU test and the
# smoke on it, A/B against the previous build (build/ab/libpcn_ipt_base.so) on configs
# 3, 5, 2; then the evidence of that build (not kept: the A/B lost on config 3, so
# tools/sessions/r04_final.sh reruns the evidence part on the reverted tree).
TAG=r04_final
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run ab_ipd_cfg3 400 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0,0.5,1 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
run ab_ipd_cfg5 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
CFG5_HOOK=tc run ab_ipd_cfg5_tc 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
run ab_ipd_cfg2 300 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 50 \
  --variants "jit,lib:base,jit,lib:base"
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
exit 0
