#!/bin/bash
# Round 5, session 1: the hygiene changes (provenance fields, per-rank parity,
# stream release, -ENOSPC refusals, the sweep subset in the gpu suite) on the GPU:
# every GPU test, the smoke, the headline bench line, the 2-rank test hook, and
# config 5's stage ablation (parse only / lookups / full) as the starting point.
TAG=r05_s1
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 1100 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 50 --warmup 10 --no-update
PCN_BENCH_DEVICE=0 run bench_2rank 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw \
  --no-hits --no-update
run ab_cfg5 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 --variants "jit1,jit2,jit,jit1,jit2,jit"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 --variants "jit1,jit2,jit"
exit 0
