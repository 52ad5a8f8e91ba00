#!/bin/bash
# Round 5, session 2: the sweep subset and the new parity tests; config 5 with the
# header prefetch issued after the candidate stage (PCN_PF_LATE, depth 1/2/3);
# config 3's adaptive deal window at hit rates 0.5 / 1; config 2 at 2^20 with
# prefetch depth 1/2/3 against parse only.
TAG=r05_s2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_sweep 600 tests/test_gpu_sweep.py tests/test_gpu_parity.py
L="-DPCN_PF_LATE=1"
run ab_cfg5 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:$L+-DPCN_PREFETCH_GENERIC=2,jit:$L,jit:$L+-DPCN_PREFETCH_GENERIC=3,jit,jit:$L+-DPCN_PREFETCH_GENERIC=2,jit:-DPCN_PREFETCH_GENERIC=2"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:$L+-DPCN_PREFETCH_GENERIC=2,jit:$L,jit,jit:$L+-DPCN_PREFETCH_GENERIC=2"
SETTLE=2 run ab_cfg3_deal 600 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5,1,0 --iters 30 \
  --variants "jit@DEAL_ADAPT=0,jit,jit@DEAL_ADAPT=2,jit@DEAL_ADAPT=0,jit"
run ab_cfg2 400 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 100 \
  --variants "jit,jit1,jit:-DPCN_PREFETCH_FIXED=3,jit:-DPCN_PREFETCH_FIXED=1,jit,jit1,jit:-DPCN_PREFETCH_FIXED=3"
exit 0
