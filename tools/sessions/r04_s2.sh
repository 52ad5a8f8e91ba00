#!/bin/bash
# Round 4, session 2: counter copies (flush contention) and workgroups per CU for
# the short config-2 launch; the two-item candidate deal (hit rate 1); full GPU tests.
TAG=r04_s2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
PCN_IPT_JIT_DEFS=-DPCN_DEAL2=1 pytest_gpu tests_deal2 300 tests/test_gpu_parity.py -k "chainprog or jit"
KEEP_GOING=1
run ab_cfg2_20 600 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 50 \
  --variants "jit@CTR_REPS=1,jit,jit@CTR_REPS=64,jit@WG_PER_CU=1,jit@WG_PER_CU=1;CTR_REPS=64,jit@CTR_REPS=1,jit"
run ab_cfg2_24 600 python -u tools/ablate.py --cfg 2 --log2n 24 --hits 0.5 --iters 30 \
  --variants "jit@CTR_REPS=1,jit,jit@WG_PER_CU=1,jit@WG_PER_CU=1;CTR_REPS=64,jit"
run ab_cfg3_reps 600 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5 --iters 30 \
  --variants "jit@CTR_REPS=1,jit,jit@CTR_REPS=64,jit@CTR_REPS=1,jit"
run ab_cfg3_deal2 900 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0,0.5,1 --iters 30 \
  --variants "jit,jit:-DPCN_DEAL2=1,jit,jit:-DPCN_DEAL2=1"
run ab_cfg5 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit@CTR_REPS=1,jit,jit@WG_PER_CU=1,jit@CTR_REPS=1,jit"
exit 0
