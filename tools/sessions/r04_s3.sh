#!/bin/bash
# Round 4, session 3: 12-byte candidate records, one workgroup per CU and 64 counter
# copies as defaults; the two-item deal A/B again (now spill-free) on configs 3 and 5;
# config-5 counter stages and the offset loads one prefetch ahead; header-only ring test; the bench line with its e2e legs.
TAG=r04_s3
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_parity 400 tests/test_gpu_parity.py
PCN_IPT_JIT_DEFS=-DPCN_DEAL2=2 PCN_IPT_DEBUG_WAVE_BYTES_GENERIC=2304 pytest_gpu tests_deal2 400 \
  tests/test_gpu_parity.py -k "chainprog or jit"
run ab_cfg3_deal2 900 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0,0.5,1 --iters 30 \
  --variants "jit,jit:-DPCN_DEAL2=1,jit,jit:-DPCN_DEAL2=1"
run ab_cfg5 900 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_DEAL2=2@WAVE_BYTES_GENERIC=2304,jit:-DPCN_OFF_AHEAD=0,jit5,jit6,jit8,jit1,jit,jit:-DPCN_DEAL2=2@WAVE_BYTES_GENERIC=2304,jit:-DPCN_OFF_AHEAD=0"
CFG5_HOOK=tc run ab_cfg5_tc 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_DEAL2=2@WAVE_BYTES_GENERIC=2304,jit:-DPCN_OFF_AHEAD=0,jit,jit:-DPCN_OFF_AHEAD=0"
run ab_cfg2_20 300 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 50 --variants "jit,jit5,jit1,jit"
run bench 600 python bench.py --steps 50 --warmup 10
exit 0
