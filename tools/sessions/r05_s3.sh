#!/bin/bash
# Round 5, session 3: config 5 with per-word slot masks (wfields: no PART read for
# a slot FULL at the word) and the late header prefetch, A/B against each alone and
# neither; IMIX / config-5 parity; the host-pack ingest ring (test + e2e legs).
TAG=r05_s3
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_c5 600 tests/test_gpu_parity.py -k "config5 or imix or ingest_ring or fuzz"
run ab_cfg5 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_WFIELDS=0,jit:-DPCN_PF_LATE=0,jit:-DPCN_PF_LATE=0+-DPCN_WFIELDS=0,jit,jit:-DPCN_WFIELDS=0,jit:-DPCN_PF_LATE=0+-DPCN_WFIELDS=0"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_WFIELDS=0,jit:-DPCN_PF_LATE=0+-DPCN_WFIELDS=0,jit,jit:-DPCN_WFIELDS=0"
run ab_cfg5_stages 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit1,jit2,jit3,jit4,jit6,jit"
run bench_e2e 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-ct --no-fw --no-hits --no-update
exit 0
