#!/bin/bash
# Round 4, session 4: ring zero-copy + header-only tests and bench legs; the
# two-item deal with broadcast filler items; SQ counters of the candidate stage
# (config 3 at hit 0.5 / 1, config 5) against the parse-only build.
TAG=r04_s4
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ring 300 tests/test_gpu_parity.py -k "ring"
run ab_cfg3_deal2 900 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5,1 --iters 30 \
  --variants "jit,jit:-DPCN_DEAL2=1,jit,jit:-DPCN_DEAL2=1"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"
pmcq sq_cfg3_h05 3 24 0.5 "$SQ"
pmcq sq_cfg3_h1 3 24 1 "$SQ"
pmcq sq_cfg3_h1_deal2 3 24 1 "$SQ" -DPCN_DEAL2=1
pmcq sq_cfg3_parse 3 24 0.5 "$SQ" -DPCN_ABLATE=1
pmcq sq_cfg5 5 22 0.5 "$SQ"
pmcq sq_cfg5_parse 5 22 0.5 "$SQ" -DPCN_ABLATE=1
pmcq sq_cfg5_lookups 5 22 0.5 "$SQ" -DPCN_ABLATE=2
TCC="TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"
pmcq tcc_cfg5 5 22 0.5 "$TCC"
pmcq tcc_cfg5_lookups 5 22 0.5 "$TCC" -DPCN_ABLATE=2
pmcq tcc_cfg3 3 24 0.5 "$TCC"
run bench 600 python bench.py --steps 50 --warmup 10 --no-cpu
exit 0
