#!/bin/bash
# Round 4, session 8: one atomic per counter pair instead of two (PCN_ABLATE=9, wrong
# byte counts: the bound of what packed counter copies would save) on configs 5, 3, 2;
# LDS issue stalls and array occupancy of config 3 against its parse-only build.
TAG=r04_s8
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run ab_ctr_cfg5 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_ABLATE=9,jit:-DPCN_ABLATE=5,jit,jit:-DPCN_ABLATE=9"
run ab_ctr_cfg3 300 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_ABLATE=9,jit:-DPCN_ABLATE=5,jit,jit:-DPCN_ABLATE=9"
run ab_ctr_cfg2 300 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 50 \
  --variants "jit,jit:-DPCN_ABLATE=9,jit:-DPCN_ABLATE=5,jit,jit:-DPCN_ABLATE=9"
LDS="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES"
pmcq lds_cfg3 3 24 0.5 "$LDS"
pmcq lds_cfg3_parse 3 24 0.5 "$LDS" -DPCN_ABLATE=1
pmcq lds_cfg3_lookups 3 24 0.5 "$LDS" -DPCN_ABLATE=2
exit 0
