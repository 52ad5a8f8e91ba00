#!/bin/bash
# Round 4, session 5: SQ / TCC counters of the candidate stage (config 3 at hit
# 0.5 / 1, with and without the two-item deal; config 5) against the parse-only
# and lookups-only builds.
TAG=r04_s5
source "$(dirname "$0")/../gpu_lib.sh"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"
TCC="TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"
pmcq sq_cfg3_h05 3 24 0.5 "$SQ"
pmcq sq_cfg3_h1 3 24 1 "$SQ"
pmcq sq_cfg3_h1_deal2 3 24 1 "$SQ" -DPCN_DEAL2=1
pmcq sq_cfg3_h05_deal2 3 24 0.5 "$SQ" -DPCN_DEAL2=1
pmcq sq_cfg3_parse 3 24 0.5 "$SQ" -DPCN_ABLATE=1
pmcq sq_cfg5 5 22 0.5 "$SQ"
pmcq sq_cfg5_parse 5 22 0.5 "$SQ" -DPCN_ABLATE=1
pmcq sq_cfg5_lookups 5 22 0.5 "$SQ" -DPCN_ABLATE=2
pmcq tcc_cfg5 5 22 0.5 "$TCC"
pmcq tcc_cfg5_lookups 5 22 0.5 "$TCC" -DPCN_ABLATE=2
pmcq tcc_cfg3 3 24 0.5 "$TCC"
KEEP_GOING=1
run ab_cfg3_stages 900 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0,0.5 --iters 30 \
  --variants "jit1,jit2,jit3,jit4,jit5,jit"
CFG5_HOOK=xdp run ab_cfg5_pf2 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_PREFETCH_GENERIC=2,jit,jit:-DPCN_PREFETCH_GENERIC=2"
pytest_gpu tests_cfg5 300 tests/test_gpu_parity.py -k "imix or config"
PCN_IPT_DEBUG_DENSE_PM=1 PCN_IPT_DEBUG_IP_BITS=8 pytest_gpu tests_cfg5_pm 300 tests/test_gpu_parity.py -k "imix or config"
run ab_cfg5_lds 900 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@IP_BITS=8,jit@DENSE_PM=1;IP_BITS=8,jit,jit@IP_BITS=8,jit@DENSE_PM=1;IP_BITS=8"
CFG5_HOOK=tc run ab_cfg5_lds_tc 900 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@IP_BITS=8,jit@DENSE_PM=1;IP_BITS=8,jit,jit@IP_BITS=8,jit@DENSE_PM=1;IP_BITS=8"
# (last: counter names not checked on this pool before)
TCP="TCP_PERF_SEL_TOTAL_READ_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_CC_READ_REQ_sum"
pmcq tcp_cfg5 5 22 0.5 "$TCP"
pmcq tcp_cfg5_lookups 5 22 0.5 "$TCP" -DPCN_ABLATE=2
exit 0
