#!/bin/bash
# Round 5, session 4: config 5's candidate stage.  A/B of the per-word slot masks
# as an unconditional load (PCN_WFIELDS 2) against the branch (1) and none (0);
# PMC of the full kernel against the summary-AND ablation (3): instruction mix,
# waits, LDS and L2 traffic, so the stage's cost can be attributed.
TAG=r05_s4
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run ab_cfg5 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_WFIELDS=0,jit:-DPCN_WFIELDS=1,jit,jit:-DPCN_WFIELDS=0"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_WFIELDS=0,jit,jit:-DPCN_WFIELDS=0"
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
SQ2="SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_WR"
TC="TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_CC_READ_REQ_sum"
KEEP_GOING=0
for v in "full:-DPCN_WFIELDS=0" "abl3:-DPCN_WFIELDS=0 -DPCN_ABLATE=3" "wf2:-DPCN_WFIELDS=2"; do
  n=${v%%:*}; d=${v#*:}
  pmcq sq1_$n 5 22 0.5 "$SQ1" "$d"
  pmcq sq2_$n 5 22 0.5 "$SQ2" "$d"
  pmcq tc_$n 5 22 0.5 "$TC" "$d"
done
exit 0
