#!/bin/bash
# LDS-pipe PMC passes over the chain program (full kernel and parse-only), GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
B="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
C="GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_BUSY_max"
for v in 0 1; do
  if [ $v = 0 ]; then unset PCN_IPT_JIT_DEFS; else export PCN_IPT_JIT_DEFS="-DPCN_ABLATE=$v"; fi
  JIT=1 TAG=${TAG:-pmc_lds}_v$v bash tools/pmc.sh "$A" "$B" "$C" || exit $?
done
