set -o pipefail
mkdir -p gpurun_out
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
JIT=1 TAG=pmc_s9 bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "$A" "$B" || exit $?
python tools/pmc_summary.py gpurun_out/pmc_s9 --traffic --out gpurun_out/pmc_s9/summary.json | tail -40
