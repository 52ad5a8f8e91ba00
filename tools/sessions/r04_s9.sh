#!/bin/bash
# Round 4, session 9: IP bucket entries that hold the class of a bucket without a
# boundary (those lanes skip the boundary and class reads): parity tests on it, then
# A/B against the previous build (build/ab/libpcn_ipt_base.so) on configs 3, 5, 2.
TAG=r04_s9
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_parity 600 tests/test_gpu_parity.py tests/test_gpu_horus.py tests/test_gpu_firewall.py
KEEP_GOING=1
run ab_ipd_cfg3 400 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0,0.5,1 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
run ab_ipd_cfg5 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
CFG5_HOOK=tc run ab_ipd_cfg5_tc 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:base,jit,lib:base"
run ab_ipd_cfg2 300 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 50 \
  --variants "jit,lib:base,jit,lib:base"
LDS="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES"
pmcq lds_cfg3 3 24 0.5 "$LDS"
exit 0
