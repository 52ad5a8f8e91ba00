#!/bin/bash
# Round 4, session 8: packed counter copies (one u64 atomic per counter pair,
# build/ab/libpcn_ipt_packed.so) -- GPU tests on that build, then A/B against the
# product build on configs 5, 3, 2, with the product's PCN_ABLATE=9 (byte atomic
# dropped: the bound of the saving) beside; LDS issue stalls of config 3.
TAG=r04_s8
source "$(dirname "$0")/../gpu_lib.sh"
P=$R/polycube_amd/build/ab/libpcn_ipt_packed.so
PCN_IPT_LIBRARY=$P pytest_gpu tests_packed 600 tests/test_gpu_parity.py tests/test_gpu_horus.py tests/test_gpu_firewall.py
KEEP_GOING=1
PCN_IPT_LIBRARY=$P pytest_gpu tests_packed_ct 400 tests/test_gpu_conntrack.py
run ab_ctr_cfg5 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:packed,jit:-DPCN_ABLATE=9,jit,lib:packed,jit:-DPCN_ABLATE=5"
CFG5_HOOK=tc run ab_ctr_cfg5_tc 300 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,lib:packed,jit,lib:packed"
run ab_ctr_cfg3 300 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5,1 --iters 30 \
  --variants "jit,lib:packed,jit:-DPCN_ABLATE=9,jit,lib:packed"
run ab_ctr_cfg2 300 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 50 \
  --variants "jit,lib:packed,jit:-DPCN_ABLATE=9,jit,lib:packed"
LDS="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES"
pmcq lds_cfg3 3 24 0.5 "$LDS"
pmcq lds_cfg3_parse 3 24 0.5 "$LDS" -DPCN_ABLATE=1
pmcq lds_cfg3_lookups 3 24 0.5 "$LDS" -DPCN_ABLATE=2
exit 0
