#!/bin/bash
# Round 6, session 9: dword-aligned strides on the fixed-stride path (1500-byte frames:
# three 16-byte loads from each frame's start instead of the generic 16-byte-aligned gather):
# frame-size parity, A/B against the 16-byte rule, the 1500-byte PMC traffic; the split
# rule kernel's record taken before its stage is refilled (fin_b's failure).
TAG=r06_s9
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_fs 600 tests/test_gpu_parity.py -k "frame_size_sweep or full_size_headline or split_launch or full_size_config5"
KEEP_GOING=1
export FRAME_STRIDE=1500
run ab_1500 300 python tools/ablate.py --cfg 3 --log2n 24 --hits 0.5 --variants "jit,jit@FIXED_ALIGN=16,jit,jit@FIXED_ALIGN=16"
export FRAME_STRIDE=1504
run ab_1504 300 python tools/ablate.py --cfg 3 --log2n 24 --hits 0.5 --variants "jit,jit@FIXED_ALIGN=16"
export FRAME_STRIDE=1500
KEEP_GOING=0
pmct config3_stride1500 3 24
unset FRAME_STRIDE
exit 0
