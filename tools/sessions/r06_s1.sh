#!/bin/bash
# Round 6, session 1: the new tests (frame-size sweep parity incl. 1500 B at 2^24, the
# advisor's stale-event fold test, split launches for config 5), the stateful suites on the
# scaled segment waves, config 5 split vs fused A/B, the bench line with the frame-size
# sweep, the counter calibration patterns, the 1500 B classify PMC traffic, and
# single-flow stateful timings.
TAG=r06_s1
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_split 600 tests/test_gpu_parity.py -k "split_launch or full_size_config5 or imix_config5"
run ab_cfg5_xdp 300 python tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --variants "jit,jit@SPLIT=0,jit,jit@SPLIT=0"
CFG5_HOOK=tc run ab_cfg5_tc 300 python tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --variants "jit,jit@SPLIT=0,jit,jit@SPLIT=0"
pytest_gpu tests_new 900 tests/test_gpu_parity.py -k "frame_size_sweep or fold_waits or closed_ring or full_size_headline"
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
run ct_probe 300 python tools/ct_probe.py --steps 6
run ct_probe_1flow 300 python tools/ct_probe.py --steps 3 --flows 1 --p-noise 0 --p-err 0 --p-icmp 0
run bench 600 python bench.py --steps 50 --warmup 10 --no-update
calib stream stream 24 calib_stream
calib s64 stride:64 24 calib_stride
calib s128 stride:128 24 calib_stride
calib s1500 stride:1500 24 calib_stride
calib s1536 stride:1536 24 calib_stride
calib imix imix 22 calib_imix
calib rec32 rec32 24 calib_rec32
export FRAME_STRIDE=1500
pmc pmc_stride1500 3 24
unset FRAME_STRIDE
exit 0
