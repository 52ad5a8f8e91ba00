#!/bin/bash
# Round 6, session 10: the stateful sweep with fused-stage-A trials (64-byte frames of one
# length, ICMP-heavy half of them): the suite's seeds, then a timed randomised sweep.
TAG=r06_s10
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_sweep 600 tests/test_gpu_sweep.py -k stateful
run sweep_stateful 420 python tools/parity_sweep.py --stateful --seconds 300 --seed0 70000
exit 0
