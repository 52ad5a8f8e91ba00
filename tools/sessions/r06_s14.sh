#!/bin/bash
# Round 6, session 14: randomised parity sweeps on the final kernels, strides now including
# 68 / 100 / 1500 (the dword-aligned fixed-stride path): the suite's sweeps, then timed
# stateless, big-chain and stateful sweeps.
TAG=r06_s14
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_sweep 600 tests/test_gpu_sweep.py
run sweep_stateless 360 python tools/parity_sweep.py --seconds 280 --seed0 120000
run sweep_big 300 python tools/parity_sweep.py --big --seconds 220 --seed0 130000
run sweep_stateful 300 python tools/parity_sweep.py --stateful --seconds 220 --seed0 140000
exit 0
