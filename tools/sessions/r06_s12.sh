#!/bin/bash
# Round 6, session 12: the fused stage A through the generic kernel (jit -1).
TAG=r06_s12
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_stage_a 600 tests/test_gpu_conntrack.py -k "stage_a"
exit 0
