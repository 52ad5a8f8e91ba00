#!/bin/bash
# Round 4, session 11: config 5 at its full bench size (2^22 IMIX, both hooks) and
# ten fuzz seeds, with the rest of the parity file, on the final build.
TAG=r04_s11
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_parity 900 tests/test_gpu_parity.py
exit 0
