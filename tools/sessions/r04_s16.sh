#!/bin/bash
# Round 4, session 16: randomised parity sweep over chains of 4100-8000 rules (2+
# summary blocks: the two-item deal, the global counter atomics past the LDS bins,
# the packed copies' folds), both services and every conntrack mode.
TAG=r04_s16
source "$(dirname "$0")/../gpu_lib.sh"
run sweep_big 400 python -u tools/parity_sweep.py --seconds 300 --seed0 60000 --big
exit 0
