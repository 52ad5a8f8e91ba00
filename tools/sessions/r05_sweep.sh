#!/bin/bash
# Round 5: randomised GPU-vs-oracle parity sweeps on the final tree (rule
# clustering, the adaptive deal window, the hand-written radix sort, stage A
# without counters): stateless, stateful and big-chain trials, fresh seeds.
TAG=r05_sweep
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run sweep 330 python -u tools/parity_sweep.py --seconds 300 --seed0 140000
run sweep_ct 330 python -u tools/parity_sweep.py --seconds 300 --seed0 150000 --stateful
run sweep_big 330 python -u tools/parity_sweep.py --seconds 300 --seed0 160000 --big
exit 0
