#!/bin/bash
# Round 6, session 34: randomised stateful parity sweep on the final tree (after the LRU digit passes; ct_count by
# rows, the radix up-sweep / column scan, the LRU deletion's counter changed since
# r06_s14), and a big-chain sweep.
TAG=${TAG:-r06_s34}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run sweep_stateful 360 python tools/parity_sweep.py --stateful --seconds 300 --seed0 170000
run sweep_big 300 python tools/parity_sweep.py --big --seconds 200 --seed0 180000
exit 0
