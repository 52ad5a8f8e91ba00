#!/bin/bash
# Round 5: randomised GPU-vs-oracle parity sweeps on the final tree after the
# stateful pipeline work of sessions 21-40 (bounded walk record loads, 24-bit key
# buckets, listed segment cuts, fence-free LRU passes, ct_count zeroing the next
# batch's control words, the plan and bitmap folds): stateful multi-batch trials
# and stateless trials, fresh seeds.
TAG=r05_sweep2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run sweep_ct 330 python -u tools/parity_sweep.py --seconds 300 --seed0 250000 --stateful
run sweep_big 330 python -u tools/parity_sweep.py --seconds 240 --seed0 260000 --big
exit 0
