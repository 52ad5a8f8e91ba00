#!/bin/bash
# Round 4: more randomised parity on the final build -- stateful trials and
# 4,100-8,000-rule chains with new seeds.
TAG=r04_sweep2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run sweep_ct 400 python -u tools/parity_sweep.py --seconds 280 --seed0 70000 --stateful
run sweep_big 400 python -u tools/parity_sweep.py --seconds 280 --seed0 80000 --big
exit 0
