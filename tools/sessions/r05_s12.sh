#!/bin/bash
# Round 5, session 12: where config 3's drain comes from (per-XCD workgroup
# timelines), config 5 TC with the 64-item deal repeated, a default bench line.
TAG=r05_s12
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
PCN_IPT_DEBUG_CLOCKS=1 run clocks_cfg3 200 python tools/wg_clocks.py --cfg 3 --log2n 24 --launches 4
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@DEAL2_MULTI=0,jit,jit@DEAL2_MULTI=0"
run bench 600 python bench.py
exit 0
