#!/bin/bash
# Round 5, session 19: config 5's launch anatomy (per-workgroup timelines, XDP
# and TC), config 3's again for reference.
TAG=r05_s19
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
PCN_IPT_DEBUG_CLOCKS=1 run clocks_cfg5 200 python tools/wg_clocks.py --cfg 5 --log2n 22 --launches 3
PCN_IPT_DEBUG_CLOCKS=1 CFG5_HOOK=tc run clocks_cfg5_tc 200 python tools/wg_clocks.py --cfg 5 --log2n 22 --launches 3
PCN_IPT_DEBUG_CLOCKS=1 PCN_IPT_JIT_DEFS=-DPCN_ABLATE=1 run clocks_cfg5_parse 200 python tools/wg_clocks.py --cfg 5 --log2n 22 --launches 3
exit 0
