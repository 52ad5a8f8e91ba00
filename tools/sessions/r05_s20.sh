#!/bin/bash
# Round 5, session 20: the dynamic tail of offsets/lens launches (the last
# rounds' frames claimed 64 at a time from per-XCD counters): parity first
# (the tail test at four shares, config 5 at full size, the other IMIX tests),
# then config 5 XDP / TC with the tail against without (PCN_IPT_DEBUG_TAIL=0),
# bench lines and workgroup timelines.
TAG=r05_s20
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_tail 600 tests/test_gpu_parity.py -k "dynamic_tail or config5 or imix or offsets"
KEEP_GOING=1
run ab_cfg5 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@TAIL=0,jit,jit@TAIL=0,jit@TAIL=4"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@TAIL=0,jit,jit@TAIL=0"
run bench_cfg5 200 python bench.py --config 5 --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
PCN_IPT_DEBUG_TAIL=0 run bench_cfg5_notail 200 python bench.py --config 5 --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5_tc 200 python bench.py --config 5 --hook tc --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
PCN_IPT_DEBUG_CLOCKS=1 run clocks_cfg5 200 python tools/wg_clocks.py --cfg 5 --log2n 22 --launches 3
exit 0
