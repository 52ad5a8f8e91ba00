#!/bin/bash
# Round 5, final evidence (part a) on the committed tree: every GPU test and the
# smoke; HBM traffic of the chain programs (configs 3, 2, 5 XDP / TC) into
# profiles/pmc_traffic.json; the bench lines that report it (config 3 headline with
# every leg, config 2 at 2^20, config 5 XDP and TC at 2^22) and the 2-rank self-launch.
TAG=r05_final
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
KEEP_GOING=0
pmct config3 3 24
pmct config2 2 20
pmct config5 5 22 xdp
pmct config5_tc 5 22 tc
KEEP_GOING=1
run bench 400 python bench.py --steps 50 --warmup 10
run bench_cfg2 200 python bench.py --config 2 --log2n 20 --steps 100 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5 200 python bench.py --config 5 --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5_tc 200 python bench.py --config 5 --hook tc --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
PCN_BENCH_DEVICE=0 run bench_2rank 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw \
  --no-hits --no-update
exit 0
