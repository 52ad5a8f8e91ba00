#!/bin/bash
# Round 4, last check on the committed tree (rerun after the stats-read skip): every GPU test, the smoke, the bench
# lines (headline with every leg, configs 2 and 5) and the rocprof kernel stats of
# the headline bench.  The kernel sources are those of profiles/r04_final/ (PMC
# traffic hash e076dd6a); conntrack.hip changed since (LRU scan, reverted tries).
TAG=r04_last2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 50 --warmup 10
run bench_cfg2 200 python bench.py --config 2 --log2n 20 --steps 100 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5 200 python bench.py --config 5 --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
run bench_cfg5_tc 200 python bench.py --config 5 --hook tc --log2n 22 --steps 50 --warmup 10 --no-e2e --no-ct --no-fw --no-hits --no-update
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_bench" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/prof_bench.log" 2>&1 )
echo "== prof_bench rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
exit 0
