#!/bin/bash
# Round 6, final evidence (part a): PMC traffic of every config on this build's kernel
# sources (profiles/pmc_traffic.json, the frame-size sweep's 128 / 1500-byte strides too),
# then the headline bench line (every leg) and the secondary configs' lines, the bench
# under rocprofv3 --kernel-trace --stats.
TAG=${TAG:-r06_fin_a}
source "$(dirname "$0")/../gpu_lib.sh"
pmct config3 3 24
pmct config2 2 20
pmct config5 5 22
pmct config5_tc 5 22 tc
FRAME_STRIDE=128 pmct config3_stride128 3 24
FRAME_STRIDE=1500 pmct config3_stride1500 3 24
KEEP_GOING=1
run bench 500 python bench.py --steps 50 --warmup 10
for spec in "2 xdp" "5 xdp" "5 tc"; do
  set -- $spec
  run bench_cfg$1_$2 300 python bench.py --config $1 --hook $2 --steps 20 --warmup 5 --no-e2e
done
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_bench" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/prof_bench.log" 2>&1 )
echo "== prof_bench rc=$?"
python3 tools/ktsum.py "$O/prof_bench" > "$O/prof_bench.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
exit 0
