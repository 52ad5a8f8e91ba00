#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > gpurun_out/bench_ct.json 2> gpurun_out/bench_ct.err || exit $?
cat gpurun_out/bench_ct.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ct" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-e2e > "$GRAFT_REPO_ROOT/gpurun_out/prof_ct.log" 2>&1 || exit $?
find "$GRAFT_REPO_ROOT/gpurun_out/prof_ct" -name "*kernel_stats*" -exec head -20 {} \;
