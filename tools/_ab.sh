set -u
mkdir -p gpurun_out
for a in "--warmup 5" "--warmup 5 --step-events" "--warmup 5 --settle 0" "--warmup 5" ; do
  timeout -k 10 300 python bench.py --steps 20 $a --no-cpu --no-e2e --no-ct --no-fw 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$a', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['settle'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_settle" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw > "$GRAFT_REPO_ROOT/gpurun_out/prof_settle.log" 2>&1
tail -1 "$GRAFT_REPO_ROOT/gpurun_out/prof_settle.log"
head -5 "$GRAFT_REPO_ROOT/gpurun_out/prof_settle/run_kernel_stats.csv"
