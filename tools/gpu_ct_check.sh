#!/bin/bash
# Stateful-pipeline check on one GPU box: the connection-table GPU tests, a
# bench line (stateful leg included) and a rocprofv3 kernel trace of the bench.
# Stops at the first crash/timeout.  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ct}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
echo "== pytest (stateful)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py \
  tests/test_gpu_horus.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ct_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ct_tests_$TAG.log
if fatal $rc; then exit $rc; fi
echo "== bench"
timeout -k 10 600 python bench.py --steps 50 --warmup 10 --no-cpu --no-e2e > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json
if fatal $rc; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --no-e2e --no-fw > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
