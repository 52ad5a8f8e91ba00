#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Stops at the first crash/timeout (exit 124/134/137/139); a plain test failure
# (pytest exit 1) still lets the bench run.  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
STEPS=${STEPS:-50}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

echo "== smoke"; timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  if fatal $rc; then exit $rc; fi
fi

echo "== bench"; timeout -k 10 600 python bench.py --steps $STEPS --warmup 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
if fatal $rc; then exit $rc; fi

if [ "${SKIP_MULTI:-0}" != 1 ]; then
  # bench.py launches its own ranks (--gpus 2, no WORLD_SIZE); on a one-GPU box both share
  # device 0 (PCN_BENCH_DEVICE), RCCL refuses that, and the counter blocks go through gloo
  echo "== bench --gpus 2"
  PCN_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e --no-ct --no-fw \
    > gpurun_out/bench_${TAG}_2rank.json 2> gpurun_out/bench_${TAG}_2rank.err
  rc=$?; echo "bench 2-rank rc=$rc"; cat gpurun_out/bench_${TAG}_2rank.json; tail -3 gpurun_out/bench_${TAG}_2rank.err
  if fatal $rc; then exit $rc; fi
fi

if [ "${SKIP_PROF:-0}" != 1 ]; then
  echo "== rocprofv3 kernel trace"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --no-e2e > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"
  if fatal $rc; then exit $rc; fi
  find "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -name "*stats*" | head
fi
exit 0
