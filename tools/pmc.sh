#!/bin/bash
# PMC passes over the classify kernel (one counter group per rocprofv3 run, kernel-trace only).
# Usage (GPU box): TAG=x [LIB=path/to/variant.so] bash tools/pmc.sh "<counters pass1>" "<counters pass2>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-pmc}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$ROOT/gpurun_out/$TAG/counters_list.txt" 2>&1 || true
k=0
for grp in "$@"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$TAG/p$k" -o run \
    -- python3 "$ROOT/tools/ablate.py" --child --lib "${LIB:-}" --hit ${HIT:-0.5} --iters 5 --log2n ${LOG2N:-24} --cfg ${CFG:-3} --jit ${JIT:--1} > "$ROOT/gpurun_out/$TAG/p$k.log" 2>&1
  rc=$?
  echo "pass $k ($grp) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
