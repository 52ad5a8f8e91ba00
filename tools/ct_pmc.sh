#!/bin/bash
# PMC passes over the stateful pipeline's kernels (tools/ct_probe.py), one counter group per run.
# Usage (GPU box): TAG=x bash tools/ct_pmc.sh "<counters pass1>" "<counters pass2>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-ctpmc}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
k=0
for grp in "$@"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$TAG/p$k" -o run \
    -- python3 "$ROOT/tools/ct_probe.py" --steps 1 --log2n ${LOG2N:-22} --flows ${FLOWS:-16384} > "$ROOT/gpurun_out/$TAG/p$k.log" 2>&1
  rc=$?
  echo "pass $k ($grp) rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
