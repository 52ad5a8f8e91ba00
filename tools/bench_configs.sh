#!/bin/bash
# Secondary bench lines (configs 2 and 5, XDP and TC hooks) after the headline; GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
for spec in "2 xdp" "5 xdp" "5 tc"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --hook $2 --steps 20 --warmup 5 --no-e2e \
    > gpurun_out/bench_${TAG}_cfg$1_$2.json 2> gpurun_out/bench_${TAG}_cfg$1_$2.err
  rc=$?; echo "config $1 $2 rc=$rc"; cat gpurun_out/bench_${TAG}_cfg$1_$2.json
  case $rc in 0) ;; *) tail -5 gpurun_out/bench_${TAG}_cfg$1_$2.err; exit $rc;; esac
done
