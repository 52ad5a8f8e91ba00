#!/bin/bash
# Round 6, final bench lines on the final tree (after the ring's hdr_skip leg): the headline
# line with every leg and the secondary configs' lines (the kernel sources are those of
# r06_fin3_a, whose PMC traffic entries they report); smoke.
TAG=${TAG:-r06_fin4}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 500 python bench.py --steps 50 --warmup 10
for spec in "2 xdp" "5 xdp" "5 tc"; do
  set -- $spec
  run bench_cfg$1_$2 300 python bench.py --config $1 --hook $2 --steps 20 --warmup 5 --no-e2e
done
exit 0
