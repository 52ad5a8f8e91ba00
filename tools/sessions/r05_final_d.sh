#!/bin/bash
# Round 5, final evidence (part d): the committed tree after the flow-split load changes:
# every GPU test, the smoke and the headline bench line (every leg).
TAG=r05_final_d
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 900 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 50 --warmup 10
exit 0
