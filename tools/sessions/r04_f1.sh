#!/bin/bash
# Round 4, final evidence part 1: every GPU test and the smoke on the committed tree.
TAG=r04_final
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_all 1000 tests
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
