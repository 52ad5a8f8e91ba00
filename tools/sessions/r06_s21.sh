#!/bin/bash
# Round 6, session 21: the conntrack suite again (the 10k-rule counters test with the
# chain limits it needs).
TAG=${TAG:-r06_s21}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py tests/test_gpu_flow_split.py
exit 0
