#!/bin/bash
# Round 4, session 6: the stateful walk's head wave issuing its first chunk's
# sorted indices before the key and cut checks; stateful GPU tests on it, then
# ct_probe against the previous walk (build/ab/libpcn_ipt_ct_base.so).
TAG=r04_s6
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_stateful 600 tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py
KEEP_GOING=1
NAMES="base" run ct_ab 600 bash tools/ab.sh lib
exit 0
