#!/bin/bash
# Round 6, session 13: hdr_skip (the Ethernet addresses stay on the host: 36-byte rows over
# PCIe): the ring tests, then the e2e legs (bench with every other leg off).
TAG=r06_s13
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ring 600 tests/test_gpu_parity.py -k "ingest_ring or stream_of_a_closed_ring or fold_waits"
KEEP_GOING=1
run bench_e2e 500 python bench.py --steps 20 --warmup 5 --no-cpu --no-ct --no-fw --no-hits --no-update --no-sizes
exit 0
