#!/bin/bash
# Round 5, session 5: the hand-written radix sort of the stateful pipeline
# (radix.hip; rocPRIM dropped) -- its own test first, then every conntrack /
# firewall / flow-split / horus test and the stateful sweep subset; the stateful
# batch time and its kernel trace; config 5 with the merged block queue and
# buffer-load PART cells, A/B against each off.
TAG=r05_s5
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py \
  tests/test_gpu_horus.py tests/test_gpu_sweep.py -k "not big_chain"
run ct_probe 300 python tools/ct_probe.py --steps 6
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
KEEP_GOING=1
run ab_cfg5 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_MERGE_BLOCKS=0,jit:-DPCN_BUF_LOADS=0,jit:-DPCN_MERGE_BLOCKS=0+-DPCN_BUF_LOADS=0,jit,jit:-DPCN_MERGE_BLOCKS=0"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_MERGE_BLOCKS=0+-DPCN_BUF_LOADS=0,jit,jit:-DPCN_MERGE_BLOCKS=0+-DPCN_BUF_LOADS=0"
pytest_gpu tests_c5 600 tests/test_gpu_parity.py -k "config5 or imix or ingest_ring"
exit 0
