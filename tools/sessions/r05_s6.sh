#!/bin/bash
# Round 5, session 6: the radix sort with 512-thread tiles and a 16-wide look-back
# window (its test, the conntrack tests, the stateful batch and its kernel trace);
# rule clustering inside type groups (image.cpp) A/B on configs 5 and 3, with the
# multi-block 128-candidate window on and off; parity of the new permutations.
TAG=r05_s6
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
run ct_probe 300 python tools/ct_probe.py --steps 6
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_parity 600 tests/test_gpu_parity.py tests/test_gpu_sweep.py
KEEP_GOING=1
run ab_cfg5 600 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@CLUSTER=0,jit@DEAL2_MULTI=0,jit,jit@CLUSTER=0,jit@DEAL2_MULTI=0"
CFG5_HOOK=tc run ab_cfg5_tc 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit@CLUSTER=0,jit@DEAL2_MULTI=0,jit,jit@CLUSTER=0"
SETTLE=2 run ab_cfg3 600 python -u tools/ablate.py --cfg 3 --log2n 24 --hits 0.5,1 --iters 30 \
  --variants "jit,jit@CLUSTER=0,jit,jit@CLUSTER=0"
exit 0
