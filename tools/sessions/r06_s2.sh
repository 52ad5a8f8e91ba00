#!/bin/bash
# Round 6, session 2: where the split launch's time goes (kernel trace of the gather and
# rule kernels) and its knobs against the fused kernel, config 5 XDP and TC.
TAG=r06_s2
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
ktrace kt_cfg5_split 5 22 20
PCN_IPT_DEBUG_SPLIT=0 ktrace kt_cfg5_fused 5 22 20
run ab_cfg5_xdp 400 python tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --variants \
  "jit@SPLIT=0,jit,jit:-DPCN_SPLIT_R_PF=1,jit:-DPCN_SPLIT_R_PF=1+-DPCN_SPLIT_R_LATE=1,jit@SPLIT_WG=4,jit@SPLIT_WG=8,jit@SPLIT=0"
CFG5_HOOK=tc run ab_cfg5_tc 300 python tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --variants "jit@SPLIT=0,jit,jit@SPLIT=0"
pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
run ct_probe 300 python tools/ct_probe.py --steps 6
run ct_probe_1flow 300 python tools/ct_probe.py --steps 3 --flows 1 --p-noise 0 --p-err 0 --p-icmp 0
run ct_probe_16flow 300 python tools/ct_probe.py --steps 3 --flows 16
python3 tools/ktsum.py "$O/kt_cfg5_split" > "$O/kt_cfg5_split.txt" 2>&1 || true
python3 tools/ktsum.py "$O/kt_cfg5_fused" > "$O/kt_cfg5_fused.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
exit 0
