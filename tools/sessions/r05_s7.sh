#!/bin/bash
# Round 5, session 7: the radix sort with 1024-thread tiles + windowed look-back
# (tests, stateful batch against a rocPRIM build of the same tree, kernel trace);
# config 2 at 2^20: per-workgroup timelines (full and parse only) and A/B of the
# shallow prefetch and 8 waves per SIMD; config 5 prefetch depth 2 after clustering.
TAG=r05_s7
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_LIBRARY=$R/polycube_amd/build/ab/libpcn_ipt_ct_rocprim.so run ct_probe_rocprim_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
find "$O" -name "*kernel_trace.csv" -delete
PCN_IPT_DEBUG_CLOCKS=1 run clocks_cfg2 200 python tools/wg_clocks.py --cfg 2 --log2n 20
PCN_IPT_DEBUG_CLOCKS=1 PCN_IPT_JIT_DEFS=-DPCN_ABLATE=1 run clocks_cfg2_parse 200 python tools/wg_clocks.py --cfg 2 --log2n 20
PCN_IPT_DEBUG_CLOCKS=1 run clocks_cfg3 200 python tools/wg_clocks.py --cfg 3 --log2n 24 --launches 3
run ab_cfg2 400 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 100 \
  --variants "jit,jit@SHALLOW=0,jit:-DPCN_WAVES_PER_SIMD=8@WG_PER_CU=2,jit1,jit,jit@SHALLOW=0"
run ab_cfg5 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_PREFETCH_GENERIC=2,jit,jit:-DPCN_PREFETCH_GENERIC=2"
exit 0
