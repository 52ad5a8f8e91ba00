#!/bin/bash
# Round 6, session 4: counted output stores (PCN_STORE_COUNT: buffer stores every wave
# issues, the header wait counts them) and the early image stage (PCN_STAGE_EARLY), as
# chain-program defines: parity under both, A/B on configs 3 / 2 / 5 and the stateful probe.
TAG=r06_s4
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
BOTH="-DPCN_STORE_COUNT=1 -DPCN_STAGE_EARLY=1"
PCN_IPT_JIT_DEFS="$BOTH" pytest_gpu tests_par 600 tests/test_gpu_parity.py -k "config_parity or full_size_headline or frame_size_sweep or full_size_config5 or fuzz"
PCN_IPT_JIT_DEFS="$BOTH" pytest_gpu tests_ct 900 tests/test_gpu_conntrack.py
V="jit,jit:-DPCN_STORE_COUNT=1,jit:-DPCN_STAGE_EARLY=1,jit:-DPCN_STORE_COUNT=1+-DPCN_STAGE_EARLY=1,jit"
run ab_cfg3 600 python tools/ablate.py --cfg 3 --log2n 24 --hits 0,0.5,1 --variants "$V"
run ab_cfg2 300 python tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --variants "$V,jit:-DPCN_STORE_COUNT=1+-DPCN_STAGE_EARLY=1"
run ab_cfg5 300 python tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --variants "jit,jit:-DPCN_STAGE_EARLY=1,jit,jit:-DPCN_STAGE_EARLY=1"
for r in 1 2; do
  run ct_fused_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_STORE_COUNT=1" run ct_fused_sc_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_JIT_DEFS="-DPCN_STORE_COUNT=1" PCN_IPT_DEBUG_CT_FUSED=0 run ct_prep_sc_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && PCN_IPT_JIT_DEFS="-DPCN_STORE_COUNT=1" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$O/ct_prof_sc" -o run -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof_sc.log" 2>&1 )
echo "== ct_prof_sc rc=$?"
python3 tools/ktsum.py "$O/ct_prof_sc" > "$O/ct_prof_sc.txt" 2>&1 || true
find "$O" -name "*kernel_trace.csv" -delete
exit 0
