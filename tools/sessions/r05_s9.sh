#!/bin/bash
# Round 5, session 9: super-tile reduce-then-scan radix passes (no look-back,
# no histogram kernel) against the onesweep; config 5 ablation ladder after the
# rule clustering (parse only / lookups / no candidate stage).
TAG=r05_s9
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_radix 300 tests/test_gpu_radix.py
KEEP_GOING=1
for r in 1 2; do
  PCN_IPT_DEBUG_RADIX=rts run ct_probe_rts_$r 300 python tools/ct_probe.py --steps 6
  PCN_IPT_DEBUG_RADIX=rts512 run ct_probe_rts512_$r 300 python tools/ct_probe.py --steps 6
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
for m in rts rts512; do
  export PCN_IPT_DEBUG_RADIX=$m
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof_$m" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof_$m.log" 2>&1 )
  echo "== ct_prof_$m rc=$?"
done
find "$O" -name "*kernel_trace.csv" -delete
export PCN_IPT_DEBUG_RADIX=rts
pytest_gpu tests_ct_rts 600 tests/test_gpu_conntrack.py
unset PCN_IPT_DEBUG_RADIX
run abl_cfg5 400 python -u tools/ablate.py --cfg 5 --log2n 22 --hits 0.5 --iters 30 \
  --variants "jit,jit:-DPCN_ABLATE=1,jit:-DPCN_ABLATE=2,jit:-DPCN_ABLATE=3,jit"

run abl_cfg2 400 python -u tools/ablate.py --cfg 2 --log2n 20 --hits 0.5 --iters 100 \
  --variants "jit,jit:-DPCN_ABLATE=1,jit:-DPCN_ABLATE=2,jit:-DPCN_ABLATE=3,jit"
exit 0
