#!/bin/bash
# One runner for the GPU-box A/B measurements (run through gpurun from the repo root):
#
#   bash tools/ab.sh tests [pytest files...]     GPU tests (default: all -m gpu) -> gpurun_out/ab_tests.log
#   DEFS="-DX=1" bash tools/ab.sh jit            chain-program defines: parity tests with PCN_IPT_JIT_DEFS,
#                                                then tools/ablate.py jit vs jit:$DEFS (two rounds, HITS=0,0.5,1)
#   AB="v1,v2" [CFG=2] bash tools/ab.sh ablate   tools/ablate.py --variants "$AB" (any variant list)
#   NAMES="a b" [TESTS=1] bash tools/ab.sh lib   conntrack variant libraries polycube_amd/ab/libpcn_ipt_ct_<name>.so
#                                                (make ct_variant) against the default on tools/ct_probe.py,
#                                                PROBE_ARGS passed through; TESTS=1 runs the stateful tests on each
#   NAMES="a" bash tools/ab.sh prof              rocprofv3 --kernel-trace --stats of ct_probe: default vs variants
#   [VARS='a;b'] [OUT=dir] bash tools/ab.sh ctvar  ct_probe traffic variants under a kernel trace (NOTEST=1: no tests)
#
# Every GPU step runs under its own timeout and the first failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mode=${1:-tests}
shift || true
mkdir -p "$R/gpurun_out"
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
STATEFUL="tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py"

lib_of() { if [ "$1" = default ]; then echo "$R/polycube_amd/libpcn_ipt.so"; else echo "$R/polycube_amd/build/ab/libpcn_ipt_ct_$1.so"; fi; }

case $mode in
tests)
  files=${*:-tests}
  timeout -k 10 900 $PYT -m gpu $files > "$R/gpurun_out/ab_tests.log" 2>&1; rc=$?
  tail -5 "$R/gpurun_out/ab_tests.log"
  exit $rc ;;
jit)
  PCN_IPT_JIT_DEFS="$DEFS" timeout -k 10 500 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_firewall.py \
    tests/test_gpu_horus.py > "$R/gpurun_out/abjit_tests.log" 2>&1 || { tail -30 "$R/gpurun_out/abjit_tests.log"; exit 1; }
  tail -1 "$R/gpurun_out/abjit_tests.log"
  V="jit:${DEFS// /+}"
  timeout -k 10 600 python -u tools/ablate.py --variants "jit,$V,jit,$V" --hits "${HITS:-0,0.5,1}" --iters 30 ;;
ablate)
  timeout -k 10 600 python -u tools/ablate.py --cfg "${CFG:-3}" --variants "$AB" --hits "${HITS:-0,0.5,1}" ;;
lib)
  for nm in ${NAMES:-}; do
    if [ -n "${TESTS:-}" ]; then
      PCN_IPT_LIBRARY=$(lib_of "$nm") timeout -k 10 400 $PYT $STATEFUL > "$R/gpurun_out/ab_${nm}_t.log" 2>&1 \
        || { tail -30 "$R/gpurun_out/ab_${nm}_t.log"; exit 1; }
      echo "$nm tests: $(tail -1 "$R/gpurun_out/ab_${nm}_t.log")"
    fi
  done
  for r in 1 2; do
    for L in default ${NAMES:-}; do
      echo "== $L run $r"
      PCN_IPT_LIBRARY=$(lib_of "$L") timeout -k 10 200 python tools/ct_probe.py --steps 6 ${PROBE_ARGS:-} 2>&1 | tail -1 || exit 1
    done
  done ;;
prof)
  cd /tmp && export TMPDIR=/tmp
  for L in default ${NAMES:-}; do
    PCN_IPT_LIBRARY=$(lib_of "$L") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/abprof_$L" -o run \
      --output-format csv -- python3 "$R/tools/ct_probe.py" --steps 6 ${PROBE_ARGS:-} > "$R/gpurun_out/abprof_$L.log" 2>&1 || exit 1
    tail -1 "$R/gpurun_out/abprof_$L.log"
  done ;;
ctvar)
  O=$R/gpurun_out/${OUT:-ctvar}
  mkdir -p "$O"
  if [ -z "${NOTEST:-}" ]; then
    timeout -k 10 300 $PYT $STATEFUL > "$O/t.log" 2>&1; rc=$?; tail -2 "$O/t.log"; [ $rc = 0 ] || exit $rc
  fi
  cd /tmp && export TMPDIR=/tmp
  k=0
  IFS=';' read -ra VS <<< "${VARS:---flows 65536;--flows 4096 --p-icmp 0 --p-err 0;--flows 1048576}"
  for args in "${VS[@]}"; do
    k=$((k+1))
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/v$k" -o run -- python3 "$R/tools/ct_probe.py" \
      --steps 2 $args > "$O/v$k.log" 2>&1 || exit 1
    echo "v$k $args: $(grep 'ms per batch' "$O/v$k.log")"
  done ;;
*)
  echo "unknown mode $mode" >&2; exit 2 ;;
esac
