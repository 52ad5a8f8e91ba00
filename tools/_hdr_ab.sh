set -u
# A/B of header-load variants of the chain program (tools/ablate.py, JIT defines), then parity under VARIANT_DEFS.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/hdr
timeout -k 10 600 python -u tools/ablate.py --variants "$AB" --hits ${HITS:-0,0.5,1} > $R/gpurun_out/hdr/ab.log 2>&1 || { tail -20 $R/gpurun_out/hdr/ab.log; exit 1; }
cat $R/gpurun_out/hdr/ab.log
if [ -n "${VARIANT_DEFS:-}" ]; then
  timeout -k 10 500 env PCN_IPT_JIT_DEFS="$VARIANT_DEFS" python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_horus.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/hdr/t.log 2>&1; rc=$?
  tail -3 $R/gpurun_out/hdr/t.log
  exit $rc
fi
