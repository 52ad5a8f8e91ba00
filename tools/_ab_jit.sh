set -u
# A/B of chain-program defines: parity tests with $DEFS, then tools/ablate.py jit vs jit:$DEFS (two rounds).
export PCN_IPT_JIT_DEFS="$DEFS"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_firewall.py tests/test_gpu_horus.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/abjit_tests.log 2>&1 || { tail -30 gpurun_out/abjit_tests.log; exit 1; }
tail -1 gpurun_out/abjit_tests.log
unset PCN_IPT_JIT_DEFS
V="jit:${DEFS// /+}"
timeout -k 10 600 python tools/ablate.py --variants "jit,$V,jit,$V" --hits ${HITS:-0,0.5,1} --iters 30
