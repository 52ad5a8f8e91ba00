set -u
# A/B of the default library against polycube_amd/ab/libpcn_ipt_ct_$NAME.so on the stateful probe,
# after the stateful GPU tests on the default build.  Logs to stdout.
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py \
  tests/test_gpu_horus.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2; do
  for L in default $NAME; do
    if [ $L = default ]; then LIB=$R/polycube_amd/libpcn_ipt.so; else LIB=$R/polycube_amd/ab/libpcn_ipt_ct_$L.so; fi
    echo "== $L run $r"
    PCN_IPT_LIBRARY=$LIB timeout -k 10 200 python tools/ct_probe.py --steps 6 ${PROBE_ARGS:-} 2>&1 | tail -1 || exit 1
  done
done
