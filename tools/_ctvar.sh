set -u
# conntrack/firewall/flow-split GPU tests, then ct_probe variants under a kernel trace.
#   OUT=<dir under gpurun_out>  VARS='args1;args2;...'  NOTEST=1 (skip the tests)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-ctv2}
mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
k=0
IFS=';' read -ra VS <<< "${VARS:---flows 65536;--flows 4096 --p-icmp 0 --p-err 0;--flows 1048576}"
for args in "${VS[@]}"; do
  k=$((k+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/v$k -o run -- python3 $R/tools/ct_probe.py --steps 2 $args > $O/v$k.log 2>&1 || exit 1
  echo "v$k $args: $(grep 'ms per batch' $O/v$k.log)"
done
