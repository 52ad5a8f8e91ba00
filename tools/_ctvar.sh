set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ctv2
timeout -k 10 300 python -u -m pytest tests/test_gpu_conntrack.py tests/test_gpu_firewall.py tests/test_gpu_flow_split.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/ctv2/t.log 2>&1; rc=$?; tail -2 $R/gpurun_out/ctv2/t.log; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
k=0
for args in "--flows 65536" "--flows 4096 --p-icmp 0 --p-err 0" "--flows 1048576"; do
  k=$((k+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ctv2/v$k -o run -- python3 $R/tools/ct_probe.py --steps 2 $args > $R/gpurun_out/ctv2/v$k.log 2>&1 || exit 1
  echo "v$k $args: $(grep 'ms per batch' $R/gpurun_out/ctv2/v$k.log)"
done
