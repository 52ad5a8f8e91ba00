set -u
# Conntrack A/B over several variant libraries (polycube_amd/ab/libpcn_ipt_ct_<name>.so) and the default:
#   TESTS="name ..." (variants that also run the conntrack GPU tests)  NAMES="name ..."  VARS=...
R=$GRAFT_REPO_ROOT
V=${VARS:-"--flows 65536;--flows 1048576;--flows 4096 --p-icmp 0 --p-err 0"}
OUT=abm_def bash tools/_ctvar.sh || exit 1
for nm in ${TESTS:-}; do
  timeout -k 10 300 env PCN_IPT_LIBRARY=$R/polycube_amd/ab/libpcn_ipt_ct_$nm.so python -u -m pytest tests/test_gpu_conntrack.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/abm_${nm}_t.log 2>&1 || { tail -30 $R/gpurun_out/abm_${nm}_t.log; exit 1; }
  echo "$nm tests: $(tail -1 $R/gpurun_out/abm_${nm}_t.log)"
done
for nm in ${NAMES:-}; do
  PCN_IPT_LIBRARY=$R/polycube_amd/ab/libpcn_ipt_ct_$nm.so NOTEST=1 OUT=abm_$nm VARS="$V" bash tools/_ctvar.sh || exit 1
done
