set -u
# A/B of a conntrack variant library (polycube_amd/ab/libpcn_ipt_ct_$NAME.so) against the default:
# the conntrack GPU tests on the variant, then ct_probe traffic on both.
R=$GRAFT_REPO_ROOT
V=${VARS:-"--flows 65536;--flows 1048576;--flows 4096 --p-icmp 0 --p-err 0"}
timeout -k 10 300 env PCN_IPT_LIBRARY=$R/polycube_amd/ab/libpcn_ipt_ct_$NAME.so python -u -m pytest tests/test_gpu_conntrack.py tests/test_gpu_firewall.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/ab_${NAME}_t.log 2>&1 || { tail -30 $R/gpurun_out/ab_${NAME}_t.log; exit 1; }
tail -1 $R/gpurun_out/ab_${NAME}_t.log
NOTEST=1 OUT=ab_${NAME}_def VARS="$V" bash tools/_ctvar.sh || exit 1
PCN_IPT_LIBRARY=$R/polycube_amd/ab/libpcn_ipt_ct_$NAME.so NOTEST=1 OUT=ab_$NAME VARS="$V" bash tools/_ctvar.sh || exit 1
