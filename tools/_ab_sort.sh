set -u
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  for L in default s8 s12; do
    if [ $L = default ]; then LIB=$R/polycube_amd/libpcn_ipt.so; else LIB=$R/polycube_amd/ab/libpcn_ipt_ct_$L.so; fi
    echo "== $L run $r"
    PCN_IPT_LIBRARY=$LIB timeout -k 10 200 python tools/ct_probe.py --steps 6 2>&1 | tail -2 || exit 1
  done
done
