set -u
# rocprofv3 kernel stats of the stateful probe: default library vs ab/libpcn_ipt_ct_$NAME.so
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in default $NAME; do
  if [ $L = default ]; then LIB=$R/polycube_amd/libpcn_ipt.so; else LIB=$R/polycube_amd/ab/libpcn_ipt_ct_$L.so; fi
  PCN_IPT_LIBRARY=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abprof_$L -o run --output-format csv \
    -- python3 $R/tools/ct_probe.py --steps 6 ${PROBE_ARGS:-} > $R/gpurun_out/abprof_$L.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/abprof_$L.log
done
