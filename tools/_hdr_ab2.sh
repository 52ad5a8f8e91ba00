set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/hdr2
V="jit,jit:-DPCN_HDR_ASM=1+-DPCN_HDR_ASM_MEM=0,jit,jit:-DPCN_HDR_ASM=1+-DPCN_HDR_ASM_MEM=0"
timeout -k 10 500 python -u tools/ablate.py --variants "$V" --hits 0,0.25,0.5,0.75,1 > $R/gpurun_out/hdr2/cfg3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ablate.py --cfg 2 --variants "$V" --hits 0.5 > $R/gpurun_out/hdr2/cfg2.log 2>&1 || exit 1
cat $R/gpurun_out/hdr2/cfg3.log $R/gpurun_out/hdr2/cfg2.log
