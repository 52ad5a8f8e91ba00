set -u
mkdir -p gpurun_out
timeout -k 10 900 python tools/ablate.py --cfg 5 --log2n 22 --variants "jit,jit:-DPCN_PREFETCH=2,jit,jit:-DPCN_PREFETCH=2" --hits 0.5 > gpurun_out/ab_pf5.log 2>&1
timeout -k 10 900 python tools/ablate.py --cfg 2 --variants "jit,jit:-DPCN_PREFETCH=2,jit,jit:-DPCN_PREFETCH=2" --hits 0.5 >> gpurun_out/ab_pf5.log 2>&1
cut -c1-170 gpurun_out/ab_pf5.log
