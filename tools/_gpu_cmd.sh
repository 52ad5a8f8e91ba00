set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/ablate.py --variants "jit,jit1,jit2,jit3,jit4,jit" --hits 0.5,0,1 --iters 30 > gpurun_out/ab_stages.log 2>&1
cut -c1-170 gpurun_out/ab_stages.log
