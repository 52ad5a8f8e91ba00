#!/bin/bash
# Round 4, session 15 (data for the next round): L2 -> memory read request sizes and
# L2 hit rates of the stateful kernels (ct_walk's 32-byte record gathers, ct_prep's
# streams) and of config 5's IMIX header gathers.
TAG=r04_s15
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
K="ct_prep ct_walk ct_heads ct_count"
pmcct ct_rdreq "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "$K"
pmcct ct_tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "$K"
pmcq rdreq_cfg5 5 22 0.5 "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
pmcq rdreq_cfg3 3 24 0.5 "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
exit 0
