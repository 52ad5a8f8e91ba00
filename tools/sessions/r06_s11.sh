#!/bin/bash
# Round 6, session 11: does uncached or fine-grained device memory let the L2 fetch less
# than a 128-byte line for a 48-byte header window?  tools/gather_calib stride patterns
# (timing + FETCH_SIZE + TCC_EA0_RDREQ split) in normal, uncached and fine-grained memory.
TAG=r06_s11
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
for al in nm uc fg; do
  export CALIB_ALLOC=$al
  calib ${al}_s128 stride:128 24 calib_stride
  calib ${al}_s1536 stride:1536 24 calib_stride
  calib ${al}_s64 stride:64 24 calib_stride
done
exit 0
