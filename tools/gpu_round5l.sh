#!/bin/bash
# Round-5 GPU pass 12: 8 streams, the round-4 tree vs the share commit (6c3c72d, with a job pool large enough
# that its fixed 2 GB bound does not bind) vs the current tree, same box.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 500 python -u tools/ab_streams.py 3 3 "cur:GPU_MAX_HW_QUEUES=8" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" "t6c3:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_PINNED_MB=8192,AB_ROOT=$R/build/t6c3" "cur8g:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_PINNED_MB=8192" > gpurun_out/ab12_streams.txt 2>&1 || exit $?
echo ok
