#!/bin/bash
# Round-5 GPU pass 23: C5 with short 4K batches hashed one frame per thread, vs the round-5 r126 policy
# (M2DEC_AMD_MD5_MIN_BATCH=2 makes the timed-out 3-frame batch count as a batch again); c3 unchanged check.
set -o pipefail
mkdir -p gpurun_out
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 4 5 "single:GPU_MAX_HW_QUEUES=8" "batch:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_MIN_BATCH=2" > gpurun_out/ab23_c5.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_env.py 2 8 "cur:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab23_c3.txt 2>&1 || exit $?
echo ok
