#!/bin/bash
# Round-5 pass 47: parse pool size, second look: c3 (12 / 13 / 14 / 16), C5 and 8 streams (14 vs 16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_env.py 3 6 "p16:GPU_MAX_HW_QUEUES=8" "p14:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=14" "p13:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=13" "p12:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=12" > gpurun_out/ab47_c3.txt 2>&1 || exit $?
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 3 4 "p16:GPU_MAX_HW_QUEUES=8" "p14:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=14" > gpurun_out/ab47_c5.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "p16:GPU_MAX_HW_QUEUES=8" "p14:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=14" > gpurun_out/ab47_streams.txt 2>&1 || exit $?
echo ok
