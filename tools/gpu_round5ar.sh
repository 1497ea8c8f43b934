#!/bin/bash
# Round-5 pass 46: parse pool size on the c3 decode (M2DEC_AMD_POOL_THREADS 16 default, 18, 20, 14).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_env.py 3 6 "p16:GPU_MAX_HW_QUEUES=8" "p18:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=18" "p20:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=20" "p14:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_THREADS=14" > gpurun_out/ab46_c3.txt 2>&1 || exit $?
echo ok
