#!/bin/bash
# Round-5 GPU pass 25: MD5 tail mode on the parse pool's pending work vs its running workers (r126): c3, 8
# streams, C5; MD5 batch counts per c3 decode.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_env.py 3 8 "pending:GPU_MAX_HW_QUEUES=8" "running:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL=2" > gpurun_out/ab25_c3.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "pending:GPU_MAX_HW_QUEUES=8" "running:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL=2" > gpurun_out/ab25_streams.txt 2>&1 || exit $?
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 3 5 "pending:GPU_MAX_HW_QUEUES=8" "running:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL=2" > gpurun_out/ab25_c5.txt 2>&1 || exit $?
M2DEC_AMD_ASYNC_STATS=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/thread_cpu.py c3 6 > gpurun_out/c3_stats25.txt 2> gpurun_out/c3_stats25.err || exit $?
echo ok
