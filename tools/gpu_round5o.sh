#!/bin/bash
# Round-5 GPU pass 16: 8 streams across the round-5 commits (bisect of the 8-stream regression), same box.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
Q=GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_PINNED_MB=8192
timeout -k 10 900 python -u tools/ab_streams.py 3 3 "r4:$Q,AB_ROOT=$R/build/r4tree" "t6c3:$Q,AB_ROOT=$R/build/t6c3" "tac13:$Q,AB_ROOT=$R/build/tac13141" "cur:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab16_streams.txt 2>&1 || exit $?

GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/thread_cpu.py streams 3 > gpurun_out/tcpu16_cur.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 AB_ROOT=$R/build/r4tree timeout -k 10 200 python -u tools/thread_cpu.py streams 3 > gpurun_out/tcpu16_r4.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/thread_cpu.py c3 8 > gpurun_out/tcpu16_c3cur.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 AB_ROOT=$R/build/r4tree timeout -k 10 200 python -u tools/thread_cpu.py c3 8 > gpurun_out/tcpu16_c3r4.txt 2>&1 || exit $?
echo ok2
