#!/bin/bash
# Round-5 GPU pass 17: 8 streams, error word behind the frame vs the round-4 synchronous read; vs round 4.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 700 python -u tools/ab_streams.py 3 3 "cur:GPU_MAX_HW_QUEUES=8" "errsync:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_ERR_SYNC=1" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" "tac13:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_POOL_PINNED_MB=8192,AB_ROOT=$R/build/tac13141" > gpurun_out/ab17_streams.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 M2DEC_AMD_ERR_SYNC=1 timeout -k 10 200 python -u tools/thread_cpu.py streams 3 > gpurun_out/tcpu17_errsync.txt 2>&1 || exit $?
echo ok
