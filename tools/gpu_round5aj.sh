#!/bin/bash
# Round-5 GPU pass 37: CPU time per thread role, exited threads included (M2DEC_AMD_THREAD_CPU=1), for the
# 8-stream leg and the c3 decode.
set -o pipefail
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 M2DEC_AMD_THREAD_CPU=1 timeout -k 10 300 python -u tools/thread_cpu.py streams 3 > gpurun_out/tc37.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 M2DEC_AMD_THREAD_CPU=1 timeout -k 10 300 python -u tools/thread_cpu.py c3 8 >> gpurun_out/tc37.txt 2>&1 || exit $?
echo ok
