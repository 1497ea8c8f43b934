#!/bin/bash
# Round-5 GPU pass 33: H.264 records uploaded by a kernel: the GPU suite, c3 / 8-stream / C5 A/B against the
# SDMA uploads, timeline of 8 decodes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t33.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_env.py 3 8 "kcopy:GPU_MAX_HW_QUEUES=8" "sdma:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY=0" > gpurun_out/ab33_c3.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "kcopy:GPU_MAX_HW_QUEUES=8" "sdma:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY=0" > gpurun_out/ab33_streams.txt 2>&1 || exit $?
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 2 5 "kcopy:GPU_MAX_HW_QUEUES=8" "sdma:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY=0" > gpurun_out/ab33_c5.txt 2>&1 || exit $?
echo ok
