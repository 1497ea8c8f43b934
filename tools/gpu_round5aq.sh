#!/bin/bash
# Round-5 pass 45: bind's copy-outs alternating over two copy streams (default with 8 hardware queues) against one
# (M2DEC_AMD_COPY_STREAMS=1): decode-path GPU tests, c3 / C5 / 8-stream A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_streams.py tests/test_gpu_boundary.py tests/test_gpu_f1.py > gpurun_out/t45.log 2>&1 || exit $?
tail -1 gpurun_out/t45.log
timeout -k 10 400 python -u tools/ab_env.py 3 6 "cs2:GPU_MAX_HW_QUEUES=8" "cs1:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_COPY_STREAMS=1" > gpurun_out/ab45_c3.txt 2>&1 || exit $?
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 3 4 "cs2:GPU_MAX_HW_QUEUES=8" "cs1:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_COPY_STREAMS=1" > gpurun_out/ab45_c5.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "cs2:GPU_MAX_HW_QUEUES=8" "cs1:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_COPY_STREAMS=1" > gpurun_out/ab45_streams.txt 2>&1 || exit $?
echo ok
