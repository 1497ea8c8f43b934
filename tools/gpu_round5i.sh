#!/bin/bash
# Round-5 GPU pass 9: the 8-stream and C3 legs against the round-4 tree on the same box (A/B, own processes),
# with / without the shared budget; the H.265 submit-step trace.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u tools/ab_streams.py 3 3 "cur:GPU_MAX_HW_QUEUES=8" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" "noshare:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_SHARE=0" > gpurun_out/ab9_streams.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_env.py 3 8 "cur:GPU_MAX_HW_QUEUES=8" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" "noshare:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_SHARE=0" > gpurun_out/ab9_c3.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/h265_timeline_run.py c_h265_1080p_pb_s1 4 > gpurun_out/h5sub9.log 2> gpurun_out/h5sub9.err || exit $?
echo ok
