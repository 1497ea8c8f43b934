#!/bin/bash
# Round-5 GPU pass 11: copies through blit kernels instead of SDMA (HSA_ENABLE_SDMA=0) A/B on the 8-stream,
# C3 and H.265 legs; the H.265 submit trace without SDMA; H.265 CTU kernel stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_streams.py 3 3 "cur:GPU_MAX_HW_QUEUES=8" "nosdma:GPU_MAX_HW_QUEUES=8,HSA_ENABLE_SDMA=0" > gpurun_out/ab11_streams.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_env.py 3 8 "cur:GPU_MAX_HW_QUEUES=8" "nosdma:GPU_MAX_HW_QUEUES=8,HSA_ENABLE_SDMA=0" > gpurun_out/ab11_c3.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b11.json 2> /dev/null || exit $?
HSA_ENABLE_SDMA=0 GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b11_nosdma.json 2> /dev/null || exit $?
HSA_ENABLE_SDMA=0 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/h265_timeline_run.py c_h265_1080p_pb_s1 4 > gpurun_out/h5sub11.log 2> gpurun_out/h5sub11.err || exit $?
M2DEC_AMD_LIB=build/dbg/libm2dec_amd_h5stamps.so M2DEC_AMD_H265_STREAMS=1 timeout -k 10 120 python -u tools/stamps_h265.py > gpurun_out/stamps_h265.txt 2>&1 || exit $?
echo ok
