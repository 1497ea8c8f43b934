set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_streams.log
timeout -k 10 120 python tools/_ab_streams.py >> gpurun_out/ab_streams.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/_ab_streams.py >> gpurun_out/ab_streams.log 2>&1 &&
M2DEC_AMD_LIB=build/var6/libm2dec_amd.so GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/_ab_streams.py >> gpurun_out/ab_streams.log 2>&1 &&
M2DEC_AMD_LIB=build/var6/libm2dec_amd.so timeout -k 10 120 python tools/_ab_streams.py >> gpurun_out/ab_streams.log 2>&1
cat gpurun_out/ab_streams.log
