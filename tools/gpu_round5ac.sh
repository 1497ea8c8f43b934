#!/bin/bash
# Round-5 GPU pass 30: H.265 per-wave LDS in int16 (two 4-wave CTU workgroups per CU): parity, legs, stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py > gpurun_out/t30.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/h265_bench.py 10 > gpurun_out/h265_b30.json 2> /dev/null || exit $?
M2DEC_AMD_LIB=build/dbg/libm2dec_amd_h5stamps.so M2DEC_AMD_H265_STREAMS=1 timeout -k 10 120 python -u tools/stamps_h265.py > gpurun_out/stamps_h265_30.txt 2>&1 || exit $?
echo ok
