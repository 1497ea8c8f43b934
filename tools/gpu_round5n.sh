#!/bin/bash
# Round-5 GPU pass 14: H.265 parity + legs + stamps (dword-wide tile stores); 8 streams with the reaper gated
# on other processes waiting, vs the round-4 tree and vs no shared budget; the concurrent-process CLI test.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py tests/test_gpu_cli.py > gpurun_out/t14.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b14.json 2> /dev/null || exit $?
M2DEC_AMD_LIB=build/dbg/libm2dec_amd_h5stamps.so M2DEC_AMD_H265_STREAMS=1 timeout -k 10 120 python -u tools/stamps_h265.py > gpurun_out/stamps_h265_14.txt 2>&1 || exit $?
timeout -k 10 500 python -u tools/ab_streams.py 3 3 "cur:GPU_MAX_HW_QUEUES=8" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" "noshare:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_SHARE=0" > gpurun_out/ab14_streams.txt 2>&1 || exit $?
echo ok
