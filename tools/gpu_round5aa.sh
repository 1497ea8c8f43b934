#!/bin/bash
# Round-5 GPU pass 28: H.265 record upload by kernel (parity, legs with / without, P / B timeline).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py > gpurun_out/t28.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/h265_bench.py 10 > gpurun_out/h265_b28_k.json 2> /dev/null || exit $?
GPU_MAX_HW_QUEUES=8 M2DEC_AMD_H265_KCOPY=0 timeout -k 10 300 python -u tools/h265_bench.py 10 > gpurun_out/h265_b28_sdma.json 2> /dev/null || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh pb28 4 c_h265_1080p_pb_s1 > gpurun_out/h5tl28.log 2>&1 || exit $?
echo ok
