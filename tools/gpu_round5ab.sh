#!/bin/bash
# Round-5 GPU pass 29: H.265 arena ring + kernel upload: parity, H.265 legs, bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py > gpurun_out/t29.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/h265_bench.py 10 > gpurun_out/h265_b29.json 2> /dev/null || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/b29.json 2> gpurun_out/b29.err || exit $?
echo ok
