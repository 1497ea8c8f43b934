#!/bin/bash
# Round-5 GPU pass 18: bench line after the error-word fix; H.264 stream tests; H.265 err A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_streams.py tests/test_gpu_cli.py tests/test_gpu_h265.py > gpurun_out/t18.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/b18.json 2> gpurun_out/b18.err || exit $?
GPU_MAX_HW_QUEUES=8 M2DEC_AMD_H265_ERR_ASYNC=1 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b18_async.json 2> /dev/null || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b18_sync.json 2> /dev/null || exit $?
echo ok
