#!/bin/bash
# Round-5 GPU pass 7: H.265 parity (coefficients staged in LDS, submit sizing before the dependency waits),
# H.265 legs at 4 and 8 hardware queues, P / B and intra timelines; C5 in the bench's order after the pools'
# LRU eviction; H.264 stream / boundary tests; the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py tests/test_gpu_streams.py tests/test_gpu_boundary.py > gpurun_out/t7.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b7_q4.json 2> gpurun_out/h265_b7.err || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b7_q8.json 2>> gpurun_out/h265_b7.err || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh pb7 4 c_h265_1080p_pb_s1 > gpurun_out/h5tl7.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh i7 4 c_h265_1080p_s1 >> gpurun_out/h5tl7.log 2>&1 || exit $?
C5_LATE=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/c5_bench_order.py > gpurun_out/c5_late7.txt 2>/dev/null || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b7.json 2> gpurun_out/b7.err || exit $?
echo ok
