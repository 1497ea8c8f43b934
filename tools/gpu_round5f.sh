#!/bin/bash
# Round-5 GPU pass 6: H.265 parity with the CTU-grid kernel and 8 streams; H.265 legs; P / B timeline; C5 late
# with the stage stats; C5 late after release_pools.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py > gpurun_out/t6.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b6.json 2> gpurun_out/h265_b6.err || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh pb6 4 c_h265_1080p_pb_s1 > gpurun_out/h5tl6.log 2>&1 || exit $?
C5_LATE=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/c5_bench_order.py > gpurun_out/c5_late_q8.txt 2>/dev/null || exit $?
C5_LATE=1 C5_RELEASE=1 timeout -k 10 300 python -u tools/c5_bench_order.py > gpurun_out/c5_late_rel.txt 2>/dev/null || exit $?
echo ok
