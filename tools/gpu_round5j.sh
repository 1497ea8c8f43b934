#!/bin/bash
# Round-5 GPU pass 10: parity after the wait reordering and the adaptive pinned-pool cap; 8 streams and C3
# against the round-4 tree; H.265 submit trace and legs; the bench line.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t10.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 3 3 "cur:GPU_MAX_HW_QUEUES=8" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" > gpurun_out/ab10_streams.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_env.py 3 8 "cur:GPU_MAX_HW_QUEUES=8" "r4:GPU_MAX_HW_QUEUES=8,AB_ROOT=$R/build/r4tree" > gpurun_out/ab10_c3.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/h265_timeline_run.py c_h265_1080p_pb_s1 4 > gpurun_out/h5sub10.log 2> gpurun_out/h5sub10.err || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b10.json 2> gpurun_out/b10.err || exit $?
echo ok
