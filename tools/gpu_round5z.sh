#!/bin/bash
# Round-5 GPU pass 27: H.265 P / B and intra timelines with the current kernels.
set -o pipefail
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh pb27 4 c_h265_1080p_pb_s1 > gpurun_out/h5tl27.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh i27 4 c_h265_1080p_s1 >> gpurun_out/h5tl27.log 2>&1 || exit $?
echo ok
