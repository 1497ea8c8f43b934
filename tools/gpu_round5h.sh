#!/bin/bash
# Round-5 GPU pass 8: the whole GPU suite (error words copied behind the frames, H.265 args in the arena),
# H.265 legs at 4 / 8 hardware queues, timelines, the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t8.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b8_q4.json 2> gpurun_out/h265_b8.err || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_b8_q8.json 2>> gpurun_out/h265_b8.err || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh pb8 4 c_h265_1080p_pb_s1 > gpurun_out/h5tl8.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/h265_timeline.sh i8 4 c_h265_1080p_s1 >> gpurun_out/h5tl8.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b8.json 2> gpurun_out/b8.err || exit $?
echo ok
