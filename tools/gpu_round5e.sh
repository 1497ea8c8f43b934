#!/bin/bash
# Round-5 GPU pass 5: C5 in bench.py's order (first seen after the 1080p legs) with the pool stats; the bench
# with a larger pinned-pool cap; the H.265 P / B timeline.
set -o pipefail
mkdir -p gpurun_out
C5_LATE=1 M2DEC_AMD_ASYNC_STATS=1 timeout -k 10 300 python -u tools/c5_bench_order.py > gpurun_out/c5_late.txt 2> gpurun_out/c5_late.err || exit $?
C5_LATE=1 M2DEC_AMD_POOL_PINNED_MB=8192 timeout -k 10 300 python -u tools/c5_bench_order.py > gpurun_out/c5_late8g.txt 2> /dev/null || exit $?
bash tools/h265_timeline.sh pb 4 c_h265_1080p_pb_s1 > gpurun_out/h5tl.log 2>&1 || exit $?
bash tools/h265_timeline.sh i 4 c_h265_1080p_s1 >> gpurun_out/h5tl.log 2>&1 || exit $?
echo ok
