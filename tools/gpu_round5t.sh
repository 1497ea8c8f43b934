#!/bin/bash
# Round-5 GPU pass 21: C5 timeline (host events + kernel / copy trace), MD5 batching stats of c3 decodes,
# rocprofv3 stats of every bench leg.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
bash tools/timeline.sh c5r127 4 c5_4k_s1 > gpurun_out/tl_c5r127.out 2>&1 || exit $?
M2DEC_AMD_ASYNC_STATS=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/thread_cpu.py c3 6 > gpurun_out/c3_stats.txt 2> gpurun_out/c3_stats.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r127_all -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_r127_all.log 2>&1 || exit $?
echo ok
