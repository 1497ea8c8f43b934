#!/bin/bash
# Round-5 GPU pass 22: MD5 batch latency on the box's host (4-lane kernel for 2-4 frames); c3 / 8-stream / C5
# decodes with the tail share of 4 vs one frame per thread (the round-4 policy).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
python3 tools/md5_batch_bench.py > gpurun_out/md5b22.txt 2>&1 || exit $?
M2DEC_AMD_MD5_NO_X4=1 python3 tools/md5_batch_bench.py > gpurun_out/md5b22_nox4.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_env.py 3 8 "share4:GPU_MAX_HW_QUEUES=8" "share0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL_SHARE=0" > gpurun_out/ab22_c3.txt 2>&1 || exit $?
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 3 5 "share4:GPU_MAX_HW_QUEUES=8" "share0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL_SHARE=0" > gpurun_out/ab22_c5.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "share4:GPU_MAX_HW_QUEUES=8" "share0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL_SHARE=0" > gpurun_out/ab22_streams.txt 2>&1 || exit $?
echo ok
