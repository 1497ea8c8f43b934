#!/bin/bash
# Round-5 GPU pass 36: MD5 batching of the shared pipe on the 8-stream leg (batches of 16 cost the same CPU
# time as batches of 8 on the box's host), MD5 thread count.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_streams.py 2 3 "dflt:GPU_MAX_HW_QUEUES=8" "b16:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_MIN_BATCH=16,M2DEC_AMD_MD5_WAIT_US=8000" "b16w4:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_MIN_BATCH=16" "t3:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAM_MD5_THREADS=3" > gpurun_out/ab36_streams.txt 2>&1 || exit $?
echo ok
