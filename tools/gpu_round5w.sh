#!/bin/bash
# Round-5 GPU pass 24: C5 (4K) decode-path grid: row-pair workgroups and inter workers per P / B picture.
set -o pipefail
mkdir -p gpurun_out
AB_STREAM=c5_4k_s1 timeout -k 10 600 python -u tools/ab_env.py 3 5 "r12:GPU_MAX_HW_QUEUES=8" "r24:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_ROW_WG=24" "r34:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_ROW_WG=34" "i128:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_INTER_WG=128" > gpurun_out/ab24_c5.txt 2>&1 || exit $?
echo ok
