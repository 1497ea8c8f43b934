#!/bin/bash
# Round-5 pass 43: more row-pair workgroups per P / B picture (16, 20, 24) on the replay and on the c3 decode.
set -o pipefail
mkdir -p gpurun_out
TAG=43 CFGS='80 12;80 16;80 20;80 24;96 20' bash tools/gpu_round5ao.sh || exit $?
timeout -k 10 400 python -u tools/ab_env.py 3 6 "r12:GPU_MAX_HW_QUEUES=8" "r16:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_ROW_WG=16" "r20:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_ROW_WG=20" > gpurun_out/ab43_c3.txt 2>&1 || exit $?
echo ok
