#!/bin/bash
# Round-5 pass 48: the MD5 tail mode's threshold (busy parse workers, M2DEC_AMD_MD5_TAIL_BUSY: 4 default, 2, 8) on c3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/ab_env.py ${ROUNDS:-3} 6 ${CFGS:-"t4:GPU_MAX_HW_QUEUES=8" "t2:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL_BUSY=2" "t8:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL_BUSY=8" "t12:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL_BUSY=12"} > gpurun_out/ab${TAG:-48}_c3.txt 2>&1 || exit $?
echo ok
