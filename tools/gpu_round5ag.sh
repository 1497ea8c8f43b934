#!/bin/bash
# Round-5 GPU pass 34: frames copied down by a kernel (M2DEC_AMD_KCOPY_D2H=1): the GPU suite with it on, c3 /
# 8-stream / C5 / H.265 A/B against the SDMA copy-out.
set -o pipefail
mkdir -p gpurun_out
M2DEC_AMD_KCOPY_D2H=1 timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t34.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_env.py 3 8 "kd2h:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY_D2H=1" "sdma:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab34_c3.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "kd2h:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY_D2H=1" "sdma:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab34_streams.txt 2>&1 || exit $?
AB_STREAM=c5_4k_s1 timeout -k 10 400 python -u tools/ab_env.py 2 5 "kd2h:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY_D2H=1" "sdma:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab34_c5.txt 2>&1 || exit $?
for i in 1 2; do
  M2DEC_AMD_KCOPY_D2H=1 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/ab34_h265_kd2h_$i.json 2>&1 || exit $?
  timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/ab34_h265_sdma_$i.json 2>&1 || exit $?
done
echo ok
