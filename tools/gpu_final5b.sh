#!/bin/bash
# Round-5 final pass B: rocprofv3 stats of every bench leg; PMC traffic of the H.265 legs and the H.264 kernels.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
TAG=${TAG:-r126}
bash tools/gpu_pmc.sh ${TAG}_h265 h265 > gpurun_out/pmc_${TAG}_h265.out 2>&1 || exit $?
bash tools/gpu_pmc.sh ${TAG}_h265pb h265_pb > gpurun_out/pmc_${TAG}_h265pb.out 2>&1 || exit $?
bash tools/gpu_pmc.sh ${TAG}_pic k_picture > gpurun_out/pmc_${TAG}_pic.out 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_all -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_all.log 2>&1 || exit $?
cd $R && GPU_MAX_HW_QUEUES=8 M2DEC_AMD_THREAD_CPU=1 timeout -k 10 300 python -u tools/thread_cpu.py c3 8 > gpurun_out/thread_cpu_${TAG}.txt 2>&1 || exit $?
echo ok
