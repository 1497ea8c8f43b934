#!/bin/bash
# Round-5 GPU pass 26: is the job's CPU share a CFS quota, and do c3 decodes get throttled?
mkdir -p gpurun_out
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>&1)"; echo "nproc $(nproc) OMP $OMP_NUM_THREADS"; cat /sys/fs/cgroup/cpu.stat 2>&1; } > gpurun_out/cg26.txt
timeout -k 10 300 python -u tools/ab_env.py 1 12 "cur:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab26_c3.txt 2>&1 || exit $?
{ echo "--- after"; cat /sys/fs/cgroup/cpu.stat 2>&1; } >> gpurun_out/cg26.txt
echo ok
