#!/bin/bash
# Diagnose the cross-process hang: the decode-path tests in this process, then the HIP harness in a child.
set -o pipefail
mkdir -p gpurun_out
export M2DEC_AMD_BUDGET_LOG=$PWD/gpurun_out/budget.log M2DEC_AMD_SHARE_REPORT=1
timeout -k 10 240 python -u -m pytest -x -v --timeout 60 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_boundary.py -k "pictures_per_launch or switch" > gpurun_out/diag.log 2>&1
rc=$?
ls -la /dev/shm >> gpurun_out/diag.log 2>&1
exit $rc
