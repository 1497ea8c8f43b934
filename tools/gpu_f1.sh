#!/bin/bash
# First GPU bring-up: dual (HIP vs oracle) per-picture diff on F1, then the gpu test suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m tests.diag_dual tests/golden/f1_realshort.264 > gpurun_out/diag_f1.log 2>&1
rc=$?
echo "diag rc=$rc"
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
