#!/bin/bash
# round-3 GPU check: the GPU test suite (incl. the boundary harness), smoke, and the default bench line
set -o pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_$TAG.log; exit $rc; fi
if [ "$2" = "bench" ]; then bash tools/gpu_smoke_bench.sh $TAG || exit $?; fi
exit 0
