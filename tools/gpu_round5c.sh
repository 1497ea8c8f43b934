#!/bin/bash
# Round-5 GPU pass 3: H.265 and CLI GPU tests (row-wait change, concurrent processes), the default bench line,
# PMC traffic of the H.265 legs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_h265.py tests/test_gpu_cli.py tests/test_gpu_boundary.py > gpurun_out/t3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b4.json 2> gpurun_out/b4.err || exit $?
bash tools/gpu_pmc.sh r122h265 h265 > gpurun_out/pmc_h265.log 2>&1 || exit $?
bash tools/gpu_pmc.sh r122h265pb h265_pb > gpurun_out/pmc_h265pb.log 2>&1 || exit $?
echo ok
