#!/bin/bash
# Round-5 GPU pass 2: the default bench line, the thread-placement A/B, PMC traffic of the H.265 legs, the
# FETCH_SIZE width calibration.  Each step under its own limit, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/b3.json 2> gpurun_out/b3.err || exit $?
timeout -k 10 400 tools/ab_place.sh > gpurun_out/ab_place.txt 2>&1 || exit $?
bash tools/gpu_pmc.sh r121h265 h265 > gpurun_out/pmc_h265.log 2>&1 || exit $?
bash tools/gpu_pmc.sh r121h265pb h265_pb > gpurun_out/pmc_h265pb.log 2>&1 || exit $?
bash tools/gpu_pmc_calib.sh > gpurun_out/pmc_calib.txt 2>&1 || exit $?
echo ok
