#!/bin/bash
# Round-5 GPU pass 35: kernel copy-out while several decoders are live (default) vs SDMA always: 8 streams, the
# bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_streams.py 2 3 "auto:GPU_MAX_HW_QUEUES=8" "sdma:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_KCOPY_D2H=0" > gpurun_out/ab35_streams.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/b35.json 2> gpurun_out/b35.err || exit $?
echo ok
