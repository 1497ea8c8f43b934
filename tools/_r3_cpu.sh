#!/bin/bash
# round-3 host-side measurements: deblock sub-step stamps, parse A/B, multi-stream sweep with CPU use
set -o pipefail
mkdir -p gpurun_out
bash tools/_std.sh || exit $?
bash tools/pb_ab.sh > gpurun_out/pb_ab2.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/sweep_streams_e2e.py ${SWEEP:-8:3 16:3} > gpurun_out/sweep_e2e_r3.txt 2>&1
