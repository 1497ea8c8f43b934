#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep_streams_e2e.py ${SWEEP:-16:3} > gpurun_out/sweep_e2e_r3b.txt 2>&1
