#!/bin/bash
# Round-5 GPU pass 40: intra_row inlined into its callers (build/var/lib_ir.so: 304 instead of 392 B of scratch
# per lane, 154 instead of 186 scratch instructions) against the default library: replay legs, c3 decode.
set -o pipefail
mkdir -p gpurun_out
V=ir bash tools/ab_replay.sh ir40 || exit $?
timeout -k 10 400 python -u tools/ab_env.py 3 6 "base:GPU_MAX_HW_QUEUES=8" "ir:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_LIB=$PWD/build/var/lib_ir.so" > gpurun_out/ab40_c3.txt 2>&1 || exit $?
echo ok
