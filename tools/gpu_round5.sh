#!/bin/bash
# Round-5 GPU pass: the -m gpu suite, per-slice intra stamps of a C5 I picture, the default bench line, and
# the host-parse PGO A/B; each step under its own limit, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t2.log 2>&1 || exit $?
M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=1 timeout -k 10 120 python -u tools/stamps_slices.py > gpurun_out/stamps_slices.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b2.json 2> gpurun_out/b2.err || exit $?
PGO_VARIANTS="A C D" timeout -k 10 120 tools/pgo_ab.sh > gpurun_out/pgo_ab.txt 2>&1 || exit $?
echo ok
