#!/bin/bash
# In-kernel timelines (stamps build): the batch per-picture timeline, then single pictures run alone.
set -o pipefail
mkdir -p gpurun_out
export M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so
timeout -k 10 120 python tools/stamps_batch.py > gpurun_out/stamps_batch.txt 2>&1 || exit $?
for n in ${@:-1 2 5}; do
  M2DEC_AMD_REPLAY_LIMIT=$n M2DEC_AMD_REPLAY_ISOLATE_LAST=1 timeout -k 10 120 python tools/stamps_pic.py > gpurun_out/stamps_pic$n.txt 2>&1 || exit $?
done
echo ok
