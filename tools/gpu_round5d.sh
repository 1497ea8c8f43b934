#!/bin/bash
# Round-5 GPU pass 4: H.264 parity after the intra hand-off prefetch, the I-picture step stamps, C5 after each
# bench leg, the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_streams.py tests/test_gpu_f1.py tests/test_gpu_batch.py tests/test_quirks.py tests/test_gpu_h265.py > gpurun_out/t4.log 2>&1 || exit $?
for s in c3_1080p_s1 c5_4k_s1; do
  M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=1 timeout -k 10 120 python -u tools/stamps_istep.py $s >> gpurun_out/stamps_istep.txt 2>&1 || exit $?
done
M2DEC_AMD_DEBUG=1 timeout -k 10 300 python -u tools/c5_bench_order.py > gpurun_out/c5_order.txt 2> gpurun_out/c5_order.err || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b5.json 2> gpurun_out/b5.err || exit $?
echo ok
