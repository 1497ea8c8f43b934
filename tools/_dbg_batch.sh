set -o pipefail
mkdir -p gpurun_out
M2DEC_AMD_DEBUG=1 M2DEC_AMD_ASYNC_STATS=2 timeout -k 10 120 python tools/_ab_streams.py > gpurun_out/dbg_batch.log 2>&1
tail -60 gpurun_out/dbg_batch.log
