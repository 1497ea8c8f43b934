set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_streams.py tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hold_tests.log 2>&1 || { tail -20 gpurun_out/hold_tests.log; exit 1; }
tail -1 gpurun_out/hold_tests.log
: > gpurun_out/ab_hold.log
for r in 1 2 3; do
for v in 1 0; do
  M2DEC_AMD_HOLD_BUSY=$v timeout -k 10 120 python tools/_ab_streams.py > gpurun_out/ab_one.log 2>&1 || { cat gpurun_out/ab_one.log >> gpurun_out/ab_hold.log; exit 1; }
  echo "hold_busy=$v $(tail -1 gpurun_out/ab_one.log)" >> gpurun_out/ab_hold.log
done
done
cat gpurun_out/ab_hold.log
