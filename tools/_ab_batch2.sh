set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_batch2.log
for r in 1 2 3; do
for v in 2 1; do
  M2DEC_AMD_PICS_PER_LAUNCH=$v timeout -k 10 120 python tools/_ab_streams.py > gpurun_out/ab_one.log 2>&1 || { cat gpurun_out/ab_one.log >> gpurun_out/ab_batch2.log; exit 1; }
  echo "pics_per_launch=$v $(tail -1 gpurun_out/ab_one.log)" >> gpurun_out/ab_batch2.log
done
done
cat gpurun_out/ab_batch2.log
