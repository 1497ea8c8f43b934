set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_md5.log
for r in 1 2 3; do
for cfg in "8 4000" "12 8000"; do
  set -- $cfg
  M2DEC_AMD_MD5_MIN_BATCH=$1 M2DEC_AMD_MD5_WAIT_US=$2 timeout -k 10 120 python tools/_ab_streams.py > gpurun_out/ab_one.log 2>&1 || { cat gpurun_out/ab_one.log >> gpurun_out/ab_md5.log; exit 1; }
  echo "min_batch=$1 wait_us=$2 $(tail -1 gpurun_out/ab_one.log)" >> gpurun_out/ab_md5.log
done
done
cat gpurun_out/ab_md5.log
