set -o pipefail
V=mb3 bash tools/ab_replay.sh mb3 > /dev/null 2>&1 || { echo replay-ab-failed; tail gpurun_out/ab_mb3.txt; exit 1; }
cat gpurun_out/ab_mb3.txt
for v in default mb3 default mb3; do
  if [ $v = default ]; then L=m2dec_amd/lib/libm2dec_amd.so; else L=build/var/lib_$v.so; fi
  M2DEC_AMD_LIB=$L timeout -k 10 120 python tools/_ab_streams.py > gpurun_out/ab_one.log 2>&1 || { cat gpurun_out/ab_one.log; exit 1; }
  echo "$v e2e: $(tail -1 gpurun_out/ab_one.log)"
done
