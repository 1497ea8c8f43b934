set -e
for g in 8 12 16 24 34; do
  M2DEC_AMD_ROW_WG=$g timeout -k 5 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/swr_$g.json 2>/dev/null
  echo "R=$g $(python3 -c "import json;d=json.load(open('gpurun_out/swr_$g.json'));print(d['value'])")"
done
