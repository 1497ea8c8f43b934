set -e
for g in 16 32 48 64 96; do
  M2DEC_AMD_INTER_WG=$g timeout -k 5 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/sw_$g.json 2>/dev/null
  echo "G=$g $(python3 -c "import json;d=json.load(open('gpurun_out/sw_$g.json'));print(d['value'])")"
done
