set -o pipefail
mkdir -p gpurun_out
for v in default 1; do
  if [ $v = default ]; then E=""; else E="M2DEC_AMD_PICS_PER_LAUNCH=$v"; fi
  env $E timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/ab_bench_$v.json 2> gpurun_out/ab_bench_$v.err || { tail -5 gpurun_out/ab_bench_$v.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab_bench_$v.json').read().strip().splitlines()[-1])
print('$v', 'c3', d['value'], 'streams', d['end_to_end_streams']['value'], d['end_to_end_streams']['passes_fps'], 'c5', d['end_to_end_c5']['value'])"
done
