#!/bin/bash
# inter workers (G) x row-pair workgroups (R) per picture: the gpu_recon leg (k_batch over C3) and the
# 8-stream replay; one line per point
set -o pipefail
mkdir -p gpurun_out
for g in ${GS:-24 32 48 64 80}; do
  for r in ${RS:-12 17 34}; do
    M2DEC_AMD_INTER_WG=$g M2DEC_AMD_ROW_WG=$r timeout -k 5 120 python bench.py --steps 5 --warmup 2 --replay-only --no-cpu-baseline > gpurun_out/grid_${g}_${r}.json 2>/dev/null || exit $?
    echo "G=$g R=$r $(python3 -c "import json;d=json.load(open('gpurun_out/grid_${g}_${r}.json'));print(d['gpu_recon']['value'], d.get('gpu_recon_streams',{}).get('value'))")"
  done
done
