#!/bin/bash
# Round-5 pass 42: re-sweep of the replay grid (inter workers per picture M2DEC_AMD_INTER_WG, default 80; row-pair
# workgroups of a P / B picture M2DEC_AMD_ROW_WG, default 12) on the current kernels, single-stream and 8-stream
# replay.  CFGS="inter row;inter row;..." picks the configurations, TAG the output name.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep${TAG:-42}.txt
: > $out
IFS=';' read -r -a cfgs <<< "${CFGS:-80 12;64 12;96 12;112 12;80 8;80 16;64 16}"
for rep in 1 2; do
  for cfg in "${cfgs[@]}"; do
    set -- $cfg
    for ns in 1 8; do
      M2DEC_AMD_INTER_WG=$1 M2DEC_AMD_ROW_WG=$2 timeout -k 10 150 python bench.py --replay-only --replay-streams $ns --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/sw.json || exit $?
      echo "inter $1 row $2 streams $ns: $(python3 -c "import json;print(json.load(open('gpurun_out/sw.json'))['value'])")" | tee -a $out
    done
  done
done
echo ok
