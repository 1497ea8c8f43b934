#!/bin/bash
# Multi-stream replay (bench.py --replay-only --replay-streams 8): inter workers per picture x row-pair
# workgroups per P/B picture.  Fewer workgroups per picture = more pictures resident at once (1024 slots).
# Usage: bash tools/sweep_streams.sh [TAG]  -> gpurun_out/sweep_streams_TAG.txt
set -o pipefail
TAG=${1:-r45}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
OUT=$R/gpurun_out/sweep_streams_$TAG.txt
: > $OUT
for G in ${GS:-16 24 32 48 80}; do
  for RW in ${RWS:-6 12}; do
    M2DEC_AMD_INTER_WG=$G M2DEC_AMD_ROW_WG=$RW timeout -k 10 120 python3 $R/bench.py --replay-only --replay-streams ${NS:-8} \
      --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/sw_${G}_${RW}.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('inter_wg', sys.argv[2], 'row_wg', sys.argv[3], 'fps', d['value'], 'ms', d['ms_per_step'])" \
      $R/gpurun_out/sw_${G}_${RW}.json $G $RW | tee -a $OUT
  done
done
