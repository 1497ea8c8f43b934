#!/bin/bash
# Host thread split of the single-stream decode path (parse-ahead workers x MD5 threads) under the
# box's CPU quota: bench.py's headline value per setting.  Usage: bash tools/sweep_threads.sh TAG
set -o pipefail
TAG=${1:-sweep}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
out=gpurun_out/threads_$TAG.txt
: > $out
for pt in ${PTS:-8 10 12 14}; do
  for mt in ${MTS:-3 5 8}; do
    v=$(M2DEC_AMD_PARSE_THREADS=$pt M2DEC_AMD_MD5_THREADS=$mt timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 8 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["wall_fps"])') || exit 1
    echo "parse $pt md5 $mt: $v" | tee -a $out
  done
done
