#!/bin/bash
# The 8-stream end-to-end leg (bench end_to_end_streams) by parse-ahead workers per stream.
# Usage: bash tools/sweep_stream_threads.sh TAG -> gpurun_out/stream_threads_TAG.txt
set -o pipefail
TAG=${1:-st}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
out=gpurun_out/stream_threads_$TAG.txt
: > $out
for pt in ${PTS:-1 2 3 1 2 3}; do
  v=$(M2DEC_AMD_STREAM_PARSE_THREADS=$pt timeout -k 10 200 python -c "
import time, m2dec_amd, bench, json
golden = json.load(open('tests/golden/synthetic.json'))
datas = [bench.gen_stream('c3', s, 60) for s in range(1, 9)]
m2dec_amd.decode_streams(datas)
t0 = time.perf_counter(); got = m2dec_amd.decode_streams(datas); dt = time.perf_counter() - t0
ok = all(g == golden[bench.golden_name('c3', s)]['md5'] for g, s in zip(got, range(1, 9)))
print(round(sum(len(x) for x in got) / dt, 1), ok)") || exit 1
  echo "per-stream parse workers $pt: $v" | tee -a $out
done
