#!/bin/bash
# The driver's round-end sequence in one call: smoke() on cuda:0, then the default bench line.
# Usage: bash tools/gpu_smoke_bench.sh TAG  -> gpurun_out/bench_TAG.json
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 - gpurun_out/bench_$TAG.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["gpu_recon_streams"]
print("value", d["value"], "traffic", d["roofline"]["traffic"], "gpu_recon", d["gpu_recon"]["value"],
      "streams", s["value"], s["roofline"]["traffic"], "c5", d["end_to_end_c5"]["value"])
PY
