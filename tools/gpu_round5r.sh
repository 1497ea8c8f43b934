#!/bin/bash
# Round-5 GPU pass 19: is the first timed c3 decode an outlier (warmup 2 vs 4, 8 steps)?
set -o pipefail
mkdir -p gpurun_out
for w in 2 4 2; do
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 8 --warmup $w > gpurun_out/b19_w$w.json 2> gpurun_out/b19.err || exit $?
python3 -c "import json;b=json.load(open('gpurun_out/b19_w$w.json'));print('warmup $w', b['value'], b['decode_ms'])" | tee -a gpurun_out/b19.txt
done
echo ok
