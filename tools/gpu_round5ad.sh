#!/bin/bash
# Round-5 GPU pass 31: main leg with the quota settle before the timed steps (3 runs of 5 steps).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/b31_$i.json 2> gpurun_out/b31.err || exit $?
python3 -c "import json;b=json.load(open('gpurun_out/b31_$i.json'));print(b['value'], b['decode_ms'], b.get('cpu_quota'))" | tee -a gpurun_out/b31.txt
done
echo ok
