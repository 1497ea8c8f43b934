#!/bin/bash
# The end-to-end C3 leg with the shared budget (reaper polling) and with a process-local budget, interleaved;
# the first run with M2DEC_AMD_DEBUG for the pictures-per-launch decision.
set -o pipefail
M2DEC_AMD_DEBUG=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/abs_dbg.json 2> gpurun_out/abs_dbg.err || exit $?
for r in 1 2; do
  for v in "M2DEC_AMD_SHARE=1" "M2DEC_AMD_SHARE=0"; do
    out=$(env $v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras) || exit $?
    echo "$r [$v] $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["stages_ms_per_frame"]["parse_cpu"], d["roofline"]["pictures_per_launch"])')"
  done
done
