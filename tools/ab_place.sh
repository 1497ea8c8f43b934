#!/bin/bash
# A/B of the library threads' placement on the end-to-end C3 leg: NUMA off, NUMA node, NUMA node one thread
# per core; interleaved, 3 rounds, bench.py --no-extras (value, parse_cpu).
set -o pipefail
for r in 1 2 3; do
  for v in "M2DEC_AMD_NUMA=0" "M2DEC_AMD_NUMA=1" "M2DEC_AMD_NUMA=1 M2DEC_AMD_NUMA_SMT=1"; do
    out=$(env $v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras) || exit $?
    echo "$r [$v] $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["stages_ms_per_frame"]["parse_cpu"])')"
  done
done
