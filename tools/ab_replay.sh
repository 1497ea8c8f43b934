#!/bin/bash
# A/B of kernel variants on the replay legs: bench.py --replay-only (single stream) and --replay-streams 8,
# alternating the default library and build/var/lib_$V.so.  Usage: V=pf bash tools/ab_replay.sh TAG
set -o pipefail
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
out=gpurun_out/ab_$TAG.txt
: > $out
for rep in 1 2; do
  for v in base $V; do
    lib=$R/m2dec_amd/lib/libm2dec_amd.so; [ $v != base ] && lib=$R/build/var/lib_$v.so
    for ns in 1 8; do
      M2DEC_AMD_LIB=$lib timeout -k 10 150 python bench.py --replay-only --replay-streams $ns --no-cpu-baseline --steps 5 --warmup 1 \
        > gpurun_out/ab_${v}_$ns.json || exit $?
      echo "$v streams $ns: $(python3 -c "import json;print(json.load(open('gpurun_out/ab_${v}_$ns.json'))['value'])")" | tee -a $out
    done
  done
done
