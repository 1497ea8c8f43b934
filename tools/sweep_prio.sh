#!/bin/bash
# Deblocking wave priority sweep (s_setprio of the filter / loader / storer waves of deblock_pair).
# Build the variants first (on the CPU host), e.g.:
#   make variant V=p33 FLAGS="-DM2DEC_DBK_PRIO_FILTER=3 -DM2DEC_DBK_PRIO_OTHER=3"
#   make variant V=p31 FLAGS="-DM2DEC_DBK_PRIO_FILTER=3 -DM2DEC_DBK_PRIO_OTHER=1"
#   make variant V=p00 FLAGS="-DM2DEC_DBK_PRIO_FILTER=0 -DM2DEC_DBK_PRIO_OTHER=0"
#   make variant V=l3s2 FLAGS="-DM2DEC_DBK_PRIO_FILTER=3 -DM2DEC_DBK_PRIO_OTHER=3 -DM2DEC_DBK_PRIO_STORER=2"
#   make variant V=l2s3 FLAGS="-DM2DEC_DBK_PRIO_FILTER=3 -DM2DEC_DBK_PRIO_OTHER=2 -DM2DEC_DBK_PRIO_STORER=3"
#   make variant V=l3s1 FLAGS="-DM2DEC_DBK_PRIO_FILTER=3 -DM2DEC_DBK_PRIO_OTHER=3 -DM2DEC_DBK_PRIO_STORER=1"
# "base" is the default build (filter 3, loader + storer 2).  Every run writes its own result file
# (gpurun_out/pr_<index>_<variant>.json), so a variant listed twice measures the run-to-run noise.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd $R
i=0
for v in ${VARIANTS:-base p33 p31 p00 base}; do
  i=$((i + 1))
  lib=$R/m2dec_amd/lib/libm2dec_amd.so; [ $v != base ] && lib=$R/build/var/lib_$v.so
  out=gpurun_out/pr_${i}_$v
  M2DEC_AMD_LIB=$lib timeout -k 5 120 python bench.py --steps 10 --warmup 2 --replay-only > $out.json 2> $out.err || { echo "$v failed"; tail -n 5 $out.err; exit 1; }
  echo "$i $v $(python3 -c "import json;d=json.load(open('$out.json'));print(d['gpu_recon']['value'], d['data'])")"
done
