#!/bin/bash
# deblocking wave priority sweep (s_setprio of filter / loader+storer waves); variants from
# make variant V=pXY FLAGS="-DM2DEC_DBK_PRIO_FILTER=X -DM2DEC_DBK_PRIO_OTHER=Y"
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for v in ${VARIANTS:-base p33 p31 p00 base}; do
  lib=$R/m2dec_amd/lib/libm2dec_amd.so; [ $v != base ] && lib=$R/build/var/lib_$v.so
  M2DEC_AMD_LIB=$lib timeout -k 5 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/pr_$v.json 2> gpurun_out/pr_$v.err || { echo "$v failed"; tail -n 5 gpurun_out/pr_$v.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/pr_$v.json'));print(d['value'], d['data'])")"
done
