#!/bin/bash
# HBM traffic of the bench's k_batch launches from rocprofv3 PMC counters, one counter group per pass
# (MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2, so
# they cannot share a pass).  Usage: bash tools/gpu_pmc.sh TAG   -> gpurun_out/pmc_TAG.json
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-end-to-end"
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_$TAG/$N -o run --output-format csv -- $CMD \
    > $R/gpurun_out/pmc_${TAG}_$N.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmc_${TAG}_$N.log; exit $rc; fi
done
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.json && cat gpurun_out/pmc_$TAG.json
