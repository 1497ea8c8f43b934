#!/bin/bash
# HBM traffic of the bench's k_batch launches from rocprofv3 PMC counters, one counter group per pass
# (MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2, so
# they cannot share a pass).  Usage: bash tools/gpu_pmc.sh TAG [KERNEL]  -> gpurun_out/pmc_TAG.json
# KERNEL k_batch (default): the replay leg; k_batch8: the 8-stream replay; k_picture: the decode path of the end-to-end leg (one
# launch per picture; counter collection serialises the launches, the bytes are per launch).
set -o pipefail
TAG=${1:-r01}
K=${2:-k_batch}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
if [ "$K" = k_batch ]; then
  CMD="python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --replay-only"
elif [ "$K" = k_batch8 ]; then  # the 8-stream replay (bench gpu_recon_streams)
  CMD="python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --replay-only --replay-streams 8"
elif [ "$K" = h265 ]; then  # the bench's H.265 intra leg: every k_h265_* kernel of its pictures
  CMD="python3 $R/tools/h265_bench.py 2 c_h265_1080p_s1"
elif [ "$K" = h265_pb ]; then  # the H.265 P / B leg
  CMD="python3 $R/tools/h265_bench.py 2 c_h265_1080p_pb_s1"
else
  CMD="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras"
fi
# the 4th group is the wave-state split of MI355X_MICROARCH.md §PMC (quad-cycles, disjoint:
# WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES) plus VALU issue and the clock
CGROUPS=(FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
# H.265: traffic, plus the CTU kernel's wave states (LDS issue / waits split out) and instruction mix
case "$K" in h265*) CGROUPS=(FETCH_SIZE WRITE_SIZE \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH SQ_BUSY_CYCLES") ;; esac
for C in "${CGROUPS[@]}"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_$TAG/$N -o run --output-format csv -- $CMD \
    > $R/gpurun_out/pmc_${TAG}_$N.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmc_${TAG}_$N.log; exit $rc; fi
done
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG $K > gpurun_out/pmc_$TAG.json && cat gpurun_out/pmc_$TAG.json
