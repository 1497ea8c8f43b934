#!/bin/bash
# H.265 timeline: parse jobs + kernels of one decode.  Usage: bash tools/h265_timeline.sh TAG [N] [golden name]
set -o pipefail
TAG=${1:-r01}
N=${2:-4}
S=${3:-c_h265_1080p_pb_s1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/h5tl_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/h5tl_$TAG -o run --output-format csv -- \
  python3 $R/tools/h265_timeline_run.py $S $N $R/gpurun_out/h5tl_$TAG/host_tl.csv > $R/gpurun_out/h5tl_$TAG/run.log 2> $R/gpurun_out/h5tl_$TAG/trace.err
rc=$?; echo "rocprof rc=$rc"; cat $R/gpurun_out/h5tl_$TAG/run.log
if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/h5tl_$TAG/trace.err; exit $rc; fi
cd $R && python3 tools/h265_timeline.py gpurun_out/h5tl_$TAG > gpurun_out/h5tl_$TAG.txt; cat gpurun_out/h5tl_$TAG.txt
