#!/bin/bash
# Host event timeline + rocprofv3 kernel / copy trace of the same c3 decodes (tools/timeline.py lines them up).
# Usage: bash tools/timeline.sh TAG [N decodes] [golden stream name, default c3_1080p_s1]
#        -> gpurun_out/tl_TAG/ (+ tl_TAG.txt summary)
set -o pipefail
TAG=${1:-r01}
N=${2:-4}
S=${3:-c3_1080p_s1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/tl_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/tl_$TAG -o run --output-format csv -- \
  python3 $R/tools/timeline_run.py $R/gpurun_out/tl_$TAG/host.csv $N $S > $R/gpurun_out/tl_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep decode $R/gpurun_out/tl_$TAG.log
if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/tl_$TAG.log; exit $rc; fi
cd $R && python3 tools/timeline.py gpurun_out/tl_$TAG > gpurun_out/tl_$TAG.txt; tail -60 gpurun_out/tl_$TAG.txt
