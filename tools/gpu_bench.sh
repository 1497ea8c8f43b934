#!/bin/bash
# GPU bench (default command line) + rocprofv3 kernel-trace summary of the same command.
# Usage: bash tools/gpu_bench.sh TAG
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $R/gpurun_out/prof_$TAG.log
find $R/gpurun_out/prof_$TAG -name "*stats*"
exit $rc
