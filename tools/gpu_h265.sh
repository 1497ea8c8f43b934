#!/bin/bash
# H.265 on the GPU box: the GPU parity tests, the bench's H.265 leg, and a rocprofv3 kernel-trace summary
# of the same leg.  Usage: bash tools/gpu_h265.sh TAG
set -o pipefail
TAG=${1:-h265}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_h265.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h265_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/h265_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/h265_tests_$TAG.log
timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_bench_$TAG.json 2> gpurun_out/h265_bench_$TAG.err || exit $?
cat gpurun_out/h265_bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_h265_$TAG -o run --output-format csv -- python3 $R/tools/h265_bench.py 3 > $R/gpurun_out/prof_h265_$TAG.log 2>&1 || exit $?
find $R/gpurun_out/prof_h265_$TAG -name "*kernel_stats.csv" -exec cat {} \;
