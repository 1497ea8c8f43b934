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
# two profiles, one per roofline of the bench line, so each kernel's average is over exactly the launches
# its roofline is quoted on: the value leg (k_picture, one launch per 1080p picture) and the
# single-stream replay leg (k_batch, one launch per 60-picture pass)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $R/gpurun_out/prof_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_replay -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --replay-only > $R/gpurun_out/prof_${TAG}_replay.log 2>&1
rc=$?; echo "rocprof replay rc=$rc"; tail -2 $R/gpurun_out/prof_${TAG}_replay.log
if [ $rc -ne 0 ]; then exit $rc; fi
# every leg of the default bench (decode path, replay, H.265 I and P / B, MPEG-2): one summary naming
# k_picture, k_batch, k_h265_mc / k_h265_ctu_rows / k_h265_deblock / k_h265_sao and k_m2v
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_all -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_all.log 2>&1
rc=$?; echo "rocprof all rc=$rc"; tail -2 $R/gpurun_out/prof_${TAG}_all.log
find $R/gpurun_out/prof_$TAG $R/gpurun_out/prof_${TAG}_replay $R/gpurun_out/prof_${TAG}_all -name "*kernel_stats*"
exit $rc
