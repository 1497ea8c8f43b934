#!/bin/bash
# Round-5 final pass A: the whole GPU suite, smoke(), the bench line, rocprofv3 kernel stats of the decode and
# replay legs.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/tfinal.log 2>&1 || exit $?
tail -2 gpurun_out/tfinal.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
cat gpurun_out/smoke_final.log
TAG=${TAG:-r126}
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_replay -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --replay-only > $R/gpurun_out/prof_${TAG}_replay.log 2>&1 || exit $?
echo ok
