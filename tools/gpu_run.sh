#!/bin/bash
# One GPU call = a list of steps, each under its own time limit, stopping at the first failure (gpurun rules:
# no GPU step after a fault, an abort or a time limit).  Replaces the one-shot tools/gpu_round5*.sh scripts.
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# steps (outputs under gpurun_out/, named with TAG):
#   tests[=KEXPR]    pytest -m gpu (thread timeouts, one process; -k KEXPR) -> pytest_TAG.log
#   smoke            __graft_entry__.smoke()
#   bench[=ARGS]     python bench.py ARGS (default: the driver's line)   -> bench_TAG.json / .err
#   bench20          the driver's own command line (--steps 20 --warmup 5)
#   ab=R,N,CFG;CFG   tools/ab_env.py R N CFG CFG ... (c3 decode medians) -> ab_TAG.txt
#   diff=V,STREAM    tools/replay_diff.py STREAM with build/var/lib_V.so ("base": the product library)
#   prof             rocprofv3 --kernel-trace --stats of the default bench (decode path, replay, all legs)
#   pmc=KERNEL       tools/gpu_pmc.sh TAG KERNEL (FETCH_SIZE / WRITE_SIZE / SQ passes)
#   h265ab=R,VAR,A,B interleaved A/B of VAR=A / VAR=B on the bench's two H.265 legs (R rounds)  -> h265ab_TAG.txt
#   h265tl=N,STREAM  tools/h265_timeline.sh (rocprof kernel trace + parse jobs of N decodes)   -> h5tl_TAG.txt
#   h5stamps[=STREAM] tools/stamps_h265.py with the stamps build (make h5stamps: build/h5s/, delete after use) -> h5stamps_TAG.txt
#   md5host          tools/md5_batch_bench.py with and without the stitched 2-3 frame kernel -> md5host_TAG.txt
#   md5gpu[=N]       tools/_build/md5_gpu_probe N (one MD5 chain per wave / per lane on the GPU) -> md5gpu_TAG.txt
set -o pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
O=gpurun_out
for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $name $arg ($(date +%T))"
  case $name in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${arg:+-k "$arg"} \
        > $O/pytest_$TAG.log 2>&1
      rc=$?; tail -3 $O/pytest_$TAG.log ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()"; rc=$? ;;
    bench)
      timeout -k 10 900 python bench.py $arg > $O/bench_$TAG.json 2> $O/bench_$TAG.err
      rc=$?; tail -c 600 $O/bench_$TAG.json; echo ;;
    bench20)
      timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$TAG.json 2> $O/bench20_$TAG.err
      rc=$?; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('value', d['value'], 'cpu_quota', d.get('cpu_quota'), 'host_cpu', d.get('host_cpu'), 'decode_ms', d.get('decode_ms'))" $O/bench20_$TAG.json ;;
    ab)
      IFS=',' read -r rounds n cfgs <<< "$arg"
      IFS=';' read -ra cl <<< "$cfgs"
      timeout -k 10 900 python -u tools/ab_env.py $rounds $n "${cl[@]}" > $O/ab_$TAG.txt 2>&1
      rc=$?; tail -4 $O/ab_$TAG.txt ;;
    diff)
      IFS=',' read -r v s <<< "$arg"
      lib=$R/m2dec_amd/lib/libm2dec_amd.so; [ "$v" != base ] && lib=$R/build/var/lib_$v.so
      M2DEC_AMD_LIB=$lib timeout -k 10 200 python -u tools/replay_diff.py $s > $O/diff_${TAG}_$v.txt 2>&1
      rc=$?; grep "pictures differ\|best oracle" $O/diff_${TAG}_$v.txt; tail -2 $O/diff_${TAG}_$v.txt ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$TAG -o run --output-format csv -- \
         python3 $R/bench.py --no-cpu-baseline > $R/$O/prof_$TAG.log 2>&1)
      rc=$?; find $O/prof_$TAG -name "*kernel_stats*" ;;
    h265ab)
      IFS=',' read -r rounds var va vb <<< "$arg"
      for ((i = 0; i < rounds; i++)); do
        for v in $va $vb; do
          echo "$var=$v $(env $var=$v timeout -k 10 300 python tools/h265_bench.py 10)" >> $O/h265ab_$TAG.txt || exit 1
        done
      done
      rc=$?; python3 tools/h265_ab_summary.py $O/h265ab_$TAG.txt ;;
    h265tl)
      IFS=',' read -r n st <<< "$arg"
      timeout -k 10 400 bash tools/h265_timeline.sh $TAG ${n:-4} ${st:-c_h265_1080p_s1}; rc=$? ;;
    h5stamps)
      M2DEC_AMD_LIB=$R/build/h5s/libm2dec_amd_h5stamps.so M2DEC_AMD_H265_STREAMS=1 timeout -k 10 200 \
        python -u tools/stamps_h265.py ${arg:-c_h265_1080p_s1} > $O/h5stamps_$TAG.txt 2>&1
      rc=$?; head -30 $O/h5stamps_$TAG.txt ;;
    md5host)
      { for st in 1 0; do echo "M2DEC_AMD_MD5_STITCH=$st"; M2DEC_AMD_MD5_STITCH=$st timeout -k 10 120 python tools/md5_batch_bench.py || exit 1; done; } \
        > $O/md5host_$TAG.txt 2>&1
      rc=$?; cat $O/md5host_$TAG.txt ;;
    md5gpu)
      timeout -k 10 300 tools/_build/md5_gpu_probe ${arg:-64} > $O/md5gpu_$TAG.txt 2>&1
      rc=$?; cat $O/md5gpu_$TAG.txt ;;
    pmc)
      timeout -k 10 900 bash tools/gpu_pmc.sh $TAG $arg; rc=$? ;;
    *)
      echo "unknown step $name"; rc=2 ;;
  esac
  echo "== $name rc=$rc ($(date +%T))"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
