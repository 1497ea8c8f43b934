#!/bin/bash
# Round-4 GPU checks on the box, each step under its own time limit, stopping at the first failure:
#   h265    the H.265 GPU parity tests (I and P / B goldens) + the H.265 bench legs
#   tl      host + rocprof timeline of one C3 decode (tools/timeline.sh)
#   streams interleaved end-to-end A/B of the launch stream count (tools/ab_env.py)
#   ext     decode-path GPU tests + A/B of uploads from the parser's pinned records (M2DEC_AMD_EXTERNAL)
#   gpu     the whole GPU test suite
# Usage: bash tools/gpu_round4.sh TAG STEP...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for step in "$@"; do
  case $step in
  h265)
    timeout -k 10 300 python -u -m pytest tests/test_gpu_h265.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h265_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/h265_tests_$TAG.log; exit 1; }
    tail -1 gpurun_out/h265_tests_$TAG.log
    timeout -k 10 300 python -u tools/h265_bench.py 3 > gpurun_out/h265_bench_$TAG.json 2> gpurun_out/h265_bench_$TAG.err || { tail -5 gpurun_out/h265_bench_$TAG.err; exit 1; }
    cat gpurun_out/h265_bench_$TAG.json ;;
  tl)
    bash tools/timeline.sh $TAG 4 || exit 1 ;;
  streams)
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "s3:" "s4q5:M2DEC_AMD_STREAMS=4,GPU_MAX_HW_QUEUES=5" "s4q8:M2DEC_AMD_STREAMS=4,GPU_MAX_HW_QUEUES=8" "s3q8:GPU_MAX_HW_QUEUES=8" > gpurun_out/ab_streams_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_streams_$TAG.txt; exit 1; }
    tail -6 gpurun_out/ab_streams_$TAG.txt ;;
  hold)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py -k "c3_1080p or reflists or mmco5" > gpurun_out/pytest_hold_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_hold_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_hold_$TAG.log
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "hold1:" "hold0:M2DEC_AMD_HOLD=0" "hold1s4:M2DEC_AMD_STREAMS=4,GPU_MAX_HW_QUEUES=5" > gpurun_out/ab_hold_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_hold_$TAG.txt; exit 1; }
    tail -4 gpurun_out/ab_hold_$TAG.txt ;;
  crew)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py -k "c3_1080p or reflists" > gpurun_out/pytest_crew_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_crew_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_crew_$TAG.log
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "crew3:" "crew0:M2DEC_AMD_COPY_CREW=0" "crew3hold0:M2DEC_AMD_HOLD=0" > gpurun_out/ab_crew_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_crew_$TAG.txt; exit 1; }
    tail -4 gpurun_out/ab_crew_$TAG.txt ;;
  md5)
    lscpu | grep -E "Model name|Flags" | cut -c1-200 > gpurun_out/md5_batch_$TAG.txt
    timeout -k 10 120 python3 tools/md5_batch_bench.py >> gpurun_out/md5_batch_$TAG.txt 2>&1 && M2DEC_AMD_MD5_LANES8=0 timeout -k 10 120 python3 tools/md5_batch_bench.py | sed 's/^/lanes16 /' >> gpurun_out/md5_batch_$TAG.txt 2>&1 || exit 1
    cat gpurun_out/md5_batch_$TAG.txt ;;
  tail)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_cli.py -k "c3_1080p or md5 or reflists" > gpurun_out/pytest_tail_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_tail_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_tail_$TAG.log
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "tail1:" "tail0:M2DEC_AMD_MD5_TAIL=0,M2DEC_AMD_MD5_THREADS=3" "tail1t8:M2DEC_AMD_MD5_THREADS=8" > gpurun_out/ab_tail_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_tail_$TAG.txt; exit 1; }
    tail -4 gpurun_out/ab_tail_$TAG.txt ;;
  prio)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py -k "c3_1080p or reflists or mmco5 or poc" > gpurun_out/pytest_prio_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_prio_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_prio_$TAG.log
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "prio1:" "prio0:M2DEC_AMD_PARSE_PRIO=0" > gpurun_out/ab_prio_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_prio_$TAG.txt; exit 1; }
    tail -3 gpurun_out/ab_prio_$TAG.txt ;;
  sync)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_cli.py -k "c3_1080p or md5 or reflists" > gpurun_out/pytest_sync_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_sync_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_sync_$TAG.log
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "crew3:" "crew0:M2DEC_AMD_COPY_CREW=0" > gpurun_out/ab_sync_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_sync_$TAG.txt; exit 1; }
    tail -3 gpurun_out/ab_sync_$TAG.txt ;;
  ext)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_cli.py tests/test_gpu_batch.py tests/test_gpu_boundary.py > gpurun_out/pytest_ext_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_ext_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_ext_$TAG.log
    timeout -k 10 600 python3 tools/ab_env.py 3 10 "ext1:" "ext0:M2DEC_AMD_EXTERNAL=0" > gpurun_out/ab_ext_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_ext_$TAG.txt; exit 1; }
    tail -3 gpurun_out/ab_ext_$TAG.txt ;;
  prio2)
    timeout -k 10 900 python3 tools/ab_env.py 5 16 "prio1:" "prio0:M2DEC_AMD_PARSE_PRIO=0" "prio1s4:M2DEC_AMD_STREAMS=4,GPU_MAX_HW_QUEUES=8" "prio0s4:M2DEC_AMD_PARSE_PRIO=0,M2DEC_AMD_STREAMS=4,GPU_MAX_HW_QUEUES=8" > gpurun_out/ab_prio2_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_prio2_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_prio2_$TAG.txt ;;
  win)
    timeout -k 10 900 python3 tools/ab_env.py 4 16 "w20:GPU_MAX_HW_QUEUES=8" "w12:M2DEC_AMD_PARSE_PRIO=12,GPU_MAX_HW_QUEUES=8" "w32:M2DEC_AMD_PARSE_PRIO=32,GPU_MAX_HW_QUEUES=8" > gpurun_out/ab_win_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_win_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_win_$TAG.txt ;;
  col)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_cli.py tests/test_gpu_batch.py tests/test_gpu_boundary.py > gpurun_out/pytest_col_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_col_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_col_$TAG.log
    timeout -k 10 900 python3 tools/ab_env.py 4 16 "col1:GPU_MAX_HW_QUEUES=8" "col0:M2DEC_AMD_COL_PIPE=0,GPU_MAX_HW_QUEUES=8" "col1w0:M2DEC_AMD_PARSE_PRIO=0,GPU_MAX_HW_QUEUES=8" "col1w8:M2DEC_AMD_PARSE_PRIO=8,GPU_MAX_HW_QUEUES=8" > gpurun_out/ab_col_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_col_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_col_$TAG.txt ;;
  tlq8)
    GPU_MAX_HW_QUEUES=8 bash tools/timeline.sh $TAG 4 || exit 1 ;;
  lane)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_batch.py > gpurun_out/pytest_lane_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_lane_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_lane_$TAG.log
    V=hoist timeout -k 10 600 bash tools/ab_replay.sh lane_$TAG || exit 1
    cat gpurun_out/ab_lane_$TAG.txt
    timeout -k 10 900 python3 tools/ab_env.py 4 12 "lane1:GPU_MAX_HW_QUEUES=8" "hoist:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_LIB=$R/build/var/lib_hoist.so" > gpurun_out/ab_lane_e2e_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_lane_e2e_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_lane_e2e_$TAG.txt ;;
  sab)
    timeout -k 10 900 python3 tools/ab_streams.py 2 3 "def:GPU_MAX_HW_QUEUES=8" "col0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_COL_PIPE=0" "s3:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=3" "tail0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL=0" "prio0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_PARSE_PRIO=0" "ext0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_EXTERNAL=0" "crew0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_COPY_CREW=0" "hold0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_HOLD=0" > gpurun_out/ab_streams8_$TAG.txt 2>&1 || { tail -20 gpurun_out/ab_streams8_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_streams8_$TAG.txt ;;
  dp)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_cli.py tests/test_gpu_boundary.py tests/test_gpu_f1.py > gpurun_out/pytest_dp_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_dp_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_dp_$TAG.log
    timeout -k 10 900 python3 tools/ab_env.py 4 12 "s4:GPU_MAX_HW_QUEUES=8" "s5:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=5" "s6i64:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=6,M2DEC_AMD_INTER_WG=64" "s4i64:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_INTER_WG=64" > gpurun_out/ab_dp_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_dp_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_dp_$TAG.txt ;;
  pb)
    bash tools/pb_ab3.sh > gpurun_out/pb_ab3_$TAG.txt 2>&1 || exit 1
    cat gpurun_out/pb_ab3_$TAG.txt ;;
  s5)
    timeout -k 10 120 tools/_build/ipprof tools/_build/c3.264 3 bm > gpurun_out/ipprof_bm_$TAG.txt 2> gpurun_out/ipprof_bm_$TAG.err || exit 1
    timeout -k 10 900 python3 tools/ab_env.py 5 12 "s5:GPU_MAX_HW_QUEUES=8" "s4:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=4" "s6:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=6" > gpurun_out/ab_s5_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_s5_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_s5_$TAG.txt
    GPU_MAX_HW_QUEUES=8 bash tools/timeline.sh $TAG 4 || exit 1 ;;
  dbk)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_batch.py tests/test_gpu_f1.py > gpurun_out/pytest_dbk_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_dbk_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_dbk_$TAG.log
    V=dbkbyte timeout -k 10 600 bash tools/ab_replay.sh dbk_$TAG || exit 1
    cat gpurun_out/ab_dbk_$TAG.txt
    timeout -k 10 900 python3 tools/ab_env.py 4 12 "dw:GPU_MAX_HW_QUEUES=8" "byte:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_LIB=$R/build/var/lib_dbkbyte.so" > gpurun_out/ab_dbk_e2e_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_dbk_e2e_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_dbk_e2e_$TAG.txt ;;
  iw)
    timeout -k 10 900 python3 tools/ab_env.py 4 12 "i80:GPU_MAX_HW_QUEUES=8" "i160:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_INTER_WG=160" "i120r17:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_INTER_WG=120,M2DEC_AMD_ROW_WG=17" "i80r17:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_ROW_WG=17" > gpurun_out/ab_iw_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_iw_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_iw_$TAG.txt ;;
  c5)
    AB_STREAM=c5_4k_s1 timeout -k 10 900 python3 tools/ab_env.py 4 8 "def:GPU_MAX_HW_QUEUES=8" "p1:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_PICS_PER_LAUNCH=1" "s3:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=3" > gpurun_out/ab_c5_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_c5_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_c5_$TAG.txt ;;
  p1)
    timeout -k 10 900 python3 tools/ab_env.py 4 12 "def:GPU_MAX_HW_QUEUES=8" "s6p1:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_STREAMS=6,M2DEC_AMD_PICS_PER_LAUNCH=1" "s8p1:GPU_MAX_HW_QUEUES=12,M2DEC_AMD_STREAMS=8,M2DEC_AMD_PICS_PER_LAUNCH=1" "s8p1h0:GPU_MAX_HW_QUEUES=12,M2DEC_AMD_STREAMS=8,M2DEC_AMD_PICS_PER_LAUNCH=1,M2DEC_AMD_HOLD=0" > gpurun_out/ab_p1_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_p1_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_p1_$TAG.txt ;;
  early)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_cli.py tests/test_gpu_boundary.py tests/test_gpu_f1.py > gpurun_out/pytest_early_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_early_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_early_$TAG.log
    timeout -k 10 900 python3 tools/ab_env.py 5 12 "e1:GPU_MAX_HW_QUEUES=8" "e0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_EARLY=0" > gpurun_out/ab_early_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_early_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_early_$TAG.txt
    GPU_MAX_HW_QUEUES=8 bash tools/timeline.sh $TAG 4 || exit 1 ;;
  item)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_batch.py > gpurun_out/pytest_item_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_item_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_item_$TAG.log
    V=noitem timeout -k 10 600 bash tools/ab_replay.sh item_$TAG || exit 1
    cat gpurun_out/ab_item_$TAG.txt ;;
  md5t)
    timeout -k 10 900 python3 tools/ab_env.py 4 12 "def:GPU_MAX_HW_QUEUES=8" "mb4:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_MIN_BATCH=4" "mb16:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_MIN_BATCH=16" "tail0:GPU_MAX_HW_QUEUES=8,M2DEC_AMD_MD5_TAIL=0" > gpurun_out/ab_md5t_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_md5t_$TAG.txt; exit 1; }
    grep "^all" gpurun_out/ab_md5t_$TAG.txt ;;
  gpu)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
    tail -2 gpurun_out/pytest_gpu_$TAG.log ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
