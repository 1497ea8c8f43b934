set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dbk_pytest.log 2>&1 || { tail -30 gpurun_out/dbk_pytest.log; exit 1; }
tail -1 gpurun_out/dbk_pytest.log
for v in base_stampd libm2dec_amd_stampd; do
  M2DEC_AMD_LIB=build/dbg/$v.so M2DEC_AMD_REPLAY_LIMIT=2 M2DEC_AMD_REPLAY_ISOLATE_LAST=1 timeout -k 10 120 python tools/stamps_dbk.py > gpurun_out/dbk_$v.txt 2>&1 || { tail gpurun_out/dbk_$v.txt; exit 1; }
  echo "== $v"; tail -8 gpurun_out/dbk_$v.txt
done
timeout -k 10 120 python bench.py --replay-only --no-cpu-baseline --steps 5 > gpurun_out/dbk_replay.json 2>&1 || exit 1
tail -1 gpurun_out/dbk_replay.json | cut -c1-200
