set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
for v in base sg8 sg8r32; do
  lib=$R/m2dec_amd/lib/libm2dec_amd.so; [ $v != base ] && lib=$R/build/var/lib_$v.so
  M2DEC_AMD_LIB=$lib timeout -k 5 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/sg_$v.json 2> gpurun_out/sg_$v.err || { echo "$v failed"; tail -n 5 gpurun_out/sg_$v.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/sg_$v.json'));print(d['value'])")"
  (cd /tmp && M2DEC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/sgpmc_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/sgpmc_$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
  python3 - $R/gpurun_out/sgpmc_$v <<'PY'
import sys; sys.path.insert(0, 'tools'); import pmc_traffic as p, statistics
w = p.per_dispatch(sys.argv[1]); print("  write MB", round(statistics.median(x["WRITE_SIZE"] for x in w) * 1024 / 1e6, 1))
PY
done
