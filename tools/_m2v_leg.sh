set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpeg2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m2v_tests.log 2>&1 || { tail -20 gpurun_out/m2v_tests.log; exit 1; }
tail -1 gpurun_out/m2v_tests.log
timeout -k 10 200 python -c "import json, bench; print(json.dumps(bench.m2v_leg(0, 5, 2)))" > gpurun_out/m2v_leg.json 2>&1 || { tail gpurun_out/m2v_leg.json; exit 1; }
tail -1 gpurun_out/m2v_leg.json
