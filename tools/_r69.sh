set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_h265.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r69_h265_tests.log 2>&1 || { tail -30 gpurun_out/r69_h265_tests.log; exit 1; }
tail -1 gpurun_out/r69_h265_tests.log
timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_bench_r69.json 2>&1 || exit 1
tail -1 gpurun_out/h265_bench_r69.json
