set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_h265.sh r68 > gpurun_out/r68_h265.txt 2>&1 || { tail -40 gpurun_out/r68_h265.txt; exit 1; }
tail -12 gpurun_out/r68_h265.txt
M2DEC_AMD_H265_BLOCKS=1 timeout -k 10 200 python -u tools/h265_bench.py 5 > gpurun_out/h265_bench_r68_blocks.json 2>&1 || exit 1
cat gpurun_out/h265_bench_r68_blocks.json | tail -1
timeout -k 10 120 python tools/_ab_streams.py > gpurun_out/r68_ab.txt 2>&1 || { cat gpurun_out/r68_ab.txt; exit 1; }
cat gpurun_out/r68_ab.txt
