#!/bin/bash
# round-3 final evidence: bench + rocprofv3 kernel-trace summaries, then PMC traffic of both rooflines' kernels
set -o pipefail
bash tools/gpu_bench.sh r74p > gpurun_out/gpu_bench_r74p.txt 2>&1 || { tail -20 gpurun_out/gpu_bench_r74p.txt; exit 1; }
tail -8 gpurun_out/gpu_bench_r74p.txt
bash tools/gpu_pmc.sh r74pic k_picture > gpurun_out/pmc_r74pic.txt 2>&1 || { tail -20 gpurun_out/pmc_r74pic.txt; exit 1; }
tail -6 gpurun_out/pmc_r74pic.txt
bash tools/gpu_pmc.sh r74 k_batch > gpurun_out/pmc_r74.txt 2>&1 || { tail -20 gpurun_out/pmc_r74.txt; exit 1; }
tail -6 gpurun_out/pmc_r74.txt
