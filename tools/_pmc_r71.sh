set -o pipefail
bash tools/gpu_pmc.sh r71pic k_picture > gpurun_out/pmc_r71pic.txt 2>&1 || { tail -20 gpurun_out/pmc_r71pic.txt; exit 1; }
tail -30 gpurun_out/pmc_r71pic.txt
bash tools/gpu_pmc.sh r71 k_batch > gpurun_out/pmc_r71.txt 2>&1 || { tail -20 gpurun_out/pmc_r71.txt; exit 1; }
tail -30 gpurun_out/pmc_r71.txt
