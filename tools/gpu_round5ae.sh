#!/bin/bash
# Round-5 GPU pass 32: timeline of the slowest and of the fastest of 8 c3 decodes.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
bash tools/timeline.sh c3var 8 c3_1080p_s1 > gpurun_out/tl_c3var.out 2>&1 || exit $?
cd $R && TL_DECODE=slowest python3 tools/timeline.py gpurun_out/tl_c3var > gpurun_out/tl_c3var_slow.txt && python3 tools/timeline.py gpurun_out/tl_c3var > gpurun_out/tl_c3var_last.txt
echo ok
