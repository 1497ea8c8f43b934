#!/bin/bash
# parse cost of the host bS derivation: tools/_build/abA built with bS skipped under M2DEC_NO_BS
set -o pipefail
S=tools/_build/c3.264
for i in 1 2 3; do
  echo "bS   $(LD_LIBRARY_PATH=tools/_build/abA taskset -c 2 timeout -k 5 60 tools/_build/parse_bench $S 2 | tail -1)"
  echo "noBS $(M2DEC_NO_BS=1 LD_LIBRARY_PATH=tools/_build/abA taskset -c 2 timeout -k 5 60 tools/_build/parse_bench $S 2 | tail -1)"
done
