#!/bin/bash
# A/B of the host parse (tools/parse_bench.c) between two builds of the library: B = the tree's, A =
# tools/_build/abA; alternating runs, one core each
set -o pipefail
S=${S:-tools/_build/c3.264}
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=tools/_build/abA; else L=m2dec_amd/lib; fi
    echo "$v $(LD_LIBRARY_PATH=$L taskset -c 2 timeout -k 5 60 tools/_build/parse_bench $S 2 | tail -1)"
  done
done
