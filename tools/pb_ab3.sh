#!/bin/bash
# A/B/C of the host parse (tools/parse_bench.c, one core, sequential parse) between library builds:
# A = tools/_build/abA, B = tools/_build/abB, T = the tree's; alternating runs, best of 3 passes each
set -o pipefail
S=${S:-tools/_build/c3.264}
for i in 1 2 3 4 5; do
  for v in A B T; do
    case $v in A) L=tools/_build/abA ;; B) L=tools/_build/abB ;; T) L=m2dec_amd/lib ;; esac
    echo "$v $(LD_LIBRARY_PATH=$L taskset -c 2 timeout -k 5 60 tools/_build/parse_bench $S 3 2>/dev/null | sort -n | head -1)"
  done
done
