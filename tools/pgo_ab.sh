#!/bin/bash
# A/B of the host parse (null back end, one thread) between two builds of the library:
# tools/_build/pgoA (plain -O3) and tools/_build/pgoB (profile-guided), alternating, c3 seed 1.
set -e -o pipefail
tools/_build/h264gen --preset c3 --seed 1 --frames 60 -o /tmp/pgo_ab_c3.264 2>/dev/null
for i in 1 2 3 4 5; do
  for v in ${PGO_VARIANTS:-A B}; do
    echo -n "$v "; LD_LIBRARY_PATH=tools/_build/pgo$v timeout -k 5 60 tools/_build/parse_bench /tmp/pgo_ab_c3.264 3 | awk '{print $1}' | tr '\n' ' '; echo
  done
done
