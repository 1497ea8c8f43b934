#!/bin/bash
# Round-5 parse A/B: single-thread host parse (null back end, tools/parse_bench.c) of the c3 stream, the library
# in build/abA (before the change under test) against the current one, interleaved.
set -o pipefail
mkdir -p gpurun_out
python3 -c "
import sys; sys.path.insert(0, '.')
from tests._streams import stream
open('/tmp/c3_ab.264', 'wb').write(stream('c3_1080p_s1'))
" || exit $?
for r in 1 2 3 4; do
  echo "A $(LD_LIBRARY_PATH=build/abA timeout -k 5 60 build/abtools/parse_bench /tmp/c3_ab.264 4 | awk '{printf "%s ", $1}')" >> gpurun_out/parse_ab.txt || exit $?
  echo "B $(LD_LIBRARY_PATH=m2dec_amd/lib timeout -k 5 60 build/abtools/parse_bench /tmp/c3_ab.264 4 | awk '{printf "%s ", $1}')" >> gpurun_out/parse_ab.txt || exit $?
done
LD_LIBRARY_PATH=m2dec_amd/lib timeout -k 5 60 build/abtools/parse_bench /tmp/c3_ab.264 2 >> gpurun_out/parse_ab.txt 2>&1 || exit $?
echo ok
