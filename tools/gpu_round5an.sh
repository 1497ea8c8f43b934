#!/bin/bash
# Round-5 pass 41: cycle-sampling profile of the single-thread host parse of c3 on the box's host
# (tools/ipprof.c, null back end), current library.
set -o pipefail
mkdir -p gpurun_out
python3 -c "
import sys; sys.path.insert(0, '.')
from tests._streams import stream
open('/tmp/c3_ip.264', 'wb').write(stream('c3_1080p_s1'))
" || exit $?
timeout -k 5 120 build/abtools/ipprof /tmp/c3_ip.264 6 > gpurun_out/ipprof41.txt 2> gpurun_out/ipprof41.err || exit $?
echo ok
