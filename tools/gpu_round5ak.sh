#!/bin/bash
# Round-5 GPU pass 38: time the parse workers spend waiting for co-located rows (col_wait) in c3 decodes.
set -o pipefail
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 M2DEC_AMD_ASYNC_STATS=1 timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import stream, GOLDEN
d = stream('c3_1080p_s1')
for i in range(6):
    st = m2dec_amd.Stats()
    assert m2dec_amd.decode_stream_md5(d, device=0, stats=st) == GOLDEN['c3_1080p_s1']['md5']
    print('decode %.2f ms parse_cpu/pic %.3f ms' % (1e3 * (st.t_end - st.t_start), 1e3 * st.parse_cpu_s / st.pictures), flush=True)
" > gpurun_out/cw38.txt 2>&1 || exit $?
echo ok
