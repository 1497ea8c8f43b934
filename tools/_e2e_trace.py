"""Decode c3 a few times (the last one is the traced one for kernel-timeline analysis)."""
import sys, time
sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import stream, GOLDEN
d = stream('c3_1080p_s1')
for i in range(4):
    st = m2dec_amd.Stats()
    t0 = time.time_ns()
    md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
    t1 = time.time_ns()
    print('decode', i, md5 == GOLDEN['c3_1080p_s1']['md5'], 'interval %.1f ms' % (1e3 * (st.t_end - st.t_start)), 'wall_ns', t0, t1, flush=True)
