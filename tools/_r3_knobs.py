"""single-stream C3 end-to-end fps under env knob settings (each: 2 warmup + 5 timed decodes)"""
import os, sys, json
sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import stream, GOLDEN
d = stream('c3_1080p_s1')
gold = GOLDEN['c3_1080p_s1']['md5']
for spec in sys.argv[1:]:
    for kv in spec.split(','):
        k, v = kv.split('=')
        os.environ[k] = v
    fps = []
    for i in range(7):
        st = m2dec_amd.Stats()
        md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
        assert md5 == gold
        if i >= 2:
            fps.append(60 / (st.t_end - st.t_start))
    print(spec, ' '.join('%.0f' % f for f in fps), 'median %.0f' % sorted(fps)[2], flush=True)
