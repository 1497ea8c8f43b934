"""A/B of decode-path variants on the c3 stream: interval per decode (best / median of N)."""
import os, sys, time, statistics
sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import stream, GOLDEN
d = stream('c3_1080p_s1')
ok = True
iv = []
for i in range(12):
    st = m2dec_amd.Stats()
    md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
    ok &= md5 == GOLDEN['c3_1080p_s1']['md5']
    if i >= 2:
        iv.append(1e3 * (st.t_end - st.t_start))
print(os.environ.get('M2DEC_AMD_LIB', 'default'), os.environ.get('GPU_MAX_HW_QUEUES', '-'), 'bit-exact', ok,
      'interval ms: best %.1f median %.1f -> %.0f fps' % (min(iv), statistics.median(iv), 60e3 / statistics.median(iv)), flush=True)
