# One c3 stream through the decode path with M2DEC_AMD_ASYNC_STATS: where the caller's thread spends
# its time (lookahead, record copies, submit, drain / sync, MD5-ring copies).  Extra env passes through.
cd $GRAFT_REPO_ROOT
export M2DEC_AMD_ASYNC_STATS=1
timeout -k 10 200 python -u - <<'PY' 2>&1 | tee gpurun_out/e2e_one.txt
import os, sys, time, ctypes
sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import GOLDEN, stream
data = stream("c3_1080p_s1")
m2dec_amd.decode_stream_md5(data)
for dpb in (-1, 16):
    st = m2dec_amd.Stats()
    got = m2dec_amd.decode_stream_md5(data, dpb=dpb, stats=st)
    print("md5 path dpb", dpb, round(len(got) / (st.t_end - st.t_start), 1), "fps", got == GOLDEN["c3_1080p_s1"]["md5"], flush=True)
n = [0]
st = m2dec_amd.Stats()
m2dec_amd.decode_stream(data, md5=False, on_frame=lambda f: n.__setitem__(0, n[0] + 1), stats=st)
print("no-md5 decode path", round(n[0] / (st.t_end - st.t_start), 1), "fps, ahead", st.ahead, flush=True)
PY
