"""One c3 decode under M2DEC_AMD_TIMELINE (host events) — run it under rocprofv3 --kernel-trace
--memory-copy-trace and line both up with tools/timeline.py.  Usage: python3 tools/timeline_run.py OUT.csv [N]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["M2DEC_AMD_TIMELINE"] = os.path.abspath(sys.argv[1])
import m2dec_amd  # noqa: E402
from tests._streams import stream, GOLDEN  # noqa: E402

name = sys.argv[3] if len(sys.argv) > 3 else "c3_1080p_s1"
d = stream(name)
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
    st = m2dec_amd.Stats()
    md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
    print("decode", i, "ok", md5 == GOLDEN[name]["md5"], "interval %.2f ms" % (1e3 * (st.t_end - st.t_start)), flush=True)
