"""Sweep of parse-ahead workers for the single-stream decode path (h264d_func + MD5 thread)."""
import os, sys, time, json, subprocess
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402
data = stream("c3_1080p_s1")
res = {}
for th in [int(x) for x in sys.argv[1:]] or [0, 2, 4, 8, 12]:
    os.environ["M2DEC_AMD_PARSE_THREADS"] = str(th)
    m2dec_amd.decode_stream_md5(data)  # warm
    t0 = time.perf_counter()
    got = m2dec_amd.decode_stream_md5(data)
    dt = time.perf_counter() - t0
    res[th] = (round(len(got) / dt, 1), got == GOLDEN["c3_1080p_s1"]["md5"])
    print(th, res[th], flush=True)
