"""Single-stream end-to-end rate of the decode path by stage: parse only (null back end), decode without
MD5, decode with the MD5 threads — at a few parse-worker counts (M2DEC_AMD_PARSE_THREADS is read per
decoder).  Usage: python tools/e2e_matrix.py [workers ...]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from m2dec_amd import Backend  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402

L = m2dec_amd.lib()
L.m2dec_amd_null_backend_create.argtypes = [ctypes.POINTER(Backend)]
data = stream("c3_1080p_s1")
gold = GOLDEN["c3_1080p_s1"]["md5"]
m2dec_amd.decode_stream_md5(data)


def best(fn, reps=4):
    return max(fn() for _ in range(reps))


for th in [int(x) for x in sys.argv[1:]] or [8, 12]:
    os.environ["M2DEC_AMD_PARSE_THREADS"] = str(th)

    def parse_only():
        be = Backend()
        L.m2dec_amd_null_backend_create(ctypes.byref(be))
        t0 = time.perf_counter()
        m2dec_amd.decode_stream(data, backend=be, md5=False, parse_threads=th)
        dt = time.perf_counter() - t0
        ctypes.CFUNCTYPE(None, ctypes.c_void_p)(be.destroy)(be.self)
        return 60 / dt

    def no_md5():
        n = [0]
        st = m2dec_amd.Stats()
        m2dec_amd.decode_stream(data, md5=False, on_frame=lambda f: n.__setitem__(0, n[0] + 1), stats=st)
        return n[0] / (st.t_end - st.t_start)

    def with_md5():
        st = m2dec_amd.Stats()
        got = m2dec_amd.decode_stream_md5(data, stats=st)
        assert got == gold
        return len(got) / (st.t_end - st.t_start)

    print(f"workers {th}: parse only {best(parse_only):.0f} fps, decode no MD5 {best(no_md5):.0f} fps, "
          f"decode + MD5 {best(with_md5):.0f} fps", flush=True)
