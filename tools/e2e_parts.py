"""Where the single-stream end-to-end time goes: host parse alone (null back end) vs parse-ahead
workers, the decode path without MD5, and with the MD5 threads (tools for DESIGN.md §6)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from m2dec_amd import Backend  # noqa: E402
from tests._streams import stream  # noqa: E402

L = m2dec_amd.lib()
L.m2dec_amd_null_backend_create.argtypes = [ctypes.POINTER(Backend)]
data = stream("c3_1080p_s1")
for th in (0, 4, 8, 12):
    be = Backend()
    L.m2dec_amd_null_backend_create(ctypes.byref(be))
    t0 = time.perf_counter()
    m2dec_amd.decode_stream(data, backend=be, md5=False, parse_threads=th)
    dt = time.perf_counter() - t0
    ctypes.CFUNCTYPE(None, ctypes.c_void_p)(be.destroy)(be.self)
    print("host parse only (null back end), workers", th, round(60 / dt, 1), "fps", flush=True)
for th in (0, 8):
    m2dec_amd.decode_stream(data, md5=False, parse_threads=th)
    cnt = [0]
    t0 = time.perf_counter()
    m2dec_amd.decode_stream(data, md5=False, on_frame=lambda f: cnt.__setitem__(0, cnt[0] + 1), parse_threads=th)
    print("decode path, no MD5, workers", th, round(cnt[0] / (time.perf_counter() - t0), 1), "fps", flush=True)
t0 = time.perf_counter()
n = len(m2dec_amd.decode_stream_md5(data))
print("decode path + MD5 threads (default workers)", round(n / (time.perf_counter() - t0), 1), "fps")
