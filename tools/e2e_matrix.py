"""Single-stream end-to-end rate of the decode path by stage: parse only (null back end), decode without
MD5, decode with the MD5 threads — at a few parse-worker counts (M2DEC_AMD_PARSE_THREADS is read per
decoder).  Usage: python tools/e2e_matrix.py [workers ...]"""
import ctypes
import os
import resource
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


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def best(fn, reps=4):
    """best rate of `reps` runs, and the process CPU time per frame (ms) over them"""
    c0 = cpu_s()
    rates = [fn() for _ in range(reps)]
    return max(rates), (cpu_s() - c0) / (60 * reps) * 1e3


def throttled():
    try:
        st = dict(line.split() for line in open("/sys/fs/cgroup/cpu.stat"))
        return int(st.get("nr_throttled", 0)), int(st.get("throttled_usec", 0))
    except OSError:
        return 0, 0


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

    out = []
    for name, fn in (("parse only", parse_only), ("decode no MD5", no_md5), ("decode + MD5", with_md5)):
        t0 = throttled()
        fps, cpu = best(fn)
        t1 = throttled()
        out.append(f"{name} {fps:.0f} fps ({cpu:.2f} CPU-ms/frame, throttled {t1[0] - t0[0]}x {(t1[1] - t0[1]) / 1e3:.0f} ms)")
    print(f"workers {th}: " + ", ".join(out), flush=True)
