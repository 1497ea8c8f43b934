"""Diagnostic: per-iteration phases of the pipelined intra luma wave (rows 0, 1, 2) of ONE picture.
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=1 python tools/stamps_luma.py"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"))
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(1); rp.sync()
L.m2dec_amd_debug_stamps_clear()
rp.run(1); rp.sync()
N = 160 * 4 * 256
buf = (ctypes.c_ulonglong * N)()
L.m2dec_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.m2dec_amd_debug_stamps(buf, N) > 0
a = np.frombuffer(buf, np.uint64).reshape(160, 4, 256)
t = (a >> np.uint64(16)).astype(np.int64)
v = (a & np.uint64(0xffff)).astype(np.int64)
print("iteration: xt, prep, chain, write-back+signal, gap-to-next (us)")
for y in (0, 1, 2, 9):
    print("row", y)
    for it in range(31):
        e = t[y, 1, 128 + it * 4:128 + it * 4 + 4]
        n = t[y, 1, 128 + (it + 1) * 4]
        if (e > 0).all():
            d = [round(float(x), 2) for x in np.diff(e) / 100.0]
            print(it, int(v[y, 1, 128 + it * 4]), d, round((n - e[3]) / 100.0, 2) if n > 0 else None)
