"""Diagnostic: deblocking filter sub-steps (stamps build with -DM2DEC_STAMPD): per MB, the wait for its
inputs, the vertical-edge pass and the horizontal-edge pass, over the rows of one picture run alone.
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stampd.so M2DEC_AMD_REPLAY_LIMIT=N M2DEC_AMD_REPLAY_ISOLATE_LAST=1 \
        python tools/stamps_dbk.py"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"))
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(1); rp.sync()
N = 160 * 3 * 128
buf = (ctypes.c_ulonglong * N)()
L.m2dec_amd_debug_dstamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.m2dec_amd_debug_dstamps(buf, N) > 0
t = np.frombuffer(buf, np.uint64).reshape(160, 3, 128).astype(np.int64)
Hmb, Wmb = tr.height // 16, tr.width // 16
v, h, step, wait = [], [], [], []
for y in range(Hmb):
    for x in range(Wmb):
        e0, e1, e2 = t[y, 0, x], t[y, 1, x], t[y, 2, x]
        if e0 > 0 and e1 > e0 and e2 > e1:
            v.append(e1 - e0); h.append(e2 - e1)
        if x + 1 < Wmb and t[y, 0, x + 1] > 0 and e2 > 0:
            wait.append(t[y, 0, x + 1] - e2)
        if x > 0 and e0 > 0 and t[y, 0, x - 1] > 0:
            step.append(e0 - t[y, 0, x - 1])
for name, a in (("vertical", v), ("horizontal", h), ("wait before next MB", wait), ("MB step", step)):
    a = np.array(a) / 100.0
    print(f"{name:22s} n={len(a):6d} mean {a.mean():6.3f} us  median {np.median(a):6.3f}  p10 {np.percentile(a, 10):6.3f}  p90 {np.percentile(a, 90):6.3f}")
