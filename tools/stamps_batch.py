"""Diagnostic: per-picture timeline inside one k_batch launch (in-kernel stamps).
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so python tools/stamps_batch.py [stream]"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"))
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(2); rp.sync()
buf = (ctypes.c_ulonglong * 1024)()
L.m2dec_amd_debug_pstamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.m2dec_amd_debug_pstamps(buf, 1024) > 0
a = np.frombuffer(buf, np.uint64).reshape(256, 4).astype(np.int64)[:tr.npics]
t0 = a[:, 0].min()
rel = (a - t0) / 100.0
print("pic  type  start  inter_done  rows_done  span")
for i in range(tr.npics):
    p = tr.pics[i]
    kind = "I" if p.n_inter == 0 else "P/B"
    print(f"{i:3d} {kind:4s} {rel[i, 0]:8.1f} {rel[i, 1]:10.1f} {rel[i, 2]:10.1f} {rel[i, 2] - rel[i, 0]:8.1f}")
end = rel[:, 2].max()
print("launch span us", end, "per picture", end / tr.npics)
# pictures in flight over time
ts = np.linspace(0, end, 200)
inflight = [int(((rel[:, 0] <= x) & (rel[:, 2] > x)).sum()) for x in ts]
print("in flight: mean", np.mean(inflight), "max", max(inflight))
