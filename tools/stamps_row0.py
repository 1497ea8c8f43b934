"""Diagnostic: deblocking filter step per MB on row 0 (no row above to wait for) of one isolated picture."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402
L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"))
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(1); rp.sync()
N = 160 * 4 * 256
buf = (ctypes.c_ulonglong * N)()
L.m2dec_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.m2dec_amd_debug_stamps(buf, N) > 0
a = np.frombuffer(buf, np.uint64).reshape(160, 4, 256)
t = (a >> np.uint64(16)).astype(np.int64)
Hmb, Wmb = tr.height // 16, tr.width // 16
f = t[0, 1, :Wmb + 1]
f = f[f > 0]
print("row 0 filter step median us", np.median(np.diff(f)) / 100.0, "mean", np.mean(np.diff(f)) / 100.0)
ends = [t[y, 3, 4] for y in range(Hmb) if t[y, 3, 4] > 0]
t0 = t[t > 0].min()
print("picture span us", (max(ends) - t0) / 100.0)
