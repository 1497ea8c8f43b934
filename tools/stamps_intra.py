"""Diagnostic: per-row phase and per-MB intra timing of ONE picture from in-kernel stamps.
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=1 python tools/stamps_intra.py [stream]"""
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
Hmb, Wmb = tr.height // 16, tr.width // 16
t0 = t[:Hmb][t[:Hmb] > 0].min()
us = lambda v: round((v - t0) / 100.0, 1) if v > 0 else None
print("row: phases(start, A1, A2, intra, deblock) | intra MB0 end, MB-last end, median MB step")
for y in list(range(0, 8)) + list(range(Hmb - 4, Hmb)):
    ph = [us(t[y, 3, i]) for i in range(5)]
    mb = t[y, 3, 16:16 + Wmb]
    ok = mb[mb > 0]
    step = np.median(np.diff(ok)) / 100.0 if len(ok) > 2 else None
    print(y, ph, "|", us(ok[0]) if len(ok) else None, us(ok[-1]) if len(ok) else None, step)
print("intra sub-phases (us) for MBs 1..15 of rows 0 and 1: gather, chroma pred, luma, chroma res, store, signal")
for y in (0, 1):
    for x in range(1, 16):
        ev = t[y, 3, 160 + x * 6:160 + x * 6 + 6]
        prev = t[y, 3, 16 + x - 1]
        if (ev > 0).all() and prev > 0:
            d = np.diff(np.concatenate([[prev], ev])) / 100.0
            print(y, x, [round(float(v), 2) for v in d])
