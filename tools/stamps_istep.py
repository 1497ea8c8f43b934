"""The I-picture intra MB step from in-kernel stamps: replays the first picture of a stream
(an I picture) and prints, per MB row, the median time between consecutive intra MBs' ends, for the first row
of each slice (no upper hand-off) and for the rows below (upper hand-off words polled).
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=1 python tools/stamps_istep.py [stream]"""
import ctypes
import os
import sys

import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"
L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(name))
p0 = tr.pics[0]
Wmb, Hmb = p0.width_mbs, p0.height_mbs
recs = tr.records()
mbs = np.frombuffer(recs, np.uint8, count=32 * Wmb * Hmb, offset=p0.off_mb).reshape(Hmb, Wmb, 32)
row_slice = mbs[:, 0, 10].astype(np.int64) | (mbs[:, 0, 11].astype(np.int64) << 8)
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(1)
rp.sync()
L.m2dec_amd_debug_stamps_clear()
rp.run(1)
rp.sync()
N = 160 * 4 * 256
buf = (ctypes.c_ulonglong * N)()
L.m2dec_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.m2dec_amd_debug_stamps(buf, N) > 0
a = np.frombuffer(buf, np.uint64).reshape(160, 4, 256)
t = (a >> np.uint64(16)).astype(np.int64)
end = t[:Hmb, 3, 16:16 + Wmb]
top, below = [], []
for y in range(Hmb):
    e = end[y][end[y] > 0]
    if len(e) < 8:
        continue
    step = float(np.median(np.diff(e))) / 100.0  # s_memrealtime: 100 MHz
    (top if y == 0 or row_slice[y] != row_slice[y - 1] else below).append(step)
t0 = end[end > 0].min()
print(f"{name}: picture 0, {Wmb}x{Hmb} MBs; intra end {(end.max() - t0) / 100.0:.1f} us")
print(f"median intra MB step: slice top rows {np.median(top):.2f} us ({len(top)} rows), rows below {np.median(below):.2f} us "
      f"({len(below)} rows)")
