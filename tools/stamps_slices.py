"""Per-slice intra wavefronts of one multi-slice I picture, from in-kernel stamps.
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=1 python tools/stamps_slices.py [stream]
Replays the first picture of the stream (C5: a 3840x2160 I picture of 8 row-aligned slices) and prints, per MB
row, when its first and last intra MB finished (us from the picture's first stamp) and the slice the row
starts in.  With slice-aware waits every slice's first row starts at once (8 chains of Wmb + 2 rows steps);
without, row y's first MB ends ~2 MB steps after row y - 1's (one chain of Wmb + 2 Hmb steps)."""
import ctypes
import os
import sys

import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c5_4k_s1"
L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(name))
p0 = tr.pics[0]
Wmb, Hmb = p0.width_mbs, p0.height_mbs
# slice of each MB row's first MB from the first picture's MB records (m2r_mb_t.slice, byte offset 10)
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
mb_end = t[:Hmb, 3, 16:16 + Wmb]
t0 = mb_end[mb_end > 0].min()
us = lambda v: (v - t0) / 100.0  # noqa: E731  (s_memrealtime: 100 MHz)
print(f"{name}: {Wmb}x{Hmb} MBs, picture 0 ({p0.n_intra} intra MBs, {len(set(row_slice.tolist()))} slices)")
print("row  slice  first_mb_end_us  last_mb_end_us")
tops = {}
for y in range(Hmb):
    ok = mb_end[y][mb_end[y] > 0]
    if not len(ok):
        continue
    sl = int(row_slice[y])
    top = y == 0 or row_slice[y - 1] != sl
    if top:
        tops[sl] = us(ok[0])
    print(f"{y:3d}  {sl:5d}{'*' if top else ' '} {us(ok[0]):15.1f}  {us(ok[-1]):14.1f}")
print("first MB of each slice's top row done at (us):", {k: round(v, 1) for k, v in sorted(tops.items())})
print("picture intra end: %.1f us" % us(mb_end.max()))
