"""Diagnostic: timeline of ONE picture (the last of the first N, run alone after the others):
row phases and inter-worker activity from in-kernel stamps.
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so M2DEC_AMD_REPLAY_LIMIT=N M2DEC_AMD_REPLAY_ISOLATE_LAST=1 \
        python tools/stamps_pic.py [stream]"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"))
lim = int(os.environ.get("M2DEC_AMD_REPLAY_LIMIT", "1"))
p = tr.pics[lim - 1]
print(f"picture {lim - 1}: n_inter {p.n_inter} n_intra {p.n_intra} slot {p.slot}")
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(1); rp.sync()
N = 160 * 4 * 256
buf = (ctypes.c_ulonglong * N)()
L.m2dec_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.m2dec_amd_debug_stamps(buf, N) > 0
a = np.frombuffer(buf, np.uint64).reshape(160, 4, 256)
t = (a >> np.uint64(16)).astype(np.int64)
v = (a & np.uint64(0xffff)).astype(np.int64)
Hmb, Wmb = tr.height // 16, tr.width // 16
t0 = t[t > 0].min()
us = lambda x: round((x - t0) / 100.0, 1) if x > 0 else None
print("row: start, A1 inter-done, A2, intra-done, deblock-done")
for y in list(range(0, 12, 2)) + list(range(Hmb // 2 - 2, Hmb // 2 + 4, 2)) + list(range(Hmb - 6, Hmb, 2)):
    print(y, [us(t[y, 3, i]) for i in range(5)])
ends = [t[y, 3, 4] for y in range(Hmb) if t[y, 3, 4] > 0]
print("picture span us", us(max(ends)))
# inter workers: rows 96..159, role 0 = dequeued item, 1 = after ref wait, 2 = segment done
wait_tot, work_tot, items = 0.0, 0.0, 0
p0_tot, n_p0 = 0.0, 0
first = []
for w in range(64):
    r = 96 + w
    for i in range(256):
        if t[r, 0, i] <= 0 or t[r, 2, i] <= 0:
            continue
        items += 1
        wait_tot += (t[r, 1, i] - t[r, 0, i]) / 100.0
        work_tot += (t[r, 2, i] - t[r, 1, i]) / 100.0
        if t[r, 3, i] > 0:
            p0_tot += (t[r, 3, i] - t[r, 1, i]) / 100.0
            n_p0 += 1
        first.append((us(t[r, 0, i]), int(v[r, 0, i]), round((t[r, 1, i] - t[r, 0, i]) / 100.0, 1), round((t[r, 2, i] - t[r, 1, i]) / 100.0, 1)))
if items:
    print(f"inter items {items}: ref-wait {wait_tot / items:.1f} us/item, work {work_tot / items:.1f} us/item (8 MBs)")
    if n_p0:
        print(f"  of which inter MBs (pass 0, 4 waves): {p0_tot / n_p0:.1f} us/item")
    first.sort()
    print("first items (t, item, wait, work):", first[:8])
    print("last items:", first[-5:])
print("deblock detail: rows 10, 11 - filter MB times (us), loader got-events, storer lim-events")
for y in (10, 12):
    f = t[y, 1, :Wmb + 1]
    print(y, "filter", [us(f[i]) for i in range(0, 24)])
    print(y, "loader", [(us(t[y, 0, i]), int(v[y, 0, i])) for i in range(0, 14) if t[y, 0, i] > 0])
    print(y, "storer", [(us(t[y, 2, i]), int(v[y, 2, i])) for i in range(0, 14) if t[y, 2, i] > 0])
    fs = f[f > 0]
    print(y, "filter step median", np.median(np.diff(fs)) / 100.0)
