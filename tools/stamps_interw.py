"""Diagnostic: inter MB phase durations inside the inter workers (stamps build with -DM2DEC_STAMPW).
    M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stampw.so M2DEC_AMD_REPLAY_LIMIT=N M2DEC_AMD_REPLAY_ISOLATE_LAST=1 \
        python tools/stamps_interw.py
events: 0 start, 1 windows loaded, 2 prediction done, 3 dequantised, 4 transformed, 5 added (6 = done
without residual)"""
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
a = np.frombuffer(buf, np.uint64).reshape(160, 4, 256)[72:88]
t = (a >> np.uint64(16)).astype(np.int64)
ph = {k: [] for k in ["win", "pred", "deq", "idct", "add", "total_res", "total_nores"]}
for r in range(16):
    for w in range(4):
        for m in range(32):
            e = t[r, w, m * 8:m * 8 + 8]
            if e[0] <= 0 or e[1] <= 0 or e[2] <= 0:
                continue
            ph["win"].append(e[1] - e[0])
            ph["pred"].append(e[2] - e[1])
            if e[5] > 0 and e[5] > e[0]:
                ph["deq"].append(e[3] - e[2]); ph["idct"].append(e[4] - e[3]); ph["add"].append(e[5] - e[4])
                ph["total_res"].append(e[5] - e[0])
            elif e[6] > 0:
                ph["total_nores"].append(e[6] - e[0])
for k, v in ph.items():
    if v:
        v = np.array(v) / 100.0
        print(f"{k:12s} n={len(v):5d} mean {v.mean():6.2f} us  median {np.median(v):6.2f}  p90 {np.percentile(v, 90):6.2f}")
