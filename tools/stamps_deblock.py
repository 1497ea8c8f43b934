"""Diagnostic: per-row timing of the deblocking wavefront from in-kernel s_memrealtime stamps.
Run with M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stamps.so (make stamps)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import stream  # noqa: E402

L = m2dec_amd.lib()
tr = m2dec_amd.Trace(stream(sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"))
rp = m2dec_amd.HipReplay(tr, 0)
rp.run(1)
rp.sync()
N = 160 * 4 * 256
buf = (ctypes.c_ulonglong * N)()
L.m2dec_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
L.m2dec_amd_debug_stamps_clear()
# run only the last picture again (deblocked) so the stamps are from one picture
rp.run(1)
rp.sync()
assert L.m2dec_amd_debug_stamps(buf, N) > 0
a = np.frombuffer(buf, np.uint64).reshape(160, 4, 256)
t = (a >> np.uint64(16)).astype(np.int64)
v = (a & np.uint64(0xffff)).astype(np.int64)
Hmb = tr.height // 16
Wmb = tr.width // 16
t0 = t[:Hmb][t[:Hmb] > 0].min()
out = {"rows": []}
for y in range(Hmb):
    f = t[y, 1, :Wmb + 1]
    fs = (f - t0) / 100.0  # us (100 MHz)
    ld = [(int((t[y, 0, i] - t0) / 100), int(v[y, 0, i])) for i in range(256) if t[y, 0, i] > 0]
    st = [(int((t[y, 2, i] - t0) / 100), int(v[y, 2, i])) for i in range(256) if t[y, 2, i] > 0]
    steps = np.diff(fs)
    out["rows"].append({"y": y, "start": round(fs[0], 2), "end": round(fs[Wmb], 2),
                        "step_med": round(float(np.median(steps)), 3), "step_max": round(float(steps.max()), 2),
                        "loader": ld[:12], "storer": st[:12]})
for r in out["rows"][:6] + out["rows"][-3:]:
    print(r)
ends = [r["end"] for r in out["rows"]]
print("picture span us", max(ends))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/stamps_deblock.json", "w"))
