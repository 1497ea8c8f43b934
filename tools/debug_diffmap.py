"""Where do full-speed HIP frames differ from the oracle's?  Per output frame: differing MBs, and a
histogram of the differing luma pixel rows inside an MB (0..15) and chroma rows (0..7)."""
import os, sys, ctypes, faulthandler
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(250, exit=True)
import m2dec_amd
from tests._oracle import OracleBackend
from tests._streams import stream


def grab(data, backend=None):
    out = []

    def cb(f):
        w, h = f.width, f.height
        y = np.ctypeslib.as_array(ctypes.cast(f.luma, ctypes.POINTER(ctypes.c_uint8)), shape=(h, w)).copy()
        c = np.ctypeslib.as_array(ctypes.cast(f.chroma, ctypes.POINTER(ctypes.c_uint8)), shape=(h // 2, w)).copy()
        out.append((y, c))
    m2dec_amd.decode_stream(data, backend=backend, on_frame=cb, md5=False)
    return out


for n in sys.argv[1:]:
    data = stream(n)
    with OracleBackend() as ob:
        ref = grab(data, ob.be)
    for rep in range(2):
        got = grab(data)
        print(f"== {n} run {rep}: {len(got)} frames", flush=True)
        for i, ((gy, gc), (oy, oc)) in enumerate(zip(got, ref)):
            h, w = oy.shape
            dy = gy != oy
            dc = gc != oc
            if not dy.any() and not dc.any():
                continue
            mb = dy.reshape(h // 16, 16, w // 16, 16).any(axis=(1, 3)) | dc.reshape(h // 16, 8, w // 16, 16).any(axis=(1, 3))
            rows_l = dy.reshape(h // 16, 16, w).any(axis=(0, 2))
            rows_c = dc.reshape(h // 16, 8, w).any(axis=(0, 2))
            ys, xs = np.nonzero(mb)
            print(f" frame {i}: {mb.sum()} MBs differ; MB rows {sorted(set(ys.tolist()))[:12]}; "
                  f"luma px rows {np.nonzero(rows_l)[0].tolist()} chroma px rows {np.nonzero(rows_c)[0].tolist()}; "
                  f"max |d| {max(np.abs(gy.astype(int) - oy).max(), np.abs(gc.astype(int) - oc).max())}", flush=True)
