"""Host-side H.265 parse cost per picture: decode the 1080p intra golden through h265d_func with a back end
whose calls do nothing, so only the parser (NAL / slice header / CABAC / records) is timed. CPU only."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import m2dec_amd  # noqa: E402
from test_h265_cpu import h265_stream  # noqa: E402

SF = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)
SB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
SY = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int)
DE = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c_h265_1080p_s1"
    data = h265_stream(name)
    fns = SF(lambda *a: 0), SB(lambda *a: 0), SY(lambda *a: 0), DE(lambda *a: None)
    be = m2dec_amd.Backend265()
    be.set_frames, be.submit, be.sync_frame, be.destroy = (ctypes.cast(f, ctypes.c_void_p) for f in fns)
    m2dec_amd.decode_h265(data, backend=be)
    n, t = 0, time.perf_counter()
    while time.perf_counter() - t < 3.0:
        n += len(m2dec_amd.decode_h265(data, backend=be)[0])
    dt = time.perf_counter() - t
    print(f"{name}: {n} frames, host parse {dt / n * 1e3:.2f} ms/frame, {len(data) * 8 / 1e6 / 8:.2f} Mbit/picture")


if __name__ == "__main__":
    main()
