"""Where the gfx950 H.265 reconstruction differs from the CPU oracle: decodes one golden stream both ways
and prints, per output frame, whether the planes agree and the first differing samples (luma x, y / chroma
pair x, y, component).  Needs the GPU (decode) and the oracle library (the checker).
Usage: python3 tools/h265_diff.py GOLDEN_NAME [max_lines]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctypes  # noqa: E402

import m2dec_amd  # noqa: E402
from _oracle import Oracle265Backend  # noqa: E402
from test_h265_cpu import h265_stream  # noqa: E402


def grab(data, backend=None):
    out = []

    def on_frame(f):
        w, h = f.width, f.height
        y = ctypes.string_at(f.luma, w * h)
        c = ctypes.string_at(f.chroma, w * h // 2)
        out.append((w, h, y, c))

    if backend is None:
        m2dec_amd.decode_h265(data, device=0, on_frame=on_frame)
    else:
        m2dec_amd.decode_h265(data, backend=backend, on_frame=on_frame)
    return out


def main():
    name = sys.argv[1]
    lim = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    data = h265_stream(name)
    gpu = grab(data)
    with Oracle265Backend() as o:
        ref = grab(data, o.be)
    print(f"{name}: {len(gpu)} GPU frames, {len(ref)} oracle frames")
    for i, (g, r) in enumerate(zip(gpu, ref)):
        w, h = g[0], g[1]
        bad = [(k % w, k // w) for k in range(w * h) if g[2][k] != r[2][k]]
        badc = [((k % w) >> 1, k // w, k & 1) for k in range(w * h // 2) if g[3][k] != r[3][k]]
        print(f"frame {i}: luma diffs {len(bad)}, chroma diffs {len(badc)}")
        for x, y in bad[:lim]:
            print(f"  Y ({x},{y}) gpu {g[2][y * w + x]} oracle {r[2][y * w + x]}")
        for x, y, c in badc[:lim]:
            print(f"  C{c} ({x},{y}) gpu {g[3][y * w + 2 * x + c]} oracle {r[3][y * w + 2 * x + c]}")


if __name__ == "__main__":
    main()
