"""Where an H.265 intra picture's CTU kernel time goes (k_h265_ctu_rows, H265_STAMPS build):
M2DEC_AMD_LIB=build/dbg/libm2dec_amd_h5stamps.so M2DEC_AMD_H265_STREAMS=1 python3 tools/stamps_h265.py [golden]
One warm decode, then one stamped decode (pictures one after another on one stream); for its first picture:
the kernel's span, per CTU the wait for the row above / the blocks / the store, the per-block cost by size,
prediction and residual kind, and the CTU chain that ends the picture."""
import ctypes
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import m2dec_amd  # noqa: E402
from test_h265_cpu import h265_stream  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c_h265_1080p_s1"
g = json.load(open(os.path.join(ROOT, "tests", "golden", "h265.json")))[name]
data = h265_stream(name)
L = m2dec_amd.lib()
L.m2dec_amd_h265_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
N = 1 << 20
T = (ctypes.c_ulonglong * N)()
I = (ctypes.c_uint * N)()
with m2dec_amd.H265HipBackend(0) as be:
    assert m2dec_amd.decode_h265_md5(data, backend=be.be)[0] == g["md5"]
    assert L.m2dec_amd_h265_stamps(T, I, N) >= 0, "not a stamps build"
    assert m2dec_amd.decode_h265_md5(data, backend=be.be)[0] == g["md5"]
    n = L.m2dec_amd_h265_stamps(T, I, N)
ev = sorted((T[i], I[i] & 15, (I[i] >> 4) & 255, (I[i] >> 12) & 255, I[i] >> 20) for i in range(n))
# pictures: a CTU (0, 0) start opens one
pics, cur = [], None
for e in ev:
    if e[1] == 0 and e[2] == 0 and e[3] == 0:
        cur = []
        pics.append(cur)
    if cur is not None:
        cur.append(e)
print(f"{name}: {n} events, {len(pics)} pictures")
us = lambda d: d / 100.0  # noqa: E731  (100 MHz clock)
for pi, p in enumerate(pics[:2]):
    t0 = p[0][0]
    span = us(max(e[0] for e in p) - t0)
    ctu = defaultdict(dict)
    blocks = []
    last = {}
    for t, k, r, c, aux in p:
        if k in (0, 1, 3):
            ctu[(r, c)][k] = t
            if k == 1:
                last[(r, c, 0)] = last[(r, c, 1)] = t
        elif k == 2:
            ctu[(r, c)][f"w{aux}"] = t
        elif k == 4:
            w = (aux >> 7) & 1  # (the plane; with two waves per plane a block's duration spans the other wave's too)
            st = last.get((r, c, w), t)
            blocks.append((aux & 7, (aux >> 3) & 1, (aux >> 4) & 7, w, us(t - st)))
            last[(r, c, w)] = t
    waits = [us(v[1] - v[0]) for v in ctu.values() if 0 in v and 1 in v]
    # per plane: the last of its waves (two waves per plane when the kernel runs 4 waves: w2 / w3 seen)
    four = any("w2" in v for v in ctu.values())
    luma_w, chroma_w = (("w0", "w1"), ("w2", "w3")) if four else (("w0",), ("w1",))
    end = lambda v, ws: max(v[w] for w in ws if w in v) if any(w in v for w in ws) else None  # noqa: E731
    body0 = [us(end(v, luma_w) - v[1]) for v in ctu.values() if 1 in v and end(v, luma_w)]
    body1 = [us(end(v, chroma_w) - v[1]) for v in ctu.values() if 1 in v and end(v, chroma_w)]
    tail = [us(v[3] - max(end(v, luma_w) or 0, end(v, chroma_w) or 0)) for v in ctu.values() if 3 in v and end(v, luma_w)]
    print(f"\npicture {pi}: span {span:.0f} us, {len(ctu)} CTUs, {len(blocks)} blocks")
    q = lambda xs: f"median {statistics.median(xs):6.1f} mean {statistics.mean(xs):6.1f} max {max(xs):7.1f}" if xs else "-"  # noqa: E731
    print(f"  CTU wait for the row above + row load  {q(waits)} us")
    print(f"  CTU luma blocks ({'waves 0-1' if four else 'wave 0'})           {q(body0)} us")
    print(f"  CTU chroma blocks ({'waves 2-3' if four else 'wave 1'})         {q(body1)} us")
    print(f"  CTU join + store + progress           {q(tail)} us")
    print("  blocks by (plane, log2, intra, residual kind): n, median us, sum us")
    groups = defaultdict(list)
    for lg, pr, rs, w, d in blocks:
        groups[(w, lg, pr, rs)].append(d)
    for key in sorted(groups, key=lambda k: -sum(groups[k]))[:14]:
        xs = groups[key]
        print(f"    plane {key[0]} n{1 << key[1]:2d} pred {key[2]} res {key[3]}: {len(xs):5d}  {statistics.median(xs):6.2f}  {sum(xs):8.0f}")
    # block phases (kind 5, per workgroup and wave): start -> residual -> reference samples -> prediction + store;
    # "gap" = from the wave's previous block end to this block's start (next record, dependency waits)
    seqs = defaultdict(list)
    for t, k, r, c, aux in p:
        if k == 5:
            seqs[(c, r)].append((t, aux >> 8, aux & 255))
    ph = defaultdict(lambda: [[], [], [], [], []])
    for key, evs in seqs.items():
        evs.sort()
        prev_end, cur = None, None
        for t, phase, sz in evs:
            if phase == 0:
                cur = {0: t, "sz": sz, "gap": us(t - prev_end) if prev_end is not None else None}
            elif cur is not None:
                cur[phase] = t
                if phase == 3:
                    g = ph[(sz >> 3, 1 << (sz & 7))]
                    w = cur.get(4, cur.get(1))
                    if 1 in cur:
                        g[0].append(us(cur[1] - cur[0]))
                    if 4 in cur and 1 in cur:
                        g[1].append(us(cur[4] - cur[1]))
                    if 2 in cur and w is not None:
                        g[2].append(us(cur[2] - w))
                    if 2 in cur:
                        g[3].append(us(t - cur[2]))
                    if cur["gap"] is not None:
                        g[4].append(cur["gap"])
                    prev_end, cur = t, None
    if ph:
        print("  intra block phases (median us): plane, size: n, residual, wait for neighbours, reference samples, "
              "prediction + store, gap before")
        md = lambda xs: f"{statistics.median(xs):6.2f}" if xs else "     -"  # noqa: E731
        for key in sorted(ph):
            g = ph[key]
            print(f"    plane {key[0]} n{key[1]:2d}: {len(g[3]):5d}  {md(g[0])}  {md(g[1])}  {md(g[2])}  {md(g[3])}  {md(g[4])}")
    # the chain: the CTU finishing last, and per row when its last CTU ended
    rows = defaultdict(list)
    for (r, c), v in ctu.items():
        if 3 in v:
            rows[r].append((c, us(v[3] - t0)))
    print("  row: first CTU end .. last CTU end (us)")
    for r in sorted(rows)[:40]:
        xs = sorted(rows[r])
        print(f"    {r:3d}: {xs[0][1]:8.1f} .. {xs[-1][1]:8.1f}  ({len(xs)} CTUs, {(xs[-1][1] - xs[0][1]) / max(1, len(xs) - 1):.1f} us per CTU)")
