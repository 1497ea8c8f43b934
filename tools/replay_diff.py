"""Locate wrong macroblocks of a GPU replay: one checked k_batch pass of a golden stream (the library named
by M2DEC_AMD_LIB, default the in-tree one), every picture captured in decoding order, compared with the
CPU oracle's picture MB by MB.  Per differing picture: its kind (I / P-B), differing MBs per plane, the
first differing MB in raster order with its record kind, and the pixel rows inside the MB that differ
(rows 13..15 / chroma 5..7 only point at deblocking across the MB row edge).

    python tools/replay_diff.py c3_1080p_s1 [passes_before]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._oracle import OracleBackend  # noqa: E402
from tests._streams import stream  # noqa: E402

KIND = {0: "I4x4", 1: "I8x8", 2: "I16x16", 3: "PCM", 4: "INTER"}


def oracle_frames(data):
    out = []

    def cb(f):
        w, h = f.width, f.height
        y = np.ctypeslib.as_array(ctypes.cast(f.luma, ctypes.POINTER(ctypes.c_uint8)), shape=(h, w)).copy()
        c = np.ctypeslib.as_array(ctypes.cast(f.chroma, ctypes.POINTER(ctypes.c_uint8)), shape=(h // 2, w)).copy()
        out.append((y, c))

    with OracleBackend() as ob:
        m2dec_amd.decode_stream(data, backend=ob.be, on_frame=cb, md5=False)
    return out


def intra_dump(tr, recs):
    """-DM2DEC_DBG_INTRA builds: MB (0, 0) of the first I picture as intra_row saw it, against its records."""
    L = m2dec_amd.lib()
    L.m2dec_amd_debug_intra.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = (ctypes.c_int * 2048)()
    if L.m2dec_amd_debug_intra(buf, 2048) < 0:
        print("no intra dump in this build")
        return
    d = np.array(buf[:], dtype=np.int64)
    p = tr.pics[0]
    want_m = np.frombuffer(recs[p.off_mb:p.off_mb + 32], dtype=np.int32)
    print("record words  dev:", [hex(int(v) & 0xffffffff) for v in d[:8]])
    print("record words want:", [hex(int(v) & 0xffffffff) for v in want_m])
    coef = int(want_m[7])
    pool = np.frombuffer(recs[p.off_coef + 2 * coef:p.off_coef + 2 * coef + 2 * 448], dtype=np.int16)
    q = d[16:16 + 448]
    bad = np.nonzero(q[:448] != pool[:448])[0]
    print(f"qb {d[15]} done {d[14]}; coefficient staging: {len(bad)} of 448 differ (first {bad[:12].tolist()})")
    print(" dev Q[0:32] ", q[:32].tolist())
    print(" pool[0:32]  ", pool[:32].tolist())
    lb = d[512:512 + 17 * 25].reshape(17, 25)
    la = d[1024:1024 + 17 * 25].reshape(17, 25)
    print(" L before row 0:", lb[0].tolist(), " col 0:", lb[:, 0].tolist())
    print(" L after (MB samples):\n", la[1:, 1:17])
    print(" R[0:32]:", d[1536:1568].tolist())
    print(" DC:", d[1936:1952].tolist(), " HV:", d[1952:1956].tolist())


def rows_dump(tr, recs):
    """-DM2DEC_DBG_ROWS builds: per row workgroup / wave of the I picture, the row intra_row worked on and its
    first MB's record kind / coefficient offset, against the expected row of that workgroup and wave."""
    L = m2dec_amd.lib()
    L.m2dec_amd_debug_rows.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = (ctypes.c_uint * 2048)()
    if L.m2dec_amd_debug_rows(buf, 2048) < 0:
        print("no row dump in this build")
        return
    d = list(buf)
    p = tr.pics[0]
    Wmb = tr.width // 16
    for b in range(256):
        for w in range(4):
            a, c = d[(b * 4 + w) * 2], d[(b * 4 + w) * 2 + 1]
            if (a >> 24) != 0xab:
                continue
            y, part, wave = a & 0xff, (a >> 8) & 0xf, (a >> 12) & 0xf
            want_kind = recs[p.off_mb + 32 * (y * Wmb)]
            want_coef = int.from_bytes(recs[p.off_mb + 32 * (y * Wmb) + 20:p.off_mb + 32 * (y * Wmb) + 24], "little")
            print(f"block {b} wave {w}: y {y} part {part} wave-arg {wave} y0 {c & 0xffff} kind {(c >> 16) & 0xff} "
                  f"(record {want_kind}) coef&255 {c >> 24} (record {want_coef & 255})")


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"
    before = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    data = open(name, "rb").read() if os.path.exists(name) else stream(name)
    ref_out = oracle_frames(data)
    tr = m2dec_amd.Trace(data)
    W, H = tr.width, tr.height
    ref = [None] * tr.npics
    for k, d in enumerate(tr.output_order):
        ref[d] = ref_out[k]
    pics = tr.pics
    rp = m2dec_amd.HipReplay(tr)
    if before:
        rp.run(before)
        rp.sync()
    raw = np.frombuffer(rp.capture(), dtype=np.uint8)
    fb = W * H * 3 // 2
    recs = tr.records()
    nbad = 0
    for i in range(tr.npics):
        g = raw[i * fb:(i + 1) * fb]
        gy, gc = g[:W * H].reshape(H, W), g[W * H:].reshape(H // 2, W)
        oy, oc = ref[i]
        dy, dc = gy != oy, gc != oc
        if not dy.any() and not dc.any():
            continue
        nbad += 1
        p = pics[i]
        mby = dy.reshape(H // 16, 16, W // 16, 16).any(axis=(1, 3))
        mbc = dc.reshape(H // 16, 8, W // 16, 16).any(axis=(1, 3))
        anyb = mby | mbc
        ys, xs = np.nonzero(anyb)
        y0, x0 = int(ys[0]), int(xs[0])
        # the first differing MB's record kind (m2r_mb_t: 32 bytes, kind in byte 0)
        kind = recs[p.off_mb + 32 * (y0 * (W // 16) + x0)]
        ry = np.nonzero(dy[y0 * 16:(y0 + 1) * 16, x0 * 16:(x0 + 1) * 16].any(axis=1))[0].tolist()
        rc = np.nonzero(dc[y0 * 8:(y0 + 1) * 8, x0 * 16:(x0 + 1) * 16].any(axis=1))[0].tolist()
        print(f"picture {i} ({'I' if p.n_inter == 0 else 'P/B'}, slot {p.slot}): {int(mby.sum())} luma MBs, "
              f"{int(mbc.sum())} chroma MBs differ; first MB ({x0}, {y0}) {KIND.get(kind, kind)}: luma rows {ry} "
              f"chroma rows {rc}; MB rows hit {sorted(set(ys.tolist()))[:16]}", flush=True)
        if nbad == 1:
            print("  differing MBs per MB row:", anyb.sum(axis=1).tolist(), flush=True)
            # which MB row of the oracle's picture each row of the device's matches best (a shifted or swapped row)
            gr = gy.reshape(H // 16, 16 * W).astype(np.int32)
            orr = oy.reshape(H // 16, 16 * W).astype(np.int32)
            match = [int(np.abs(orr - gr[r]).sum(axis=1).argmin()) for r in range(H // 16)]
            print("  best oracle MB row per device MB row:", match, flush=True)
            if os.environ.get("DIFF_SAVE"):
                np.savez_compressed(os.environ["DIFF_SAVE"], got_y=gy, got_c=gc, want_y=oy, want_c=oc)
            blk = (slice(y0 * 16, y0 * 16 + 16), slice(x0 * 16, x0 * 16 + 16))
            print("  got luma:\n" + str(gy[blk]) + "\n  want luma:\n" + str(oy[blk]), flush=True)
    print(f"{name}: {nbad} of {tr.npics} pictures differ", flush=True)
    if os.environ.get("DBG_INTRA"):
        intra_dump(tr, recs)
    if os.environ.get("DBG_ROWS"):
        rows_dump(tr, recs)
    rp.close()


if __name__ == "__main__":
    main()
