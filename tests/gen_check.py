"""Cross-check of the host parser against the stream generator (test infrastructure).

The generator (tools/h264gen) writes, next to each stream, a dump of what it encoded per
macroblock: type, cbp, QP, intra modes, reference indices, motion vectors (exact in I/P pictures)
and every coefficient level.  Direct-predicted blocks (B_Skip, B_Direct_16x16, direct sub-MBs)
carry the generator's own spec restatement of spatial / temporal direct (8.4.1.2), so B-picture
reference indices and vectors are compared like any other.  Here the stream is parsed by libm2dec_amd's host parser (with the
CPU oracle as the back end so that decoding completes), the per-picture records are captured at
submit time, and every field is compared with the dump.  This checks CABAC/CAVLC syntax decoding,
scans, QP tracking, intra-mode and motion-vector prediction independently of reconstruction.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

import m2dec_amd
from m2dec_amd import Backend, Frame
from tests._oracle import OracleBackend

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "tools", "_build", "h264gen")

MB_DT = np.dtype([("kind", "u1"), ("cbp", "u1"), ("avail_luma", "u1"), ("avail_chroma", "u1"), ("qpy", "i1"),
                  ("qpc", "i1", 2), ("pred_mode", "u1"), ("chroma_mode", "u1"), ("flags", "u1"), ("slice", "<u2"),
                  ("ipred", "<u4", 2), ("coef", "<u4"), ("nz", "<u4"), ("inter", "<u4")])
INTER_DT = np.dtype([("mv", "<i2", (2, 16, 2)), ("slot", "i1", (2, 4)), ("refidx", "i1", (2, 4))])
DUMP_DT = np.dtype([("pic", "<i4"), ("mbaddr", "<i4"), ("kind", "u1"), ("cbp", "u1"), ("qp", "i1"), ("t8x8", "u1"),
                    ("exact_mv", "u1"), ("i16_pred", "u1"), ("cmode", "u1"), ("dir8", "u1"), ("ipm", "i1", 16),
                    ("ref", "i1", (2, 4)), ("mv", "<i2", (2, 16, 2)), ("ldc", "<i2", 16), ("luma", "<i2", 256),
                    ("cdc", "<i2", (2, 4)), ("cac", "<i2", (2, 4, 16))])
REFDUMP_DT = np.dtype([("pic", "<i4"), ("first_mb", "<i4"), ("slice_type", "<i4"), ("poc", "<i4"), ("n", "<i4", 2),
                       ("poc_l", "<i4", (2, 16)), ("lt", "i1", (2, 16))])
assert MB_DT.itemsize == 32 and INTER_DT.itemsize == 144 and DUMP_DT.itemsize == 984 and REFDUMP_DT.itemsize == 184


class Picture(ctypes.Structure):
    _fields_ = [("width_mbs", ctypes.c_int32), ("height_mbs", ctypes.c_int32), ("slot", ctypes.c_int32),
                ("n_inter", ctypes.c_int32), ("n_coef", ctypes.c_int32), ("n_slices", ctypes.c_int32),
                ("n_intra", ctypes.c_int32), ("deblock", ctypes.c_int32), ("mb", ctypes.c_void_p),
                ("dbk", ctypes.c_void_p), ("slice", ctypes.c_void_p), ("inter", ctypes.c_void_p),
                ("coef", ctypes.c_void_p), ("cap_slices", ctypes.c_int32), ("cap_inter", ctypes.c_int32),
                ("cap_coef", ctypes.c_int32), ("flags", ctypes.c_int32)]


SET_FRAMES = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Frame), ctypes.c_int,
                              ctypes.c_int)
ACQUIRE = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)
SUBMIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(Picture))
SYNC = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int)
DESTROY = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


def _arr(ptr, dtype, n):
    if n == 0:
        return np.zeros(0, dtype)
    buf = (ctypes.c_char * (n * dtype.itemsize)).from_address(ptr)
    return np.frombuffer(bytes(buf), dtype=dtype, count=n)


class RecordingBackend:
    """Forwards to an inner back end and keeps a copy of every submitted picture's records."""

    def __init__(self, inner: Backend):
        self.inner = inner
        self.pics = []
        self._cbs = [SET_FRAMES(self._set_frames), ACQUIRE(self._acquire), SUBMIT(self._submit), SYNC(self._sync),
                     DESTROY(lambda s: None)]
        self.be = Backend(None, *[ctypes.cast(c, ctypes.c_void_p).value for c in self._cbs])

    def _set_frames(self, _s, n, frames, w, h):
        return SET_FRAMES(self.inner.set_frames)(self.inner.self, n, frames, w, h)

    def _acquire(self, _s, wm, hm):
        return ACQUIRE(self.inner.acquire)(self.inner.self, wm, hm)

    def _submit(self, _s, pic):
        p = pic.contents
        n = p.width_mbs * p.height_mbs
        self.pics.append({
            "w": p.width_mbs, "h": p.height_mbs, "slot": p.slot,
            "mb": _arr(p.mb, MB_DT, n).copy(),
            "inter": _arr(p.inter, INTER_DT, p.n_inter).copy(),
            "coef": _arr(p.coef, np.dtype("<i2"), p.n_coef).copy(),
            "dbk": _arr(p.dbk, np.dtype([("bs_v", "<u4"), ("bs_h", "<u4"), ("qpy", "i1"), ("qpc", "i1", 2),
                                         ("flags", "u1"), ("alpha", "i1"), ("beta", "i1"), ("pad", "u1", 2)]), n).copy(),
        })
        return SUBMIT(self.inner.submit)(self.inner.self, pic)

    def _sync(self, _s, slot):
        return SYNC(self.inner.sync_frame)(self.inner.self, slot)


def generate(preset, out, dump=None, seed=1, extra=(), refdump=None):
    cmd = [GEN, "--preset", preset, "--seed", str(seed), "-o", out]
    if dump:
        cmd += ["--dump", dump]
    if refdump:
        cmd += ["--dump-refs", refdump]
    for kv in extra:
        cmd += ["--set", kv]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def _pool_blocks(rec, coef):
    """Split an MB's coefficient pool into {('ldc',), ('luma', i), ('cdc', c), ('cac', c, b)} raster arrays."""
    nz = int(rec["nz"])
    t8 = bool(rec["flags"] & 1)
    off = int(rec["coef"])
    out = {}
    if nz & (1 << 16):
        out[("ldc",)] = coef[off:off + 16]
        off += 16
    for b in range(16):
        if nz & (1 << b):
            n = 64 if t8 else 16
            out[("luma", b)] = coef[off:off + n]
            off += n
    for c in range(2):
        if nz & (1 << (17 + c)):
            out[("cdc", c)] = coef[off:off + 4]
            off += 4
    for c in range(2):
        for b in range(4):
            if nz & (1 << (19 + 4 * c + b)):
                out[("cac", c, b)] = coef[off:off + 16]
                off += 16
    return out


def compare(pics, dump, max_errors=20, stats=None):
    errs = []
    stats = {"direct": 0, "mv": 0} if stats is None else stats
    kind_map = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 4}

    def err(d, msg):
        if len(errs) < max_errors:
            errs.append(f"pic {int(d['pic'])} mb {int(d['mbaddr'])} (kind {int(d['kind'])}): {msg}")

    for d in dump:
        pi, a = int(d["pic"]), int(d["mbaddr"])
        if pi >= len(pics):
            err(d, "picture missing in decoder output")
            break
        P = pics[pi]
        r = P["mb"][a]
        k = int(d["kind"])
        if int(r["kind"]) != kind_map[k]:
            err(d, f"kind {int(r['kind'])} != {kind_map[k]}")
            continue
        if k == 3:
            continue
        if int(r["qpy"]) != int(d["qp"]):
            err(d, f"qp {int(r['qpy'])} != {int(d['qp'])}")
        if k in (0, 1, 4) and (int(r["cbp"]) & 0x3f) != int(d["cbp"]):
            err(d, f"cbp {int(r['cbp']):#x} != {int(d['cbp']):#x}")
        if k == 5 and (int(r["cbp"]) & 0x3f) != 0:
            err(d, "skip with cbp")
        if k in (0, 1, 2) and int(r["chroma_mode"]) != int(d["cmode"]):
            err(d, f"chroma mode {int(r['chroma_mode'])} != {int(d['cmode'])}")
        if k == 2 and int(r["pred_mode"]) != int(d["i16_pred"]):
            err(d, f"i16 mode {int(r['pred_mode'])} != {int(d['i16_pred'])}")
        if k in (0, 1):
            nb = 16 if k == 0 else 4
            for b in range(nb):
                m = (int(r["ipred"][b >> 3]) >> (4 * (b & 7))) & 15
                if m != int(d["ipm"][b]):
                    err(d, f"intra mode blk {b}: {m} != {int(d['ipm'][b])}")
                    break
        if bool(r["flags"] & 1) != bool(d["t8x8"]) and (k == 1 or (k == 4 and (int(d["cbp"]) & 15))):
            err(d, f"t8x8 {int(r['flags'] & 1)} != {int(d['t8x8'])}")
        if k in (4, 5):
            I = P["inter"][int(r["inter"])]
            for lx in range(2):
                for b8 in range(4):
                    gref = int(d["ref"][lx][b8])
                    if (int(d["dir8"]) >> b8) & 1:
                        stats["direct"] += 1
                    used = int(I["slot"][lx][b8]) >= 0
                    if (gref >= 0) != used:
                        err(d, f"L{lx} 8x8 {b8}: used {used} vs generator ref {gref}")
                        continue
                    if gref >= 0:
                        if int(I["refidx"][lx][b8]) != gref:
                            err(d, f"L{lx} 8x8 {b8}: refidx {int(I['refidx'][lx][b8])} != {gref}")
                        if d["exact_mv"]:
                            stats["mv"] += 1
                            for blk in range(4):
                                x = (b8 & 1) * 2 + (blk & 1)
                                y = (b8 >> 1) * 2 + (blk >> 1)
                                got = tuple(int(v) for v in I["mv"][lx][y * 4 + x])
                                want = tuple(int(v) for v in d["mv"][lx][y * 4 + x])
                                if got != want:
                                    err(d, f"L{lx} mv at ({x},{y}) {got} != {want}")
                                    break
        # coefficients
        blocks = _pool_blocks(r, P["coef"])
        want = {}
        if np.any(d["ldc"]):
            want[("ldc",)] = d["ldc"]
        t8 = bool(d["t8x8"])
        for b in range(16):
            if t8:
                if b % 4 == 0 and np.any(d["luma"][(b // 4) * 64:(b // 4) * 64 + 64]):
                    want[("luma", b)] = d["luma"][(b // 4) * 64:(b // 4) * 64 + 64]
            elif np.any(d["luma"][b * 16:b * 16 + 16]):
                want[("luma", b)] = d["luma"][b * 16:b * 16 + 16]
        for c in range(2):
            if np.any(d["cdc"][c]):
                want[("cdc", c)] = d["cdc"][c]
            for b in range(4):
                if np.any(d["cac"][c][b]):
                    want[("cac", c, b)] = d["cac"][c][b]
        gk = {kk for kk, v in blocks.items() if np.any(v)}
        if gk != set(want):
            err(d, f"coded blocks {sorted(gk ^ set(want))[:6]} differ")
        else:
            for kk, v in want.items():
                if not np.array_equal(np.asarray(blocks[kk], np.int32), np.asarray(v, np.int32)):
                    err(d, f"levels of {kk} differ: {list(blocks[kk])[:16]} vs {list(v)[:16]}")
                    break
    return errs


def compare_refs(gen, dec, max_errors=20):
    """Every P / B slice's active lists (POC and long-term flag per entry): generator vs parser."""
    errs = []
    got = {(int(r["pic"]), int(r["first_mb"])): r for r in dec}
    for g in gen:
        key = (int(g["pic"]), int(g["first_mb"]))
        d = got.get(key)
        if d is None:
            errs.append(f"pic {key[0]} slice at {key[1]}: no list dump from the parser")
        elif int(d["slice_type"]) != int(g["slice_type"]) or int(d["poc"]) != int(g["poc"]) or list(d["n"]) != list(g["n"]):
            errs.append(f"pic {key[0]} slice at {key[1]}: type/poc/n {int(d['slice_type'])}/{int(d['poc'])}/{list(d['n'])} != "
                        f"{int(g['slice_type'])}/{int(g['poc'])}/{list(g['n'])}")
        else:
            for lx in range(2):
                n = int(g["n"][lx])
                a = [(int(p), int(t)) for p, t in zip(d["poc_l"][lx][:n], d["lt"][lx][:n])]
                b = [(int(p), int(t)) for p, t in zip(g["poc_l"][lx][:n], g["lt"][lx][:n])]
                if a != b:
                    errs.append(f"pic {key[0]} slice at {key[1]} L{lx}: (poc, lt) {a} != {b}")
        if len(errs) >= max_errors:
            break
    return errs


def check(preset, seed=1, extra=(), tmpdir="/tmp", refs=True):
    out = os.path.join(tmpdir, f"gc_{preset}_{seed}.264")
    dmp = out + ".dump"
    rdg, rdd = out + ".refs", out + ".decrefs"
    generate(preset, out, dmp, seed, extra, refdump=rdg if refs else None)
    data = open(out, "rb").read()
    dump = np.fromfile(dmp, dtype=DUMP_DT)
    L = m2dec_amd.lib()
    L.m2dec_amd_h264_set_refdump.argtypes = [ctypes.c_char_p]
    if refs:
        assert L.m2dec_amd_h264_set_refdump(rdd.encode()) == 0
    try:
        with OracleBackend() as ob:
            rec = RecordingBackend(ob.be)
            err = None
            try:
                m2dec_amd.decode_stream(data, backend=rec.be)
            except RuntimeError as e:
                err = str(e)
    finally:
        if refs:
            L.m2dec_amd_h264_set_refdump(None)
    errs = compare(rec.pics, dump)
    if refs:
        errs = compare_refs(np.fromfile(rdg, dtype=REFDUMP_DT), np.fromfile(rdd, dtype=REFDUMP_DT)) + errs
    npics = int(dump["pic"].max()) + 1 if len(dump) else 0
    if err:
        errs.insert(0, f"decode error: {err}")
    if len(rec.pics) != npics:
        errs.insert(0, f"decoded {len(rec.pics)} pictures, generator wrote {npics}")
    return errs


if __name__ == "__main__":
    presets = sys.argv[1:] or ["cov_cavlc", "cov_cabac4x4", "cov_cabac", "cov_wp", "cov_slices"]
    bad = 0
    for p in presets:
        e = check(p)
        print(p, "OK" if not e else f"{len(e)} errors")
        for x in e:
            print("   ", x)
        bad += bool(e)
    sys.exit(1 if bad else 0)
