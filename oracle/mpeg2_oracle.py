"""CPU restatement of the reference's MPEG-1/2 decode path — TEST INFRASTRUCTURE ONLY.

Only tests/ (and tools/make_m2v_goldens.py) use this module: it is the checker of the product's
MPEG-2 decoder (m2dec_amd/csrc/host/mpeg2_dec.c, behind m2d_func), never part of it.

It follows /root/reference/src/lib/mpeg2.cpp + idct.cpp + motioncomp.cpp + src/app/m2decoder.h step by
step (intra, P and B frame pictures: macroblock types, skipped macroblocks, frame / field / dual-prime
motion vectors and their predictors, half-sample prediction, non-intra blocks), written
independently of the product's C and reading its variable-length codes from
tests/golden/mpeg2_vlc.json — the codewords of the REFERENCE's own tables (vld.h) as its decoder walks
them (tools/gen_mpeg2_vlc_golden.py) — so a transcription error in the product's Annex-B tables
cannot hide behind a shared table.  Pure Python: small pictures only (the coverage streams,
176x144); the 720x480 C1 stream's golden MD5s were produced by the product and cross-checked here on
a prefix of its pictures (tools/make_m2v_goldens.py).

Parity is pinned by the reference's own test vectors (the DCT-VLC table of mpeg2.cpp:1743-1753 and the
intra-DC table of m2dec.cpp:142-217, tests/golden/mpeg2_kat.json) and by the reference's VLC tables;
whole-picture output has no reference-produced golden (the reference is unbuildable here,
DESIGN.md §4): "parity unpinned" for complete streams.
"""
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W1, W2, W3, W5, W6, W7 = 2841, 2676, 2408, 1609, 1108, 565  # idct.cpp:35-40

SCAN = [  # 7.3 zig-zag and alternate scans (mpeg2.cpp uses vld.h m2d_zigzag)
    [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21,
     28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
     47, 55, 62, 63],
    [0, 8, 16, 24, 1, 9, 2, 10, 17, 25, 32, 40, 48, 56, 57, 49, 41, 33, 26, 18, 3, 11, 4, 12, 19, 27, 34, 42, 50, 58, 35,
     43, 51, 59, 20, 28, 5, 13, 6, 14, 21, 29, 36, 44, 52, 60, 37, 45, 53, 61, 22, 30, 7, 15, 23, 31, 38, 46, 54, 62, 39,
     47, 55, 63]]
Q_SCALE = [[2] + [2 * i for i in range(1, 32)],
           [1, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 18, 20, 22, 24, 28, 32, 36, 40, 44, 48, 52, 56, 64, 72, 80, 88, 96,
            104, 112]]
DEFAULT_INTRA = [8, 16, 19, 22, 26, 27, 29, 34, 16, 16, 22, 24, 27, 29, 34, 37, 19, 22, 26, 27, 29, 34, 34, 38,
                 22, 22, 26, 27, 29, 34, 37, 40, 22, 26, 27, 29, 32, 35, 40, 48, 26, 27, 29, 32, 35, 40, 48, 58,
                 26, 27, 29, 34, 38, 46, 56, 69, 27, 29, 35, 38, 46, 56, 69, 83]


def _codes():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "mpeg2_vlc.json")))
    return {k: {c[0]: tuple(c[1:]) for c in v} for k, v in g.items() if k != "source"}


class Bits:
    def __init__(self, data):
        self.s = "".join(format(b, "08b") for b in data) + "0" * 64  # reads past the end see zeros
        self.p = 0

    def get(self, n):
        t = self.s[self.p:self.p + n].ljust(n, "0")
        self.p += n
        return int(t, 2) if n else 0

    def show(self, n):
        return int(self.s[self.p:self.p + n].ljust(n, "0"), 2) if n else 0

    def vlc(self, table, maxlen=18):
        for n in range(1, maxlen + 1):
            c = self.s[self.p:self.p + n]
            if c in table:
                self.p += n
                return table[c]
        raise ValueError("undefined code")


def units(data):
    """(code, payload) per start code (m2d_find_mpeg_data, m2d.cpp:130-155)."""
    out, i, n = [], 0, len(data)
    starts = []
    while True:
        j = data.find(b"\x00\x00\x01", i)
        if j < 0 or j + 3 >= n:
            break
        starts.append(j)
        i = j + 3
    for k, j in enumerate(starts):
        end = starts[k + 1] if k + 1 < len(starts) else n
        payload = data[j + 4:end]
        out.append((data[j + 3], payload.rstrip(b"\x00")))
    return out


def idct_block(coef):
    """intra: idct_raw clipped (ClipStore, idct.cpp:364-370)"""
    out = idct_raw(coef)
    for r in range(8):
        for k in range(8):
            v = out[r][k]
            assert -256 <= v <= 767, "CLIP255C argument outside the reference table (UB)"
            out[r][k] = 0 if v < 0 else 255 if v > 255 else v
    return out


def idct_raw(coef):
    """idct.cpp:69-236 (rows, stored as int16) + 286-358 (columns, (x + 8192) >> 14); rows without
    AC coefficients take the DC-only branch there (idct.cpp:147-159), which gives the same values."""
    def s16(v):
        v &= 0xffff
        return v - 0x10000 if v & 0x8000 else v
    c = list(coef)
    for r in range(8):
        s = c[8 * r:8 * r + 8]
        a0, a1 = s[0] * 2048 + 128, s[4] * 2048
        e0, e1 = a0 - a1, a0 + a1
        o4 = W7 * (s[1] + s[7]) + (W1 - W7) * s[1]
        o5 = W7 * (s[1] + s[7]) - (W1 + W7) * s[7]
        o6 = W3 * (s[5] + s[3]) - (W3 - W5) * s[5]
        o7 = W3 * (s[5] + s[3]) - (W3 + W5) * s[3]
        p4, p6, p5, p7 = o4 - o6, o4 + o6, o5 - o7, o5 + o7
        q5 = ((p4 + p5) * 181 + 128) >> 8
        q4 = ((p4 - p5) * 181 + 128) >> 8
        x2 = W6 * (s[2] + s[6]) - (W2 + W6) * s[6]
        x3 = W6 * (s[2] + s[6]) + (W2 - W6) * s[2]
        e0, x2 = e0 - x2, e0 + x2
        e1, x3 = e1 - x3, e1 + x3
        c[8 * r:8 * r + 8] = [s16((x3 + p6) >> 8), s16((x2 + q5) >> 8), s16((e0 + q4) >> 8), s16((e1 + p7) >> 8),
                              s16((e1 - p7) >> 8), s16((e0 - q4) >> 8), s16((x2 - q5) >> 8), s16((x3 - p6) >> 8)]
    out = [[0] * 8 for _ in range(8)]
    for k in range(8):
        s = [c[8 * r + k] for r in range(8)]
        x8 = W3 * (s[5] + s[3]) + 4
        x6, x7 = (x8 - (W3 - W5) * s[5]) >> 3, (x8 - (W3 + W5) * s[3]) >> 3
        x8 = W7 * (s[1] + s[7]) + 4
        x4, x5 = (x8 + (W1 - W7) * s[1]) >> 3, (x8 - (W1 + W7) * s[7]) >> 3
        x1 = W6 * (s[2] + s[6]) + 4
        x2, x3 = (x1 - (W2 + W6) * s[6]) >> 3, (x1 + (W2 - W6) * s[2]) >> 3
        x1, x4, x6, x5 = x4 + x6, x4 - x6, x5 + x7, x5 - x7
        x0 = s[0] * 256 + 8192
        x7 = s[4] * 256
        x8, x0 = x0 + x7, x0 - x7
        x7, x8 = x8 + x3, x8 - x3
        x3, x0 = x0 + x2, x0 - x2
        x2 = ((x4 + x5) * 181 + 128) >> 8
        x4 = ((x4 - x5) * 181 + 128) >> 8
        col = [(x7 + x1) >> 14, (x3 + x2) >> 14, (x0 + x4) >> 14, (x8 + x6) >> 14,
               (x8 - x6) >> 14, (x0 - x4) >> 14, (x3 - x2) >> 14, (x7 - x1) >> 14]
        for r in range(8):
            out[r][k] = col[r]
    return out


class Decoder:
    """m2d_context + M2Decoder (outbuf 0: 3 frames) for intra, P and B frame pictures."""

    def __init__(self):
        self.c = _codes()
        self.mpeg2 = 0
        self.intra_vlc = 0
        self.conceal = 0
        self.dc_scale, self.dc_max = 3, 255
        self.frame_mode = 3
        self.scan = SCAN[0]
        self.qst = 0
        self.qm = [DEFAULT_INTRA, [16] * 64]
        self.store = [[0] * 64 for _ in range(4)]
        self.frames = None
        self.num = 0
        self.lru = [0] * 16
        self.ref = [0, 0]
        self.index = -1
        self.out_state = 0
        self.copy_src = -1
        self.coding_type = 0
        self.mb_x, self.mb_y = -1, 0
        self.mb_type = 0
        self.dif = [None, None]
        self.r_size = [[0, 0], [0, 0]]
        self.pmv = [[[0, 0], [0, 0]], [[0, 0], [0, 0]]]
        self.out = []

    # ---- frames / output (mpeg2.cpp:130-194, 1543-1573; m2decoder.h:54-80, 132-157)
    def set_frames(self):
        w, h = (self.hsize + 15) & ~15, (self.vsize + 15) & ~15
        if self.frames is None or self.fsize != (w, h):
            self.fsize = (w, h)
            self.frames = [[bytearray(w * h), bytearray(w * h // 2)] for _ in range(3)]
            self.num = 3
            self.index = -1

    def update_frames(self, ctype):
        if self.index < 0:
            self.out_state = 2 if ctype in (1, 2) else 0
            self.index = 0
            return
        mi, mv = -1, -1
        for i in range(self.num):
            if i != self.ref[0] and i != self.ref[1]:
                v = self.lru[i]
                self.lru[i] = v + 1
                if mv < v:
                    mv, mi = v, i
        if mi < 0:
            mi = self.ref[0]
        self.lru[mi] = 0
        if ctype in (1, 2):
            self.ref = [self.ref[1], mi]
            if self.out_state < 4:
                self.out_state += 2
        else:
            self.out_state |= 1
        self.index = mi
        self.copy_src = self.ref[0]
        self.dif = [self.ref[0], self.ref[1]]

    def peek(self, is_end):
        if self.coding_type == 3:
            idx = self.index
        elif is_end and 0 < self.out_state < 4:
            idx = self.ref[1]
        else:
            idx = self.ref[0]
        if self.coding_type != 3:
            s = self.out_state >> 1
            if s == 0:
                return None
            if s == 1:
                return idx if is_end else None
            return idx
        return idx if self.out_state & 1 else None

    def get(self, is_end):
        idx = self.peek(is_end)
        if idx is not None:
            if self.coding_type == 3:
                self.out_state &= ~1
            else:
                self.out_state -= 2
        return idx

    def emit(self, idx):
        y, c = self.frames[idx]
        w, h = self.hsize, self.vsize  # stride = horizontal_size_value (store_frame_info)
        m = hashlib.md5()
        for r in range(h):
            m.update(bytes(y[r * w:r * w + w]))
        for r in range(h // 2):
            m.update(bytes(c[r * w:r * w + w]))
        self.out.append(m.hexdigest())

    # ---- headers (mpeg2.cpp:320-623)
    def seq_header(self, b):
        self.hsize, self.vsize = b.get(12), b.get(12)
        b.get(4 + 4 + 18 + 1 + 10 + 1)
        for i in range(2):
            if b.get(1):
                q = self.store[i]
                for k in range(64):
                    q[SCAN[0][k]] = b.get(8)
                self.qm[i] = q
            else:
                self.qm[i] = DEFAULT_INTRA if i == 0 else [16] * 64
        self.set_frames()

    def extension(self, b):
        eid = b.get(4)
        if eid == 1:
            b.get(8 + 1 + 2)
            self.hsize |= b.get(2) << 12
            self.vsize |= b.get(2) << 12
            self.mpeg2 = 1
            self.set_frames()
        elif eid == 3:
            for i in range(4):
                if b.get(1):
                    q = self.store[i]
                    for k in range(64):
                        q[self.scan[k]] = b.get(8)
                    if i < 2:
                        self.qm[i] = q
        elif eid == 8:
            f = b.get(16)
            self.r_size = [[(f >> 12) - 1, ((f >> 8) & 15) - 1], [((f >> 4) & 15) - 1, (f & 15) - 1]]
            if not self.coding_type:
                self.coding_type = (1 if (f & 0xff00) == 0xff00 else 2) if (f & 0xff) == 0xff else 3
            bits = b.get(14)
            prec, struct = (bits >> 12) & 3, (bits >> 10) & 3
            fpfd, self.conceal, self.qst = (bits >> 8) & 1, (bits >> 7) & 1, (bits >> 6) & 1
            self.intra_vlc, alt = (bits >> 5) & 1, (bits >> 4) & 1
            self.dc_scale, self.dc_max = 3 - prec, (1 << (prec + 8)) - 1
            self.scan = SCAN[alt]
            if struct in (1, 2):
                self.frame_mode = 0
            elif struct == 3:
                self.frame_mode = 3 if fpfd else 1

    # ---- macroblocks (mpeg2.cpp:834-1187, 1427-1524)
    def dc(self, b, cc):
        size = b.vlc(self.c["dc_chroma" if cc else "dc_luma"])[0]
        d = self.pred[cc]
        if size:
            diff = b.get(size)
            half = 1 << (size - 1)
            if not diff & half:
                diff = diff + 1 - 2 * half
            d += diff
            self.pred[cc] = d
            d = max(0, min(self.dc_max, d))
        return d << self.dc_scale

    def coefs(self, b, coef, idx, inter):
        """parse_coef (mpeg2.cpp:1021-1097): coefficients from scan index idx (coef[0] kept when idx > 0),
        dequantised, saturated, then mismatch control (MPEG-2) or oddification (MPEG-1)"""
        tab = self.c["dct1" if (self.intra_vlc and not inter) else "dct0"]
        qm = self.qm[1 if inter else 0]
        mismatch = coef[0] if idx else 0
        for k in range(idx, 64):
            coef[k] = 0
        while True:
            run, level = b.vlc(tab)
            if run >= 0:
                idx += run
            elif level:
                break
            else:
                idx += b.get(6)
                if self.mpeg2:
                    v = b.get(12)
                    sign = v >> 11
                    level = ((v ^ (-sign & 0xfff)) + sign) * 2 | sign
                else:
                    v = b.get(8)
                    if v & 0x7f == 0:
                        v = b.get(8) - (v & 0x80) * 2
                    elif v >= 128:
                        v -= 256
                    level = (-v * 2) | 1 if v < 0 else v * 2
            if idx >= 64:
                break
            z = self.scan[idx]
            q = qm[z] * self.qs
            t = (((level | 1) * q) >> 5) if inter else (((level >> 1) * q) >> 4)
            v = -t if level & 1 else t
            v = max(-2048, min(2047, v))
            mismatch += v
            coef[z] = v
            idx += 1
        if self.mpeg2:
            if not mismatch & 1:
                coef[63] ^= 1
        else:
            for k in range(64):
                c = coef[k]
                if c and not c & 1:
                    coef[k] = c - 1 if c > 0 else c + 1
        return coef

    def block(self, b, dcv):
        """an intra block: DC + AC (m2d_parse_intra_block_*), reconstructed samples (ClipStore)"""
        coef = [0] * 64
        coef[0] = dcv
        return idct_block(self.coefs(b, coef, 1, False))

    def inter_block(self, b):
        """m2d_parse_inter_block (mpeg2.cpp:1317-1341): a first coefficient "1s" is level 1 at scan 0,
        dequantised without saturation; the residual (AddStore adds it)"""
        coef = [0] * 64
        idx = 0
        bits = b.show(2)
        if bits & 2:
            b.get(2)
            t = ((bits | 1) * (self.qs * self.qm[1][0])) >> 5
            coef[0] = -t if bits & 1 else t
            idx = 1
        return idct_raw(self.coefs(b, coef, idx, True))

    def cur(self):
        return self.frames[self.index if self.index >= 0 else 0]

    def refframe(self, s):
        """diff_to_ref[s] (set_ptrdiff): the frame of idx_of_ref[s] at the last update; before any, the
        current frame itself (diff 0)"""
        return self.cur() if self.dif[s] is None else self.frames[self.dif[s]]

    def mb_reset(self):
        """m2d_mb_reset: intra DC and motion vector predictors"""
        r = (self.dc_max + 1) >> 1
        self.pred = [r] * 3
        self.pmv = [[[0, 0], [0, 0]], [[0, 0], [0, 0]]]

    def copy_mb(self):
        """m2d_skip_mb_P's copy of the co-located MB of diff_to_ref[0] (in place before any update)"""
        fw = self.fsize[0]
        src, dst = self.refframe(0), self.cur()
        if src is dst:
            return
        for r in range(16):
            o = (self.mb_y * 16 + r) * fw + self.mb_x * 16
            dst[0][o:o + 16] = src[0][o:o + 16]
        for r in range(8):
            o = (self.mb_y * 8 + r) * fw + self.mb_x * 16
            dst[1][o:o + 16] = src[1][o:o + 16]

    def inc_pos(self):
        x = self.mb_x + 1
        w = self.fsize[0] // 16
        if w <= x:
            iy = 0
            while True:
                x -= w
                iy += 1
                if not w < x:
                    break
            self.mb_y += iy
        self.mb_x = x

    def mb_inc(self, b):
        if b.get(1):
            return 1
        val = 0
        while True:
            v = b.vlc(self.c["mb_inc_after0"])[0]
            val += v
            if v:
                return val
            val += 33
            if b.get(1):
                return val + 1

    # ---- prediction (motioncomp.cpp:28-546; mpeg2.cpp:1277-1308, 740-808)
    def predict(self, ref, cur, src, dst, stride, mvx, mvy, h, chroma, avg):
        """m2d_motion_compensation_{luma,chroma}[_add]: 16 bytes x h rows at byte offset dst of plane cur
        (row stride `stride`) from plane ref at byte offset src moved by the vector (half samples; chroma:
        the vector halved toward zero, Cb / Cr interleaved); avg: AveStore (the second direction)"""
        W = self.fsize[0]
        if chroma:
            mvx, mvy = int(mvx / 2), int(mvy / 2)
            dx, gap = mvx & ~1, 2
        else:
            dx, gap = mvx >> 1, 1
        hx, hy = mvx & 1, mvy & 1
        s0 = src + stride * (mvy >> 1) + dx
        col = src % W + dx
        assert 0 <= col and col + 15 + gap * hx < W and s0 >= 0 and s0 + (h - 1 + hy) * stride + 15 + gap * hx < len(ref), \
            "prediction outside the reference frame (the reference reads outside its buffers: UB)"
        for r in range(h):
            a0 = s0 + r * stride
            b0 = a0 + stride
            d0 = dst + r * stride
            for c in range(16):
                a = ref[a0 + c]
                if hx and hy:
                    v = (a + ref[a0 + c + gap] + ref[b0 + c] + ref[b0 + c + gap] + 2) >> 2
                elif hx:
                    v = (a + ref[a0 + c + gap] + 1) >> 1
                elif hy:
                    v = (a + ref[b0 + c] + 1) >> 1
                else:
                    v = a
                cur[d0 + c] = (cur[d0 + c] + v + 1) >> 1 if avg else v

    def motion_comp(self, s, avg, mvxy, ref_field):
        """m2d_motion_comp: one direction of the current MB (frame: one vector; field: one per parity,
        from the selected reference field, into the lines of that parity)"""
        W = self.fsize[0]
        ref, cur = self.refframe(s), self.cur()
        lo = self.mb_y * 16 * W + self.mb_x * 16
        co = self.mb_y * 8 * W + self.mb_x * 16
        if self.mt[0] == 1:
            self.predict(ref[0], cur[0], lo, lo, W, mvxy[0], mvxy[1], 16, False, avg)
            self.predict(ref[1], cur[1], co, co, W, mvxy[0], mvxy[1], 8, True, avg)
        else:
            for i in range(2):
                so = W if ref_field[i] else 0
                mx, my = mvxy[2 * i], mvxy[2 * i + 1]
                self.predict(ref[0], cur[0], lo + so, lo + i * W, 2 * W, mx, my, 8, False, avg)
                self.predict(ref[1], cur[1], co + so, co + i * W, 2 * W, mx, my, 4, True, avg)

    def skip_b(self, inc):
        """m2d_skip_mb_B: the skipped MBs predicted like the last coded one — its directions, frame
        prediction with the first vector predictor of each"""
        d = self.mb_type & 3
        bi = d == 3
        one = 0 if bi else d >> 1
        W = self.fsize[0]
        for _ in range(inc - 1):
            self.inc_pos()
            lo = self.mb_y * 16 * W + self.mb_x * 16
            co = self.mb_y * 8 * W + self.mb_x * 16
            cur = self.cur()
            dirs = [(0, False), (1, True)] if bi else [(one, False)]
            for s, avg in dirs:
                ref = self.refframe(s)
                mx, my = self.pmv[s][0]
                self.predict(ref[0], cur[0], lo, lo, W, mx, my, 16, False, avg)
                self.predict(ref[1], cur[1], co, co, W, mx, my, 8, True, avg)

    # ---- motion vectors (mpeg2.cpp:1189-1275)
    def one_mv(self, b, pm, comp, r, is_field):
        p = pm[comp]
        if b.get(1) == 0:
            code = b.vlc(self.c["motion_code"])[0]
            res = 1 + b.get(r) if r > 0 else 1
            mv = ((code - 1) << r) + res if code >= 0 else ((code + 1) << r) - res
            mv += p >> is_field
            lim = 16 << r
            if mv < -lim:
                mv += 2 * lim
            elif mv >= lim:
                mv -= 2 * lim
        else:
            mv = p >> is_field
        pm[comp] = mv << is_field
        return mv

    def motion_vectors(self, b, s):
        count, fmt_field, dmv = self.mt
        pm = self.pmv[s]
        rs = self.r_size[s]
        if count == 1:
            if fmt_field and not dmv:
                b.get(1)  # motion_vertical_field_select (not used)
            mx = self.one_mv(b, pm[0], 0, rs[0], 0)
            if dmv and b.get(1):
                b.get(1)
            my = self.one_mv(b, pm[0], 1, rs[1], 1 if fmt_field else 0)
            if dmv and b.get(1):
                b.get(1)
            pm[1][0], pm[1][1] = pm[0][0], pm[0][1]
            return [mx, my], None
        out, rf = [], []
        for i in range(2):
            rf.append(b.get(1))
            out.append(self.one_mv(b, pm[i], 0, rs[0], 0))
            out.append(self.one_mv(b, pm[i], 1, rs[1], 1))
        return out, rf

    # ---- macroblocks (mpeg2.cpp:834-872, 1136-1187, 1343-1417)
    MT = [[(2, 1, 0), (2, 1, 0), (1, 0, 0), (1, 1, 1)], [(1, 1, 0), (1, 1, 0), (2, 1, 0), (1, 1, 1)]]

    def mb_modes(self, b):
        ct = self.coding_type
        if ct == 2:
            t = b.vlc(self.c["mb_type_p"])[0]
        elif ct == 3:
            t = b.vlc(self.c["mb_type_b"])[0]
        elif b.show(1):
            b.get(1)
            t = 4
        else:
            b.get(2)
            t = 20
        fm = self.frame_mode
        if t & 3:
            if fm & 1:
                self.mt = self.MT[0][b.get(2) if fm == 1 else 2]
            else:
                self.mt = self.MT[1][b.get(2)]
        else:
            k = 1 if fm == 0 else 0
            self.mt = self.MT[k][2 - k]
        if fm == 1 and t & 12:
            self.dct_type = b.get(1)
        else:
            self.dct_type = 0 if fm else 1
        return t

    def put_block(self, px, i, add):
        """m2d_idct_{intra,inter}_{luma,chroma}: block i of the current MB (LUMA_BLOCK_OFFSET, stride
        W << dct_type; chroma interleaved), ClipStore / AddStore"""
        f = self.cur()
        fw = self.fsize[0]
        if i < 4:
            plane = f[0]
            bx = self.mb_x * 16 + (i & 1) * 8
            rows = [self.mb_y * 16 + ((i >> 1) + 2 * r if self.dct_type else (i >> 1) * 8 + r) for r in range(8)]
            offs = [[y * fw + bx + k for k in range(8)] for y in rows]
        else:
            plane = f[1]
            offs = [[(self.mb_y * 8 + r) * fw + self.mb_x * 16 + 2 * k + (i - 4) for k in range(8)] for r in range(8)]
        for r in range(8):
            for k in range(8):
                o = offs[r][k]
                v = plane[o] + px[r][k] if add else px[r][k]
                assert -256 <= v <= 767, "CLIP255C argument outside the reference table (UB)"
                plane[o] = 0 if v < 0 else 255 if v > 255 else v

    def macroblock(self, b):
        """m2d_parse_macroblock"""
        prev_intra = self.mb_type & 4
        t = self.mb_modes(b)
        self.mb_type = t
        if t & 4:
            if not prev_intra:
                self.pred = [(self.dc_max + 1) >> 1] * 3
            if t & 16:
                self.qs = Q_SCALE[self.qst][b.get(5)]
            if self.conceal:
                self.motion_vectors(b, 0)
                b.get(1)
            for i in range(4):
                self.put_block(self.block(b, self.dc(b, 0)), i, False)
            for cc in range(2):
                self.put_block(self.block(b, self.dc(b, 1 + cc)), 4 + cc, False)
            return
        if prev_intra:
            self.pmv = [[[0, 0], [0, 0]], [[0, 0], [0, 0]]]
        if t & 16:
            self.qs = Q_SCALE[self.qst][b.get(5)]
        if t & 3:
            fwd = t & 1
            if fwd:
                mvxy, rf = self.motion_vectors(b, 0)
                self.motion_comp(0, False, mvxy, rf)
            if t & 2:
                mvxy, rf = self.motion_vectors(b, 1)
                self.motion_comp(1, fwd != 0, mvxy, rf)
        else:  # m2d_skip_mb_P(mb, 0)
            self.copy_mb()
            self.mb_reset()
        if t & 8:
            cbp = b.vlc(self.c["cbp"])[0]
            for i in range(6):
                if cbp & (1 << (5 - i)):
                    self.put_block(self.inter_block(b), i, True)

    def slice(self, b, code):
        """m2d_read_slice + m2d_decode_macroblocks (mpeg2.cpp:625-660, 1502-1524)"""
        vpos = code - 1
        self.qs = Q_SCALE[self.qst][b.get(5)]
        if vpos == 0:
            self.update_frames(self.coding_type)
        mbh = self.fsize[1] // 16
        fw = self.fsize[0]
        if mbh <= vpos:
            return 0
        if 1 < vpos - self.mb_y:  # m2d_copy_slice
            src, dst = self.refframe(0), self.cur()
            if src is not dst:
                lo, n = (self.mb_y + 1) * 16 * fw, fw * (vpos - self.mb_y - 1) * 16
                dst[0][lo:lo + n] = src[0][lo:lo + n]
                dst[1][lo // 2:lo // 2 + n // 2] = src[1][lo // 2:lo // 2 + n // 2]
        self.mb_x, self.mb_y = -1, vpos
        if b.get(1):
            b.get(8)
            while b.get(1):
                b.get(8)
        self.mb_reset()
        while True:
            inc = self.mb_inc(b)
            if inc > 1:
                if self.coding_type == 3:
                    self.skip_b(inc)
                else:  # m2d_skip_mb_P (also the I table's entry)
                    for _ in range(inc - 1):
                        self.inc_pos()
                        self.copy_mb()
                    self.mb_reset()
            self.inc_pos()
            self.macroblock(b)
            if (self.mb_y == mbh - 1 and fw // 16 - 1 <= self.mb_x) or mbh <= self.mb_y:
                self.mb_x, self.mb_y = -1, 0
                return 1
            if b.show(23) == 0:
                return 0

    def decode_picture(self, it):
        """m2d_decode_data: 1 per picture, -1 at the end of the data"""
        self.coding_type = 0
        for code, payload in it:
            b = Bits(payload)
            if code == 0:
                b.get(10)
                self.coding_type = b.get(3)
                b.get(16)
                if self.coding_type not in (1, 2, 3):
                    raise ValueError("D pictures")
                self.mb_x, self.mb_y = -1, 0
                if self.coding_type in (2, 3):  # full_pel + f_code as one value - 1 (mpeg2.cpp:608-618)
                    r = b.get(4) - 1
                    self.r_size[0] = [r, r]
                    if self.coding_type == 3:
                        r = b.get(4) - 1
                        self.r_size[1] = [r, r]
            elif code < 0xb0:
                try:
                    if self.slice(b, code) == 1:
                        return 1
                except ValueError:
                    pass  # undefined code: the reference abandons the slice (longjmp)
            elif code == 0xb3:
                self.seq_header(b)
            elif code == 0xb5:
                self.extension(b)
        return -1


def decode(data):
    """MD5 per output frame, in output order, as `h264dec -O` (M2Decoder::decode, no emptify)."""
    d = Decoder()
    it = iter(units(data))
    while True:
        while True:
            idx = d.peek(0)
            if idx is not None:
                break
            if d.decode_picture(it) < 0:
                while True:
                    idx = d.get(1)
                    if idx is None:
                        return d.out
                    d.emit(idx)
        d.emit(d.get(0))
        if d.decode_picture(it) < 0:
            while True:
                idx = d.get(1)
                if idx is None:
                    return d.out
                d.emit(idx)
