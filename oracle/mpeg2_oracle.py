"""CPU restatement of the reference's MPEG-1/2 intra decode path — TEST INFRASTRUCTURE ONLY.

Only tests/ (and tools/make_m2v_goldens.py) use this module: it is the checker of the product's
MPEG-2 decoder (m2dec_amd/csrc/host/mpeg2_dec.c, behind m2d_func), never part of it.

It follows /root/reference/src/lib/mpeg2.cpp + idct.cpp + src/app/m2decoder.h step by step, written
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
    """idct.cpp:69-236 (rows, stored as int16) + 286-358 (columns, (x + 8192) >> 14)."""
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
            v = col[r]
            assert -256 <= v <= 767, "CLIP255C argument outside the reference table (UB)"
            out[r][k] = 0 if v < 0 else 255 if v > 255 else v
    return out


class Decoder:
    """m2d_context + M2Decoder (outbuf 0: 3 frames) for intra pictures."""

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
        self.prev_intra = 0
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
            self.r_size = [(f >> 12) - 1, ((f >> 8) & 15) - 1]
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

    def block(self, b, dcv):
        coef = [0] * 64
        coef[0] = dcv
        tab = self.c["dct1" if self.intra_vlc else "dct0"]
        mismatch, idx = dcv, 1
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
            t = ((level >> 1) * (self.qm[0][z] * self.qs)) >> 4
            v = -t if level & 1 else t
            v = max(-2048, min(2047, v))
            mismatch += v
            coef[z] = v
            idx += 1
        if self.mpeg2:
            if not mismatch & 1:
                coef[63] ^= 1
        else:
            coef = [(c - 1 if c > 0 else c + 1) if c and not c & 1 else c for c in coef]
        return idct_block(coef)

    def cur(self):
        return self.frames[self.index if self.index >= 0 else 0]

    def copy_mb(self):
        if self.copy_src < 0:
            return
        fw = self.fsize[0]
        src, dst = self.frames[self.copy_src], self.cur()
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

    def one_mv(self, b, r):
        if b.get(1) == 0:
            b.vlc(self.c["motion_code"])
            if r > 0:
                b.get(r)

    def slice(self, b, code):
        vpos = code - 1
        self.qs = Q_SCALE[self.qst][b.get(5)]
        if vpos == 0:
            self.update_frames(self.coding_type)
        mbh = self.fsize[1] // 16
        fw = self.fsize[0]
        if mbh <= vpos:
            return 0
        if 1 < vpos - self.mb_y and self.copy_src >= 0:
            src, dst = self.frames[self.copy_src], self.cur()
            if src is not dst:
                lo, n = (self.mb_y + 1) * 16 * fw, fw * (vpos - self.mb_y - 1) * 16
                dst[0][lo:lo + n] = src[0][lo:lo + n]
                dst[1][lo // 2:lo // 2 + n // 2] = src[1][lo // 2:lo // 2 + n // 2]
        self.mb_x, self.mb_y = -1, vpos
        if b.get(1):
            b.get(8)
            while b.get(1):
                b.get(8)
        reset = (self.dc_max + 1) >> 1
        self.pred = [reset] * 3
        while True:
            inc = self.mb_inc(b)
            if inc > 1:
                for _ in range(inc - 1):
                    self.inc_pos()
                    self.copy_mb()
                self.pred = [reset] * 3
            self.inc_pos()
            quant = 0
            if b.show(1):
                b.get(1)
            else:
                b.get(2)
                quant = 1
            if not self.prev_intra:
                self.pred = [reset] * 3
            self.prev_intra = 1
            if self.frame_mode == 1:
                dct_type = b.get(1)
            else:
                dct_type = 0 if self.frame_mode else 1
            if quant:
                self.qs = Q_SCALE[self.qst][b.get(5)]
            if self.conceal:
                if self.frame_mode == 0:
                    b.get(1)
                self.one_mv(b, self.r_size[0])
                self.one_mv(b, self.r_size[1])
                b.get(1)
            f = self.cur()
            for i in range(4):
                px = self.block(b, self.dc(b, 0))
                bx = self.mb_x * 16 + (i & 1) * 8
                for r in range(8):
                    y = self.mb_y * 16 + ((i >> 1) + 2 * r if dct_type else (i >> 1) * 8 + r)
                    f[0][y * fw + bx:y * fw + bx + 8] = bytes(px[r])
            for cc in range(2):
                px = self.block(b, self.dc(b, 1 + cc))
                for r in range(8):
                    y = self.mb_y * 8 + r
                    for k in range(8):
                        f[1][y * fw + self.mb_x * 16 + 2 * k + cc] = px[r][k]
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
                if self.coding_type != 1:
                    raise ValueError("only intra pictures")
                self.mb_x, self.mb_y = -1, 0
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
