#!/usr/bin/env python3
"""Generate m2dec_amd/csrc/hip/intra_tables.h: table-driven 4x4 / 8x8 intra prediction.

Every directional intra sample (spec 8.3.1.2 / 8.3.2.2; the reference's pred4x4_* / pred8x8l_*,
h264.cpp:2510-2997 and 3301-3929) is (w0*N[i0] + w1*N[i1] + w2*N[i2] + rnd) >> s over the block's
neighbour array N, rnd = (1 << s) >> 1.  The tables hold, per (mode, x, y), the three neighbour
indices, weights and the shift; DC (mode 2) is computed separately.  The formulas below restate
pred4_px / pred8_px of recon_hip.hip branch for branch, and main() checks the tables against them
on random neighbours before writing the header.

4x4 neighbour index: 0 = top-left, 1..8 = top P0..P7 (P4..P7 = top-right), 9..12 = left L0..L3.
8x8 neighbour index (filtered): 0..15 = top pt0..pt15, 16..23 = left lf0..lf7, 24 = top-left.
"""
import os
import random
import sys

TL4, P4, L4 = 0, 1, 9
LW = 25  # luma context row stride (recon_hip.hip)
TL8, PT8, LF8 = 24, 0, 16


def taps4(mode, x, y):
    P = lambda i: P4 + i
    L = lambda i: L4 + i
    PP = lambda i: TL4 if i < 0 else P(i)
    LL = lambda i: TL4 if i < 0 else L(i)
    if mode == 0:
        return [(P(x), 1)], 0
    if mode == 1:
        return [(L(y), 1)], 0
    if mode == 3:
        if x == 3 and y == 3:
            return [(P(6), 1), (P(7), 3)], 2
        return [(P(x + y), 1), (P(x + y + 1), 2), (P(x + y + 2), 1)], 2
    if mode == 4:
        if x > y:
            return [(PP(x - y - 2), 1), (PP(x - y - 1), 2), (P(x - y), 1)], 2
        if x < y:
            return [(LL(y - x - 2), 1), (LL(y - x - 1), 2), (L(y - x), 1)], 2
        return [(P(0), 1), (TL4, 2), (L(0), 1)], 2
    if mode == 5:
        z, i = 2 * x - y, x - (y >> 1)
        if z >= 0 and not (z & 1):
            return [(PP(i - 1), 1), (P(i), 1)], 1
        if z >= 0:
            return [(PP(i - 2), 1), (PP(i - 1), 2), (P(i), 1)], 2
        if z == -1:
            return [(L(0), 1), (TL4, 2), (P(0), 1)], 2
        return [(L(y - 1), 1), (L(y - 2), 2), (LL(y - 3), 1)], 2
    if mode == 6:
        z, i = 2 * y - x, y - (x >> 1)
        if z >= 0 and not (z & 1):
            return [(LL(i - 1), 1), (L(i), 1)], 1
        if z >= 0:
            return [(LL(i - 2), 1), (LL(i - 1), 2), (L(i), 1)], 2
        if z == -1:
            return [(L(0), 1), (TL4, 2), (P(0), 1)], 2
        return [(P(x - 1), 1), (P(x - 2), 2), (PP(x - 3), 1)], 2
    if mode == 7:
        i = x + (y >> 1)
        if not (y & 1):
            return [(P(i), 1), (P(i + 1), 1)], 1
        return [(P(i), 1), (P(i + 1), 2), (P(i + 2), 1)], 2
    if mode == 8:
        z, i = x + 2 * y, y + (x >> 1)
        if z > 5:
            return [(L(3), 1)], 0
        if z == 5:
            return [(L(2), 1), (L(3), 3)], 2
        if not (z & 1):
            return [(L(i), 1), (L(i + 1), 1)], 1
        return [(L(i), 1), (L(i + 1), 2), (L(i + 2), 1)], 2
    raise ValueError(mode)


def taps8(mode, x, y):
    pt = lambda i: PT8 + i
    lf = lambda i: LF8 + i
    PT = lambda i: TL8 if i < 0 else pt(i)
    LF = lambda i: TL8 if i < 0 else lf(i)
    if mode == 0:
        return [(pt(x), 1)], 0
    if mode == 1:
        return [(lf(y), 1)], 0
    if mode == 3:
        if x == 7 and y == 7:
            return [(pt(14), 1), (pt(15), 3)], 2
        return [(pt(x + y), 1), (pt(x + y + 1), 2), (pt(x + y + 2), 1)], 2
    if mode == 4:
        if x > y:
            return [(PT(x - y - 2), 1), (PT(x - y - 1), 2), (pt(x - y), 1)], 2
        if x < y:
            return [(LF(y - x - 2), 1), (LF(y - x - 1), 2), (lf(y - x), 1)], 2
        return [(pt(0), 1), (TL8, 2), (lf(0), 1)], 2
    if mode == 5:
        z, i = 2 * x - y, x - (y >> 1)
        if z >= 0 and not (z & 1):
            return [(PT(i - 1), 1), (pt(i), 1)], 1
        if z >= 0:
            return [(PT(i - 2), 1), (PT(i - 1), 2), (pt(i), 1)], 2
        if z == -1:
            return [(lf(0), 1), (TL8, 2), (pt(0), 1)], 2
        return [(LF(y - 2 * x - 1), 1), (LF(y - 2 * x - 2), 2), (LF(y - 2 * x - 3), 1)], 2
    if mode == 6:
        z, i = 2 * y - x, y - (x >> 1)
        if z >= 0 and not (z & 1):
            return [(LF(i - 1), 1), (lf(i), 1)], 1
        if z >= 0:
            return [(LF(i - 2), 1), (LF(i - 1), 2), (lf(i), 1)], 2
        if z == -1:
            return [(lf(0), 1), (TL8, 2), (pt(0), 1)], 2
        return [(PT(x - 2 * y - 1), 1), (PT(x - 2 * y - 2), 2), (PT(x - 2 * y - 3), 1)], 2
    if mode == 7:
        i = x + (y >> 1)
        if not (y & 1):
            return [(pt(i), 1), (pt(i + 1), 1)], 1
        return [(pt(i), 1), (pt(i + 1), 2), (pt(i + 2), 1)], 2
    if mode == 8:
        z, i = x + 2 * y, y + (x >> 1)
        if z > 13:
            return [(lf(7), 1)], 0
        if z == 13:
            return [(lf(6), 1), (lf(7), 3)], 2
        if not (z & 1):
            return [(lf(i), 1), (lf(i + 1), 1)], 1
        return [(lf(i), 1), (lf(i + 1), 2), (lf(i + 2), 1)], 2
    raise ValueError(mode)


def pack(taps, s, bits):
    taps = list(taps) + [(taps[0][0], 0)] * (3 - len(taps))
    w = 0
    for k, (i, wt) in enumerate(taps):
        assert 0 <= i < (1 << bits) and 0 <= wt <= 3
        w |= i << (bits * k)
        w |= wt << (3 * bits + 2 * k)
    return w | (s << (3 * bits + 6))


def unpack(word, bits):
    m = (1 << bits) - 1
    idx = [(word >> (bits * k)) & m for k in range(3)]
    wts = [(word >> (3 * bits + 2 * k)) & 3 for k in range(3)]
    s = (word >> (3 * bits + 6)) & 3
    return idx, wts, s


def evaluate(word, bits, N):
    idx, wts, s = unpack(word, bits)
    return (sum(w * N[i] for i, w in zip(idx, wts)) + ((1 << s) >> 1)) >> s


def main():
    t4 = [[pack(*taps4(m, p & 3, p >> 2), 4) if m != 2 else 0 for p in range(16)] for m in range(9)]
    t8 = [[pack(*taps8(m, p & 7, p >> 3), 5) if m != 2 else 0 for p in range(64)] for m in range(9)]
    rnd = random.Random(1)
    for _ in range(200):  # the packed tables reproduce the formulas exactly
        N4 = [rnd.randrange(256) for _ in range(13)]
        N8 = [rnd.randrange(256) for _ in range(25)]
        for m in range(9):
            if m == 2:
                continue
            for p in range(16):
                taps, s = taps4(m, p & 3, p >> 2)
                assert evaluate(t4[m][p], 4, N4) == (sum(w * N4[i] for i, w in taps) + ((1 << s) >> 1)) >> s
            for p in range(64):
                taps, s = taps8(m, p & 7, p >> 3)
                assert evaluate(t8[m][p], 5, N8) == (sum(w * N8[i] for i, w in taps) + ((1 << s) >> 1)) >> s
    # offset form of the 4x4 table over the luma context L[17][LW] (see recon_hip.hip IntraLDS)
    def off4(i, tr):
        if i == 0:
            return 0
        if i <= 8:
            return min(i, 4) if tr else i
        return (i - 8) * LW
    t4o = [[[0] * 16 for _ in range(9)] for _ in range(2)]
    for tr in range(2):
        for m in range(9):
            if m == 2:
                continue
            for p in range(16):
                idx, wts, sh = unpack(t4[m][p], 4)
                w = sum(off4(i, tr) << (8 * k) for k, i in enumerate(idx))
                w |= sum(wt << (24 + 2 * k) for k, wt in enumerate(wts)) | (sh << 30)
                t4o[tr][m][p] = w
    for _ in range(200):  # the offset form reads the same samples out of a context array
        ctx = [rnd.randrange(256) for _ in range(5 * LW)]
        for tr in range(2):
            N4 = [ctx[0]] + [ctx[min(i, 4) if tr else i] for i in range(1, 9)] + [ctx[k * LW] for k in range(1, 5)]
            for m in range(9):
                if m == 2:
                    continue
                for p in range(16):
                    w = t4o[tr][m][p]
                    o = [(w >> (8 * k)) & 255 for k in range(3)]
                    wt = [(w >> (24 + 2 * k)) & 3 for k in range(3)]
                    sh = w >> 30
                    got = (sum(a * ctx[b] for a, b in zip(wt, o)) + ((1 << sh) >> 1)) >> sh
                    assert got == evaluate(t4[m][p], 4, N4)
    REQ4 = [2, 1, 0, 0, 3, 3, 3, 0, 1]
    REQ8 = [2, 1, 0, 2, 11, 11, 11, 2, 1]
    out = ["/* Generated by tools/gen_intra_tables.py -- do not edit.  Table-driven 4x4 / 8x8 intra prediction:",
           " * word = idx0 | idx1 << B | idx2 << 2B | w0 << 3B | w1 << 3B+2 | w2 << 3B+4 | shift << 3B+6",
           " * (B = 4 for 4x4, 5 for 8x8); sample = (w0 N[idx0] + w1 N[idx1] + w2 N[idx2] + rnd) >> shift. */",
           "#pragma once",
           "#include <stdint.h>",
           "/* neighbour availability a mode needs: 4x4 avail bits (1 left, 2 top), 2 bits per mode; 8x8 (1 left,",
           " * 2 top, 8 top-left), 4 bits per mode.  Packed immediates: a per-lane index into a __constant__",
           " * array compiles to a vector memory load on the block chain. */",
           f"#define M2D_REQ4_PACKED 0x{sum(v << (2 * i) for i, v in enumerate(REQ4)):x}u",
           f"#define M2D_REQ8_PACKED 0x{sum(v << (4 * i) for i, v in enumerate(REQ8)):x}ull",
           "__device__ __forceinline__ int d_req4(int mode) { return (int)((M2D_REQ4_PACKED >> (2 * mode)) & 3u); }",
           "__device__ __forceinline__ int d_req8(int mode) { return (int)((M2D_REQ8_PACKED >> (4 * mode)) & 15u); }",
           "/* 4x4 in LDS-offset form: c_ipred4o[tr][mode][pixel] = off0 | off1 << 8 | off2 << 16 | w0 << 24 |",
           " * w1 << 26 | w2 << 28 | shift << 30, offsets from the block's top-left neighbour in the luma context",
           f" * (row stride LW = {LW}); tr = 1: top-right unavailable (P4..P7 read P3). */",
           f"#define M2D_IPRED4O_LW {LW}",
           "__constant__ static const uint32_t c_ipred4o[2][9][16] = {"]
    for tr in range(2):
        out.append("\t{")
        for m in range(9):
            out.append("\t\t{" + ", ".join(f"0x{w:08x}" for w in t4o[tr][m]) + "},")
        out.append("\t},")
    out.append("};")
    out.append("__constant__ static const uint32_t c_ipred8[9][64] = {")
    for m in range(9):
        out.append("\t{" + ", ".join(f"0x{w:07x}" for w in t8[m]) + "},")
    out.append("};")
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "m2dec_amd", "csrc", "hip", "intra_tables.h")
    open(path, "w").write("\n".join(out) + "\n")
    print("wrote", path)


if __name__ == "__main__":
    sys.exit(main())
