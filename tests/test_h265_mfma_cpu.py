"""The int8-MFMA inverse DCT of the H.265 CTU kernels (m2dec_amd/csrc/hip/h265_mfma.h), emulated on the CPU slot
by slot: each int16 operand split into hi = v >> 8 and lo = (v & 255) - 128, the A / B fragments built with the
k-assignment the device code uses (32 x 32: k = 16 h + j in pass 1, the accumulator row of register j in pass 2;
16 x 16: k = 4 q + j, j < 4), the accumulator read back through the gfx950 C/D map — against the reference's
two-pass integer transform (h265.cpp:2142 dispatch; spec 8.6.4.2).  The hardware lane maps themselves are
checked on the GPU by tools/mfma_idct_probe.hip (tests/test_gpu_h265.py::test_mfma_idct_probe)."""
import numpy as np

COS = [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
       61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0]


def t32(k, n):
    m, sign = ((2 * n + 1) * k) & 127, 1
    if m > 64:
        m = 128 - m
    if m > 32:
        m, sign = 64 - m, -1
    return sign * COS[m]


def sat16(v):
    return np.clip(v, -32768, 32767)


def reference(c, n):
    t = np.array([[t32(k * 32 // n, x) for x in range(n)] for k in range(n)], dtype=np.int64)
    g = sat16((t.T @ c.astype(np.int64) + 64) >> 7)       # g[y][x] = sum_k T[k][y] C[k][x]
    return sat16((g @ t + 2048) >> 12)                    # r[y][x] = sum_k T[k][x] g[y][k]


def acc_row(n, i, lane):
    return (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5) if n == 32 else 4 * (lane >> 4) + i


def split(v):
    v = np.asarray(v, dtype=np.int64)
    hi, lo = v >> 8, (v & 255) - 128
    assert ((hi >= -128) & (hi <= 127) & (lo >= -128) & (lo <= 127)).all()
    assert (256 * hi + lo + 128 == v).all()
    return hi, lo


def mfma(a_frag, b_frag, n, kslot):
    """D[row][col] = sum over the lane groups g and elements j of A(row, g)[j] * B(col, g)[j]."""
    groups = 64 // n
    d = np.zeros((n, n), dtype=np.int64)
    for g in range(groups):
        for j in range(kslot):
            a = np.array([a_frag[r + n * g][j] for r in range(n)], dtype=np.int64)
            b = np.array([b_frag[c + n * g][j] for c in range(n)], dtype=np.int64)
            d += np.outer(a, b)
    return d


def emulate(c, n):
    groups, kslot = 64 // n, (16 if n == 32 else 4)
    k1 = lambda lane, j: 16 * (lane >> 5) + j if n == 32 else 4 * (lane >> 4) + j  # noqa: E731
    t = lambda k, x: t32(k * 32 // n, x)  # noqa: E731
    colsum = [sum(t(k, x) for k in range(n)) for x in range(n)]
    lanes = range(64)
    # pass 1: A[x][k] = C[k][x] (lane = x + n g), B[k][y] = T[k][y]
    av = [[c[k1(l, j), l % n] for j in range(kslot)] for l in lanes]
    ahi = [split(r)[0] for r in av]
    alo = [split(r)[1] for r in av]
    b1 = [[t(k1(l, j), l % n) for j in range(kslot)] for l in lanes]
    d = 256 * mfma(ahi, b1, n, kslot) + mfma(alo, b1, n, kslot) + 128 * np.array(colsum)[None, :]
    g = sat16((d + 64) >> 7)                              # g = D, D[x][y] = G[y][x]
    # pass 2: lane (y = col, group) element j = the accumulator register j = G[y][x = acc_row(j)]
    gv = [[g[acc_row(n, j, l), l % n] for j in range(kslot)] for l in lanes]
    b2 = [[t(acc_row(n, j, l), l % n) for j in range(kslot)] for l in lanes]
    r = 256 * mfma([split(x)[0] for x in gv], b2, n, kslot) + mfma([split(x)[1] for x in gv], b2, n, kslot) \
        + 128 * np.array(colsum)[None, :]
    assert groups * kslot == n
    return sat16((r + 2048) >> 12)


def test_split_identity_covers_int16():
    hi, lo = split(np.arange(-32768, 32768))
    assert hi.min() == -128 and hi.max() == 127 and lo.min() == -128 and lo.max() == 127


def test_emulated_mfma_idct_matches_reference():
    rng = np.random.default_rng(7)
    for n in (16, 32):
        for kind in range(4):
            if kind == 0:
                c = np.where(rng.random((n, n)) < 0.15, rng.integers(-256, 256, (n, n)), 0)
            elif kind == 1:
                c = rng.integers(-32768, 32768, (n, n))
            elif kind == 2:
                c = np.where(rng.random((n, n)) < 0.3, np.where(rng.random((n, n)) < 0.5, 32767, -32768), 0)
            else:
                c = np.zeros((n, n), dtype=np.int64)
                c[0, 0], c[0, 1], c[1, 0] = rng.integers(-2048, 2048, 3)
            c = c.astype(np.int64)
            assert (emulate(c, n) == reference(c, n)).all(), (n, kind)
