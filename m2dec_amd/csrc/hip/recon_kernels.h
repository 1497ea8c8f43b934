/*
 * Device-side building blocks of the gfx950 reconstruction kernels.  Each helper restates one
 * reference routine (paths under /root/reference/src/lib) on sample arrays in registers / LDS;
 * the CPU oracle (oracle/recon_oracle.c) restates the same routines and is the parity checker.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "m2d_recon.h"

__device__ __forceinline__ int d_clip255(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int d_clip3(int lo, int hi, int v) { return min(max(v, lo), hi); }
__device__ __forceinline__ int d_sat16(int v) { return min(max(v, -32768), 32767); }

/* 4x4 block index (decoding order, spec 6.4.3) <-> position in the MB, as bit arithmetic (a per-lane
 * index into a __constant__ table compiles to a vector memory load) */
__device__ __forceinline__ int d_blk_x(int blk) { return (blk & 1) | ((blk >> 1) & 2); }
__device__ __forceinline__ int d_blk_y(int blk) { return ((blk >> 1) & 1) | ((blk >> 2) & 2); }
__device__ __forceinline__ int d_rast2blk(int lb) /* raster 4x4 position (ry * 4 + rx) -> block index */
{
	const int rx = lb & 3, ry = lb >> 2;
	return (rx & 1) | ((ry & 1) << 1) | ((rx & 2) << 1) | ((ry & 2) << 2);
}
__constant__ static const uint8_t c_alpha[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28,
                                                 32, 36, 40, 45, 50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
__constant__ static const uint8_t c_beta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8,
                                                9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
__constant__ static const uint8_t c_tc0[52][3] = {
	{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
	{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1},
	{0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2},
	{1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6},
	{4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20},
	{11, 15, 23}, {13, 17, 25}};

/* ---------------------------------------------------------------- dequantisation (h264.cpp:964-1054) */
/* dequantisation scale LevelScale(qp % 6, x, y) << (qp / 6) (spec 8.5.9).  The norm columns are
 * packed into immediates (6 x 5 / 6 bits, one per position class) so that a per-lane class never
 * turns into a per-lane constant-memory load (norm4 / norm8 of the spec, columns = classes). */
__device__ __forceinline__ int d_scale4(int qp, int x, int y)
{
	const uint32_t w0 = 0x2507356au, w1 = 0x3b9bd250u, w2 = 0x2f4941cdu;
	const uint32_t w = (((x | y) & 1) == 0) ? w0 : (((x & y) & 1) ? w1 : w2);
	return (int)((w >> (5 * (qp % 6))) & 31) << (qp / 6);
}

__device__ __forceinline__ int d_scale8(int qp, int x, int y)
{
	const uint64_t w0 = 0x000000092071a594ull, w1 = 0x000000081c6574d2ull, w2 = 0x0000000eb3b6a8e0ull;
	const uint64_t w3 = 0x000000089e698553ull, w4 = 0x0000000ba88e1719ull, w5 = 0x0000000ae685f698ull;
	const int x3 = x & 3, y3 = y & 3;
	uint64_t w;
	if (x3 == 0 && y3 == 0) w = w0;
	else if ((x & 1) && (y & 1)) w = w1;
	else if (x3 == 2 && y3 == 2) w = w2;
	else if ((x3 == 0 && (y & 1)) || ((x & 1) && y3 == 0)) w = w3;
	else if ((x3 == 0 && y3 == 2) || (x3 == 2 && y3 == 0)) w = w4;
	else w = w5;
	const int v = (int)((w >> (6 * (qp % 6))) & 63);
	const int sh = qp / 6 - 2;
	return sh >= 0 ? v << sh : v >> (-sh);
}

/* ---------------------------------------------------------------- 1-D inverse transforms (spec 8.5.12) */
__device__ __forceinline__ void d_idct4_1d(int &a, int &b, int &c, int &d)
{
	int e0 = a + c, e1 = a - c, e2 = (b >> 1) - d, e3 = b + (d >> 1);
	a = e0 + e3;
	b = e1 + e2;
	c = e1 - e2;
	d = e0 - e3;
}

__device__ __forceinline__ void d_idct8_1d(int *s)
{
	int a0 = s[0] + s[4], a4 = s[0] - s[4];
	int a2 = (s[2] >> 1) - s[6], a6 = s[2] + (s[6] >> 1);
	int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
	int a1 = -s[3] + s[5] - s[7] - (s[7] >> 1);
	int a3 = s[1] + s[7] - s[3] - (s[3] >> 1);
	int a5 = -s[1] + s[7] + s[5] + (s[5] >> 1);
	int a7 = s[3] + s[5] + s[1] + (s[1] >> 1);
	int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2);
	int b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
	s[0] = b0 + b7;
	s[1] = b2 + b5;
	s[2] = b4 + b3;
	s[3] = b6 + b1;
	s[4] = b6 - b1;
	s[5] = b4 - b3;
	s[6] = b2 - b5;
	s[7] = b0 - b7;
}

/* DC-only byte-replicated saturating add (m2d.h:286-341, Appendix A #17): byte `x` of the word */
__device__ __forceinline__ int d_swar(int p, int dc, int x, int n)
{
	int adj = (dc + 32) >> 6;
	uint64_t v = (uint64_t)(adj < 0 ? -(int64_t)adj : adj);
	uint64_t w = (n == 4) ? (uint64_t)(uint32_t)(v * 0x01010101u) : v * 0x0101010101010101ull;
	int b = (int)((w >> (8 * x)) & 255);
	return adj < 0 ? max(p - b, 0) : min(p + b, 255);
}

/* offset (int16 units) of luma block `bit` (blkIdx, or 4*b8) in an MB's pool segment */
__device__ __forceinline__ int d_luma_off(const m2r_mb_t &m, int bit)
{
	uint32_t before = m.nz & ((1u << bit) - 1);
	int off = (m.nz & M2R_NZ_LUMA_DC) ? 16 : 0;
	return off + __popc(before & 0xffffu) * ((m.flags & M2R_FLAG_T8x8) ? 64 : 16);
}

/* offset of a chroma block (DC of component c: bit = 17 + c; AC: 19 + 4c + b) */
__device__ __forceinline__ int d_chroma_off(const m2r_mb_t &m, int bit)
{
	uint32_t before = m.nz & ((1u << bit) - 1);
	int off = (before & M2R_NZ_LUMA_DC) ? 16 : 0;
	off += __popc(before & 0xffffu) * ((m.flags & M2R_FLAG_T8x8) ? 64 : 16);
	off += __popc(before & (M2R_NZ_CDC(0) | M2R_NZ_CDC(1))) * 4;
	off += __popc(before & (0xffu << 19)) * 16;
	return off;
}

/* branch-free select: c ? a : b without letting the compiler sink a or b into a divergent branch */
__device__ __forceinline__ int d_sel(bool c, int a, int b)
{
	return b ^ ((a ^ b) & -(int)c);
}

/* int16 words of the pool an MB owns (PCM: 384 sample bytes) */
#define M2R_MB_COEF_MAX 416
__device__ __forceinline__ int d_mb_ncoef(const m2r_mb_t &m)
{
	return m.kind == M2R_MB_PCM ? 192 : d_chroma_off(m, 27);
}

/* chroma DC of 4x4 block b of component c (intra_chroma_dc_transform, h264.cpp:4387-4404) */
/* `q` points at the MB's own coefficients (pool + m.coef, or a staged copy) */
__device__ __forceinline__ int d_chroma_dc(const m2r_mb_t &m, const int16_t *q, int c, int b)
{
	if (!(m.nz & M2R_NZ_CDC(c))) return 0;
	const int16_t *p = q + d_chroma_off(m, 17 + c);
	int s = d_scale4(c ? m.qpc[1] : m.qpc[0], 0, 0);
	int c0 = p[0] * s, c1 = p[1] * s, c2 = p[2] * s, c3 = p[3] * s;
	switch (b) {
	case 0: return (c0 + c1 + c2 + c3) >> 1;
	case 1: return (c0 - c1 + c2 - c3) >> 1;
	case 2: return (c0 + c1 - c2 - c3) >> 1;
	default: return (c0 - c1 - c2 + c3) >> 1;
	}
}
