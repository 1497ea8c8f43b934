/*
 * H.265 inverse DCT 16 x 16 / 32 x 32 on the matrix cores (gfx950 int8 MFMA), bit-exact.
 *
 * The reference's two passes (h265.cpp:2142 transform dispatch; spec 8.6.4.2):
 *   g[y][x]   = sat16((sum_k T[k][y] C[k][x] + 64) >> 7)       (columns)
 *   r[y][x]   = sat16((sum_k T[k][x] g[y][k] + 2048) >> 12)    (rows)
 * with T the N-point DCT matrix (T_N[k][n] = T_32[k 32 / N][n], |T| <= 90: an int8) and C, g int16.
 * An int16 v is split into two int8 operands, v = 256 hi + (lo + 128) with hi = v >> 8 and lo = (v & 255) - 128
 * (both in [-128, 127]), so sum_k T v = 256 (T . hi) + (T . lo) + 128 sum_k T: two int8 MFMAs and a per-column
 * constant, all exact in int32 (|sum| <= 32 * 32768 * 90 < 2^31).
 *
 * Orientation (cdna_hip_programming.md §3, "an accumulator tile as the next MFMA's operand"): pass 1 computes
 * D = C^T T, i.e. D[x][y] = G[y][x] before rounding, whose accumulator holds column y of D on the lane and rows
 * x in the registers — exactly the A fragment (rows y, sums over x) of pass 2, R = G T, so the two passes need
 * no lane movement and no LDS between them.  Which k an operand element carries is free as long as the A and B
 * fragments agree (the hardware pairs element j of a lane half of A with element j of the same half of B); the
 * accumulator maps are the gfx950 ones (dtype-independent): 32x32 col = lane & 31, row = (i & 3) + 8 (i >> 2) +
 * 4 (lane >> 5); 16x16 col = lane & 15, row = 4 (lane >> 4) + i.
 *
 * 32 x 32: one v_mfma_i32_32x32x32_i8 per split per pass (K = 32 exactly); lane half h carries k = 16 h + j in
 * pass 1 and k = row(j, h) in pass 2.  16 x 16: v_mfma_i32_16x16x64_i8 with K = 16 of its 64 used (lane quarter q
 * carries k = 4 q + j in its elements j < 4, zeros above).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace h265mfma {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

/* T_32[k][n] (spec eq. 8-315 as tabulated: 64 sqrt(2) cos((2n + 1) k pi / 64) rounded as the standard's table) */
__host__ __device__ constexpr int t32(int k, int n)
{
	constexpr int cosv[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
	                          61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
	int m = ((2 * n + 1) * k) & 127, sign = 1;
	if (m > 64) m = 128 - m;
	if (m > 32) {
		m = 64 - m;
		sign = -1;
	}
	return sign * cosv[m];
}

/* the accumulator row of register i (the pass-2 k of element i) */
template <int N>
__host__ __device__ constexpr int acc_row(int i, int lane)
{
	return N == 32 ? (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5) : 4 * (lane >> 4) + i;
}
template <int N>
__host__ __device__ constexpr int acc_col(int lane)
{
	return lane & (N - 1);
}
/* results per lane */
template <int N>
__host__ __device__ constexpr int per_lane()
{
	return N * N / 64;
}

/* per lane, the B fragments of both passes (T's column, int8 bytes) and T's column sum: built once per workgroup */
struct Tabs {
	v4i b32[2][64], b16[2][64];
	int cs32[32], cs16[16];
};

__device__ inline void tabs_init(Tabs &tb, int tid, int nt)
{
	for (int i = tid; i < 4 * 64; i += nt) {
		const int which = i >> 6, lane = i & 63;
		const int n = which >> 1, pass = which & 1; /* n 0: 32-point, 1: 16-point */
		v4i f = {0, 0, 0, 0};
		for (int j = 0; j < 16; ++j) {
			int v = 0;
			if (n == 0) {
				const int col = lane & 31;
				const int k = pass == 0 ? 16 * (lane >> 5) + j : acc_row<32>(j, lane);
				v = t32(k, col);
			} else if (j < 4) {
				const int col = lane & 15, k = 4 * (lane >> 4) + j;
				v = t32(2 * k, col);
			}
			f[j >> 2] |= (int)((uint32_t)(v & 255) << (8 * (j & 3)));
		}
		if (n == 0) tb.b32[pass][lane] = f;
		else tb.b16[pass][lane] = f;
	}
	for (int i = tid; i < 48; i += nt) {
		int s = 0;
		if (i < 32)
			for (int k = 0; k < 32; ++k) s += t32(k, i);
		else
			for (int k = 0; k < 16; ++k) s += t32(2 * k, i - 32);
		if (i < 32) tb.cs32[i] = s;
		else tb.cs16[i - 32] = s;
	}
}

/* 4 int16 values (low halves of a, b, c, d) -> the hi / lo int8 operand dwords of split4 */
__device__ __forceinline__ void split4(int a, int b, int c, int d, v4i &hi, v4i &lo, int q)
{
	const uint32_t p0 = ((uint32_t)a & 0xffffu) | ((uint32_t)b << 16), p1 = ((uint32_t)c & 0xffffu) | ((uint32_t)d << 16);
	/* v_perm_b32: bytes of {p1, p0}; selector bytes 0-3 pick p0's, 4-7 p1's */
	hi[q] = (int)__builtin_amdgcn_perm(p1, p0, 0x07050301u);
	lo[q] = (int)(__builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u);
}

__device__ __forceinline__ int sat16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

/* The residual of one N x N block (N = 16, 32): coefficients C[k][x] at coef (row-major, int16, any address
 * space via a generic pointer) -> res[i] = r[acc_row<N>(i, lane)][acc_col<N>(lane)], i < per_lane<N>(). */
template <int N>
__device__ __forceinline__ void idct(const int16_t *coef, const Tabs &tb, int lane, int *res)
{
	if (N == 32) {
		const int col = lane & 31, h = lane >> 5;
		/* pass 1: A[x = col][k = 16 h + j] = C[k][x] */
		int v[16];
#pragma unroll
		for (int j = 0; j < 16; ++j) v[j] = coef[(16 * h + j) * 32 + col];
		v4i ahi, alo;
#pragma unroll
		for (int q = 0; q < 4; ++q) split4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3], ahi, alo, q);
		const v4i b1 = tb.b32[0][lane], b2 = tb.b32[1][lane];
		const v16i z = {};
		const v16i dh = __builtin_amdgcn_mfma_i32_32x32x32_i8(ahi, b1, z, 0, 0, 0);
		const v16i dl = __builtin_amdgcn_mfma_i32_32x32x32_i8(alo, b1, z, 0, 0, 0);
		const int c128 = 128 * tb.cs32[col];
		int g[16];
#pragma unroll
		for (int i = 0; i < 16; ++i) g[i] = sat16((dh[i] * 256 + dl[i] + c128 + 64) >> 7);
		/* pass 2: A[y = col][k = acc_row(j)] = g[y][k] = element j */
#pragma unroll
		for (int q = 0; q < 4; ++q) split4(g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3], ahi, alo, q);
		const v16i rh = __builtin_amdgcn_mfma_i32_32x32x32_i8(ahi, b2, z, 0, 0, 0);
		const v16i rl = __builtin_amdgcn_mfma_i32_32x32x32_i8(alo, b2, z, 0, 0, 0);
#pragma unroll
		for (int i = 0; i < 16; ++i) res[i] = sat16((rh[i] * 256 + rl[i] + c128 + 2048) >> 12);
	} else {
		const int col = lane & 15, q4 = lane >> 4;
		int v[4];
#pragma unroll
		for (int j = 0; j < 4; ++j) v[j] = coef[(4 * q4 + j) * 16 + col];
		v4i ahi = {0, 0, 0, 0}, alo = {0, 0, 0, 0};
		split4(v[0], v[1], v[2], v[3], ahi, alo, 0);
		const v4i b1 = tb.b16[0][lane], b2 = tb.b16[1][lane];
		const v4i z = {0, 0, 0, 0};
		const v4i dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahi, b1, z, 0, 0, 0);
		const v4i dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(alo, b1, z, 0, 0, 0);
		const int c128 = 128 * tb.cs16[col];
		int g[4];
#pragma unroll
		for (int i = 0; i < 4; ++i) g[i] = sat16((dh[i] * 256 + dl[i] + c128 + 64) >> 7);
		split4(g[0], g[1], g[2], g[3], ahi, alo, 0);
		const v4i rh = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahi, b2, z, 0, 0, 0);
		const v4i rl = __builtin_amdgcn_mfma_i32_16x16x64_i8(alo, b2, z, 0, 0, 0);
#pragma unroll
		for (int i = 0; i < 4; ++i) res[i] = sat16((rh[i] * 256 + rl[i] + c128 + 2048) >> 12);
	}
}

} /* namespace h265mfma */
