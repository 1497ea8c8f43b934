/*
 * gfx950 reconstruction of H.265 pictures (h265d_func): the records of one picture (include/m2d_recon.h
 * h265r_*, made by m2dec_amd/csrc/host/h265_dec.c) in, the picture's NV12 samples in its device frame out.
 * It restates the reference decoder's reconstruction (h265.cpp:1693-2913 intra prediction and residual,
 * :4125-4384 deblocking, :4386-4729 SAO), exactly as oracle/h265_oracle.c does on the CPU.
 *
 * k_h265_intra — the transform blocks in decoding order, one 64-lane wave (= one workgroup) at a time,
 *   persistent: a wave takes the next block from a counter, waits until the blocks that own its
 *   neighbour samples are done (the 4x4-unit owner map: one lane per neighbour unit, at most 33), then
 *   predicts (reference samples gathered straight from the frame with the substitution folded into a
 *   clamp — the available samples of a block always form one run of the substitution order —, [1 2 1] /
 *   strong smoothing in LDS, planar / DC / angular per sample), inverse-transforms the residual in LDS
 *   (DCT 4..32 / DST 4 as two matrix passes with the int16 clip between, the reference's DC-only and
 *   transform-skip shortcuts), adds, stores, releases and raises the block's done flag.  Luma and chroma
 *   blocks are independent chains and run side by side; the dependency graph, not the CTU raster, bounds
 *   the picture (a block starts as soon as its left / top / top-right / bottom-left owners are done).
 * k_h265_deblock — one thread per 4-sample edge segment on the 8x8 grid, vertical edges of the whole
 *   picture, then (second launch) horizontal edges: HEVC's edges 8 samples apart never touch the same
 *   sample, so every segment of a direction is independent.  Chroma rides on the luma segment (bS 2,
 *   16-sample grid).
 * k_h265_sao — one thread per 4 bytes of an NV12 row, from a copy of the deblocked frame, dword stores.
 * k_h265_mc — P / B pictures, before the blocks: one 64-lane workgroup per prediction block (grid-stride),
 *   each list's reference window ((w + 7) x (h + 7) luma bytes, (w / 2 + 3) x (h / 2 + 3) CbCr pairs, positions
 *   clamped to the picture as the reference's address_umv does) staged in LDS, then every sample computed
 *   from LDS: the 8-tap luma filters (1-D with shift - 6, 2-D through int16 horizontal sums) and the
 *   reference's packed two-component chroma arithmetic in 64-bit integers, bi-prediction averaged through an
 *   int16 LDS buffer.  The CTU kernel then starts each CTU from these samples and adds the residuals.
 * Bounds: the intra kernel is latency-bound on the block chain (a 32x32 block is a 2 x 32^3 MAC inverse
 * transform on one wave); deblocking and SAO are HBM-bound (each reads and writes the frame once).
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <mutex>
#include <vector>
#include "m2d_recon.h"
#include "h265_dec.h"
#include "h265_mfma.h"

extern "C" void m2dec_par_memcpy(int crew, int n, void *const *dst, const void *const *src, const size_t *len);
enum { M2DEC_CREW_SYNC_ = 1 }; /* = M2DEC_CREW_SYNC (h264_dec.h) */

#define H265_CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "m2dec_amd HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -1; } } while (0)
#define H265_SPIN_LIMIT (1 << 26) /* ~30-60 s of polls: every wait points at a workgroup dispatched earlier (a slow one means a shared GPU: waited on); only a bug ends the picture */

namespace {

typedef int __attribute__((address_space(1))) gi32;

struct H265Args {
	const h265r_tu_t *tu;
	const int16_t *coef;
	const int32_t *map;
	const uint8_t *bs_v, *bs_h;
	const h265r_sao_t *sao;
	uint8_t *frame;   /* NV12, stride W */
	uint8_t *copy;    /* the deblocked frame (SAO input) */
	int *done;        /* per block (block kernel) */
	int *counter;     /* next block (block kernel) */
	int *progress;    /* per CTU row: CTUs finished (CTU kernel) */
	int *ctu_first;   /* [ctu_cols * ctu_rows + 1]: the first record of each CTU (CTU kernel) */
	int ctu_cols, ctu_rows;
	int *err;         /* sticky: a hand-off that never came */
	int W, H, pic_w, pic_h, ctb_log2, n_tu, flags;
	int beta_offset, tc_offset, cb_qp_offset, cr_qp_offset;
	/* P / B pictures */
	const h265r_pu_t *pu;
	const uint8_t *frames; /* every frame (the references), fsz bytes apart */
	size_t fsz;
	int n_pu;
};

/* H265_STAMPS (build/dbg/libm2dec_amd_h5stamps.so, tools/stamps_h265.py): the CTU kernels' steps on the
 * device's constant 100 MHz clock — per CTU its start, the end of its wait for the row above, each wave's last
 * block and its end; per block its end with the block's size / prediction / residual kind */
#ifdef H265_STAMPS
#define H5ST_N (1 << 20)
__device__ unsigned long long g_h5t[H5ST_N];
__device__ unsigned g_h5i[H5ST_N];
__device__ unsigned g_h5n;
__device__ __forceinline__ void h5st(int kind, int row, int col, int aux)
{
	const unsigned i = atomicAdd(&g_h5n, 1u);
	if (i < H5ST_N) {
		g_h5t[i] = wall_clock64();
		g_h5i[i] = (unsigned)kind | ((unsigned)row << 4) | ((unsigned)col << 12) | ((unsigned)aux << 20);
	}
}
#define H5ST(lane, ...) do { if ((lane) == 0) h5st(__VA_ARGS__); } while (0)
/* block phases (kind 5, H265_STAMPS_PHASES: heavy, ~0.3 us per stamp): per workgroup and wave, phase 0 = the block
 * starts, 1 its residual, 4 its neighbours done, 2 its reference samples, 3 its end; aux = phase << 8 | plane << 3 | log2 */
#ifdef H265_STAMPS_PHASES
#define H5PH(lane, t, ph) H5ST(lane, 5, __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6, blockIdx.x & 255, ((ph) << 8) | ((t).plane << 3) | (t).log2)
#else
#define H5PH(lane, t, ph) do { } while (0)
#endif
#else
#define H5PH(lane, t, ph) do { } while (0)
#define H5ST(lane, ...) do { } while (0)
#endif

__constant__ int c_cos[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                              61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
__constant__ int c_dst[16] = {29, 55, 74, 84, 74, 74, 0, -74, 84, -29, -74, 55, 55, -84, 74, -29};
__constant__ int c_ang[35] = {0,   0,   32,  26,  21,  17,  13,  9,  5,  2,  0,  -2, -5, -9, -13, -17, -21, -26,
                              -32, -26, -21, -17, -13, -9,  -5,  -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
__constant__ int c_inv[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482, -390, -315,
                              -256, -315, -390, -482, -630, -910, -1638, -4096, 0, 0, 0, 0, 0, 0, 0, 0, 0};
__constant__ uint8_t c_beta[36] = {6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28,
                                   30, 32, 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
__constant__ uint8_t c_tc[38] = {0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3,
                                 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int sat16(int v) { return clampi(v, -32768, 32767); }

/* the 32-point DCT coefficient of basis k, sample n (spec 8.6.4.2, eq. 8-315: 64 sqrt(2) cos((2n + 1) k pi / 64)
 * as tabulated); the N-point matrix is T_N[k][n] = T_32[k * 32 / N][n] */
__device__ __forceinline__ int dct32_coef(int k, int n)
{
	int m = ((2 * n + 1) * k) & 127, sign = 1;
	if (m > 64) m = 128 - m;
	if (m > 32) {
		m = 64 - m;
		sign = -1;
	}
	return sign * c_cos[m];
}

/* wave-private LDS of one block */
struct Lds {
	int16_t seq[2][132];   /* reference samples per component: [0 .. 4n] substitution order, filtered */
	int16_t raw[132];      /* unfiltered copy (filter input) */
	int16_t mat32[32 * 32]; /* the 32-point DCT matrix (built once per workgroup) */
	int16_t mat[32 * 32];  /* transform matrix of this block's size: mat[k * n + s]; the butterfly's first-pass output */
	int16_t t0[32 * 32];   /* coefficients, then the first-stage output */
	int16_t pred[2][32 * 32]; /* prediction, then prediction + residual, saturated to int16 (the store clamps to
	                           * 0..255: clamp(sat16(x)) == clamp(x)); the CTU kernels' small blocks: the residual.
	                           * int16 keeps a wave's LDS at ~11 KB: the 4-wave CTU kernels fit two per CU */
};

/* wave-private LDS of the CTU kernels' blocks: only the reference samples — the transforms stay in registers
 * (4 x 4 / 8 x 8: cross-lane DPP / swizzle, small_block; 16 x 16 / 32 x 32: the matrix cores, big_block) */
struct LdsCtu {
	int16_t seq[2][132]; /* reference samples per component: [0 .. 4n] substitution order, filtered */
};
/* per workgroup, read by all its waves: the 32-point DCT matrix and the MFMA lane fragments (h265_mfma.h) */
struct CtuConst {
	int16_t mat32[32 * 32];
	int16_t dst4[16], dct4[16]; /* M[j][n] = m[j * 4 + n] */
	h265mfma::Tabs tb;
};
__device__ __forceinline__ void ctu_const_init(CtuConst &k, int tid, int nt)
{
	for (int i = tid; i < 32 * 32; i += nt) k.mat32[i] = (int16_t)dct32_coef(i >> 5, i & 31);
	if (tid < 16) {
		k.dst4[tid] = (int16_t)c_dst[tid];
		k.dct4[tid] = (int16_t)dct32_coef((tid >> 2) << 3, tid & 3);
	}
	h265mfma::tabs_init(k.tb, tid, nt);
}

/* 4 x 4 inverse DST / DCT in registers: lane y 4 + x (lanes 0..15; the others compute a copy) holds r[y][x].
 * Pass 1 reads its column of coefficients; pass 2 takes row y of the first-stage output from the lanes of its quad
 * (DPP quad_perm broadcasts, no LDS).  m[j * 4 + n] = M[j][n]. */
__device__ __forceinline__ int tr4_regs(const int16_t *d, const int16_t *m, int lane)
{
	const int x = lane & 3, y = (lane >> 2) & 3;
	int e = 0;
#pragma unroll
	for (int j = 0; j < 4; ++j) e += m[j * 4 + y] * d[j * 4 + x];
	const int g = sat16((e + 64) >> 7);
	const int g0 = __builtin_amdgcn_mov_dpp(g, 0x00, 0xf, 0xf, false), g1 = __builtin_amdgcn_mov_dpp(g, 0x55, 0xf, 0xf, false);
	const int g2 = __builtin_amdgcn_mov_dpp(g, 0xaa, 0xf, 0xf, false), g3 = __builtin_amdgcn_mov_dpp(g, 0xff, 0xf, 0xf, false);
	return sat16((m[x] * g0 + m[4 + x] * g1 + m[8 + x] * g2 + m[12 + x] * g3 + 2048) >> 12);
}

/* 8 x 8 inverse DCT in registers: lane y 8 + x holds r[y][x]; pass 2 takes row y of the first-stage output from the 8
 * lanes of its group (ds_swizzle bit mode: lane (l & 0x18) | j within each 32, no memory access) */
__device__ __forceinline__ int tr8_regs(const int16_t *d, const int16_t *mat32, int lane)
{
	const int x = lane & 7, y = lane >> 3;
	int e = 0;
#pragma unroll
	for (int j = 0; j < 8; ++j) e += mat32[(j << 2) * 32 + y] * d[j * 8 + x];
	const int g = sat16((e + 64) >> 7);
	int gr[8];
	gr[0] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (0 << 5));
	gr[1] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (1 << 5));
	gr[2] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (2 << 5));
	gr[3] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (3 << 5));
	gr[4] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (4 << 5));
	gr[5] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (5 << 5));
	gr[6] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (6 << 5));
	gr[7] = __builtin_amdgcn_ds_swizzle(g, 0x18 | (7 << 5));
	int f = 0;
#pragma unroll
	for (int j = 0; j < 8; ++j) f += mat32[(j << 2) * 32 + x] * gr[j];
	return sat16((f + 2048) >> 12);
}

__device__ __forceinline__ uint8_t *plane_px(const H265Args &a, int plane, int comp, int x, int y)
{
	return plane ? a.frame + (size_t)a.W * a.H + (size_t)y * a.W + (size_t)x * 2 + comp : a.frame + (size_t)y * a.W + x;
}

/* Block hand-off (cdna_hip_programming.md §6, Guideline 16; as recon_hip.hip's): a block's samples go out
 * as 32-bit write-through stores (agent-scope relaxed atomics = sc1), drained before its done flag; a
 * consumer polls the flags, then reads neighbour samples with sc1 loads — no L2 write-back / invalidate. */
__device__ __forceinline__ int ld_px(const H265Args &a, int plane, int comp, int x, int y)
{
	const uint8_t *p = plane_px(a, plane, comp, x, y);
	const uint32_t w = (uint32_t)__hip_atomic_load((gi32 *)((uintptr_t)p & ~(uintptr_t)3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	return (int)((w >> (8 * ((uintptr_t)p & 3))) & 255);
}

__device__ __forceinline__ void st_word(uint8_t *p, uint32_t v)
{
	__hip_atomic_store((gi32 *)p, (int)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* LDS ordering among the lanes of one wave (every block runs on one wave; the CTU kernel's two waves
 * must not wait for each other per block) */
__device__ __forceinline__ void wsync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* One pass of the N-point inverse DCT (N = 8, 16, 32) over all N lines of a block, even / odd split:
 * out[b] = E + O and out[N - 1 - b] = E - O with E / O the sums over the even / odd frequencies j of
 * T[j][b] in[j] (T[j][N - 1 - b] = (-1)^j T[j][b]), exactly the matrix product's integers in half the
 * multiplies.  Lane: line a = lane & (N - 1) (its N inputs held in registers), output pairs b =
 * (lane >> log2 N) + k 64 / N.  COLS: pass 1 (line = column x: in[j] = src[j][x], out to dst[b][x] as
 * sat16((v + 64) >> 7)); else pass 2 (line = row y: in[j] = src[y][j], dst[y][b] += sat16((v + 2048) >> 12)). */
template <int N, bool COLS, bool ACC = true>
__device__ __forceinline__ void idct_pass(const int16_t *src, int16_t *dst, const int16_t *mat32, int lane)
{
	constexpr int L = N == 8 ? 3 : (N == 16 ? 4 : 5), PAIRS = N * N / 2, PPL = PAIRS < 64 ? 1 : PAIRS / 64;
	const int a = lane & (N - 1);
	int in[N];
#pragma unroll
	for (int j = 0; j < N; ++j) in[j] = COLS ? src[j * N + a] : src[a * N + j];
#pragma unroll
	for (int k = 0; k < PPL; ++k) {
		const int b = (lane >> L) + k * (64 >> L);
		if (b < N / 2) {
			int e = 0, o = 0;
#pragma unroll
			for (int j = 0; j < N; j += 2) {
				e += mat32[(j << (5 - L)) * 32 + b] * in[j];
				o += mat32[((j + 1) << (5 - L)) * 32 + b] * in[j + 1];
			}
			if (COLS) {
				dst[b * N + a] = sat16((e + o + 64) >> 7);
				dst[(N - 1 - b) * N + a] = sat16((e - o + 64) >> 7);
			} else if (ACC) {
				dst[a * N + b] = (int16_t)sat16(dst[a * N + b] + sat16((e + o + 2048) >> 12));
				dst[a * N + N - 1 - b] = (int16_t)sat16(dst[a * N + N - 1 - b] + sat16((e - o + 2048) >> 12));
			} else {
				dst[a * N + b] = sat16((e + o + 2048) >> 12);
				dst[a * N + N - 1 - b] = sat16((e - o + 2048) >> 12);
			}
		}
	}
}

template <int N, bool ACC = true>
__device__ __forceinline__ void idct_block(int16_t *t0, int16_t *tmp, int16_t *pred, const int16_t *mat32, int lane)
{
	idct_pass<N, true>(t0, tmp, mat32, lane);
	wsync();
	idct_pass<N, false, ACC>(tmp, pred, mat32, lane);
	wsync();
}

/* samples straight from / to the frame (block kernel) */
struct FrameSamples {
	const H265Args &a;
	__device__ int ld(int plane, int comp, int x, int y) const { return ld_px(a, plane, comp, x, y); }
	/* 4 luma samples / 2 CbCr pairs of one row, little-endian in v */
	__device__ void st(int plane, int x, int y, uint32_t v) const { st_word(plane_px(a, plane, 0, x, y), v); }
};

/* one block (wave-wide); Src: where neighbour samples come from and the block's samples go */
template <class Src>
__device__ void do_block(const H265Args &a, const h265r_tu_t &t, Lds &s, int lane, const Src &src, const int16_t *cbase, uint32_t clo)
{
	const int n = 1 << t.log2, log2 = t.log2, n2 = n * n;
	const int ncomp = t.plane ? 2 : 1;
	const bool luma = t.plane == 0;
	/* ---- prediction */
	for (int c = 0; c < ncomp; ++c) {
		int16_t *pred = s.pred[c];
		if (!(t.flags & H265R_TU_PRED)) {
			for (int i = lane; i < n2; i += 64) pred[i] = src.ld(t.plane, c, t.x + (i & (n - 1)), t.y + (i >> log2));
			continue;
		}
		const int at = t.avail_top > 2 * n ? 2 * n : t.avail_top, al = t.avail_left > 2 * n ? 2 * n : t.avail_left;
		const bool top = at > 0, left = al > 0;
		/* the available run [lo, hi] of the substitution order p[-1][2n-1] .. corner .. p[2n-1][-1] */
		const int corner = 2 * n;
		const int lo = left ? corner - al : (top ? corner + 1 : 0);
		const int hi = top ? corner + at : (left ? corner - 1 : 0);
		for (int i = lane; i <= 4 * n; i += 64) {
			int v = 128;
			if (top || left) {
				const int k = clampi(i, lo, hi);
				const int xx = k < corner ? -1 : (k == corner ? -1 : k - corner - 1);
				const int yy = k < corner ? corner - 1 - k : -1;
				v = src.ld(t.plane, c, t.x + xx, t.y + yy);
			}
			s.raw[i] = (int16_t)v;
		}
		wsync();
		const int mode = t.mode;
		bool filt = false;
		if (luma && mode != 1 && n != 4) {
			const int d26 = abs(mode - 26), d10 = abs(mode - 10);
			const int dist = d26 < d10 ? d26 : d10;
			const int thres = n == 8 ? 7 : (n == 16 ? 1 : 0);
			filt = mode == 0 || dist > thres;
		}
		const int last = 4 * n;
		bool strong = false;
		if (filt && t.strong && n == 32) {
			const int cc = s.raw[corner], bl = s.raw[0], tr = s.raw[last];
			strong = abs(cc + tr - 2 * s.raw[corner + n]) < 8 && abs(cc + bl - 2 * s.raw[corner - n]) < 8;
		}
		for (int i = lane; i <= last; i += 64) {
			int v = s.raw[i];
			if (strong) {
				const int cc = s.raw[corner];
				if (i > 0 && i < corner) v = ((63 - (corner - 1 - i)) * cc + (corner - i) * s.raw[0] + 32) >> 6;
				else if (i > corner && i < last) v = ((63 - (i - corner - 1)) * cc + (i - corner) * s.raw[last] + 32) >> 6;
			} else if (filt && i > 0 && i < last) {
				v = (s.raw[i - 1] + 2 * s.raw[i] + s.raw[i + 1] + 2) >> 2;
			}
			s.seq[c][i] = (int16_t)v;
		}
		wsync();
		const int16_t *q = s.seq[c];
#define LL(yy) ((int)q[corner - 1 - (yy)]) /* p[-1][y], y >= -1 */
#define TT(xx) ((int)q[corner + 1 + (xx)]) /* p[x][-1], x >= -1 */
		if (mode == 0) {
			for (int i = lane; i < n2; i += 64) {
				const int x = i & (n - 1), y = i >> log2;
				pred[i] = ((n - 1 - x) * LL(y) + (x + 1) * TT(n) + (n - 1 - y) * TT(x) + (y + 1) * LL(n) + n) >> (log2 + 1);
			}
		} else if (mode == 1) {
			int sum = 0;
			for (int i = lane; i < n; i += 64) sum += TT(i) + LL(i);
			for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
			const int dc = (sum + n) >> (log2 + 1);
			for (int i = lane; i < n2; i += 64) {
				const int x = i & (n - 1), y = i >> log2;
				int v = dc;
				if (luma && n < 32) {
					if (x == 0 && y == 0) v = (LL(0) + 2 * dc + TT(0) + 2) >> 2;
					else if (y == 0) v = (TT(x) + 3 * dc + 2) >> 2;
					else if (x == 0) v = (LL(y) + 3 * dc + 2) >> 2;
				}
				pred[i] = v;
			}
		} else {
			const int ang = c_ang[mode], inv = c_inv[mode];
			const bool vert = mode >= 18;
			for (int i = lane; i < n2; i += 64) {
				const int x = i & (n - 1), y = i >> log2;
				const int p = vert ? y : x, qq = vert ? x : y;
				const int idx = ((p + 1) * ang) >> 5, fr = ((p + 1) * ang) & 31;
				int r1, r2;
				{
					const int k = qq + idx + 1;
					int kk = k;
					if (kk >= 0) r1 = vert ? TT(kk - 1) : LL(kk - 1);
					else r1 = vert ? LL(-1 + ((kk * inv + 128) >> 8)) : TT(-1 + ((kk * inv + 128) >> 8));
					kk = k + 1;
					if (kk >= 0) r2 = vert ? TT(kk - 1) : LL(kk - 1);
					else r2 = vert ? LL(-1 + ((kk * inv + 128) >> 8)) : TT(-1 + ((kk * inv + 128) >> 8));
				}
				int v = fr ? ((32 - fr) * r1 + fr * r2 + 16) >> 5 : r1;
				if (luma && n < 32) {
					if (mode == 26 && x == 0) v = clampi(TT(0) + ((LL(y) - LL(-1)) >> 1), 0, 255);
					if (mode == 10 && y == 0) v = clampi(LL(0) + ((TT(x) - TT(-1)) >> 1), 0, 255);
				}
				pred[i] = v;
			}
		}
#undef LL
#undef TT
		wsync();
	}
	/* ---- residual */
	for (int c = 0; c < ncomp; ++c) {
		const int kind = t.res[c];
		int16_t *pred = s.pred[c];
		if (kind == H265R_RES_NONE) continue;
		const int16_t *d = cbase + (t.coef[c] - clo); /* (the pool, or the CTU's coefficients staged in LDS) */
		if (kind == H265R_RES_DC) {
			const int dc = (d[0] + 64) >> 7; /* acNxNtransform_dconly<N, 7> (m2d.h:306-341) */
			for (int i = lane; i < n2; i += 64) pred[i] = (int16_t)sat16(pred[i] + dc);
			continue;
		}
		if (kind == H265R_RES_SKIP) {
			for (int i = lane; i < n2; i += 64) pred[i] = (int16_t)sat16(pred[i] + ((d[i] + 16) >> 5));
			continue;
		}
		for (int i = lane; i < n2; i += 64) s.t0[i] = d[i];
		const bool dstm = kind == H265R_RES_DST;
		if (!dstm && n >= 8) {
			wsync();
			if (n == 8) idct_block<8>(s.t0, s.mat, pred, s.mat32, lane);
			else if (n == 16) idct_block<16>(s.t0, s.mat, pred, s.mat32, lane);
			else idct_block<32>(s.t0, s.mat, pred, s.mat32, lane);
			continue;
		}
		for (int i = lane; i < n2; i += 64) {
			const int k = i >> log2, sm = i & (n - 1);
			s.mat[i] = dstm ? c_dst[k * 4 + sm] : s.mat32[(k << (5 - log2)) * 32 + sm];
		}
		wsync();
		/* first stage (columns): g[y][x] = sat16((sum_j M[j][y] d[j][x] + 64) >> 7) */
		int g[16];
		for (int r = 0, i = lane; i < n2; i += 64, ++r) {
			const int x = i & (n - 1), y = i >> log2;
			int e = 0;
			for (int j = 0; j < n; ++j) e += s.mat[j * n + y] * s.t0[j * n + x];
			g[r] = sat16((e + 64) >> 7);
		}
		wsync();
		for (int r = 0, i = lane; i < n2; i += 64, ++r) s.t0[i] = g[r];
		wsync();
		/* second stage (rows): r[y][x] = sat16((sum_j M[j][x] g[y][j] + 2048) >> 12) */
		for (int i = lane; i < n2; i += 64) {
			const int x = i & (n - 1), y = i >> log2;
			int e = 0;
			for (int j = 0; j < n; ++j) e += s.mat[j * n + x] * s.t0[y * n + j];
			pred[i] = (int16_t)sat16(pred[i] + sat16((e + 2048) >> 12));
		}
		wsync();
	}
	/* ---- out: 32-bit write-through words (luma: 4 samples of a row; chroma: 2 CbCr pairs) */
	if (luma) {
		const int wpr = n >> 2;
		for (int w = lane; w < n2 >> 2; w += 64) {
			const int y = w / wpr, x = (w - y * wpr) * 4;
			const int16_t *q = s.pred[0] + y * n + x;
			const uint32_t v = (uint32_t)clampi(q[0], 0, 255) | ((uint32_t)clampi(q[1], 0, 255) << 8) |
			                   ((uint32_t)clampi(q[2], 0, 255) << 16) | ((uint32_t)clampi(q[3], 0, 255) << 24);
			src.st(0, t.x + x, t.y + y, v);
		}
	} else {
		const int wpr = n >> 1;
		for (int w = lane; w < n2 >> 1; w += 64) {
			const int y = w / wpr, x = (w - y * wpr) * 2;
			const int16_t *cb = s.pred[0] + y * n + x, *cr = s.pred[1] + y * n + x;
			const uint32_t v = (uint32_t)clampi(cb[0], 0, 255) | ((uint32_t)clampi(cr[0], 0, 255) << 8) |
			                   ((uint32_t)clampi(cb[1], 0, 255) << 16) | ((uint32_t)clampi(cr[1], 0, 255) << 24);
			src.st(1, t.x + x, t.y + y, v);
		}
	}
}

__global__ __launch_bounds__(64) void k_h265_intra(const H265Args *ap)
{
	const H265Args a = *ap;
	__shared__ Lds s;
	const int lane = threadIdx.x;
	for (int i = lane; i < 32 * 32; i += 64) s.mat32[i] = (int16_t)dct32_coef(i >> 5, i & 31);
	__syncthreads();
	for (;;) {
		const int v = __hip_atomic_fetch_add((gi32 *)&a.counter[0], lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const int idx = __builtin_amdgcn_readfirstlane(v);
		if (idx >= a.n_tu) break;
		const h265r_tu_t t = a.tu[idx];
		/* wait for the owners of the neighbour samples: lane k < 2n/4 the top units, next the left units, last the corner */
		{
			const int n = 1 << t.log2;
			const int at = t.avail_top > 2 * n ? 2 * n : t.avail_top, al = t.avail_left > 2 * n ? 2 * n : t.avail_left;
			const int ntop = at > 0 ? (at + 3) >> 2 : 0, nleft = al > 0 ? (al + 3) >> 2 : 0;
			const int mw = t.plane ? a.W / 8 : a.W / 4;
			const int32_t *map = a.map + (t.plane ? (size_t)(a.W / 4) * (a.H / 4) : 0);
			int dep = -1;
			if (lane < ntop) dep = map[(size_t)((t.y >> 2) - 1) * mw + (t.x >> 2) + lane];
			else if (lane < ntop + nleft) dep = map[(size_t)((t.y >> 2) + lane - ntop) * mw + (t.x >> 2) - 1];
			else if (lane == ntop + nleft && ntop && nleft) dep = map[(size_t)((t.y >> 2) - 1) * mw + (t.x >> 2) - 1];
			unsigned spins = 0;
			for (;;) {
				const bool ok = dep < 0 || dep >= idx ||
				                __hip_atomic_load((gi32 *)&a.done[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
				if (__all(ok)) break;
				if (++spins > H265_SPIN_LIMIT) {
					__hip_atomic_store((gi32 *)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					break;
				}
				if (__hip_atomic_load((gi32 *)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
				__builtin_amdgcn_s_sleep(1);
			}
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keeps the sample loads below the poll */
		}
		do_block(a, t, s, lane, FrameSamples{a}, a.coef, 0);
		/* publish: the write-through sample stores drained, then the flag */
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__hip_atomic_store((gi32 *)&a.done[idx], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}

/* ---- the CTU wavefront (default): one workgroup per CTU row, CTUs left to right; wave 0 reconstructs the
 * CTU's luma blocks, wave 1 its chroma blocks, each in decoding order, entirely in LDS: the CTU's samples,
 * the column left of it (kept from the previous CTU) and the row above it from the left-above corner to
 * the end of the above-right CTU (loaded once per CTU after that CTU row published it).  A CTU starts when
 * the row above finished the CTU above-right of it (HEVC's intra references reach no further), so the
 * picture is a 2-CTU-lag wavefront of cols + 2 (rows - 1) CTU steps, each with two global round trips
 * (the row above in, the CTU out) instead of two per block. */
#define H265_CTB_MAX 64
#define H265_CTU_RECS 256
struct CtuTile {
	uint8_t y[H265_CTB_MAX][H265_CTB_MAX];      /* luma */
	uint8_t c[H265_CTB_MAX / 2][H265_CTB_MAX];  /* CbCr pairs */
	uint8_t ly[H265_CTB_MAX], lc[H265_CTB_MAX];  /* the column left of the CTU (CbCr pairs) */
	uint8_t ty[2 * H265_CTB_MAX + 4];            /* the row above: [0] the left-above corner, [1 + i] x0 + i */
	uint8_t tc[2 * H265_CTB_MAX + 4];            /* CbCr pairs: [2 (1 + i) + comp] */
};

struct CtuSamples {
	CtuTile &tl;
	int x0, y0; /* the CTU's luma origin */
	__device__ int ld(int plane, int comp, int x, int y) const
	{
		if (!plane) {
			const int dx = x - x0, dy = y - y0;
			return dy < 0 ? tl.ty[dx + 1] : (dx < 0 ? tl.ly[dy] : tl.y[dy][dx]);
		}
		const int dx = x - (x0 >> 1), dy = y - (y0 >> 1);
		return dy < 0 ? tl.tc[2 * (dx + 1) + comp] : (dx < 0 ? tl.lc[2 * dy + comp] : tl.c[dy][2 * dx + comp]);
	}
	__device__ void st(int plane, int x, int y, uint32_t v) const
	{
		if (!plane) *(uint32_t *)&tl.y[y - y0][x - x0] = v;
		else *(uint32_t *)&tl.c[y - (y0 >> 1)][2 * (x - (x0 >> 1))] = v;
	}
};

/* the record with every field in scalar registers (all lanes read the same LDS record: without this the
 * compiler keeps them in VGPRs and every size / mode / kind test is a divergent branch) */
__device__ __forceinline__ h265r_tu_t uniform_tu(const h265r_tu_t &r)
{
	static_assert(sizeof(h265r_tu_t) == 24, "h265r_tu_t layout");
	h265r_tu_t t;
	const uint32_t *src = (const uint32_t *)&r;
	uint32_t *dst = (uint32_t *)&t;
#pragma unroll
	for (int i = 0; i < 6; ++i) dst[i] = __builtin_amdgcn_readfirstlane(src[i]);
	return t;
}

/* 16 x 16 and 32 x 32 blocks of the CTU kernels (N; chroma: 16 x 16 CbCr pairs), sample-parallel in the matrix
 * cores' accumulator layout: lane l owns the samples (h265mfma::acc_row<N>(i, l), acc_col<N>(l)), i < N N / 64, of
 * each component.  The residual of a full transform comes out of h265mfma::idct in exactly those registers (int8
 * MFMAs, bit-exact), so the prediction, the residual add, the clip and the tile store of a sample happen in one
 * lane with no LDS round trip between them; only the reference samples go through LDS, gathered and filtered in
 * one pass (as do_block_ctu's phase 2).  The loops have compile-time trip counts: a lane's samples issue their
 * LDS reads together instead of one dependent round trip per 64 samples (r124 stamps: a 32 x 32 intra block with
 * a residual 13.6 us, of which ~7.7 us the two butterfly passes on one wave). */
/* LDS byte offset (from the tile's start) of sample (dx, dy) relative to the CTU's origin, dy = -1 the row above,
 * dx = -1 the column left (chroma: CbCr pairs, component comp); selects, not branches, so that a lane's reads of
 * several samples issue together */
__device__ __forceinline__ int tile_off(bool luma, int comp, int dx, int dy)
{
	if (luma) return dy < 0 ? (int)offsetof(CtuTile, ty) + dx + 1 : (dx < 0 ? (int)offsetof(CtuTile, ly) + dy : dy * H265_CTB_MAX + dx);
	return dy < 0 ? (int)offsetof(CtuTile, tc) + 2 * (dx + 1) + comp
	              : (dx < 0 ? (int)offsetof(CtuTile, lc) + 2 * dy + comp : (int)offsetof(CtuTile, c) + dy * H265_CTB_MAX + 2 * dx + comp);
}

/* The reference samples of an intra block into seq[c][0 .. 4n] (substitution order, unavailable ones substituted by
 * clamping the index into the available run), [1 2 1] or strong smoothing folded in: each lane reads the up to three
 * unfiltered samples it needs straight from the tile.  NC components side by side.  Ends with wsync. */
template <int N, int NC, bool LUMA>
__device__ __forceinline__ void ref_samples(const h265r_tu_t &t, const CtuTile &tl, LdsCtu &s, int lane, int bx, int by)
{
	const uint8_t *tb = (const uint8_t *)&tl;
	constexpr int corner = 2 * N, last = 4 * N, NREF = NC * (last + 1);
	const int at = t.avail_top > 2 * N ? 2 * N : t.avail_top, al = t.avail_left > 2 * N ? 2 * N : t.avail_left;
	const bool top = at > 0, left = al > 0;
	const int lo = left ? corner - al : (top ? corner + 1 : 0);
	const int hi = top ? corner + at : (left ? corner - 1 : 0);
	const bool none = !top && !left;
	auto raw = [&](int c, int k) -> int {
		const int kk = clampi(k, lo, hi);
		const int xx = max(kk - corner - 1, -1), yy = max(corner - 1 - kk, -1);
		return none ? 128 : (int)tb[tile_off(LUMA, c, bx + xx, by + yy)];
	};
	const int mode = t.mode;
	bool filt = false;
	if (LUMA && N > 4 && mode != 1) {
		const int d26 = abs(mode - 26), d10 = abs(mode - 10);
		const int dist = d26 < d10 ? d26 : d10;
		filt = mode == 0 || dist > (N == 8 ? 7 : (N == 16 ? 1 : 0));
	}
	if (N == 32 && filt && t.strong) {
		const int cc = raw(0, corner), bl = raw(0, 0), tr = raw(0, last);
		if (abs(cc + tr - 2 * raw(0, corner + N)) < 8 && abs(cc + bl - 2 * raw(0, corner - N)) < 8) {
#pragma unroll
			for (int r = 0; r < (NREF + 63) / 64; ++r) {
				const int k = lane + 64 * r;
				if (k <= last) {
					int v;
					if (k > 0 && k < corner) v = ((63 - (corner - 1 - k)) * cc + (corner - k) * bl + 32) >> 6;
					else if (k > corner && k < last) v = ((63 - (k - corner - 1)) * cc + (k - corner) * tr + 32) >> 6;
					else v = k == 0 ? bl : (k == corner ? cc : tr);
					s.seq[0][k] = (int16_t)v;
				}
			}
			wsync();
			return;
		}
	}
#pragma unroll
	for (int r = 0; r < (NREF + 63) / 64; ++r) {
		const int i = lane + 64 * r;
		if (i < NREF) {
			const int c = NC == 2 && i > last, k = i - c * (last + 1);
			const int v0 = raw(c, k);
			int v = v0;
			if (filt) {
				const int vm = raw(c, k - 1), vp = raw(c, k + 1);
				if (k > 0 && k < last) v = (vm + 2 * v0 + vp + 2) >> 2;
			}
			s.seq[c][k] = (int16_t)v;
		}
	}
	wsync();
}

/* seq index of the angular predictor's reference k (spec 8.4.4.2.6: the projected row / column for k < 0) */
__device__ __forceinline__ int ang_idx(int corner, bool vert, int k, int inv)
{
	const int off = k >= 0 ? k : -((k * inv + 128) >> 8);
	return vert ? corner + off : corner - off;
}

/* Prediction of the samples (x, ys[i]) of one lane, NS of them, component c (q = seq[c]), into pv: the mode is
 * uniform, so the loops are per mode and carry no branch (selects only) */
template <int N, int NS, bool EDGE>
__device__ __forceinline__ void predict_samples(const int16_t *q, int mode, int x, const int *ys, int dcv, int *pv)
{
	constexpr int corner = 2 * N, LOG2 = N == 4 ? 2 : (N == 8 ? 3 : (N == 16 ? 4 : 5));
#define LL(yy) ((int)q[corner - 1 - (yy)]) /* p[-1][y], y >= -1 */
#define TT(xx) ((int)q[corner + 1 + (xx)]) /* p[x][-1], x >= -1 */
	if (mode == 0) {
		const int tn = TT(N), ln = LL(N), tx = TT(x);
#pragma unroll
		for (int i = 0; i < NS; ++i) {
			const int y = ys[i];
			pv[i] = ((N - 1 - x) * LL(y) + (x + 1) * tn + (N - 1 - y) * tx + (y + 1) * ln + N) >> (LOG2 + 1);
		}
	} else if (mode == 1) {
		if (EDGE) {
			const int tx = TT(x), l0 = LL(0), t0 = TT(0);
#pragma unroll
			for (int i = 0; i < NS; ++i) {
				const int y = ys[i], ly = LL(y);
				pv[i] = x == 0 && y == 0 ? (l0 + 2 * dcv + t0 + 2) >> 2
				                         : (y == 0 ? (tx + 3 * dcv + 2) >> 2 : (x == 0 ? (ly + 3 * dcv + 2) >> 2 : dcv));
			}
		} else {
#pragma unroll
			for (int i = 0; i < NS; ++i) pv[i] = dcv;
		}
	} else {
		const int ang = c_ang[mode], inv = c_inv[mode];
		const bool vert = mode >= 18;
#pragma unroll
		for (int i = 0; i < NS; ++i) {
			const int y = ys[i];
			const int p = vert ? y : x, qq = vert ? x : y;
			const int idx = ((p + 1) * ang) >> 5, fr = ((p + 1) * ang) & 31;
			const int k = qq + idx + 1;
			const int r1 = q[ang_idx(corner, vert, k, inv)], r2 = q[ang_idx(corner, vert, k + 1, inv)];
			pv[i] = fr ? ((32 - fr) * r1 + fr * r2 + 16) >> 5 : r1;
		}
		if (EDGE && (mode == 26 || mode == 10)) {
			const int t0 = TT(0), l0 = LL(0), c0 = LL(-1), tx = TT(x);
#pragma unroll
			for (int i = 0; i < NS; ++i) {
				const int y = ys[i], ly = LL(y);
				if (mode == 26) pv[i] = x == 0 ? clampi(t0 + ((ly - c0) >> 1), 0, 255) : pv[i];
				else pv[i] = y == 0 ? clampi(l0 + ((tx - c0) >> 1), 0, 255) : pv[i];
			}
		}
	}
#undef LL
#undef TT
}

/* DC value of component c (lanes 0..N-1 add their top + left sample; wave-wide butterfly) */
template <int N>
__device__ __forceinline__ int dc_value(const int16_t *q, int lane)
{
	constexpr int corner = 2 * N, LOG2 = N == 4 ? 2 : (N == 8 ? 3 : (N == 16 ? 4 : 5));
	int sum = lane < N ? (int)q[corner + 1 + lane] + (int)q[corner - 1 - lane] : 0;
	for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
	return (sum + N) >> (LOG2 + 1);
}

template <int N, bool LUMA, class Wait>
__device__ void big_block(const h265r_tu_t &t, CtuTile &tl, LdsCtu &s, const h265mfma::Tabs &tb, int lane, int x0, int y0,
                          const int16_t *cbase, uint32_t clo, const Wait &wait)
{
	constexpr int PL = N * N / 64, NC = LUMA ? 1 : 2, LOG2 = N == 16 ? 4 : 5;
	const int bx = LUMA ? t.x - x0 : t.x - (x0 >> 1), by = LUMA ? t.y - y0 : t.y - (y0 >> 1);
	const int x = h265mfma::acc_col<N>(lane);
	/* ---- 1. the residual of each component, in the lane's samples */
	int res[NC][PL];
	bool any_res = false;
#pragma unroll
	for (int c = 0; c < NC; ++c) {
		const int kind = t.res[c];
		const int16_t *d = cbase + (t.coef[c] - clo);
		if (kind == H265R_RES_FULL) {
			h265mfma::idct<N>(d, tb, lane, res[c]);
		} else if (kind == H265R_RES_DC) {
			const int dc = (d[0] + 64) >> 7; /* acNxNtransform_dconly<N, 7> (m2d.h:306-341) */
#pragma unroll
			for (int i = 0; i < PL; ++i) res[c][i] = dc;
		} else if (kind == H265R_RES_SKIP) {
#pragma unroll
			for (int i = 0; i < PL; ++i) res[c][i] = (d[h265mfma::acc_row<N>(i, lane) * N + x] + 16) >> 5;
		} else {
#pragma unroll
			for (int i = 0; i < PL; ++i) res[c][i] = 0;
		}
		any_res |= kind != H265R_RES_NONE;
	}
	H5PH(lane, t, 1);
	wait(); /* (the residual does not depend on the neighbours: computed before their done flags) */
	H5PH(lane, t, 4);
	if (!(t.flags & H265R_TU_PRED)) {
		/* inter: the residual onto the motion-compensated samples */
		if (any_res) {
#pragma unroll
			for (int i = 0; i < PL; ++i) {
				const int y = h265mfma::acc_row<N>(i, lane);
				if (LUMA) {
					uint8_t &p = tl.y[by + y][bx + x];
					p = (uint8_t)clampi((int)p + res[0][i], 0, 255);
				} else {
					uint16_t &p = *(uint16_t *)&tl.c[by + y][2 * (bx + x)];
					const int cb = clampi((int)(p & 255) + res[0][i], 0, 255), cr = clampi((int)(p >> 8) + res[NC - 1][i], 0, 255);
					p = (uint16_t)(cb | (cr << 8));
				}
			}
			wsync();
		}
		return;
	}
	/* ---- 2. reference samples, filtered (both chroma components side by side) */
	ref_samples<N, NC, LUMA>(t, tl, s, lane, bx, by);
	H5PH(lane, t, 2);
	/* ---- 3. prediction + residual, clipped, into the tile */
	int ys[PL];
#pragma unroll
	for (int i = 0; i < PL; ++i) ys[i] = h265mfma::acc_row<N>(i, lane);
	int pv[NC][PL];
#pragma unroll
	for (int c = 0; c < NC; ++c) {
		const int dcv = t.mode == 1 ? dc_value<N>(s.seq[c], lane) : 0;
		predict_samples<N, PL, LUMA && N < 32>(s.seq[c], t.mode, x, ys, dcv, pv[c]);
	}
#pragma unroll
	for (int i = 0; i < PL; ++i) {
		const int y = ys[i];
		if (LUMA) {
			tl.y[by + y][bx + x] = (uint8_t)clampi(pv[0][i] + res[0][i], 0, 255);
		} else {
			const int cb = clampi(pv[0][i] + res[0][i], 0, 255), cr = clampi(pv[NC - 1][i] + res[NC - 1][i], 0, 255);
			*(uint16_t *)&tl.c[by + y][2 * (bx + x)] = (uint16_t)(cb | (cr << 8));
		}
	}
	wsync();
	H5PH(lane, t, 3);
}

/* 4 x 4 and 8 x 8 blocks of the CTU kernels (the many: three quarters of a picture's blocks), the same integers as
 * do_block in three wave-serial phases (round-5 stamps: a 4x4 block cost ~2 us of phase latency, the CTU's ~25 luma
 * blocks one after another):
 *   1. the residual first, into s.pred (it does not depend on the prediction): full / DST transforms;
 *      DC-only and transform-skip are added per sample in phase 3;
 *   2. reference samples gathered AND filtered in one pass (ref_samples), both chroma components side by side;
 *   3. prediction + residual, clipped and stored straight into the tile: lane l owns sample (l & (N - 1), l >> log2 N)
 *      of every component (lanes past N N idle).
 * An inter block (no prediction) adds its residual to the motion-compensated tile samples in place, or does
 * nothing without one. */
template <int N, bool LUMA, class Wait>
__device__ void small_block(const h265r_tu_t &t, CtuTile &tl, LdsCtu &s, const CtuConst &kc, int lane, int x0, int y0,
                            const int16_t *cbase, uint32_t clo, const Wait &wait)
{
	constexpr int LOG2 = N == 4 ? 2 : 3, N2 = N * N, NC = LUMA ? 1 : 2;
	const int bx = LUMA ? t.x - x0 : t.x - (x0 >> 1), by = LUMA ? t.y - y0 : t.y - (y0 >> 1);
	/* ---- 1. full / DST transforms in registers (lane l: sample (l & (N - 1), l >> log2 N)) */
	int tres[NC];
#pragma unroll
	for (int c = 0; c < NC; ++c) {
		const int kind = t.res[c];
		tres[c] = 0;
		if (kind != H265R_RES_FULL && kind != H265R_RES_DST) continue;
		const int16_t *d = cbase + (t.coef[c] - clo);
		if (N == 8) tres[c] = tr8_regs(d, kc.mat32, lane);
		else if (kind == H265R_RES_DST) tres[c] = tr4_regs(d, kc.dst4, lane);
		else tres[c] = tr4_regs(d, kc.dct4, lane);
	}
	H5PH(lane, t, 1);
	wait(); /* (the residual does not depend on the neighbours: computed before their done flags) */
	H5PH(lane, t, 4);
	const bool act = lane < N2;
	const int x = lane & (N - 1), y = (lane >> LOG2) & (N - 1);
	int res[NC];
#pragma unroll
	for (int c = 0; c < NC; ++c) {
		const int kind = t.res[c];
		const int16_t *d = cbase + (t.coef[c] - clo);
		if (kind == H265R_RES_NONE) res[c] = 0;
		else if (kind == H265R_RES_DC) res[c] = (d[0] + 64) >> 7; /* acNxNtransform_dconly<N, 7> (m2d.h:306-341) */
		else if (kind == H265R_RES_SKIP) res[c] = (d[y * N + x] + 16) >> 5;
		else res[c] = tres[c];
	}
	if (!(t.flags & H265R_TU_PRED)) {
		/* inter: the residual onto the motion-compensated samples */
		if (t.res[0] != H265R_RES_NONE || (NC == 2 && t.res[1] != H265R_RES_NONE)) {
			if (act) {
				if (LUMA) {
					uint8_t &p = tl.y[by + y][bx + x];
					p = (uint8_t)clampi((int)p + res[0], 0, 255);
				} else {
					uint16_t &p = *(uint16_t *)&tl.c[by + y][2 * (bx + x)];
					const int cb = clampi((int)(p & 255) + res[0], 0, 255), cr = clampi((int)(p >> 8) + res[NC - 1], 0, 255);
					p = (uint16_t)(cb | (cr << 8));
				}
			}
			wsync();
		}
		return;
	}
	/* ---- 2. reference samples, filtered (both components side by side) */
	ref_samples<N, NC, LUMA>(t, tl, s, lane, bx, by);
	H5PH(lane, t, 2);
	/* ---- 3. prediction + residual into the tile */
	int pv[NC];
#pragma unroll
	for (int c = 0; c < NC; ++c) {
		const int dcv = t.mode == 1 ? dc_value<N>(s.seq[c], lane) : 0;
		predict_samples<N, 1, LUMA>(s.seq[c], t.mode, x, &y, dcv, &pv[c]);
	}
	if (act) {
		if (LUMA) {
			tl.y[by + y][bx + x] = (uint8_t)clampi(pv[0] + res[0], 0, 255);
		} else {
			const int cb = clampi(pv[0] + res[0], 0, 255), cr = clampi(pv[NC - 1] + res[NC - 1], 0, 255);
			*(uint16_t *)&tl.c[by + y][2 * (bx + x)] = (uint16_t)(cb | (cr << 8));
		}
	}
	wsync();
	H5PH(lane, t, 3);
}

/* One block of a CTU kernel (wave-wide): dispatch on size and plane (uniform).  wait() returns once the blocks whose
 * samples this one reads are done; it runs between the residual and the reference samples. */
template <class Wait>
__device__ void do_block_ctu(const h265r_tu_t &t, CtuTile &tl, LdsCtu &s, const CtuConst &kc, int lane, int x0, int y0,
                             const int16_t *cbase, uint32_t clo, const Wait &wait)
{
	H5PH(lane, t, 0);
	/* (chroma blocks are at most 16 x 16) */
	if (t.plane) {
		if (t.log2 == 2) small_block<4, false>(t, tl, s, kc, lane, x0, y0, cbase, clo, wait);
		else if (t.log2 == 3) small_block<8, false>(t, tl, s, kc, lane, x0, y0, cbase, clo, wait);
		else big_block<16, false>(t, tl, s, kc.tb, lane, x0, y0, cbase, clo, wait);
	} else {
		if (t.log2 == 2) small_block<4, true>(t, tl, s, kc, lane, x0, y0, cbase, clo, wait);
		else if (t.log2 == 3) small_block<8, true>(t, tl, s, kc, lane, x0, y0, cbase, clo, wait);
		else if (t.log2 == 4) big_block<16, true>(t, tl, s, kc.tb, lane, x0, y0, cbase, clo, wait);
		else big_block<32, true>(t, tl, s, kc.tb, lane, x0, y0, cbase, clo, wait);
	}
}

/* the coefficients of records [c0, c0 + m) (staged in recs) into LDS when their pool range fits: one bulk
 * coalesced read per CTU instead of one dependent global round trip per block.  Returns the base / offset the
 * blocks read through. */
#define H265_CTU_COEF 6144 /* a 64 x 64 CTU's luma + chroma coefficients */
template <int NT>
__device__ __forceinline__ const int16_t *stage_coef(const H265Args &a, const h265r_tu_t *recs, int m, int16_t *cc, int *red,
                                                     int tid, uint32_t &clo)
{
	uint32_t lo = 0xffffffffu, hi = 0;
	for (int k = tid; k < m; k += NT) {
		const h265r_tu_t &t = recs[k];
		const uint32_t n2 = 1u << (2 * t.log2);
		for (int c = 0; c < 2; ++c)
			if (t.res[c] != H265R_RES_NONE && (c == 0 || t.plane)) {
				lo = min(lo, t.coef[c]);
				hi = max(hi, t.coef[c] + n2);
			}
	}
	if (tid == 0) {
		red[0] = -1;
		red[1] = 0;
	}
	__syncthreads();
	if (lo <= hi) {
		atomicMin((unsigned *)&red[0], lo);
		atomicMax((unsigned *)&red[1], hi);
	}
	__syncthreads();
	lo = (uint32_t)red[0];
	hi = (uint32_t)red[1];
	if (lo > hi || hi - lo > H265_CTU_COEF) {
		clo = 0;
		return a.coef;
	}
	const uint32_t base = lo & ~1u, nw = (hi - base + 1) >> 1; /* whole dwords from an even offset */
	const uint32_t *src = (const uint32_t *)(a.coef + base);
	for (uint32_t w = tid; w < nw; w += NT) ((uint32_t *)cc)[w] = src[w];
	__syncthreads();
	clo = base;
	return cc;
}

/* ---- the blocks of one chunk of a CTU's records.
 * NT = 128: wave 0 the luma blocks, wave 1 the chroma blocks, each in decoding order.
 * NT = 256 (M2DEC_AMD_H265_WAVES=4): two waves per plane.  A wave takes the plane's next block (an LDS
 * counter over the plane's records in decoding order), waits until the blocks that own the samples it reads
 * inside the CTU are done (the chunk's 4 x 4-unit owner maps; samples outside the CTU — the row above, the
 * left CTU — are final before the chunk starts), reconstructs it and raises its done flag.  Every wait points
 * at an earlier block of the plane, so the earliest unfinished block always runs.  Blocks of a CTU that do not
 * read each other (an inter block's residual, intra blocks whose neighbours are done) then overlap: a CTU's
 * luma wave was the per-CTU bound (r123 stamps: ~75 us of a ~105 us CTU step). */
struct CtuSched {
	uint16_t own[2][16 * 16]; /* per plane, the 4 x 4 units of the CTU (chroma: the 8 x 8 corner): the chunk record writing it, 0xffff none */
	uint16_t list[2][H265_CTU_RECS]; /* the chunk's records of each plane, in decoding order */
	int n[2], next[2];
	int done[H265_CTU_RECS];
	int bl_total, bl_cnt; /* the blocks holding the left half of the CTU's last sample row (luma and chroma), done of them */
};

template <int NT>
__device__ __forceinline__ void ctu_blocks(const H265Args &a, const h265r_tu_t *recs, int m, CtuTile &tl, LdsCtu *ls, const CtuConst &kc,
                                           CtuSched &sc, int tid, int x0, int y0, const int16_t *cb, uint32_t clo, int row, int col,
                                           int which = 0, bool pub = false)
{
	/* which: 0 every record, 1 the residual-only (inter) ones, 2 the intra-predicted ones (the inter ones done) */
	auto take = [&](const h265r_tu_t &t) { return which == 0 || ((t.flags & H265R_TU_PRED) ? 2 : 1) == which; };
	const int lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid) >> 6;
	if (NT == 128) {
		LdsCtu &s = ls[wave];
		for (int k = 0; k < m; ++k) {
			if (recs[k].plane != wave || !take(recs[k])) continue;
			const h265r_tu_t t = uniform_tu(recs[k]);
			do_block_ctu(t, tl, s, kc, lane, x0, y0, cb, clo, [] {});
			H5ST(lane, 4, row, col, t.log2 | ((t.flags & H265R_TU_PRED) << 3) | (t.res[0] << 4) | (wave << 7) | ((t.mode & 63) << 8));
		}
		(void)sc;
		return;
	}
	const int plane = wave >> 1;
	LdsCtu &s = ls[wave];
	/* the chunk's plane lists, owner maps and done flags */
	for (int i = tid; i < 2 * 16 * 16; i += NT) (&sc.own[0][0])[i] = 0xffff;
	if (tid == 0) sc.bl_total = sc.bl_cnt = 0;
	/* pub (the row kernel, 64 x 64 CTBs): the left half of the CTU's last sample row goes out as soon as the blocks
	 * holding it are done, for the CTU row below (its top-right blocks read at most 32 samples into this CTU) */
	const int ctb = 1 << a.ctb_log2, rows_here = min(ctb, a.pic_h - y0), crows = rows_here >> 1;
	auto in_bl = [&](const h265r_tu_t &t) {
		const int n = 1 << t.log2;
		return t.plane ? (t.y - (y0 >> 1) + n >= crows && t.x - (x0 >> 1) < 16) : (t.y - y0 + n >= rows_here && t.x - x0 < 32);
	};
	for (int k = tid; k < m; k += NT) sc.done[k] = which == 2 && !(recs[k].flags & H265R_TU_PRED);
	if ((wave & 1) == 0) {
		int cnt = 0;
		for (int base = 0; base < m; base += 64) {
			const int k = base + lane;
			const bool mine = k < m && recs[k].plane == plane && take(recs[k]);
			const unsigned long long mask = __ballot(mine);
			if (mine) sc.list[plane][cnt + __popcll(mask & ((1ull << lane) - 1))] = (uint16_t)k;
			cnt += __popcll(mask);
		}
		if (lane == 0) {
			sc.n[plane] = cnt;
			sc.next[plane] = 0;
		}
	}
	__syncthreads();
	int nbl = 0;
	for (int k = tid; k < m; k += NT) {
		const h265r_tu_t &t = recs[k];
		const int u = (1 << t.log2) >> 2;
		const int ux = (t.plane ? t.x - (x0 >> 1) : t.x - x0) >> 2, uy = (t.plane ? t.y - (y0 >> 1) : t.y - y0) >> 2;
		for (int j = 0; j < u * u; ++j) sc.own[t.plane][(uy + j / u) * 16 + ux + j % u] = (uint16_t)k;
		nbl += pub && in_bl(t);
	}
	if (nbl) atomicAdd(&sc.bl_total, nbl);
	__syncthreads();
	for (;;) {
		/* (every lane adds, lane 0 by 1, and the wave takes lane 0's value: no single-lane section inside the
		 * persistent loop — DESIGN §5 compiler hazards) */
		const int pos = __builtin_amdgcn_readfirstlane(atomicAdd(&sc.next[plane], lane == 0 ? 1 : 0));
		if (pos >= __builtin_amdgcn_readfirstlane(sc.n[plane])) break;
		const int k = __builtin_amdgcn_readfirstlane(sc.list[plane][pos]);
		const h265r_tu_t t = uniform_tu(recs[k]);
		auto wait = [&] {
			if (!(t.flags & H265R_TU_PRED)) return;
			/* the owners of the samples it reads inside the CTU: lane i < ntop the units above, then the units to the
			 * left, then the corner */
			const int n = 1 << t.log2;
			const int bx = t.plane ? t.x - (x0 >> 1) : t.x - x0, by = t.plane ? t.y - (y0 >> 1) : t.y - y0;
			const int at = t.avail_top > 2 * n ? 2 * n : t.avail_top, al = t.avail_left > 2 * n ? 2 * n : t.avail_left;
			const int ntop = (by > 0 && at > 0) ? (at + 3) >> 2 : 0, nleft = (bx > 0 && al > 0) ? (al + 3) >> 2 : 0;
			const bool corner = bx > 0 && by > 0 && at > 0 && al > 0;
			int unit = -1;
			if (lane < ntop) unit = ((by >> 2) - 1) * 16 + (bx >> 2) + lane;
			else if (lane < ntop + nleft) unit = ((by >> 2) + lane - ntop) * 16 + (bx >> 2) - 1;
			else if (lane == ntop + nleft && corner) unit = ((by >> 2) - 1) * 16 + (bx >> 2) - 1;
			const int o = unit >= 0 && unit < 256 ? sc.own[t.plane][unit] : 0xffff;
			unsigned spins = 0;
			for (;;) {
				const bool ok = o == 0xffff || o >= k || __hip_atomic_load(&sc.done[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
				if (__all(ok)) break;
				if (++spins > H265_SPIN_LIMIT) {
					__hip_atomic_store((gi32 *)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					break;
				}
				if ((spins & 255) == 0 && __hip_atomic_load((gi32 *)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
				__builtin_amdgcn_s_sleep(1);
			}
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
		};
#ifdef H265_WAIT_FIRST
		wait();
		do_block_ctu(t, tl, s, kc, lane, x0, y0, cb, clo, [] {});
#else
		do_block_ctu(t, tl, s, kc, lane, x0, y0, cb, clo, wait);
#endif
		H5ST(lane, 4, row, col, t.log2 | ((t.flags & H265R_TU_PRED) << 3) | (t.res[0] << 4) | (plane << 7) | ((t.mode & 63) << 8));
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
		__hip_atomic_store(&sc.done[k], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); /* (every lane: the same word) */
		if (pub && in_bl(t)) {
			const int seen = __builtin_amdgcn_readfirstlane(atomicAdd(&sc.bl_cnt, lane == 0 ? 1 : 0));
			if (seen + 1 == __builtin_amdgcn_readfirstlane(sc.bl_total)) {
				/* the last of them: every other one's tile writes were released before its count */
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
				if (lane < 16) {
					const int c = lane >> 3, w = lane & 7; /* 8 luma words, then 8 words of CbCr pairs */
					if (c == 0) st_word(plane_px(a, 0, 0, x0 + 4 * w, y0 + rows_here - 1), *(const uint32_t *)&tl.y[rows_here - 1][4 * w]);
					else st_word(plane_px(a, 1, 0, (x0 >> 1) + 2 * w, (y0 >> 1) + crows - 1), *(const uint32_t *)&tl.c[crows - 1][4 * w]);
				}
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				__hip_atomic_store((gi32 *)&a.progress[row], 2 * col + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
		}
	}
}

/* first record of every CTU (records are in decoding order, CTUs in raster order) */
__global__ __launch_bounds__(256) void k_h265_ctu_index(const H265Args *ap)
{
	const H265Args &a = *ap;
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	const int nctu = a.ctu_cols * a.ctu_rows;
	if (i > a.n_tu) return;
	auto ctu_of = [&](int k) {
		const h265r_tu_t &t = a.tu[k];
		const int x = t.plane ? 2 * t.x : t.x, y = t.plane ? 2 * t.y : t.y;
		return (y >> a.ctb_log2) * a.ctu_cols + (x >> a.ctb_log2);
	};
	const int cur = i < a.n_tu ? ctu_of(i) : nctu;
	const int prev = i > 0 ? ctu_of(i - 1) : -1;
	for (int c = prev + 1; c <= cur && c <= nctu; ++c) a.ctu_first[c] = i;
}

template <int NT>
__global__ __launch_bounds__(NT, 2) void k_h265_ctu_rows(const H265Args *ap)
{
	const H265Args a = *ap;
	__shared__ LdsCtu ls[NT / 64];
	__shared__ CtuConst kc;
	__shared__ CtuTile tl;
	__shared__ h265r_tu_t recs[H265_CTU_RECS]; /* the CTU's records, staged (every wave reads all of them) */
	__shared__ __attribute__((aligned(16))) int16_t ccoef[H265_CTU_COEF + 2];
	__shared__ int red[2];
	__shared__ CtuSched sch;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid) >> 6; /* NT 128: 0 luma, 1 chroma; NT 256: 0-1 luma, 2-3 chroma */
	const int row = blockIdx.x;
	const int ctb = 1 << a.ctb_log2, cctb = ctb >> 1;
	ctu_const_init(kc, tid, NT); /* (read after the barrier ahead of the first CTU's blocks) */
	const int y0 = row << a.ctb_log2;
	const int rows_here = min(ctb, a.pic_h - y0), crows = rows_here >> 1;
	for (int col = 0; col < a.ctu_cols; ++col) {
		const int x0 = col << a.ctb_log2;
		const int cols_here = min(ctb, a.pic_w - x0);
		H5ST(tid, 0, row, col, 0);
		/* the column left of this CTU: the previous CTU's last column (unavailable at col 0) */
		if (tid < ctb) {
			tl.ly[tid] = col ? tl.y[tid][ctb - 1] : 128;
			tl.lc[tid] = col ? tl.c[tid >> 1][ctb - 2 + (tid & 1)] : 128;
		}
		/* P / B pictures: the CTU starts from its motion-compensated samples (k_h265_mc, an earlier launch) */
		if (a.n_pu) {
			__syncthreads(); /* (the previous CTU's last column is in tl.ly) */
			const int wpr = (cols_here + 3) >> 2;
			for (int w = tid; w < wpr * rows_here; w += NT) {
				const int yy = w / wpr, xx = (w - yy * wpr) * 4;
				*(uint32_t *)&tl.y[yy][xx] = *(const uint32_t *)plane_px(a, 0, 0, x0 + xx, y0 + yy);
			}
			for (int w = tid; w < wpr * crows; w += NT) {
				const int yy = w / wpr, xx = (w - yy * wpr) * 4;
				*(uint32_t *)&tl.c[yy][xx] = *(const uint32_t *)plane_px(a, 1, 0, (x0 >> 1) + (xx >> 1), (y0 >> 1) + yy);
			}
		}
		/* the CTU's first chunk of records and its coefficients into LDS before the wait for the row above: the
		 * staging (two dependent global round trips) overlaps that wait, which is the wavefront's critical path */
		const int c = row * a.ctu_cols + col;
		const int i0 = a.ctu_first[c], i1 = a.ctu_first[c + 1];
		const int m0 = min(H265_CTU_RECS, i1 - i0);
		__syncthreads(); /* (the previous CTU's records / coefficients are consumed) */
		for (int k = tid; k < m0 * (int)(sizeof(h265r_tu_t) / 4); k += NT) ((uint32_t *)recs)[k] = ((const uint32_t *)(a.tu + i0))[k];
		__syncthreads();
		uint32_t clo0;
		const int16_t *cb0 = stage_coef<NT>(a, recs, m0, ccoef, red, tid, clo0);
		/* does a block of this CTU read the row above?  Only an intra-predicted block on the CTU's top edge does
		 * (a block below it reads the tile; inter blocks start from the motion-compensated samples, an earlier
		 * launch).  A CTU without one neither waits for the row above nor loads it: in P / B pictures, where
		 * most CTUs hold only inter blocks, the CTU rows run side by side instead of as a 2-CTU-lag wavefront */
		int above = 0;
		if (row > 0) {
			for (int k = tid; k < i1 - i0; k += NT) {
				const h265r_tu_t &t = k < m0 ? recs[k] : a.tu[i0 + k];
				if ((t.flags & H265R_TU_PRED) && (t.plane ? 2 * t.y : t.y) == y0) above = 1;
			}
			above = __syncthreads_or(above);
		}
		/* the row above, once that CTU row finished the CTU above-right */
		if (above) {
			if (wave == 0) {
				/* progress is in half CTUs: 2 c + 1 once CTU c's last row's left half is out (64 x 64 CTBs only), 2 (c + 1)
				 * once CTU c is done; with 64 x 64 CTBs (transform blocks <= 32) a CTU reads the row above at most 32
				 * samples into the CTU above-right, with smaller CTBs possibly all of it (then no half step is
				 * published and the wait is for the whole CTU) */
				const int need = col + 1 < a.ctu_cols ? 2 * (col + 1) + 1 : 2 * a.ctu_cols;
				unsigned spins = 0;
				for (;;) {
					const int got = __hip_atomic_load((gi32 *)&a.progress[row - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if (got >= need) break;
					if (++spins > H265_SPIN_LIMIT) {
						__hip_atomic_store((gi32 *)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						break;
					}
					if (__hip_atomic_load((gi32 *)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
					__builtin_amdgcn_s_sleep(1);
				}
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			}
			__syncthreads();
			for (int i = tid; i <= 2 * ctb; i += NT) {
				const int x = x0 - 1 + i;
				tl.ty[i] = (x >= 0 && x < a.pic_w) ? (uint8_t)ld_px(a, 0, 0, x, y0 - 1) : 128;
			}
			for (int i = tid; i < 2 * (ctb + 1); i += NT) {
				const int x = (x0 >> 1) - 1 + (i >> 1);
				tl.tc[i] = (x >= 0 && x < (a.pic_w >> 1)) ? (uint8_t)ld_px(a, 1, i & 1, x, (y0 >> 1) - 1) : 128;
			}
		}
		__syncthreads();
		H5ST(tid, 1, row, col, above);
		/* the CTU's blocks (luma on waves 0-1, chroma on waves 2-3, each plane in decoding order): the staged first
		 * chunk, then any further chunk of a CTU with more than H265_CTU_RECS records */
		if (m0 > 0)
			ctu_blocks<NT>(a, recs, m0, tl, ls, kc, sch, tid, x0, y0, cb0, clo0, row, col, 0,
			               m0 == i1 - i0 && row + 1 < a.ctu_rows && a.ctb_log2 == 6 && !(a.flags & (1 << 28)));
		for (int c0 = i0 + m0; c0 < i1; c0 += H265_CTU_RECS) {
			const int m = min(H265_CTU_RECS, i1 - c0);
			__syncthreads(); /* (the previous chunk is consumed) */
			for (int k = tid; k < m * (int)(sizeof(h265r_tu_t) / 4); k += NT)
				((uint32_t *)recs)[k] = ((const uint32_t *)(a.tu + c0))[k];
			__syncthreads();
			uint32_t clo;
			const int16_t *cb = stage_coef<NT>(a, recs, m, ccoef, red, tid, clo);
			ctu_blocks<NT>(a, recs, m, tl, ls, kc, sch, tid, x0, y0, cb, clo, row, col);
		}
		H5ST(lane, 2, row, col, wave);
		__syncthreads();
		/* out: the CTU's samples (inside the picture) as write-through words, drained, then the progress word */
		{
			const int wpr = (cols_here + 3) >> 2;
			for (int w = tid; w < wpr * rows_here; w += NT) {
				const int yy = w / wpr, xx = (w - yy * wpr) * 4;
				st_word(plane_px(a, 0, 0, x0 + xx, y0 + yy), *(const uint32_t *)&tl.y[yy][xx]);
			}
			const int cw = (cols_here + 3) >> 2; /* words of CbCr pairs per chroma row: cols_here bytes */
			for (int w = tid; w < cw * crows; w += NT) {
				const int yy = w / cw, xx = (w - yy * cw) * 4;
				st_word(plane_px(a, 1, 0, (x0 >> 1) + (xx >> 1), (y0 >> 1) + yy), *(const uint32_t *)&tl.c[yy][xx]);
			}
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			__syncthreads();
			if (tid == 0) __hip_atomic_store((gi32 *)&a.progress[row], 2 * (col + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			H5ST(tid, 3, row, col, 0);
		}
	}
	(void)cctb;
}

/* ---- P / B pictures: one workgroup per CTU (k_h265_ctu_rows's body without the row carry).  Most CTUs of an
 * inter picture hold only inter blocks: they start from the motion-compensated samples and add their residuals,
 * side by side with every other CTU.  A CTU with an intra-predicted block on its left / top edge waits for the
 * neighbour CTUs that block reads (left, above-left, above, above-right: lower raster indices, i.e. workgroups
 * dispatched earlier, so a wait always ends) and loads their published edge samples; the row kernel's 17
 * workgroups of a 1080p picture instead walked their 30 CTUs one after another. */
template <int NT>
__global__ __launch_bounds__(NT, 2) void k_h265_ctu_grid(const H265Args *ap)
{
	const H265Args a = *ap;
	__shared__ LdsCtu ls[NT / 64];
	__shared__ CtuConst kc;
	__shared__ CtuTile tl;
	__shared__ h265r_tu_t recs[H265_CTU_RECS];
	__shared__ __attribute__((aligned(16))) int16_t ccoef[H265_CTU_COEF + 2];
	__shared__ int red[2];
	__shared__ CtuSched sch;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid) >> 6; /* 0 luma, 1 chroma */
	const int c = blockIdx.x, row = c / a.ctu_cols, col = c - row * a.ctu_cols;
	const int ctb = 1 << a.ctb_log2;
	const int x0 = col << a.ctb_log2, y0 = row << a.ctb_log2;
	const int rows_here = min(ctb, a.pic_h - y0), crows = rows_here >> 1, cols_here = min(ctb, a.pic_w - x0);
	const int i0 = a.ctu_first[c], i1 = a.ctu_first[c + 1];
	gi32 *done = (gi32 *)(a.ctu_first + a.ctu_cols * a.ctu_rows + 1);
	__shared__ int s_need;
	if (i0 < i1) {
		ctu_const_init(kc, tid, NT);
		/* the neighbour CTUs the CTU's edge intra blocks read: 1 left, 2 above-left, 4 above, 8 above-right */
		int need = 0;
		if (tid == 0) s_need = 0;
		__syncthreads();
		for (int k = i0 + tid; k < i1; k += NT) {
			const h265r_tu_t &t = a.tu[k];
			if (!(t.flags & H265R_TU_PRED)) continue;
			const int n = 1 << t.log2, sc = t.plane ? 2 : 1, lx = sc * t.x, ly = sc * t.y;
			const int at = t.avail_top > 2 * n ? 2 * n : t.avail_top, al = t.avail_left > 2 * n ? 2 * n : t.avail_left;
			const bool top = at > 0, left = al > 0;
			if (lx == x0 && left) need |= 1;
			if (lx == x0 && ly == y0 && top && left) need |= 2;
			if (ly == y0 && top) need |= 4 | (lx + sc * at > x0 + ctb ? 8 : 0);
		}
		if (need) atomicOr(&s_need, need);
		__syncthreads();
		need = s_need;
		/* the motion-compensated samples (k_h265_mc, an earlier launch) */
		if (a.n_pu) {
			const int wpr = (cols_here + 3) >> 2;
			for (int w = tid; w < wpr * rows_here; w += NT) {
				const int yy = w / wpr, xx = (w - yy * wpr) * 4;
				*(uint32_t *)&tl.y[yy][xx] = *(const uint32_t *)plane_px(a, 0, 0, x0 + xx, y0 + yy);
			}
			for (int w = tid; w < wpr * crows; w += NT) {
				const int yy = w / wpr, xx = (w - yy * wpr) * 4;
				*(uint32_t *)&tl.c[yy][xx] = *(const uint32_t *)plane_px(a, 1, 0, (x0 >> 1) + (xx >> 1), (y0 >> 1) + yy);
			}
		}
		/* A CTU whose intra blocks wait for neighbour CTUs first adds the residuals of its inter blocks (which read
		 * nothing outside themselves), then waits, then reconstructs its intra blocks in decoding order (an intra
		 * block reads only earlier blocks' samples: the inter ones are final by then): the inter work leaves the
		 * chain of intra CTUs (r166: the neighbour waits were ~75 % of the 1080p P / B CTU pass).  A CTU with more
		 * records than one LDS chunk keeps the single pass. */
		const bool split = need && i1 - i0 <= H265_CTU_RECS && !(a.flags & (1 << 29));
		uint32_t clo0 = 0;
		const int16_t *cb0 = nullptr;
		if (split) {
			__syncthreads(); /* (the tile) */
			for (int k = tid; k < (i1 - i0) * (int)(sizeof(h265r_tu_t) / 4); k += NT) ((uint32_t *)recs)[k] = ((const uint32_t *)(a.tu + i0))[k];
			__syncthreads();
			cb0 = stage_coef<NT>(a, recs, i1 - i0, ccoef, red, tid, clo0);
			ctu_blocks<NT>(a, recs, i1 - i0, tl, ls, kc, sch, tid, x0, y0, cb0, clo0, row, col, 1);
		}
		/* wave 0 lanes 0..3 poll one neighbour each */
		if (wave == 0 && need && !(a.flags & (1 << 30))) {
			int dep = -1;
			if (lane == 0 && (need & 1)) dep = c - 1;
			if (lane == 1 && (need & 2)) dep = c - a.ctu_cols - 1;
			if (lane == 2 && (need & 4)) dep = c - a.ctu_cols;
			if (lane == 3 && (need & 8) && col + 1 < a.ctu_cols) dep = c - a.ctu_cols + 1;
			unsigned spins = 0;
			for (;;) {
				const bool ok = dep < 0 || __hip_atomic_load(&done[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
				if (__all(ok)) break;
				if (++spins > H265_SPIN_LIMIT) {
					__hip_atomic_store((gi32 *)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					break;
				}
				if (__hip_atomic_load((gi32 *)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
				__builtin_amdgcn_s_sleep(1);
			}
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		}
		__syncthreads();
		/* the neighbours' edge samples (published as write-through words: read at agent scope) */
		if (need & 1)
			for (int i = tid; i < 2 * ctb; i += NT) {
				if (i < ctb) tl.ly[i] = i < rows_here ? (uint8_t)ld_px(a, 0, 0, x0 - 1, y0 + i) : 128;
				else tl.lc[i - ctb] = (i - ctb) < rows_here ? (uint8_t)ld_px(a, 1, (i - ctb) & 1, (x0 >> 1) - 1, (y0 >> 1) + ((i - ctb) >> 1)) : 128;
			}
		if (need & 14) {
			for (int i = tid; i <= 2 * ctb; i += NT) {
				const int x = x0 - 1 + i;
				const bool in = x >= 0 && x < a.pic_w && (i > 0 || (need & 2)) && (i <= ctb || (need & 8));
				tl.ty[i] = in ? (uint8_t)ld_px(a, 0, 0, x, y0 - 1) : 128;
			}
			for (int i = tid; i < 2 * (ctb + 1); i += NT) {
				const int x = (x0 >> 1) - 1 + (i >> 1);
				const bool in = x >= 0 && x < (a.pic_w >> 1) && (i > 1 || (need & 2)) && (i < ctb + 2 || (need & 8));
				tl.tc[i] = in ? (uint8_t)ld_px(a, 1, i & 1, x, (y0 >> 1) - 1) : 128;
			}
		}
		/* the CTU's blocks (luma on waves 0-1, chroma on waves 2-3, each plane in decoding order): the intra ones of a
		 * split CTU, else all of them */
		if (split) {
			__syncthreads(); /* (the edge samples) */
			ctu_blocks<NT>(a, recs, i1 - i0, tl, ls, kc, sch, tid, x0, y0, cb0, clo0, row, col, 2);
		}
		for (int c0 = i0; c0 < i1 && !split; c0 += H265_CTU_RECS) {
			const int m = min(H265_CTU_RECS, i1 - c0);
			__syncthreads(); /* (the tile / the previous chunk) */
			for (int k = tid; k < m * (int)(sizeof(h265r_tu_t) / 4); k += NT) ((uint32_t *)recs)[k] = ((const uint32_t *)(a.tu + c0))[k];
			__syncthreads();
			uint32_t clo;
			const int16_t *cb = stage_coef<NT>(a, recs, m, ccoef, red, tid, clo);
			ctu_blocks<NT>(a, recs, m, tl, ls, kc, sch, tid, x0, y0, cb, clo, row, col);
		}
		__syncthreads();
		/* out: the CTU's samples as write-through words, drained before the done flag */
		const int wpr = (cols_here + 3) >> 2;
		for (int w = tid; w < wpr * rows_here; w += NT) {
			const int yy = w / wpr, xx = (w - yy * wpr) * 4;
			st_word(plane_px(a, 0, 0, x0 + xx, y0 + yy), *(const uint32_t *)&tl.y[yy][xx]);
		}
		for (int w = tid; w < wpr * crows; w += NT) {
			const int yy = w / wpr, xx = (w - yy * wpr) * 4;
			st_word(plane_px(a, 1, 0, (x0 >> 1) + (xx >> 1), (y0 >> 1) + yy), *(const uint32_t *)&tl.c[yy][xx]);
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
	}
	if (tid == 0) __hip_atomic_store(&done[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* ---- the picture's records from the pinned arena into device memory (16 bytes per thread, grid-stride) */
/* a copy by a kernel (records up from the pinned arena, frames down to pinned staging); `zero` (nzero ints): the
 * picture's scratch words cleared in the same launch (one HIP call fewer per picture on the serial submission) */
__global__ __launch_bounds__(256) void k_h265_upload(const uint4 *src, uint4 *dst, size_t n16, int *zero, size_t nzero)
{
	const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
	for (size_t i = t; i < n16; i += step) dst[i] = src[i];
	for (size_t i = t; i < nzero; i += step) zero[i] = 0;
}

/* ---- motion compensation (h265.cpp:3132-3595; oracle/h265_oracle.c mc_picture) */
__constant__ int8_t c_luma_fir[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0}, {-1, 4, -10, 58, 17, -5, 1, 0}, {-1, 4, -11, 40, 40, -11, 4, -1}, {0, 1, -5, 17, 58, -10, 4, -1}};
__constant__ int8_t c_chroma_fir[8][4] = {{0, 64, 0, 0}, {2, 58, 10, 2}, {4, 54, 16, 2}, {6, 46, 28, 4}, {4, 36, 36, 4}, {4, 28, 46, 6}, {2, 16, 54, 4}, {2, 10, 58, 2}};

#define MC_WIN 72 /* luma window row pitch: 64 + 7 */
struct McLds {
	uint8_t win[(64 + 7) * MC_WIN];     /* luma reference window */
	uint8_t cwin[(32 + 3) * (32 + 3) * 2]; /* CbCr pairs */
	int16_t acc[64 * 64];               /* bi-prediction: the first list's luma */
	int16_t cacc[32 * 64];              /* ... and chroma (Cb, Cr interleaved) */
};

__device__ __forceinline__ int mc_clampx(int v, int m) { return v < 0 ? 0 : (v >= m ? m - 1 : v); }

/* store_pix<1> / store_pix<0> / add_store_pix, with the reference's 32-bit wrap */
__device__ __forceinline__ uint8_t mc_uni(int v, int sh) { return (uint8_t)mc_clampx((int)((unsigned)v + (1u << (sh - 1))) >> sh, 256); }
__device__ __forceinline__ int16_t mc_bi0(int v, int sh) { return (int16_t)(v >> sh); }
__device__ __forceinline__ uint8_t mc_bi1(int16_t d, int v, int sh) { return (uint8_t)mc_clampx((int)((unsigned)d + (unsigned)(v >> sh) + 64u) >> 7, 256); }

__device__ __forceinline__ uint64_t mc_chroma_h(const uint8_t *cw, int pitch, int r, int x, int fx)
{
	const uint8_t *q = cw + (size_t)(r * pitch + x) * 2;
	const uint64_t a0 = ((uint64_t)q[0] << 32) | q[1], a1 = ((uint64_t)q[2] << 32) | q[3];
	const uint64_t a2 = ((uint64_t)q[4] << 32) | q[5], a3 = ((uint64_t)q[6] << 32) | q[7];
	const uint64_t c0 = (uint64_t)c_chroma_fir[fx][0], c1 = (uint64_t)c_chroma_fir[fx][1], c2 = (uint64_t)c_chroma_fir[fx][2],
	               c3 = (uint64_t)c_chroma_fir[fx][3];
	return (((c1 * a1 + c2 * a2) | 0x80000000ull) - (c0 * a0 + c3 * a3)) & ~0xf8000000ull;
}

__global__ __launch_bounds__(64) void k_h265_mc(const H265Args *ap)
{
	const H265Args &a = *ap;
	__shared__ McLds s;
	const int lane = threadIdx.x;
	const int W = a.W, pw = a.pic_w, ph = a.pic_h, cw = a.pic_w >> 1, chh = a.pic_h >> 1;
	for (int pi = blockIdx.x; pi < a.n_pu; pi += gridDim.x) {
		const h265r_pu_t u = a.pu[pi];
		const int w = u.w, h = u.h;
		const bool bi = u.ref[0] >= 0 && u.ref[1] >= 0;
		const int full = bi ? 6 : 12;
		uint8_t *luma = a.frame, *chroma = a.frame + (size_t)W * a.H;
		bool first = true;
		for (int l = 0; l < 2; ++l) {
			if (u.ref[l] < 0) continue;
			const uint8_t *rl = a.frames + (size_t)u.ref[l] * a.fsz, *rc = rl + (size_t)W * a.H;
			const int mvx = u.mv[l][0], mvy = u.mv[l][1];
			const int fx = mvx & 3, fy = mvy & 3, xi = u.x + (mvx >> 2) - 3, yi = u.y + (mvy >> 2) - 3;
			const int cfx = mvx & 7, cfy = mvy & 7, cxi = (u.x >> 1) + (mvx >> 3) - 1, cyi = (u.y >> 1) + (mvy >> 3) - 1;
			const int ww = w + 7, wh = h + 7, cww = (w >> 1) + 3, cwh = (h >> 1) + 3;
			__syncthreads(); /* (the previous list's / block's windows are consumed) */
			for (int i = lane; i < ww * wh; i += 64) {
				const int r = i / ww, c = i - r * ww;
				s.win[r * MC_WIN + c] = rl[(size_t)mc_clampx(yi + r, ph) * W + mc_clampx(xi + c, pw)];
			}
			for (int i = lane; i < cww * cwh; i += 64) {
				const int r = i / cww, c = i - r * cww;
				const uint8_t *q = rc + (size_t)mc_clampx(cyi + r, chh) * W + (size_t)mc_clampx(cxi + c, cw) * 2;
				s.cwin[(r * cww + c) * 2] = q[0];
				s.cwin[(r * cww + c) * 2 + 1] = q[1];
			}
			__syncthreads();
			for (int i = lane; i < w * h; i += 64) {
				const int y = i / w, x = i - y * w;
				int v = 0, sh = full;
				if (!fx && !fy) {
					v = (int)s.win[(y + 3) * MC_WIN + x + 3] << 12;
				} else if (!fy) {
					const uint8_t *q = &s.win[(y + 3) * MC_WIN + x];
#pragma unroll
					for (int k = 0; k < 8; ++k) v += c_luma_fir[fx][k] * (int)q[k];
					sh = full - 6;
				} else if (!fx) {
					const uint8_t *q = &s.win[y * MC_WIN + x + 3];
#pragma unroll
					for (int k = 0; k < 8; ++k) v += c_luma_fir[fy][k] * (int)q[k * MC_WIN];
					sh = full - 6;
				} else {
#pragma unroll
					for (int r = 0; r < 8; ++r) {
						const uint8_t *q = &s.win[(y + r) * MC_WIN + x];
						int hs = 0;
#pragma unroll
						for (int k = 0; k < 8; ++k) hs += c_luma_fir[fx][k] * (int)q[k];
						v += c_luma_fir[fy][r] * (int)(int16_t)hs;
					}
				}
				uint8_t *o = luma + (size_t)(u.y + y) * W + u.x + x;
				if (!bi) *o = mc_uni(v, sh);
				else if (first) s.acc[y * 64 + x] = mc_bi0(v, sh);
				else *o = mc_bi1(s.acc[y * 64 + x], v, sh);
			}
			for (int i = lane; i < (w >> 1) * (h >> 1); i += 64) {
				const int y = i / (w >> 1), x = i - y * (w >> 1);
				const uint64_t h0 = mc_chroma_h(s.cwin, cww, y, x, cfx), h1 = mc_chroma_h(s.cwin, cww, y + 1, x, cfx);
				const uint64_t h2 = mc_chroma_h(s.cwin, cww, y + 2, x, cfx), h3 = mc_chroma_h(s.cwin, cww, y + 3, x, cfx);
				const uint64_t k0 = (uint64_t)c_chroma_fir[cfy][0], k1 = (uint64_t)c_chroma_fir[cfy][1], k2 = (uint64_t)c_chroma_fir[cfy][2],
				               k3 = (uint64_t)c_chroma_fir[cfy][3];
				const uint64_t wv = ((h1 * k1 + h2 * k2) | 0x80000000ull) - (h0 * k0 + h3 * k3);
				const int vb = (int)(uint32_t)(wv >> 32), vr = (int)((uint32_t)wv ^ 0x80000000u);
				uint8_t *o = chroma + (size_t)((u.y >> 1) + y) * W + u.x + 2 * x;
				int16_t *ca = &s.cacc[y * 64 + 2 * x];
				if (!bi) {
					o[0] = mc_uni(vb, full);
					o[1] = mc_uni(vr, full);
				} else if (first) {
					ca[0] = mc_bi0(vb, full);
					ca[1] = mc_bi0(vr, full);
				} else {
					o[0] = mc_bi1(ca[0], vb, full);
					o[1] = mc_bi1(ca[1], vr, full);
				}
			}
			first = false;
		}
	}
}

/* ---- deblocking (8.7.2; oracle/h265_oracle.c luma_edge / chroma_edge) */
__device__ __forceinline__ void luma_edge(uint8_t *sp, int xs, int ls, int bs, int qp, int beta_off, int tc_off)
{
	const int bq = clampi(qp + beta_off, 0, 51), tq = clampi(qp + 2 * (bs - 1) + tc_off, 0, 51); /* tc QP clipped to 51 (reference) */
	const int beta = bq < 16 ? 0 : c_beta[bq - 16], tc = tq < 16 ? 0 : c_tc[tq - 16];
#define P(i, k) sp[(k) * ls - ((i) + 1) * xs]
#define Q(i, k) sp[(k) * ls + (i) * xs]
	const int dp0 = abs(P(2, 0) - 2 * P(1, 0) + P(0, 0)), dp3 = abs(P(2, 3) - 2 * P(1, 3) + P(0, 3));
	const int dq0 = abs(Q(2, 0) - 2 * Q(1, 0) + Q(0, 0)), dq3 = abs(Q(2, 3) - 2 * Q(1, 3) + Q(0, 3));
	if (!(dp0 + dq0 + dp3 + dq3 < beta)) return;
	bool strong = true;
	for (int k = 0; k < 4; k += 3) {
		const int dpq = 2 * ((k ? dp3 : dp0) + (k ? dq3 : dq0));
		if (!(dpq < (beta >> 2) && abs(P(3, k) - P(0, k)) + abs(Q(0, k) - Q(3, k)) < (beta >> 3) &&
		      abs(P(0, k) - Q(0, k)) < ((5 * tc + 1) >> 1)))
			strong = false;
	}
	const int dep = (dp0 + dp3) < ((beta + (beta >> 1)) >> 3), deq = (dq0 + dq3) < ((beta + (beta >> 1)) >> 3);
	for (int k = 0; k < 4; ++k) {
		const int p0 = P(0, k), p1 = P(1, k), p2 = P(2, k), p3 = P(3, k);
		const int q0 = Q(0, k), q1 = Q(1, k), q2 = Q(2, k), q3 = Q(3, k);
		if (strong) {
			const int t2 = 2 * tc;
			P(0, k) = (uint8_t)clampi((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, p0 - t2, p0 + t2);
			P(1, k) = (uint8_t)clampi((p2 + p1 + p0 + q0 + 2) >> 2, p1 - t2, p1 + t2);
			P(2, k) = (uint8_t)clampi((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3, p2 - t2, p2 + t2);
			Q(0, k) = (uint8_t)clampi((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, q0 - t2, q0 + t2);
			Q(1, k) = (uint8_t)clampi((p0 + q0 + q1 + q2 + 2) >> 2, q1 - t2, q1 + t2);
			Q(2, k) = (uint8_t)clampi((p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3, q2 - t2, q2 + t2);
		} else {
			int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
			if (abs(delta) < tc * 10) {
				delta = clampi(delta, -tc, tc);
				P(0, k) = (uint8_t)clampi(p0 + delta, 0, 255);
				Q(0, k) = (uint8_t)clampi(q0 - delta, 0, 255);
				if (dep) P(1, k) = (uint8_t)clampi(p1 + clampi((((p2 + p0 + 1) >> 1) - p1 + delta) >> 1, -(tc >> 1), tc >> 1), 0, 255);
				if (deq) Q(1, k) = (uint8_t)clampi(q1 + clampi((((q2 + q0 + 1) >> 1) - q1 - delta) >> 1, -(tc >> 1), tc >> 1), 0, 255);
			}
		}
	}
#undef P
#undef Q
}

__device__ __forceinline__ int qpc_deb(int qpi)
{
	if (qpi < 30) return qpi;
	if (qpi >= 43) return qpi - 6;
	const int t[13] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37};
	return t[qpi - 30];
}

__device__ __forceinline__ void chroma_edge(uint8_t *sp, int xs, int ls, int qp, int qp_off, int tc_off)
{
	const int q = clampi(qpc_deb(qp + qp_off) + 2 + tc_off, 0, 53);
	if (q < 16) return;
	const int tc = c_tc[q - 16];
	for (int k = 0; k < 2; ++k) {
		uint8_t *l = sp + k * ls;
		const int p1 = l[-2 * xs], p0 = l[-xs], q0 = l[0], q1 = l[xs];
		const int delta = clampi((((q0 - p0) * 4) + p1 - q1 + 4) >> 3, -tc, tc);
		if (delta) {
			l[-xs] = (uint8_t)clampi(p0 + delta, 0, 255);
			l[0] = (uint8_t)clampi(q0 - delta, 0, 255);
		}
	}
}

__global__ __launch_bounds__(256) void k_h265_deblock(const H265Args *ap, int dir)
{
	const H265Args &a = *ap;
	const int W = a.W, H = a.H;
	const int rows = dir ? H / 8 : H / 4, cols = dir ? W / 4 : W / 8;
	const int id = blockIdx.x * blockDim.x + threadIdx.x;
	if (id >= rows * cols) return;
	const int j = id / cols, i = id - j * cols;
	const int v = (dir ? a.bs_h : a.bs_v)[id], b = v & 3, qp = v >> 2;
	if (!b) return;
	const int ex = dir ? 4 * i : 8 * i, ey = dir ? 8 * j : 4 * j;
	uint8_t *luma = a.frame + (size_t)ey * W + ex;
	if (dir == 0) luma_edge(luma, 1, W, b, qp, a.beta_offset, a.tc_offset);
	else luma_edge(luma, W, 1, b, qp, a.beta_offset, a.tc_offset);
	if (b == 2 && ((dir == 0 ? ex : ey) & 15) == 0) {
		const int cx = ex >> 1, cy = ey >> 1;
		for (int c = 0; c < 2; ++c) {
			uint8_t *sp = a.frame + (size_t)W * H + (size_t)cy * W + (size_t)(2 * cx + c);
			const int off = c ? a.cr_qp_offset : a.cb_qp_offset;
			if (dir == 0) chroma_edge(sp, 2, W, qp, off, a.tc_offset);
			else chroma_edge(sp, W, 2, qp, off, a.tc_offset);
		}
	}
}

/* ---- SAO (8.7.3; oracle/h265_oracle.c sao) */
/* SAO of one sample (sao_bo_block / sao_eo_block, h265.cpp:4386-4729): plane ci (0 luma, 1 Cb, 2 Cr) at sample
 * (x, y) of a plane of pw x ph samples, `step` bytes apart in rows of W bytes; v its deblocked value */
__device__ __forceinline__ int sao_sample(const H265Args &a, const uint8_t *src, int ci, int x, int y, int pw, int ph, int step, int v)
{
	const int W = a.W;
	const int sub = ci ? 1 : 0, cs = (1 << a.ctb_log2) >> sub;
	const int cols = (a.pic_w + (1 << a.ctb_log2) - 1) >> a.ctb_log2;
	const h265r_sao_t &sa = a.sao[(y / cs) * cols + x / cs];
	const int type = sa.type[ci];
	if (!type) return v;
	int o = 0;
	if (type == 1) {
		const int k = (v >> 3) - sa.band[ci]; /* no band-table wrap (sao_bo_block, reference quirk) */
		if (k >= 0 && k < 4) o = sa.off[ci][k];
	} else {
		const int e = sa.eo[ci];
		const int dx0 = e == 1 ? 0 : (e == 3 ? 1 : -1), dy0 = e == 0 ? 0 : -1;
		const int ax = x + dx0, ay = y + dy0, bx = x - dx0, by = y - dy0;
		if (ax < 0 || ay < 0 || bx < 0 || by < 0 || ax >= pw || bx >= pw || ay >= ph || by >= ph) return v;
		const int pa = src[(size_t)ay * W + (size_t)ax * step], pb = src[(size_t)by * W + (size_t)bx * step];
		const int ei = 2 + (v > pa) - (v < pa) + (v > pb) - (v < pb);
		const int cat = ei == 0 ? 1 : (ei == 1 ? 2 : (ei == 3 ? 3 : (ei == 4 ? 4 : 0)));
		if (cat) o = sa.off[ci][cat - 1];
	}
	return clampi(v + o, 0, 255);
}

/* one thread per 4 bytes of an NV12 row (4 luma samples, or 2 CbCr pairs), from the copy of the deblocked frame,
 * written back as one dword: bytes outside the picture or without SAO keep their (deblocked) value, which the
 * frame already holds.  (r122: one byte store per sample wrote 21 MB per 1080p picture, PMC WRITE_SIZE;
 * profiles/r122_pmc_h265.json) */
__global__ __launch_bounds__(256) void k_h265_sao(const H265Args *ap)
{
	const H265Args &a = *ap;
	const int W = a.W, H = a.H, wpr = W >> 2;
	const int ch = a.pic_h >> 1;
	const int id = blockIdx.x * blockDim.x + threadIdx.x;
	if (id >= (a.pic_h + ch) * wpr) return;
	const bool chroma = id >= a.pic_h * wpr;
	const int row = chroma ? id / wpr - a.pic_h : id / wpr, x4 = (id % wpr) * 4;
	if (chroma ? !(a.flags & H265R_PIC_SAO_CHROMA) : !(a.flags & H265R_PIC_SAO_LUMA)) return;
	const uint8_t *src = a.copy + (chroma ? (size_t)W * H : 0);
	uint8_t *dst = a.frame + (chroma ? (size_t)W * H : 0);
	const uint32_t in = *(const uint32_t *)(src + (size_t)row * W + x4);
	uint32_t out = 0;
#pragma unroll
	for (int b = 0; b < 4; ++b) {
		int v = (int)((in >> (8 * b)) & 255);
		if (!chroma) {
			if (x4 + b < a.pic_w) v = sao_sample(a, src, 0, x4 + b, row, a.pic_w, a.pic_h, 1, v);
		} else {
			const int x = (x4 + b) >> 1, comp = (x4 + b) & 1;
			if (x < (a.pic_w >> 1)) v = sao_sample(a, src + comp, 1 + comp, x, row, a.pic_w >> 1, ch, 2, v);
		}
		out |= (uint32_t)v << (8 * b);
	}
	if (out != in) *(uint32_t *)(dst + (size_t)row * W + x4) = out;
}

/* ------------------------------------------------------------------ runtime
 * Pictures are dealt over up to 8 HIP streams (M2DEC_AMD_H265_STREAMS; default 8 when the process has 8 hardware
 * queues — GPU_MAX_HW_QUEUES, m2dec_amd_configure_queues — else 4), each with its own scratch words and SAO copy
 * buffer; the record arenas are one ring.  Dependencies between pictures are host-ordered with events (no
 * kernel waits on another launch, so nothing here needs a workgroup budget):
 *   - read-after-write: a P / B picture's stream waits for the kernels of every reference frame's last picture;
 *   - write-after-read / -write: a picture's stream waits for the pictures that read its frame's previous
 *     content (their kernels) and for that content's copy-out to the staging buffer.
 * Independent pictures (an all-intra stream, the B pictures of one hierarchy level) then reconstruct side by
 * side: a 1080p CTU-row kernel has 17 workgroups, far from filling 256 CUs. */
struct H265Gpu {
	static const int NS = 8;
	static const int NEV = 512; /* recycled per-picture events: far more than a dependency can span */
	int dev = 0, cus = 0, ns = NS;
	hipStream_t st[NS] = {};
	int W = 0, H = 0, n = 0;
	size_t fsz = 0;
	uint8_t *frames = nullptr;
	m2d_frame_t caller[H265R_MAX_FRAMES];
	uint8_t *stg[H265R_MAX_FRAMES] = {};
	hipEvent_t ev[H265R_MAX_FRAMES] = {};   /* the frame's copy to staging is complete */
	bool pend[H265R_MAX_FRAMES] = {};
	hipEvent_t kdone[H265R_MAX_FRAMES] = {}; /* the kernels of the frame's last picture are done (null: none) */
	/* kernels of the pictures that read the frame's content: the latest one per HIP stream (events of one stream
	 * complete in order, so an older reader on the same stream is covered; ADVICE r5: a frame that stays a
	 * reference no longer collects one event per reading picture, which the 512-event ring re-records) */
	std::vector<std::pair<int, hipEvent_t>> readers[H265R_MAX_FRAMES];
	hipEvent_t evr[NEV] = {};
	int ev_next = 0;
	int *err = nullptr;     /* sticky error word */
	int *err_host = nullptr; /* page-locked: the error word as of each frame's copy-out ([H265R_MAX_FRAMES]) */
	/* record arenas: a picture's records in page-locked memory (read by k_h265_upload), filled either by a parse
	 * worker right after its parse (stage: in parallel, off the serial submission) or by submit itself.  An arena
	 * is reserved from its fill until its upload is queued, then free again once `used` fires. */
	struct Arena {
		uint8_t *host = nullptr, *dev = nullptr;
		const uint8_t *host_dev = nullptr; /* the pinned host buffer's device address (k_h265_upload reads it) */
		size_t size = 0;
		hipEvent_t used = nullptr;
		bool recorded = false; /* `used` was recorded at least once */
		bool reserved = false; /* being filled, staged, or being submitted */
		long last = 0;         /* submission order of its last use */
	};
	static const int NARENA = 48; /* > the parse pipeline's 16 staged pictures + the pictures in flight */
	Arena pool[NARENA];
	int npool = 0;
	long arena_clock = 0;
	/* pictures staged by a parse worker, found again by submit from the same record buffers */
	struct Staged {
		const void *tu = nullptr, *coef = nullptr;
		int n_tu = 0, n_coef = 0, n_pu = 0, slot = -1, width = 0, height = 0;
		int arena = -1; /* -1: entry free */
		unsigned refs = 0;
		long seq = 0;
	};
	Staged staged[32];
	long stage_clock = 0;
	int64_t staged_pictures = 0, staged_used = 0;
	std::mutex amu; /* pool, staged, grave_*, max_total */
	struct Lane {
		uint8_t *copy = nullptr; /* the deblocked frame (SAO input) */
		int *scratch = nullptr;  /* done flags + the block counter + CTU progress */
		size_t scratch_n = 0;
	} lane[NS];
	int rr = 0;
	/* timing: per picture, its kernels' start / end on its stream */
	struct Timing {
		hipEvent_t t0 = nullptr, t1 = nullptr;
		bool pending = false;
	} tr[32];
	int tr_next = 0;
	double kernel_us = 0;
	long pictures = 0;
	int64_t record_bytes = 0, frame_bytes = 0;
	std::vector<uint8_t *> grave_host, grave_dev; /* outgrown arenas (freed at set_frames / destroy) */
	bool block_kernel = false; /* M2DEC_AMD_H265_BLOCKS=1: the per-block dependency-graph kernel */
	bool trace = false;        /* M2DEC_AMD_H265_TRACE */
	bool upload_zero = true;   /* scratch cleared by the upload kernel (M2DEC_AMD_H265_UPLOAD_ZERO=0: hipMemsetAsync, A/B) */
	double trace_ms = 0.5;     /* M2DEC_AMD_H265_TRACE_MS: the submit steps reported above this */
	bool kcopy = true;         /* record upload by k_h265_upload (M2DEC_AMD_H265_KCOPY=0: hipMemcpyAsync) */
	bool kcopy_d2h = false;    /* M2DEC_AMD_KCOPY_D2H=1: the frame down by k_h265_upload writing the pinned staging buffer */
	size_t max_total = 0;      /* the largest picture's arena bytes so far */
	bool waves4 = true;        /* CTU kernels with two waves per plane (M2DEC_AMD_H265_WAVES=2: one) */
	bool err_async = true;     /* error word copied behind each frame (M2DEC_AMD_H265_ERR_ASYNC=0: read in sync) */
	bool ctu_grid = true;      /* P / B pictures: one workgroup per CTU (M2DEC_AMD_H265_CTU_GRID=0: the row kernel) */
	bool no_stage = false;     /* M2DEC_AMD_H265_STAGE=0: records copied by submit only (A/B) */
};

static size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

static void flush_timing(H265Gpu *g, H265Gpu::Timing &t)
{
	if (!t.pending) return;
	float ms = 0;
	if (hipEventSynchronize(t.t1) == hipSuccess && hipEventElapsedTime(&ms, t.t0, t.t1) == hipSuccess) g->kernel_us += 1000.0 * ms;
	t.pending = false;
}

static int sync_all(H265Gpu *g)
{
	for (int k = 0; k < g->ns; ++k) H265_CHECK(hipStreamSynchronize(g->st[k]));
	return 0;
}

int h_set_frames(void *p, int n, const m2d_frame_t *frames, int width, int height)
{
	H265Gpu *g = (H265Gpu *)p;
	if (!g || n <= 0 || n > H265R_MAX_FRAMES || width <= 0 || height <= 0 || (width & 15) || (height & 15)) return -1;
	H265_CHECK(hipSetDevice(g->dev));
	if (sync_all(g) < 0) return -1;
	const size_t fsz = ((size_t)width * height * 3 / 2 + 4095) & ~(size_t)4095;
	if (!g->frames || fsz != g->fsz || n > g->n) {
		if (g->frames) (void)hipFree(g->frames);
		g->frames = nullptr;
		for (auto &l : g->lane) {
			if (l.copy) (void)hipFree(l.copy);
			l.copy = nullptr;
		}
		H265_CHECK(hipMalloc((void **)&g->frames, fsz * (size_t)n));
		for (int k = 0; k < g->ns; ++k) H265_CHECK(hipMalloc((void **)&g->lane[k].copy, fsz));
		H265_CHECK(hipMemset(g->frames, 0, fsz * (size_t)n));
	}
	{
		/* (the decoder drains its parse pipeline before set_frames: nothing is staged or being staged now) */
		std::lock_guard<std::mutex> lk(g->amu);
		for (uint8_t *p : g->grave_host) (void)hipHostFree(p);
		for (uint8_t *p : g->grave_dev) (void)hipFree(p);
		g->grave_host.clear();
		g->grave_dev.clear();
		for (auto &e : g->staged)
			if (e.arena >= 0) {
				g->pool[e.arena].reserved = false;
				e.arena = -1;
			}
	}
	{
		/* scratch words of the largest picture the frame holds: 4 x 4 luma and chroma blocks, 16 x 16 CTUs */
		const size_t sn = (size_t)(width / 4) * (height / 4) + (size_t)(width / 8) * (height / 8) + 2 + (size_t)(height / 16 + 1) +
		                  2 * (size_t)(width / 16 + 1) * (height / 16 + 1) + 1;
		for (int k = 0; k < g->ns; ++k) {
			H265Gpu::Lane &ln = g->lane[k];
			if (sn <= ln.scratch_n) continue;
			if (ln.scratch) (void)hipFree(ln.scratch);
			ln.scratch = nullptr;
			ln.scratch_n = 0;
			H265_CHECK(hipMalloc((void **)&ln.scratch, sizeof(int) * sn));
			ln.scratch_n = sn;
		}
	}
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) {
		if (g->stg[i] && ((size_t)width * height != (size_t)g->W * g->H || i >= n)) {
			(void)hipHostFree(g->stg[i]);
			g->stg[i] = nullptr;
		}
		g->pend[i] = false;
		g->kdone[i] = nullptr;
		g->readers[i].clear();
	}
	g->fsz = fsz;
	g->n = n;
	g->W = width;
	g->H = height;
	memcpy(g->caller, frames, sizeof(m2d_frame_t) * (size_t)n);
	return 0;
}

static hipEvent_t next_event(H265Gpu *g)
{
	hipEvent_t &e = g->evr[g->ev_next];
	g->ev_next = (g->ev_next + 1) % H265Gpu::NEV;
	if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
	return e;
}

/* host-side checks of what the kernels assume; refs = the frames the picture's prediction blocks read */
static int check_picture(const H265Gpu *g, const h265r_picture_t *pic, unsigned *refs_out)
{
	if (!g->frames || pic->width != g->W || pic->height != g->H || pic->slot < 0 || pic->slot >= g->n || pic->n_tu < 0)
		return -1;
	/* blocks inside the frame and inside one CTU, CTUs in raster order (the CTU kernel's per-CTU record ranges and
	 * LDS tile), coefficients inside the pool */
	if (pic->ctb_log2 < 4 || pic->ctb_log2 > 6 || pic->pic_w > g->W || pic->pic_h > g->H) return -1;
	for (int i = 0, last_ctu = 0; i < pic->n_tu; ++i) {
		const h265r_tu_t &t = pic->tu[i];
		const int n = 1 << t.log2, pw = t.plane ? g->W / 2 : g->W, ph = t.plane ? g->H / 2 : g->H;
		if (t.log2 < 2 || t.log2 > 5 || t.x + n > pw || t.y + n > ph || t.mode > 34 || (t.x & 3) || (t.y & 3)) return -1;
		const int lx = t.plane ? 2 * t.x : t.x, ly = t.plane ? 2 * t.y : t.y, ln = t.plane ? 2 * n : n;
		const int ctb = 1 << pic->ctb_log2, cols_ = (pic->pic_w + ctb - 1) >> pic->ctb_log2;
		const int ctu = (ly >> pic->ctb_log2) * cols_ + (lx >> pic->ctb_log2);
		if (ctu < last_ctu || (lx & (ctb - 1)) + ln > ctb || (ly & (ctb - 1)) + ln > ctb) return -1;
		last_ctu = ctu;
		for (int c = 0; c < 2; ++c)
			if (t.res[c] && (int64_t)t.coef[c] + n * n > (int64_t)pic->n_coef) return -1;
	}
	/* prediction blocks: inside the frame, 4..64 samples a side, references other frames of this context */
	if (pic->n_pu < 0 || (pic->n_pu && !pic->pu)) return -1;
	unsigned refs = 0;
	for (int i = 0; i < pic->n_pu; ++i) {
		const h265r_pu_t &u = pic->pu[i];
		if (u.w < 4 || u.h < 4 || u.w > 64 || u.h > 64 || (u.w & 3) || (u.h & 3) || (u.x & 3) || (u.y & 3) || u.x + u.w > g->W ||
		    u.y + u.h > g->H || (u.ref[0] < 0 && u.ref[1] < 0))
			return -1;
		for (int l = 0; l < 2; ++l) {
			if (u.ref[l] >= g->n || (u.ref[l] >= 0 && u.ref[l] == pic->slot)) return -1;
			if (u.ref[l] >= 0) refs |= 1u << u.ref[l];
		}
	}
	*refs_out = refs;
	return 0;
}

/* where a picture's records sit in its arena */
struct ArenaLayout {
	int cols, rows;
	size_t units, nbs, o_tu, o_coef, o_map, o_bsv, o_bsh, o_sao, o_pu, o_args, total;
};

static ArenaLayout layout_of(const h265r_picture_t *pic)
{
	ArenaLayout L;
	L.units = (size_t)(pic->width / 4) * (pic->height / 4) + (size_t)(pic->width / 8) * (pic->height / 8);
	L.nbs = (size_t)(pic->height / 4) * (pic->width / 8);
	L.cols = (pic->pic_w + (1 << pic->ctb_log2) - 1) >> pic->ctb_log2;
	L.rows = (pic->pic_h + (1 << pic->ctb_log2) - 1) >> pic->ctb_log2;
	L.o_tu = 0;
	L.o_coef = al16(L.o_tu + sizeof(h265r_tu_t) * (size_t)pic->n_tu);
	L.o_map = al16(L.o_coef + sizeof(int16_t) * (size_t)pic->n_coef);
	L.o_bsv = al16(L.o_map + sizeof(int32_t) * L.units);
	L.o_bsh = al16(L.o_bsv + L.nbs);
	L.o_sao = al16(L.o_bsh + L.nbs);
	L.o_pu = al16(L.o_sao + sizeof(h265r_sao_t) * (size_t)(L.cols * L.rows));
	/* the kernels' argument block rides in the arena (one upload from page-locked memory: a hipMemcpyAsync
	 * from the stack is a pageable copy, which can block this thread until the stream — waiting on other
	 * streams' pictures — reaches it) */
	L.o_args = al16(L.o_pu + sizeof(h265r_pu_t) * (size_t)pic->n_pu);
	L.total = al16(L.o_args + sizeof(H265Args));
	return L;
}

static void arena_release(H265Gpu *g, int i);

/* a free arena of at least `total` bytes, reserved for the caller (any thread): one whose last upload is done,
 * else a new one, else the oldest in flight (waited for); -1 on a HIP error */
static int arena_acquire(H265Gpu *g, size_t total)
{
	int pick = -1;
	bool wait = false;
	{
		std::lock_guard<std::mutex> lk(g->amu);
		int small = -1, oldest = -1;
		for (int i = 0; i < g->npool; ++i) {
			H265Gpu::Arena &a = g->pool[i];
			if (a.reserved) continue;
			if (a.recorded && hipEventQuery(a.used) != hipSuccess) {
				if (oldest < 0 || a.last < g->pool[oldest].last) oldest = i;
				continue;
			}
			if (a.size >= total) {
				pick = i;
				break;
			}
			if (small < 0) small = i;
		}
		if (pick < 0 && g->npool < H265Gpu::NARENA) {
			H265Gpu::Arena &a = g->pool[g->npool];
			if (!a.used && hipEventCreateWithFlags(&a.used, hipEventDisableTiming) != hipSuccess) return -1;
			pick = g->npool++;
		}
		if (pick < 0) pick = small;
		if (pick < 0) {
			pick = oldest;
			wait = true;
		}
		if (pick < 0) return -1; /* (every arena reserved: more staged pictures than the pipeline can hold) */
		g->pool[pick].reserved = true;
	}
	H265Gpu::Arena &a = g->pool[pick];
	if (wait && hipEventSynchronize(a.used) != hipSuccess) {
		arena_release(g, pick);
		return -1;
	}
	if (a.size < total) {
		std::lock_guard<std::mutex> lk(g->amu);
		if (a.host) g->grave_host.push_back(a.host);
		if (a.dev) g->grave_dev.push_back(a.dev);
		a.host = a.dev = nullptr;
		a.size = 0;
		/* at least the largest picture seen so far, with headroom: every arena soon holds an intra picture */
		const size_t want = total > g->max_total ? total : g->max_total;
		const size_t sz = al16(want + want / 4);
		if (hipHostMalloc((void **)&a.host, sz, hipHostMallocDefault) != hipSuccess || hipMalloc((void **)&a.dev, sz) != hipSuccess) {
			a.reserved = false;
			return -1;
		}
		void *hd = nullptr;
		if (hipHostGetDevicePointer(&hd, a.host, 0) != hipSuccess) {
			a.reserved = false;
			return -1;
		}
		a.host_dev = (const uint8_t *)hd;
		a.size = sz;
	}
	{
		std::lock_guard<std::mutex> lk(g->amu);
		if (total > g->max_total) g->max_total = total;
	}
	return pick;
}

static void arena_release(H265Gpu *g, int i)
{
	std::lock_guard<std::mutex> lk(g->amu);
	g->pool[i].reserved = false;
}

static void arena_fill(H265Gpu::Arena &a, const h265r_picture_t *pic, const ArenaLayout &L)
{
	memcpy(a.host + L.o_tu, pic->tu, sizeof(h265r_tu_t) * (size_t)pic->n_tu);
	memcpy(a.host + L.o_coef, pic->coef, sizeof(int16_t) * (size_t)pic->n_coef);
	memcpy(a.host + L.o_map, pic->map, sizeof(int32_t) * L.units);
	memcpy(a.host + L.o_bsv, pic->bs_v, L.nbs);
	memcpy(a.host + L.o_bsh, pic->bs_h, L.nbs);
	memcpy(a.host + L.o_sao, pic->sao, sizeof(h265r_sao_t) * (size_t)(L.cols * L.rows));
	if (pic->n_pu) memcpy(a.host + L.o_pu, pic->pu, sizeof(h265r_pu_t) * (size_t)pic->n_pu);
}

static bool staged_match(const H265Gpu::Staged &e, const h265r_picture_t *pic)
{
	return e.arena >= 0 && e.tu == (const void *)pic->tu && e.coef == (const void *)pic->coef && e.n_tu == pic->n_tu &&
	       e.n_coef == pic->n_coef && e.n_pu == pic->n_pu && e.slot == pic->slot && e.width == pic->width && e.height == pic->height;
}

/* h265r_backend_t.stage: a parse worker hands over a parsed picture before its (serial, decode-order) submit:
 * its checks and the copy of its records into a page-locked arena happen here, on the worker, in parallel with
 * the other workers and the submissions (the round-5 intra timeline: 0.4-0.9 ms of copies per picture on the
 * submitting thread, the eighth picture's kernels starting 4.5 ms after the parse ended).  discard = 1: the
 * picture will not be submitted (a failed or abandoned job): its arena goes back.  A picture that cannot be
 * staged is simply copied by submit. */
int h_stage(void *p, const h265r_picture_t *pic, int discard)
{
	H265Gpu *g = (H265Gpu *)p;
	if (!g || !pic) return -1;
	if (discard) {
		std::lock_guard<std::mutex> lk(g->amu);
		for (auto &e : g->staged)
			if (staged_match(e, pic)) {
				g->pool[e.arena].reserved = false;
				e.arena = -1;
			}
		return 0;
	}
	if (g->no_stage) return 0;
	unsigned refs = 0;
	if (check_picture(g, pic, &refs) < 0) return 0; /* (submit checks again and refuses it) */
	H265_CHECK(hipSetDevice(g->dev));
	const ArenaLayout L = layout_of(pic);
	const int ai = arena_acquire(g, L.total);
	if (ai < 0) return 0;
	arena_fill(g->pool[ai], pic, L);
	std::lock_guard<std::mutex> lk(g->amu);
	int slot = -1;
	for (int i = 0; i < 32; ++i) {
		H265Gpu::Staged &e = g->staged[i];
		if (staged_match(e, pic) || (e.tu == (const void *)pic->tu && e.arena >= 0)) { /* (the same job staged again) */
			g->pool[e.arena].reserved = false;
			e.arena = -1;
		}
		if (e.arena < 0 && slot < 0) slot = i;
	}
	if (slot < 0) { /* (cannot happen with the pipeline's 16 jobs: the oldest entry goes) */
		slot = 0;
		for (int i = 1; i < 32; ++i)
			if (g->staged[i].seq < g->staged[slot].seq) slot = i;
		g->pool[g->staged[slot].arena].reserved = false;
	}
	H265Gpu::Staged &e = g->staged[slot];
	e.tu = pic->tu;
	e.coef = pic->coef;
	e.n_tu = pic->n_tu;
	e.n_coef = pic->n_coef;
	e.n_pu = pic->n_pu;
	e.slot = pic->slot;
	e.width = pic->width;
	e.height = pic->height;
	e.refs = refs;
	e.arena = ai;
	e.seq = ++g->stage_clock;
	g->staged_pictures++;
	return 0;
}

int h_submit(void *p, const h265r_picture_t *pic)
{
	H265Gpu *g = (H265Gpu *)p;
	if (!g || !pic) return -1;
	/* M2DEC_AMD_H265_TRACE: the steps of this call that took over 0.5 ms */
	struct timespec ts0;
	clock_gettime(CLOCK_MONOTONIC, &ts0);
	double tp = ts0.tv_sec * 1e3 + ts0.tv_nsec * 1e-6;
	auto lap = [&](const char *what) {
		if (!g->trace) return;
		struct timespec ts;
		clock_gettime(CLOCK_MONOTONIC, &ts);
		const double t = ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
		if (t - tp > g->trace_ms) fprintf(stderr, "h265 submit slot %d: %s %.3f ms\n", pic->slot, what, t - tp);
		tp = t;
	};
	unsigned refs = 0;
	int ai = -1;
	{
		std::lock_guard<std::mutex> lk(g->amu);
		for (auto &e : g->staged)
			if (staged_match(e, pic)) {
				ai = e.arena;
				refs = e.refs;
				e.arena = -1;
				g->staged_used++;
				break;
			}
	}
	if (ai < 0 && check_picture(g, pic, &refs) < 0) return -1;
	H265_CHECK(hipSetDevice(g->dev));
	const ArenaLayout L = layout_of(pic);
	if (ai < 0) {
		ai = arena_acquire(g, L.total);
		if (ai < 0) return -1;
		arena_fill(g->pool[ai], pic, L);
	}
	/* (the arena goes back to the pool on every return below; after its `used` event on success) */
	struct Release {
		H265Gpu *g;
		int i;
		~Release() { arena_release(g, i); }
	} release{g, ai};
	H265Gpu::Arena &a = g->pool[ai];
	lap("records");
	/* the stream: the first idle one after the last, else round robin */
	int k = g->rr;
	for (int i = 0; i < g->ns; ++i) {
		const int c = (g->rr + i) % g->ns;
		if (hipStreamQuery(g->st[c]) == hipSuccess) {
			k = c;
			break;
		}
	}
	g->rr = (k + 1) % g->ns;
	hipStream_t s = g->st[k];
	H265Gpu::Lane &ln = g->lane[k];
	const int cols = L.cols, rows = L.rows;
	const size_t o_tu = L.o_tu, o_coef = L.o_coef, o_map = L.o_map, o_bsv = L.o_bsv, o_bsh = L.o_bsh, o_sao = L.o_sao,
	             o_pu = L.o_pu, o_args = L.o_args, total = L.total;
	/* per-block done flags + 2 counters, then the CTU rows' progress words, the CTUs' first records and the CTUs'
	 * done flags (sized for the frame at set_frames: a block is at least 4 x 4) */
	const int nctu = cols * rows;
	const size_t sn = (size_t)pic->n_tu + 2 + (size_t)rows + 2 * (size_t)nctu + 1;
	if (sn > ln.scratch_n) return -1;
	H265Args h;
	h.tu = (const h265r_tu_t *)(a.dev + o_tu);
	h.coef = (const int16_t *)(a.dev + o_coef);
	h.map = (const int32_t *)(a.dev + o_map);
	h.bs_v = a.dev + o_bsv;
	h.bs_h = a.dev + o_bsh;
	h.sao = (const h265r_sao_t *)(a.dev + o_sao);
	h.frame = g->frames + (size_t)pic->slot * g->fsz;
	h.copy = ln.copy;
	h.done = ln.scratch;
	h.counter = ln.scratch + pic->n_tu;
	h.progress = h.counter + 2;
	h.ctu_first = h.progress + rows;
	h.ctu_cols = cols;
	h.ctu_rows = rows;
	h.err = g->err;
	h.W = g->W;
	h.H = g->H;
	h.pic_w = pic->pic_w;
	h.pic_h = pic->pic_h;
	h.ctb_log2 = pic->ctb_log2;
	h.n_tu = pic->n_tu;
	h.flags = pic->flags;
	if (getenv("M2DEC_AMD_H265_DIAG_NOWAIT")) h.flags |= 1 << 30; /* (diagnostic: CTU-grid neighbour waits skipped — wrong output) */
	if (getenv("M2DEC_AMD_H265_GRID_ONEPASS")) h.flags |= 1 << 29; /* (A/B: no inter-first split of the CTU-grid blocks) */
	if (getenv("M2DEC_AMD_H265_NO_HALF_ROW")) h.flags |= 1 << 28;   /* (A/B: a CTU's last row published only with the CTU) */
	h.beta_offset = pic->beta_offset;
	h.tc_offset = pic->tc_offset;
	h.cb_qp_offset = pic->cb_qp_offset;
	h.cr_qp_offset = pic->cr_qp_offset;
	h.pu = (const h265r_pu_t *)(a.dev + o_pu);
	h.frames = g->frames;
	h.fsz = g->fsz;
	h.n_pu = pic->n_pu;
	memcpy(a.host + o_args, &h, sizeof(h));
	const H265Args *args = (const H265Args *)(a.dev + o_args);
	lap("record copy");
	if (g->kcopy) {
		/* the upload as a kernel reading the pinned records over the host link: an SDMA copy queued behind an
		 * earlier picture's copy-out (itself waiting for that picture's kernels) held this thread 8-10 ms once
		 * per decode, the GPU idling meanwhile (round-5 H.265 timelines) */
		const size_t n16 = total / 16;
		const int grid = (int)std::min<size_t>(512, (n16 + 255) / 256);
		hipLaunchKernelGGL(k_h265_upload, dim3(grid), dim3(256), 0, s, (const uint4 *)a.host_dev, (uint4 *)a.dev, n16,
		                   g->upload_zero ? ln.scratch : (int *)nullptr, g->upload_zero ? sn : (size_t)0);
		H265_CHECK(hipGetLastError());
		if (!g->upload_zero) H265_CHECK(hipMemsetAsync(ln.scratch, 0, sizeof(int) * sn, s));
	} else {
		H265_CHECK(hipMemcpyAsync(a.dev, a.host, total, hipMemcpyHostToDevice, s));
		H265_CHECK(hipMemsetAsync(ln.scratch, 0, sizeof(int) * sn, s));
	}
	lap("upload");
	g->record_bytes += (int64_t)o_args;
	g->frame_bytes += (int64_t)g->W * g->H * 3 / 2;
	/* dependencies on other streams' pictures, after the uploads (a copy behind a wait on another stream's
	 * picture can hold this thread until that picture completes: 8-10 ms per decode in the round-5 trace) */
	for (int r = 0; r < H265R_MAX_FRAMES; ++r)
		if (((refs >> r) & 1) && g->kdone[r]) H265_CHECK(hipStreamWaitEvent(s, g->kdone[r], 0));
	for (const auto &re : g->readers[pic->slot]) H265_CHECK(hipStreamWaitEvent(s, re.second, 0));
	if (g->kdone[pic->slot]) H265_CHECK(hipStreamWaitEvent(s, g->kdone[pic->slot], 0));
	if (g->pend[pic->slot] || g->kdone[pic->slot]) H265_CHECK(hipStreamWaitEvent(s, g->ev[pic->slot], 0)); /* its copy-out */
	lap("event waits");
	H265Gpu::Timing &tm = g->tr[g->tr_next];
	g->tr_next = (g->tr_next + 1) % 32;
	flush_timing(g, tm);
	H265_CHECK(hipEventRecord(tm.t0, s));
	lap("timing");
	if (pic->n_pu) {
		const int grid = pic->n_pu < g->cus * 8 ? pic->n_pu : g->cus * 8;
		hipLaunchKernelGGL(k_h265_mc, dim3(grid), dim3(64), 0, s, args);
		H265_CHECK(hipGetLastError());
	}
	if (pic->n_tu && g->block_kernel) {
		const int grid = pic->n_tu < g->cus * 8 ? pic->n_tu : g->cus * 8;
		hipLaunchKernelGGL(k_h265_intra, dim3(grid), dim3(64), 0, s, args);
		H265_CHECK(hipGetLastError());
	} else if (pic->n_tu) {
		hipLaunchKernelGGL(k_h265_ctu_index, dim3(pic->n_tu / 256 + 1), dim3(256), 0, s, args);
		if (pic->n_pu && g->ctu_grid) {
			if (g->waves4) hipLaunchKernelGGL(k_h265_ctu_grid<256>, dim3(nctu), dim3(256), 0, s, args);
			else hipLaunchKernelGGL(k_h265_ctu_grid<128>, dim3(nctu), dim3(128), 0, s, args);
		} else if (g->waves4) {
			hipLaunchKernelGGL(k_h265_ctu_rows<256>, dim3(rows), dim3(256), 0, s, args);
		} else {
			hipLaunchKernelGGL(k_h265_ctu_rows<128>, dim3(rows), dim3(128), 0, s, args);
		}
		H265_CHECK(hipGetLastError());
	}
	lap("ctu kernels");
	if (pic->flags & H265R_PIC_DEBLOCK) {
		const int nv = (g->H / 4) * (g->W / 8), nh = (g->H / 8) * (g->W / 4);
		hipLaunchKernelGGL(k_h265_deblock, dim3((nv + 255) / 256), dim3(256), 0, s, args, 0);
		hipLaunchKernelGGL(k_h265_deblock, dim3((nh + 255) / 256), dim3(256), 0, s, args, 1);
		H265_CHECK(hipGetLastError());
	}
	lap("deblock");
	if (pic->flags & (H265R_PIC_SAO_LUMA | H265R_PIC_SAO_CHROMA)) {
		H265_CHECK(hipMemcpyAsync(ln.copy, h.frame, (size_t)g->W * g->H * 3 / 2, hipMemcpyDeviceToDevice, s));
		const int nsa = (pic->pic_h + (pic->pic_h >> 1)) * (g->W >> 2); /* (4 bytes of a row per thread) */
		hipLaunchKernelGGL(k_h265_sao, dim3((nsa + 255) / 256), dim3(256), 0, s, args);
		H265_CHECK(hipGetLastError());
	}
	lap("kernels");
	H265_CHECK(hipEventRecord(tm.t1, s));
	tm.pending = true;
	H265_CHECK(hipEventRecord(a.used, s));
	{
		std::lock_guard<std::mutex> lk(g->amu);
		a.recorded = true;
		a.last = ++g->arena_clock;
	}
	/* this picture's kernels: what later readers of its frame wait for, and what the next writers of its
	 * references' frames wait for */
	hipEvent_t kd = next_event(g);
	if (!kd) return -1;
	H265_CHECK(hipEventRecord(kd, s));
	for (int r = 0; r < H265R_MAX_FRAMES; ++r)
		if ((refs >> r) & 1) {
			auto &rd = g->readers[r];
			auto it = std::find_if(rd.begin(), rd.end(), [k](const std::pair<int, hipEvent_t> &x) { return x.first == k; });
			if (it != rd.end()) it->second = kd;
			else rd.emplace_back(k, kd);
		}
	g->readers[pic->slot].clear();
	g->kdone[pic->slot] = kd;
	lap("events");
	/* the picture to its staging buffer, behind the kernels */
	const int c = pic->slot;
	const size_t bytes = (size_t)g->W * g->H * 3 / 2;
	if (!g->stg[c]) H265_CHECK(hipHostMalloc((void **)&g->stg[c], bytes, hipHostMallocDefault));
	if (g->kcopy_d2h && bytes % 16 == 0) {
		void *dh = nullptr;
		H265_CHECK(hipHostGetDevicePointer(&dh, g->stg[c], 0));
		hipLaunchKernelGGL(k_h265_upload, dim3(256), dim3(256), 0, s, (const uint4 *)h.frame, (uint4 *)dh, bytes / 16,
		                   (int *)nullptr, (size_t)0);
		H265_CHECK(hipGetLastError());
	} else {
		H265_CHECK(hipMemcpyAsync(g->stg[c], h.frame, bytes, hipMemcpyDeviceToHost, s));
	}
	if (g->err_async) H265_CHECK(hipMemcpyAsync(&g->err_host[c], g->err, sizeof(int), hipMemcpyDeviceToHost, s));
	H265_CHECK(hipEventRecord(g->ev[c], s));
	lap("copy-out");
	g->pend[c] = true;
	g->pictures++;
	return 0;
}

int h_sync(void *p, int slot)
{
	H265Gpu *g = (H265Gpu *)p;
	if (!g || slot < 0 || slot >= H265R_MAX_FRAMES) return -1;
	if (!g->pend[slot]) return 0;
	H265_CHECK(hipEventSynchronize(g->ev[slot]));
	{
		/* a block hand-off that never came (bounded spin): the sticky error word, copied behind the frame on its
		 * stream as the H.264 back end does.  M2DEC_AMD_H265_ERR_ASYNC=0 reads it here with a synchronous hipMemcpy,
		 * whose blit runs on the null stream's hardware queue, shared with one of the picture streams: every frame
		 * then waited for that stream's last kernel (r179 timeline: frame 0 out 3.3 ms after its copy-out) */
		int err = 0;
		if (g->err_async) err = __atomic_load_n(&g->err_host[slot], __ATOMIC_ACQUIRE);
		else H265_CHECK(hipMemcpy(&err, g->err, sizeof(int), hipMemcpyDeviceToHost));
		if (err) {
			fprintf(stderr, "m2dec_amd: H.265 block hand-off timed out on the GPU\n");
			return -1;
		}
	}
	const size_t ls = (size_t)g->W * g->H;
	/* (the sync crew, parcopy.c: a 3.1 MB frame over several cores, as the H.264 back end's be_sync) */
	void *to[2] = {g->caller[slot].luma, g->caller[slot].chroma};
	const void *from[2] = {g->stg[slot], g->stg[slot] + ls};
	const size_t len[2] = {ls, ls / 2};
	m2dec_par_memcpy(M2DEC_CREW_SYNC_, 2, to, from, len);
	g->pend[slot] = false;
	return 0;
}

void h_destroy(void *p)
{
	H265Gpu *g = (H265Gpu *)p;
	if (!g) return;
	(void)hipSetDevice(g->dev);
	(void)sync_all(g);
	for (auto &a : g->pool) {
		if (a.host) (void)hipHostFree(a.host);
		if (a.dev) (void)hipFree(a.dev);
		if (a.used) (void)hipEventDestroy(a.used);
	}
	for (auto &l : g->lane) {
		if (l.scratch) (void)hipFree(l.scratch);
		if (l.copy) (void)hipFree(l.copy);
	}
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) {
		if (g->stg[i]) (void)hipHostFree(g->stg[i]);
		if (g->ev[i]) (void)hipEventDestroy(g->ev[i]);
	}
	for (auto &e : g->evr)
		if (e) (void)hipEventDestroy(e);
	for (uint8_t *p : g->grave_host) (void)hipHostFree(p);
	for (uint8_t *p : g->grave_dev) (void)hipFree(p);
	for (auto &t : g->tr) {
		if (t.t0) (void)hipEventDestroy(t.t0);
		if (t.t1) (void)hipEventDestroy(t.t1);
	}
	if (g->err) (void)hipFree(g->err);
	if (g->err_host) (void)hipHostFree(g->err_host);
	if (g->frames) (void)hipFree(g->frames);
	for (int k = 0; k < g->ns; ++k)
		if (g->st[k]) (void)hipStreamDestroy(g->st[k]);
	delete g;
}

} // namespace

extern "C" int h265_hip_backend_create(h265r_backend_t *out, int device)
{
	int n = 0;
	if (!out || hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return -1;
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) return -1;
	H265Gpu *g = new H265Gpu();
	g->dev = device;
	g->cus = prop.multiProcessorCount;
	if (const char *e = getenv("M2DEC_AMD_H265_BLOCKS")) g->block_kernel = atoi(e) != 0;
	if (const char *e = getenv("M2DEC_AMD_H265_CTU_GRID")) g->ctu_grid = atoi(e) != 0;
	g->trace = getenv("M2DEC_AMD_H265_TRACE") != nullptr;
	if (const char *e = getenv("M2DEC_AMD_H265_TRACE_MS")) g->trace_ms = atof(e);
	if (const char *e = getenv("M2DEC_AMD_H265_UPLOAD_ZERO")) g->upload_zero = atoi(e) != 0;
	if (const char *e = getenv("M2DEC_AMD_H265_WAVES")) g->waves4 = atoi(e) >= 4;
	if (const char *e = getenv("M2DEC_AMD_H265_KCOPY")) g->kcopy = atoi(e) != 0;
	if (const char *e = getenv("M2DEC_AMD_KCOPY_D2H")) g->kcopy_d2h = atoi(e) != 0;
	if (const char *e = getenv("M2DEC_AMD_H265_ERR_ASYNC")) g->err_async = atoi(e) != 0;
	if (const char *e = getenv("M2DEC_AMD_H265_STAGE")) g->no_stage = atoi(e) == 0;
	{
		const char *q = getenv("GPU_MAX_HW_QUEUES");
		g->ns = q && atoi(q) >= 8 ? 8 : 4;
	}
	if (const char *e = getenv("M2DEC_AMD_H265_STREAMS")) g->ns = atoi(e) < 1 ? 1 : (atoi(e) > H265Gpu::NS ? H265Gpu::NS : atoi(e));
	if (hipSetDevice(device) != hipSuccess) {
		delete g;
		return -1;
	}
	for (int k = 0; k < g->ns; ++k)
		if (hipStreamCreateWithFlags(&g->st[k], hipStreamNonBlocking) != hipSuccess) {
			h_destroy(g);
			return -1;
		}
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) (void)hipEventCreateWithFlags(&g->ev[i], hipEventDisableTiming);
	for (auto &t : g->tr) {
		(void)hipEventCreate(&t.t0);
		(void)hipEventCreate(&t.t1);
	}
	if (hipMalloc((void **)&g->err, sizeof(int)) != hipSuccess || hipMemset(g->err, 0, sizeof(int)) != hipSuccess ||
	    hipHostMalloc((void **)&g->err_host, sizeof(int) * H265R_MAX_FRAMES, hipHostMallocDefault) != hipSuccess) {
		h_destroy(g);
		return -1;
	}
	memset(g->err_host, 0, sizeof(int) * H265R_MAX_FRAMES);
	out->self = g;
	out->set_frames = h_set_frames;
	out->submit = h_submit;
	out->sync_frame = h_sync;
	out->destroy = h_destroy;
	out->stage = h_stage;
	return 0;
}

extern "C" int m2dec_amd_h265_hip_backend_create(h265r_backend_t *out, int device) { return h265_hip_backend_create(out, device); }

/* kernel time (HIP events per picture on its stream: pictures on different streams overlap, so this is the
 * sum of the pictures' kernel latencies), pictures, and the §8d algorithmic bytes of the pictures so far: R_pic
 * (records uploaded) and F_write (1.5 W H each); reset zeroes them */
extern "C" int m2dec_amd_h265_hip_timing(const h265r_backend_t *be, double *kernel_us, int64_t *timed_pictures,
                                         int64_t *record_bytes, int64_t *frame_bytes, int reset)
{
	if (!be || !be->self || be->submit != h_submit) return -1;
	H265Gpu *g = (H265Gpu *)be->self;
	(void)sync_all(g);
	for (auto &t : g->tr) flush_timing(g, t);
	if (kernel_us) *kernel_us = g->kernel_us;
	if (timed_pictures) *timed_pictures = g->pictures;
	if (record_bytes) *record_bytes = g->record_bytes;
	if (frame_bytes) *frame_bytes = g->frame_bytes;
	if (reset) {
		g->kernel_us = 0;
		g->record_bytes = g->frame_bytes = 0;
		g->pictures = 0;
	}
	return 0;
}

/* the H265_STAMPS events so far (and the count reset): returns how many, -1 in a build without them */
extern "C" int m2dec_amd_h265_stamps(unsigned long long *t, unsigned *info, int max)
{
#ifdef H265_STAMPS
	unsigned n = 0;
	if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_h5n), sizeof(n), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
	if (n > H5ST_N) n = H5ST_N;
	if ((int)n > max) n = (unsigned)max;
	if (n && (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_h5t), sizeof(*t) * n, 0, hipMemcpyDeviceToHost) != hipSuccess ||
	          hipMemcpyFromSymbol(info, HIP_SYMBOL(g_h5i), sizeof(*info) * n, 0, hipMemcpyDeviceToHost) != hipSuccess))
		return -1;
	const unsigned z = 0;
	if (hipMemcpyToSymbol(HIP_SYMBOL(g_h5n), &z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
	return (int)n;
#else
	(void)t;
	(void)info;
	(void)max;
	return -1;
#endif
}
