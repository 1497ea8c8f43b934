/*
 * m2dec_amd gfx950 reconstruction back end.
 *
 * Consumes the per-picture record arena (include/m2d_recon.h) produced by the host parser and
 * reconstructs the picture into a device-resident NV12 frame pool, then copies the finished
 * frame into the caller's m2d_frame_t buffer (the reference writes there directly).
 *
 * Kernels (one picture = up to three launches on one stream):
 *   k_inter   : every inter MB in parallel (one 256-thread workgroup per MB): luma qpel + chroma
 *               1/8 MC for both lists, default / explicit / implicit weighting, dequant + 4x4/8x8
 *               inverse transform + add.  Reference: inter_pred_* (h264.cpp:4763-7118),
 *               residual_luma_inter4x4/8x8 (6421-6580), residual_chroma (2374-2461).
 *   k_intra   : intra / PCM MBs as a wavefront, one wave per MB row; a row may start MB x once
 *               the row above has finished MB x+1 (progress counters, agent-scope release /
 *               acquire).  Reference: mb_intra4x4 / intra8x8 / intra16x16 (2987-4555), PCM (4736).
 *   k_deblock : in-loop filter, same 2-MB-lag wavefront, each MB filtered in an LDS tile with a
 *               4-sample halo in the exact raster order of deblock_pb (h264.cpp:10540-10663).
 * Inter MBs never read intra MBs of the same picture, so k_inter -> k_intra -> k_deblock on one
 * stream is exactly the reference's raster order in effect.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include "recon_kernels.h"
#include "intra_tables.h"

/* The workgroup's dynamic LDS.  Out-of-line device functions derive their LDS pointers from this
 * symbol instead of taking them as arguments: a pointer argument is generic, and every access
 * through it compiles to a flat_* instruction (vector-memory latency, vmcnt waits) instead of ds_*. */
extern __shared__ __attribute__((aligned(16))) uint8_t g_lds[];
/* an LDS address as a 32-bit local pointer: out-of-line functions take this (a generic pointer
 * argument would make every access flat_*, and g_lds named in a non-kernel function is looked up
 * in a dynamic-LDS offset table with a scalar load at every use) */
typedef __attribute__((address_space(3))) uint8_t lds_u8;
/* the base, made opaque at the call site (in a kernel it is a constant offset) so that the callee is
 * not specialised back onto g_lds by interprocedural constant propagation */
__device__ __forceinline__ lds_u8 *lds_base()
{
	uint32_t v = (uint32_t)(uintptr_t)(lds_u8 *)g_lds;
	asm volatile("" : "+s"(v));
	return (lds_u8 *)(uintptr_t)v;
}
#define LDS_ARG() lds_base()
template <typename T> __device__ __forceinline__ T *lds_ptr(lds_u8 *p) { return (T *)(uint8_t *)p; }
#include "recon_internal.h"
#include "m2dec_amd.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "m2dec_amd HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -1; } } while (0)

/* A wait for a hand-off ends in an error only after SPIN_ABORT polls (~30-60 s): every producer a wait points at
 * holds a workgroup reservation of the device budget (SlotBudget), so a slow hand-off means the GPU is shared with
 * other work and waiting is the recovery; only one that never comes (a bug) ends the decode.  After g_spin_report
 * polls (~1 s; M2DEC_AMD_SPIN_REPORT) a wait is reported in err[1] — the host prints it once — and goes on
 * (round 5 ended the decode there). */
#define SPIN_ABORT (1u << 26)
__device__ unsigned g_spin_report = 1u << 20;

/* Diagnostic timestamps (build with -DM2DEC_STAMPS; never in the product build): per MB row and
 * role, s_memrealtime (100 MHz) at events, read back with m2dec_amd_debug_stamps(). */
#define STAMP_ROWS 160
#define STAMP_EV 256
#ifdef M2DEC_STAMPS
__device__ unsigned long long g_stamps[STAMP_ROWS][4][STAMP_EV];
#define STAMP(row, role, idx, val)                                                                                   \
	do {                                                                                                             \
		if ((row) < STAMP_ROWS && (idx) < STAMP_EV && (threadIdx.x & 63) == 0)                                       \
			g_stamps[row][role][idx] = (__builtin_amdgcn_s_memrealtime() << 16) | (unsigned long long)((val) & 0xffff); \
	} while (0)
/* per-picture events of a batch launch: [pidx][0 first block starts, 1 inter workers done, 2 rows done] */
__device__ unsigned long long g_pstamps[256][4];
#define STAMPP(p, k) do { if ((p) < 256) g_pstamps[p][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP(row, role, idx, val) do { } while (0)
#define STAMPP(p, k) do { } while (0)
#endif
#if defined(M2DEC_STAMPS) && !defined(M2DEC_NO_STAMPI)
#define STAMPI(row, role, idx, val) STAMP(row, role, idx, val)
#else
#define STAMPI(row, role, idx, val) do { } while (0)
#endif
/* inter MB phase stamps (-DM2DEC_STAMPW): rows 72..87 = workgroup & 15, role = wave, idx = (MB count * 8 + event) */
#if defined(M2DEC_STAMPS) && defined(M2DEC_STAMPW)
#define STAMPW(cnt, ev) do { if ((threadIdx.x & 63) == 0) g_stamps[72 + (blockIdx.x & 15)][threadIdx.x >> 6][((cnt) * 8 + (ev)) & 255] = (__builtin_amdgcn_s_memrealtime() << 16) | (unsigned long long)(ev); } while (0)
#else
#define STAMPW(cnt, ev) do { } while (0)
#endif
/* deblocking filter sub-step stamps (-DM2DEC_STAMPD): [MB row][event][MB x]: 0 inputs ready, 1 vertical
 * edges done, 2 horizontal edges done */
#if defined(M2DEC_STAMPS) && defined(M2DEC_STAMPD)
__device__ unsigned long long g_dstamps[160][3][128];
#define STAMPD(row, ev, x) do { if ((threadIdx.x & 63) == 0 && (row) < 160 && (x) < 128) g_dstamps[row][ev][x] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMPD(row, ev, x) do { } while (0)
#endif
/* intra sub-phase stamps: the first 16 MBs of a row, 6 events each (role 3, idx 160..255) */
#define STAMPX(x, k) do { if ((x) < 16 && part == 0) STAMP(y, 3, 160 + (x) * 6 + (k), k); } while (0)

#ifdef M2DEC_DBG_ROWS
/* diagnostic (-DM2DEC_DBG_ROWS, never in the product build): per row workgroup and wave, the row intra_row
 * reconstructs and where its first MB's samples go (tools/replay_diff.py) */
__device__ unsigned int g_dbg_rows[256 * 4 * 2];
#endif
#ifdef M2DEC_DBG_INTRA
/* diagnostic (-DM2DEC_DBG_INTRA, never in the product build): the first I picture's MB (0, 0) luma context
 * before and after its reconstruction, read back with m2dec_amd_debug_intra (tools/replay_diff.py) */
__device__ int g_dbg[2048];
#endif

/* ======================================================================== motion compensation */
struct RefPlane {
	const uint8_t *p;
	int W, H;
};

__device__ __forceinline__ int fetch(const RefPlane &r, int x, int y)
{
	x = min(max(x, 0), r.W - 1);
	y = min(max(y, 0), r.H - 1);
	return r.p[y * r.W + x];
}

/* spec 8.4.2.2.1 (UMV == clamp); inter_pred_luma_frac* h264.cpp:6118-6261 */
__device__ int luma_mc(const RefPlane &r, int x, int y, int fx, int fy)
{
#define P(dx, dy) fetch(r, x + (dx), y + (dy))
#define TAPH(dy) (P(-2, dy) - 5 * P(-1, dy) + 20 * P(0, dy) + 20 * P(1, dy) - 5 * P(2, dy) + P(3, dy))
#define TAPV(dx) (P(dx, -2) - 5 * P(dx, -1) + 20 * P(dx, 0) + 20 * P(dx, 1) - 5 * P(dx, 2) + P(dx, 3))
	int c = fy * 4 + fx;
	if (c == 0) return P(0, 0);
	if (fy == 0) {
		int b = d_clip255((TAPH(0) + 16) >> 5);
		if (fx == 2) return b;
		return (b + P(fx == 1 ? 0 : 1, 0) + 1) >> 1;
	}
	if (fx == 0) {
		int h = d_clip255((TAPV(0) + 16) >> 5);
		if (fy == 2) return h;
		return (h + P(0, fy == 1 ? 0 : 1) + 1) >> 1;
	}
	if (fx != 2 && fy != 2) {
		/* e, g, p, r: average of two half-pel samples */
		int bh = d_clip255((TAPH(fy == 1 ? 0 : 1) + 16) >> 5);
		int vv = d_clip255((TAPV(fx == 1 ? 0 : 1) + 16) >> 5);
		return (bh + vv + 1) >> 1;
	}
	{
		int t0 = TAPH(-2), t1 = TAPH(-1), t2 = TAPH(0), t3 = TAPH(1), t4 = TAPH(2), t5 = TAPH(3);
		int j = d_clip255((t0 - 5 * t1 + 20 * t2 + 20 * t3 - 5 * t4 + t5 + 512) >> 10);
		int o;
		if (c == 10) return j;
		if (fx == 2) o = d_clip255((((fy == 1) ? t2 : t3) + 16) >> 5);         /* f: b, q: s */
		else o = d_clip255((TAPV(fx == 1 ? 0 : 1) + 16) >> 5);                /* i: h, k: m */
		return (j + o + 1) >> 1;
	}
#undef P
#undef TAPH
#undef TAPV
}

/* the same on a reference window staged in LDS: 9 rows of 12 bytes around one 4x4 block (rows from 2
 * above the block's integer position, columns from the 4-aligned byte at or left of 2 before it; `off`
 * = that distance), edge samples already clamped when it was loaded; (cx, ry) = the sample inside the
 * block */
__device__ __forceinline__ int luma_mc_win(const uint8_t *w, int off, int cx, int ry, int fx, int fy)
{
#define P(dx, dy) ((int)w[(ry + 2 + (dy)) * 12 + off + 2 + cx + (dx)])
#define TAPH(dy) (P(-2, dy) - 5 * P(-1, dy) + 20 * P(0, dy) + 20 * P(1, dy) - 5 * P(2, dy) + P(3, dy))
#define TAPV(dx) (P(dx, -2) - 5 * P(dx, -1) + 20 * P(dx, 0) + 20 * P(dx, 1) - 5 * P(dx, 2) + P(dx, 3))
	const int c = fy * 4 + fx;
	if (c == 0) return P(0, 0);
	if (fy == 0) {
		const int b = d_clip255((TAPH(0) + 16) >> 5);
		if (fx == 2) return b;
		return (b + P(fx == 1 ? 0 : 1, 0) + 1) >> 1;
	}
	if (fx == 0) {
		const int h = d_clip255((TAPV(0) + 16) >> 5);
		if (fy == 2) return h;
		return (h + P(0, fy == 1 ? 0 : 1) + 1) >> 1;
	}
	if (fx != 2 && fy != 2) {
		const int bh = d_clip255((TAPH(fy == 1 ? 0 : 1) + 16) >> 5);
		const int vv = d_clip255((TAPV(fx == 1 ? 0 : 1) + 16) >> 5);
		return (bh + vv + 1) >> 1;
	}
	{
		const int t0 = TAPH(-2), t1 = TAPH(-1), t2 = TAPH(0), t3 = TAPH(1), t4 = TAPH(2), t5 = TAPH(3);
		const int j = d_clip255((t0 - 5 * t1 + 20 * t2 + 20 * t3 - 5 * t4 + t5 + 512) >> 10);
		int o;
		if (c == 10) return j;
		if (fx == 2) o = d_clip255((((fy == 1) ? t2 : t3) + 16) >> 5);
		else o = d_clip255((TAPV(fx == 1 ? 0 : 1) + 16) >> 5);
		return (j + o + 1) >> 1;
	}
#undef P
#undef TAPH
#undef TAPV
}

/* chroma 1/8 bilinear on interleaved NV12 (filter_chroma_*, h264.cpp:4859-5057) */
__device__ __forceinline__ int chroma_mc(const uint8_t *cp, int W, int CH, int comp, int x, int y, int dx, int dy)
{
	int cw = W >> 1;
	int xa = min(max(x, 0), cw - 1), xb = min(max(x + 1, 0), cw - 1);
	int ya = min(max(y, 0), CH - 1), yb = min(max(y + 1, 0), CH - 1);
	int A = cp[ya * W + xa * 2 + comp], B = cp[ya * W + xb * 2 + comp];
	int C = cp[yb * W + xa * 2 + comp], D = cp[yb * W + xb * 2 + comp];
	return ((8 - dx) * (8 - dy) * A + dx * (8 - dy) * B + (8 - dx) * dy * C + dx * dy * D + 32) >> 6;
}

/* weighted / averaged combination of the list predictions (h264.cpp:5298-5318, 6726-7118) */
__device__ __forceinline__ int combine(const m2r_slice_t *sl, const m2r_inter_t &it, int b8, int comp, int use0, int use1, int v0, int v1)
{
	int mode = sl->wp_mode;
	if (mode == M2R_WP_EXPLICIT) {
		int sh = sl->log2wd[comp ? 1 : 0];
		if (use0 && use1) {
			int r0 = it.refidx[0][b8], r1 = it.refidx[1][b8];
			int w0 = sl->w[0][r0][comp], w1 = sl->w[1][r1][comp];
			int o0 = sl->o[0][r0][comp], o1 = sl->o[1][r1][comp];
			int t = d_sat16(v0 * w0 + (1 << sh));
			t = d_sat16(t + v1 * w1);
			t >>= sh + 1;
			t = d_sat16(t + ((o0 + o1 + 1) >> 1));
			return d_clip255(t);
		} else {
			int lx = use0 ? 0 : 1;
			int r = it.refidx[lx][b8];
			int rnd = sh ? 1 << (sh - 1) : 0;
			return d_clip255((((use0 ? v0 : v1) * sl->w[lx][r][comp] + rnd) >> sh) + sl->o[lx][r][comp]);
		}
	}
	if (use0 && use1) {
		if (mode == M2R_WP_IMPLICIT) {
			int r0 = it.refidx[0][b8], r1 = it.refidx[1][b8];
			int w0 = sl->iw[r0][r1][0], w1 = sl->iw[r0][r1][1];
			int t = d_sat16(v0 * w0 + 32);
			t = d_sat16(t + v1 * w1);
			return d_clip255(t >> 6);
		}
		return (v0 + v1 + 1) >> 1;
	}
	return use0 ? v0 : v1;
}

/* write-through hand-off primitives (cdna_hip_programming.md §6 Guideline 16, R1): every shared word is
 * a global-address-space agent-scope access; payload 8-byte sc1 stores, drained before one lane's
 * sc1 flag store; consumer polls the flag with sc1 loads and reads the payload with sc1 loads. */
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;

__device__ __forceinline__ void st_sc1(void *p, unsigned long long v)
{
	__hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st32_sc1(void *p, uint32_t v)
{
	__hip_atomic_store((gi32 *)p, (int)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* 16-byte write-through store (global_store_dwordx4 … sc1): the deblocking storer writes whole 64-byte
 * row pieces of 4 MBs with it, where 4-byte stores left a partial-line memory write per 16 bytes */
__device__ __forceinline__ void st128_sc1(void *p, uint4 v)
{
	typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
	const u32x4 d = {v.x, v.y, v.z, v.w};
	asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(d) : "memory");
}

__device__ __forceinline__ unsigned long long ld_sc1(const void *p)
{
	return __hip_atomic_load((gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* bounded spin step: false once the spin budget is spent or another workgroup has flagged an error
 * (so one failure drains the whole grid quickly instead of every row timing out in turn) */
__device__ __forceinline__ bool spin_ok(unsigned &spins, int *err, int code)
{
	__builtin_amdgcn_s_sleep(1);
	++spins;
	if ((spins & 255) == 0 && __hip_atomic_load((gi32 *)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
	if (__builtin_expect(spins == g_spin_report, 0) && (threadIdx.x & 63) == 0) atomicOr(err + 1, code); /* (reported, waits on) */
	if (spins > SPIN_ABORT) {
		if ((threadIdx.x & 63) == 0) atomicOr(err, code);
		return false;
	}
	return true;
}

/* the polls after which a wait is reported (M2DEC_AMD_SPIN_REPORT), on the current device */
extern "C" int m2dec_amd_hip_set_spin_report(unsigned polls)
{
	CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_spin_report), &polls, sizeof(polls), 0, hipMemcpyHostToDevice));
	return 0;
}

__device__ __forceinline__ bool poll_ge(int *flag, int need, int *err)
{
	unsigned spins = 0;
	while (__hip_atomic_load((gi32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
		if (!spin_ok(spins, err, 2)) return false;
	}
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keeps the payload loads below the poll */
	return true;
}

/* poll_ge returning the value seen (>= need; need - 1 after a failed spin) */
__device__ __forceinline__ int poll_get(int *flag, int need, int *err)
{
	unsigned spins = 0;
	int v;
	while ((v = __hip_atomic_load((gi32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < need) {
		if (!spin_ok(spins, err, 2)) return need - 1;
	}
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keeps the payload loads below the poll */
	return v;
}

__device__ __forceinline__ void signal_progress(int *flag, int value)
{
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* the (single) storing wave drains its sc1 stores */
	if ((threadIdx.x & 63) == 0) __hip_atomic_store((gi32 *)flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* ======================================================================== k_inter */
#ifdef M2DEC_NOINLINE
#define M2DEC_INTER_MB_ATTR __attribute__((noinline))
#else
#define M2DEC_INTER_MB_ATTR
#endif
/* wave-private residual buffers of the inter MBs in flight in a workgroup (one MB per wave) */
struct InterRes {
	int r[256 + 128]; /* luma raster 16x16, then Cb / Cr 8x8 */
	uint32_t win[2][16][9][3]; /* luma reference windows per list and raster 4x4 block (luma_mc_win) */
	uint32_t cwin[2][16][3][2]; /* chroma windows per list and 2x2 chroma block: 3 rows x 8 bytes */
};

/* wave-level step boundary for the inter MB: its lanes talk through LDS only (see WSYNC below) */
#define ISYNC()                                                  \
	do {                                                         \
		asm volatile("" ::: "memory");                           \
		__builtin_amdgcn_wave_barrier();                         \
	} while (0)

/* one inter macroblock on ONE wave (lane = 0..63; the call is wave-uniform): luma 4 samples and chroma
 * 2 samples per lane, the residual in the wave's own LDS buffer, no workgroup barrier — the four waves
 * of a worker each take a different MB of the item.  `it` is the MB's motion record staged in LDS.
 * Every global load of the MB (the luma and chroma reference windows, the coefficients) is issued
 * before the first of them is waited for: one memory round trip per MB.  The samples go to the item's
 * LDS segment. */
__device__ M2DEC_INTER_MB_ATTR void inter_mb(const int addr, const m2r_mb_t m, const m2r_inter_t &it,
                         const m2r_slice_t *__restrict__ slices, const int16_t *__restrict__ pool, uint8_t *frames,
                         size_t fsz, int W, int H, int Wmb, uint8_t *seg, InterRes *res, const int lane_in, const int scnt = 0)
{
	STAMPW(scnt, 0);
	/* the lane index through an opaque copy: every per-lane address below is then computed inside the MB
	 * loop of the caller instead of being hoisted out of it as loop invariants, which held ~60 VGPRs across
	 * the loop and spilled them to scratch at the 128-VGPR budget */
#ifndef M2DEC_NO_LANE_LAUNDER
	int lane;
	asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane_in));
#else
	const int lane = lane_in; /* r99 and before: 740 B of scratch per lane, 63 scratch operations per MB */
#endif
	const int mbx = addr % Wmb, mby = addr / Wmb;
	const m2r_slice_t *sl = &slices[m.slice];
	const int CH = H >> 1;
	int *const R = res->r;
	const int lx = lane & 15;
	const int cx = lane & 7, cy = lane >> 3;
	const int t8 = (m.flags & M2R_FLAG_T8x8) != 0;
	const bool coded = __builtin_amdgcn_readfirstlane(m.cbp) != 0;

	/* ---- phase 1: loads.  Luma windows: (list, 4x4 block, row) p = lane + 64 j, 12 bytes each (three
	 * dwords, or clamped bytes where the span leaves the picture) */
	uint32_t lw[5][3];
#pragma unroll
	for (int j = 0; j < 5; ++j) {
		const int p = lane + 64 * j;
		lw[j][0] = lw[j][1] = lw[j][2] = 0;
		if (p < 288) {
			const int l = p >= 144, rem = p - 144 * l, b = rem / 9, row = rem - 9 * b;
			const int s = it.slot[l][(b >> 3) * 2 + ((b & 3) >> 1)];
			if (s >= 0) {
				const int X = mbx * 16 + (b & 3) * 4 + (it.mv[l][b][0] >> 2), Y = mby * 16 + (b >> 2) * 4 + (it.mv[l][b][1] >> 2);
				const int xa = (X - 2) & ~3, y = min(max(Y - 2 + row, 0), H - 1);
				const uint8_t *src = frames + (size_t)s * fsz + (size_t)y * W;
				if (xa >= 0 && xa + 12 <= W) {
					const uint32_t *s32 = (const uint32_t *)(src + xa);
					lw[j][0] = s32[0];
					lw[j][1] = s32[1];
					lw[j][2] = s32[2];
				} else {
#pragma unroll
					for (int k = 0; k < 3; ++k) {
						uint32_t v = 0;
#pragma unroll
						for (int i = 0; i < 4; ++i) v |= (uint32_t)src[min(max(xa + 4 * k + i, 0), W - 1)] << (8 * i);
						lw[j][k] = v;
					}
				}
			}
		}
	}
	/* chroma windows: (list, 2x2 chroma block, row) p = lane + 64 j < 96: 3 rows of the interleaved
	 * Cb / Cr bytes of component samples X .. X + 2 (8 bytes from the 4-aligned byte at or left of 2 X) */
	uint32_t cw[2][2];
#pragma unroll
	for (int j = 0; j < 2; ++j) {
		const int p = lane + 64 * j;
		cw[j][0] = cw[j][1] = 0;
		if (p < 96) {
			const int l = p >= 48, rem = p - 48 * l, b = rem / 3, row = rem - 3 * b;
			const int s = it.slot[l][(b >> 3) * 2 + ((b & 3) >> 1)];
			if (s >= 0) {
				const int X = mbx * 8 + (b & 3) * 2 + (it.mv[l][b][0] >> 3), Y = mby * 8 + (b >> 2) * 2 + (it.mv[l][b][1] >> 3);
				const int xa = (2 * X) & ~3, y = min(max(Y + row, 0), CH - 1);
				const uint8_t *src = frames + (size_t)s * fsz + (size_t)W * H + (size_t)y * W;
				if (xa >= 0 && xa + 8 <= W) {
					const uint32_t *s32 = (const uint32_t *)(src + xa);
					cw[j][0] = s32[0];
					cw[j][1] = s32[1];
				} else {
#pragma unroll
					for (int k = 0; k < 2; ++k) {
						uint32_t v = 0;
#pragma unroll
						for (int i = 0; i < 4; ++i) {
							const int bx = xa + 4 * k + i;
							const int pos = min(max(bx >> 1, 0), (W >> 1) - 1); /* clamped component sample */
							v |= (uint32_t)src[2 * pos + (bx & 1)] << (8 * i);
						}
						cw[j][k] = v;
					}
				}
			}
		}
	}
	/* the residual's coefficients (dequantised), luma sample (lx, (lane >> 4) + 4 k), chroma (cx, cy) */
	int rl[4] = {0, 0, 0, 0}, rc[2] = {0, 0}, lv0[2] = {0, 0};
	uint64_t nzl[4] = {0, 0, 0, 0};
	if (coded) {
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const int ly = (lane >> 4) + 4 * k;
			const int lb = (ly >> 2) * 4 + (lx >> 2), lb8 = (ly >> 3) * 2 + (lx >> 3);
			if (t8) {
				const int bit = 4 * lb8;
				if (m.nz & (1u << bit)) {
					const int lv = pool[m.coef + d_luma_off(m, bit) + (ly & 7) * 8 + (lx & 7)];
					rl[k] = lv * d_scale8(m.qpy, lx & 7, ly & 7);
					nzl[k] = __ballot(lv != 0);
				}
			} else {
				const int blk = d_rast2blk(lb);
				if (m.nz & (1u << blk)) rl[k] = pool[m.coef + d_luma_off(m, blk) + (ly & 3) * 4 + (lx & 3)] * d_scale4(m.qpy, lx & 3, ly & 3);
			}
		}
		if (t8) {
			/* the DC level of this lane's two 8x8 blocks (the DC-only add below) */
#pragma unroll
			for (int h = 0; h < 2; ++h) {
				const int lb8 = h * 2 + (lx >> 3);
				if (m.nz & (1u << (4 * lb8))) lv0[h] = pool[m.coef + d_luma_off(m, 4 * lb8)];
			}
		}
		const int ccbp = m.cbp >> 4;
		const int cblk = (cy >> 2) * 2 + (cx >> 2);
		const int pos = (cy & 3) * 4 + (cx & 3);
#pragma unroll
		for (int cc = 0; cc < 2; ++cc) {
			if (ccbp) {
				if (pos == 0) {
					rc[cc] = d_chroma_dc(m, pool + m.coef, cc, cblk);
				} else if (ccbp == 2 && (m.nz & M2R_NZ_CAC(cc, cblk))) {
					const int bit = 19 + 4 * cc + cblk;
					rc[cc] = pool[m.coef + d_chroma_off(m, bit) + pos] * d_scale4(cc ? m.qpc[1] : m.qpc[0], cx & 3, cy & 3);
				}
			}
		}
	}
	/* ---- phase 2: windows and residual into the wave's LDS */
#pragma unroll
	for (int j = 0; j < 5; ++j) {
		const int p = lane + 64 * j;
		if (p < 288) {
			const int l = p >= 144, rem = p - 144 * l, b = rem / 9, row = rem - 9 * b;
			uint32_t *dst = res->win[l][b][row];
			dst[0] = lw[j][0];
			dst[1] = lw[j][1];
			dst[2] = lw[j][2];
		}
	}
#pragma unroll
	for (int j = 0; j < 2; ++j) {
		const int p = lane + 64 * j;
		if (p < 96) {
			const int l = p >= 48, rem = p - 48 * l, b = rem / 3, row = rem - 3 * b;
			uint32_t *dst = res->cwin[l][b][row];
			dst[0] = cw[j][0];
			dst[1] = cw[j][1];
		}
	}
	if (coded) {
#pragma unroll
		for (int k = 0; k < 4; ++k) R[((lane >> 4) + 4 * k) * 16 + lx] = rl[k];
#pragma unroll
		for (int cc = 0; cc < 2; ++cc) R[256 + cc * 64 + cy * 8 + cx] = rc[cc];
	}
	ISYNC();
	STAMPW(scnt, 1);
	/* ---- luma prediction: samples lane + 64 k (row (lane >> 4) + 4 k, column lane & 15) */
	int predl[4];
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const int ly = (lane >> 4) + 4 * k;
		const int lb = (ly >> 2) * 4 + (lx >> 2), lb8 = (ly >> 3) * 2 + (lx >> 3);
		int v[2] = {0, 0};
		int use[2];
		for (int l = 0; l < 2; ++l) {
			const int s = it.slot[l][lb8];
			use[l] = s >= 0;
			if (use[l]) {
				const int mx = it.mv[l][lb][0], my = it.mv[l][lb][1];
				const int X = mbx * 16 + (lb & 3) * 4 + (mx >> 2);
				v[l] = luma_mc_win((const uint8_t *)res->win[l][lb], (X - 2) & 3, lx & 3, ly & 3, mx & 3, my & 3);
			}
		}
		predl[k] = combine(sl, it, lb8, 0, use[0], use[1], v[0], v[1]);
	}
	/* ---- chroma prediction: component cc, sample (cx, cy), from the chroma windows (filter_chroma_*) */
	const int cb = (cy >> 1) * 4 + (cx >> 1), cb8 = (cy >> 2) * 2 + (cx >> 2);
	int predc[2];
#pragma unroll
	for (int cc = 0; cc < 2; ++cc) {
		int v[2] = {0, 0};
		int use[2];
		for (int l = 0; l < 2; ++l) {
			const int s = it.slot[l][cb8];
			use[l] = s >= 0;
			if (use[l]) {
				const int mx = it.mv[l][cb][0], my = it.mv[l][cb][1];
				const int dx = mx & 7, dy = my & 7;
				const int X = mbx * 8 + (cb & 3) * 2 + (mx >> 3);
				/* sample (cx, cy) sits at window row (cy & 1), component column (cx & 1) from X */
				const uint8_t *w = (const uint8_t *)res->cwin[l][cb][cy & 1];
				const int o = 2 * X - ((2 * X) & ~3) + 2 * (cx & 1) + cc;
				const int A = w[o], B = w[o + 2], C = w[o + 8], D = w[o + 10];
				v[l] = ((8 - dx) * (8 - dy) * A + dx * (8 - dy) * B + (8 - dx) * dy * C + dx * dy * D + 32) >> 6;
			}
		}
		predc[cc] = combine(sl, it, cb8, 1 + cc, use[0], use[1], v[0], v[1]);
	}
	STAMPW(scnt, 2);

	/* output: the item's LDS segment buffer (luma rows 0..15, chroma rows 16..23, SEG_ROW bytes each) */
	uint8_t *const dl = seg + (lane >> 4) * SEG_ROW + (mbx & 7) * 16 + lx;
	uint8_t *const dc = seg + (16 + cy) * SEG_ROW + (mbx & 7) * 16 + cx * 2;
	if (!coded) {
#pragma unroll
		for (int k = 0; k < 4; ++k) dl[4 * k * SEG_ROW] = (uint8_t)predl[k];
		dc[0] = (uint8_t)predc[0];
		dc[1] = (uint8_t)predc[1];
		STAMPW(scnt, 6);
		return; /* uniform: m is the same in every lane */
	}
	STAMPW(scnt, 3);
	/* ---- row pass: 8x8 luma rows on lanes 0..31 beside the chroma rows on 32..63; 4x4: luma rows on all
	 * lanes, then chroma rows */
	if (t8) {
		if (lane < 32) {
			const int b8 = lane >> 3, row = lane & 7;
			int *p = &R[((b8 >> 1) * 8 + row) * 16 + (b8 & 1) * 8];
			int v[8];
			for (int k = 0; k < 8; ++k) v[k] = p[k];
			d_idct8_1d(v);
			for (int k = 0; k < 8; ++k) p[k] = v[k];
		}
	} else {
		const int b = lane >> 2, row = lane & 3;
		int *p = &R[((b >> 2) * 4 + row) * 16 + (b & 3) * 4];
		int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
	}
	if (t8 ? lane >= 32 : lane < 32) {
		const int k = lane & 31, comp = k >> 4, b = (k >> 2) & 3, row = k & 3;
		int *p = &R[256 + comp * 64 + ((b >> 1) * 4 + row) * 8 + (b & 1) * 4];
		int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
	}
	ISYNC();
	/* ---- column pass (+32 >> 6) */
	if (t8) {
		if (lane < 32) {
			const int b8 = lane >> 3, col = lane & 7;
			int *p = &R[((b8 >> 1) * 8) * 16 + (b8 & 1) * 8 + col];
			int v[8];
			for (int k = 0; k < 8; ++k) v[k] = p[k * 16];
			d_idct8_1d(v);
			for (int k = 0; k < 8; ++k) p[k * 16] = (v[k] + 32) >> 6;
		}
	} else {
		const int b = lane >> 2, col = lane & 3;
		int *p = &R[((b >> 2) * 4) * 16 + (b & 3) * 4 + col];
		int a0 = p[0], a1 = p[16], a2 = p[32], a3 = p[48];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = (a0 + 32) >> 6; p[16] = (a1 + 32) >> 6; p[32] = (a2 + 32) >> 6; p[48] = (a3 + 32) >> 6;
	}
	if (t8 ? lane >= 32 : lane < 32) {
		const int k = lane & 31, comp = k >> 4, b = (k >> 2) & 3, col = k & 3;
		int *p = &R[256 + comp * 64 + ((b >> 1) * 4) * 8 + (b & 1) * 4 + col];
		int a0 = p[0], a1 = p[8], a2 = p[16], a3 = p[24];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = (a0 + 32) >> 6; p[8] = (a1 + 32) >> 6; p[16] = (a2 + 32) >> 6; p[24] = (a3 + 32) >> 6;
	}
	ISYNC();
	STAMPW(scnt, 4);
	/* ---- add.  8x8 blocks with only their DC level take the reference's DC-only path (d_swar): the
	 * non-zero levels per 8x8 block from the ballots of the dequantisation (samples k = 0, 1 cover the top
	 * blocks, 2, 3 the bottom ones; lanes with (lane & 15) < 8 the left ones) */
	const uint64_t LEFT = 0x00ff00ff00ff00ffull;
	const int n8[4] = {(int)(__popcll(nzl[0] & LEFT) + __popcll(nzl[1] & LEFT)), (int)(__popcll(nzl[0] & ~LEFT) + __popcll(nzl[1] & ~LEFT)),
	                   (int)(__popcll(nzl[2] & LEFT) + __popcll(nzl[3] & LEFT)), (int)(__popcll(nzl[2] & ~LEFT) + __popcll(nzl[3] & ~LEFT))};
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const int ly = (lane >> 4) + 4 * k;
		const int lb8 = (ly >> 3) * 2 + (lx >> 3);
		const int cnt = (lx >> 3) ? ((k >> 1) ? n8[3] : n8[1]) : ((k >> 1) ? n8[2] : n8[0]);
		int out;
		if (t8 && cnt == 1 && (m.nz & (1u << (4 * lb8))) && lv0[k >> 1] != 0)
			out = d_swar(predl[k], lv0[k >> 1] * d_scale8(m.qpy, 0, 0), lx & 7, 8);
		else
			out = d_clip255(predl[k] + R[ly * 16 + lx]);
		dl[4 * k * SEG_ROW] = (uint8_t)out;
	}
#pragma unroll
	for (int cc = 0; cc < 2; ++cc) dc[cc] = (uint8_t)d_clip255(predc[cc] + R[256 + cc * 64 + cy * 8 + cx]);
	STAMPW(scnt, 5);
}

/* ======================================================================== intra prediction (per sample) */
#define LW 25 /* intra luma context row: [0] = x0 - 1, [1..24] = x0 .. x0 + 23 */
static_assert(LW == M2D_IPRED4O_LW, "c_ipred4o offsets assume this luma context stride");

/* 8x8 on filtered neighbours pt[0..15], lf[0..7], tlf (spec 8.3.2.2; h264.cpp:3301-3929); the
 * directional modes go through intra_tables.h, this is used for DC */
__device__ int pred8_px(int mode, int avail, int x, int y, const int *pt, const int *lf, int tlf)
{
#define PT(i) ((i) < 0 ? tlf : pt[i])
#define LF(i) ((i) < 0 ? tlf : lf[i])
	int hasL = avail & 1, hasT = avail & 2, hasTL = avail & 8;
	switch (mode) {
	case 0: return hasT ? pt[x] : -1;
	case 1: return hasL ? lf[y] : -1;
	case 2: {
		int s = 0;
		if (hasT && hasL) { for (int i = 0; i < 8; ++i) s += pt[i] + lf[i]; return (s + 8) >> 4; }
		if (hasL) { for (int i = 0; i < 8; ++i) s += lf[i]; return (s + 4) >> 3; }
		if (hasT) { for (int i = 0; i < 8; ++i) s += pt[i]; return (s + 4) >> 3; }
		return 128;
	}
	case 3:
		if (!hasT) return -1;
		if (x == 7 && y == 7) return (pt[14] + 3 * pt[15] + 2) >> 2;
		return (pt[x + y] + 2 * pt[x + y + 1] + pt[x + y + 2] + 2) >> 2;
	case 4:
		if (!(hasT && hasL && hasTL)) return -1;
		if (x > y) return (PT(x - y - 2) + 2 * PT(x - y - 1) + pt[x - y] + 2) >> 2;
		if (x < y) return (LF(y - x - 2) + 2 * LF(y - x - 1) + lf[y - x] + 2) >> 2;
		return (pt[0] + 2 * tlf + lf[0] + 2) >> 2;
	case 5: {
		if (!(hasT && hasL && hasTL)) return -1;
		int z = 2 * x - y, i = x - (y >> 1);
		if (z >= 0 && !(z & 1)) return (PT(i - 1) + pt[i] + 1) >> 1;
		if (z >= 0) return (PT(i - 2) + 2 * PT(i - 1) + pt[i] + 2) >> 2;
		if (z == -1) return (lf[0] + 2 * tlf + pt[0] + 2) >> 2;
		return (LF(y - 2 * x - 1) + 2 * LF(y - 2 * x - 2) + LF(y - 2 * x - 3) + 2) >> 2;
	}
	case 6: {
		if (!(hasT && hasL && hasTL)) return -1;
		int z = 2 * y - x, i = y - (x >> 1);
		if (z >= 0 && !(z & 1)) return (LF(i - 1) + lf[i] + 1) >> 1;
		if (z >= 0) return (LF(i - 2) + 2 * LF(i - 1) + lf[i] + 2) >> 2;
		if (z == -1) return (lf[0] + 2 * tlf + pt[0] + 2) >> 2;
		return (PT(x - 2 * y - 1) + 2 * PT(x - 2 * y - 2) + PT(x - 2 * y - 3) + 2) >> 2;
	}
	case 7: {
		if (!hasT) return -1;
		int i = x + (y >> 1);
		if (!(y & 1)) return (pt[i] + pt[i + 1] + 1) >> 1;
		return (pt[i] + 2 * pt[i + 1] + pt[i + 2] + 2) >> 2;
	}
	default: {
		if (!hasL) return -1;
		int z = x + 2 * y, i = y + (x >> 1);
		if (z > 13) return lf[7];
		if (z == 13) return (lf[6] + 3 * lf[7] + 2) >> 2;
		if (!(z & 1)) return (lf[i] + lf[i + 1] + 1) >> 1;
		return (lf[i] + 2 * lf[i + 1] + lf[i + 2] + 2) >> 2;
	}
	}
#undef PT
#undef LF
}

/* per-block avail constants (h264.cpp:3121-3230, 4093-4118) */
__device__ __forceinline__ int avail4(int blk, int a)
{
	switch (blk) {
	case 0: return a | ((a & 2) ? 4 : 0);
	case 1: return a | ((a & 2) ? 5 : 1);
	case 2: return a | 6;
	case 4: return a | ((a & 2) ? 5 : 1);
	case 5: return a | 1;
	case 8: return a | 6;
	case 10: return a | 6;
	case 6: case 9: case 12: case 14: return 7;
	default: return 3;
	}
}

__device__ __forceinline__ int avail8(int b, int a)
{
	switch (b) {
	case 0: return (a & ~4) | ((a & 2) * 2);
	case 1: return (a & ~8) | ((a & 2) * 4) | 1;
	case 2: return 6 | ((a & 1) * 9);
	default: return 11;
	}
}

/* ======================================================================== k_intra */

/*
 * Intra / PCM macroblocks, one 64-lane workgroup per MB row, intra MBs left to right.  An intra MB
 * reads unfiltered samples of its left, top-left, top and top-right neighbours.  Inter neighbours
 * were reconstructed by k_inter before this launch (plain loads); intra neighbours of the row above
 * were written in this launch by another workgroup and are read from their 32-byte hand-off record
 * (bottom luma row + bottom chroma row, sc1 stores / sc1 loads, G16 R1), after polling that row's
 * progress word only up to the rightmost intra MB among the three upper neighbours.  P/B pictures
 * with few intra MBs therefore carry no row-to-row chain through their inter MBs.
 */

/* wave-level sync for the intra wavefront, which runs on ONE wave of its workgroup: lanes talk
 * through LDS only, so an LDS drain + wave barrier suffices (outstanding global prefetches are not
 * waited for) */
#ifdef M2DEC_WSYNC_WAIT
#define WSYNC()                                                  \
	do {                                                         \
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       \
		__builtin_amdgcn_wave_barrier();                         \
	} while (0)
#else
/* a wave's LDS operations are performed in issue order, so a later ds_read of this wave sees its
 * earlier ds_writes without waiting for them: only the compiler must not move memory operations
 * across the step boundary */
#define WSYNC()                                                  \
	do {                                                         \
		asm volatile("" ::: "memory");                           \
		__builtin_amdgcn_wave_barrier();                         \
	} while (0)
#endif

union MbWords {
	m2r_mb_t m;
	int w[8];
};

/* lane `lane`'s record, as wave-uniform values */
__device__ __forceinline__ m2r_mb_t lane_mb(const MbWords &mine, int lane)
{
	MbWords r;
#pragma unroll
	for (int i = 0; i < 8; ++i) r.w[i] = __builtin_amdgcn_readlane(mine.w[i], lane);
	return r.m;
}

/* one intra wave's LDS context (carved from the dynamic LDS: two rows run their intra at once) */
struct IntraLDS {
	uint8_t L[17][LW];   /* row 0: top neighbours; rows 1..16: MB rows; col 0: left neighbour */
	uint8_t C[2][9][9];  /* per component: row 0 top (col 0 top-left), col 0 left */
	int R[256 + 128];
	int DC[16];
	int F[32];           /* filtered 8x8 neighbours: [0..15] top, [16..23] left, [24] top-left */
	int HV[4];
	int16_t Q[2][M2R_MB_COEF_MAX]; /* the current / next intra MB's coefficients */
};

/* one part of the intra / PCM MBs of MB row y on one wave: luma (part 0) or chroma (part 1); the
 * two parts of a row run on two waves side by side (chroma prediction only reads chroma
 * neighbours).  progress: this part's per-row progress words; HBI granules 0,1 luma, 2,3 chroma. */
/* the prediction tables of intra_tables.h, staged in LDS once per workgroup */
struct IntraTables {
	uint32_t p4o[2][9][16];
	uint32_t p8[9][64];
};

__device__ __forceinline__ int ipred_taps(uint32_t w, int bits, const int *nv)
{
	const int s = (int)((w >> (3 * bits + 6)) & 3);
	const int v = (int)((w >> (3 * bits)) & 3) * nv[0] + (int)((w >> (3 * bits + 2)) & 3) * nv[1] +
	              (int)((w >> (3 * bits + 4)) & 3) * nv[2];
	return (v + ((1 << s) >> 1)) >> s;
}

/* The reconstruction of ONE intra / PCM MB in an LDS context whose row 0 / column 0 already hold the
 * unfiltered top / left neighbours (luma L[0][0] top-left, L[0][1..24] top and top-right, L[1..16][0]
 * left; chroma C[c][0][*], C[c][*][0] likewise): luma on the wave(s) with do_luma, chroma on the
 * wave(s) with do_chroma (disjoint LDS: L, R[0..255], DC, F, HV / C, R[256..383]).  q: the MB's pool
 * segment (staged in LDS).  Reference: mb_intra4x4 / intraNxN / intra16x16 / intrapcm
 * (h264.cpp:3121-3254, 4083-4127, 4407-4555, 4708-4761), residual_chroma (2374-2461). */
#ifdef M2DEC_BODY_NOINLINE
#define M2DEC_BODY_ATTR __attribute__((noinline))
#else
#define M2DEC_BODY_ATTR __forceinline__
#endif
__device__ M2DEC_BODY_ATTR void intra_mb_body(const m2r_mb_t &m, const int16_t *q, const int t_in, const bool do_luma,
                                              const bool do_chroma, IntraLDS *ctx, const IntraTables *tabs)
{
	/* the lane index laundered per call: inside intra_row's MB loop every lane-dependent address
	 * below would otherwise be hoisted out of the loop and held in registers (spills) */
	int t = t_in;
	asm volatile("" : "+v"(t));
	uint8_t(&L)[17][LW] = ctx->L;
	uint8_t(&C)[2][9][9] = ctx->C;
	int(&R)[256 + 128] = ctx->R;
	int(&DC)[16] = ctx->DC;
	int(&F)[32] = ctx->F;
	int(&HV)[4] = ctx->HV;
	if (m.kind == M2R_MB_PCM) {
		const uint8_t *s = (const uint8_t *)q;
		if (do_luma)
			for (int k = t; k < 256; k += 64) L[1 + (k >> 4)][1 + (k & 15)] = s[k];
		else
			for (int k = t; k < 128; k += 64) C[k >> 6][1 + ((k >> 3) & 7)][1 + (k & 7)] = s[256 + k];
		WSYNC();
	} else {
		/* ---- chroma prediction (h264.cpp:4559-4706); thread t: sample (t & 7, t >> 3) of both components */
		if (do_chroma) {
			int ca = m.avail_chroma, mode = m.chroma_mode;
			int px = t & 7, py = t >> 3;
			for (int c = 0; c < 2; ++c) {
				int v = -1;
				if (mode == 0) {
					int blk = (py >> 2) * 2 + (px >> 2), xo = (px >> 2) * 4, yo = (py >> 2) * 4, st = 0, sl = 0;
					int ht = (ca & 2) != 0, hl = (ca & 1) != 0;
					for (int i = 0; i < 4; ++i) { st += C[c][0][1 + xo + i]; sl += C[c][1 + yo + i][0]; }
					if (blk == 0 || blk == 3) v = (ht && hl) ? (st + sl + 4) >> 3 : (hl ? (sl + 2) >> 2 : (ht ? (st + 2) >> 2 : 128));
					else if (blk == 1) v = ht ? (st + 2) >> 2 : (hl ? (sl + 2) >> 2 : 128);
					else v = hl ? (sl + 2) >> 2 : (ht ? (st + 2) >> 2 : 128);
				} else if (mode == 1) {
					if (ca & 1) v = C[c][1 + py][0];
				} else if (mode == 2) {
					if (ca & 2) v = C[c][0][1 + px];
				} else {
					int Hh = 0, Vv = 0;
					for (int i = 0; i < 4; ++i) {
						Hh += (i + 1) * (C[c][0][1 + 4 + i] - C[c][0][1 + 2 - i]);
						Vv += (i + 1) * (C[c][1 + 4 + i][0] - C[c][1 + 2 - i][0]);
					}
					int a = 16 * (C[c][8][0] + C[c][0][8]);
					int b = (34 * Hh + 32) >> 6, cc2 = (34 * Vv + 32) >> 6;
					v = d_clip255((a + b * (px - 3) + cc2 * (py - 3) + 16) >> 5);
				}
				R[256 + c * 64 + t] = v;
			}
		}
		WSYNC();
		if (do_chroma)
			for (int c = 0; c < 2; ++c) {
				int v = R[256 + c * 64 + t];
				if (v >= 0) C[c][1 + (t >> 3)][1 + (t & 7)] = (uint8_t)v;
			}
		WSYNC();

		/* ---- luma */
		const int qp = m.qpy;
		if (!do_luma) {
			/* chroma wave: no luma */
		} else if (m.kind == M2R_MB_I4x4) {
			/* residual first (independent of the prediction): lane t < 16 dequantises and inverse
			 * transforms block t in registers */
			if (t < 16) {
				int c[16];
#pragma unroll
				for (int i = 0; i < 16; ++i) c[i] = 0;
				if ((m.nz >> t) & 1) {
					const int16_t *src = q + d_luma_off(m, t);
#pragma unroll
					for (int i = 0; i < 16; ++i) c[i] = src[i] * d_scale4(qp, i & 3, i >> 2);
				}
#pragma unroll
				for (int r = 0; r < 4; ++r) d_idct4_1d(c[4 * r], c[4 * r + 1], c[4 * r + 2], c[4 * r + 3]);
#pragma unroll
				for (int k = 0; k < 4; ++k) {
					d_idct4_1d(c[k], c[4 + k], c[8 + k], c[12 + k]);
					c[k] = (c[k] + 32) >> 6;
					c[4 + k] = (c[4 + k] + 32) >> 6;
					c[8 + k] = (c[8 + k] + 32) >> 6;
					c[12 + k] = (c[12 + k] + 32) >> 6;
				}
#pragma unroll
				for (int i = 0; i < 16; ++i) R[t * 16 + i] = c[i];
			}
			/* the block chain in anti-diagonal steps: block (bx, by) needs its left, top, top-left and
			 * top-right blocks, all on earlier steps of s = bx + 2 by, so the 16 blocks take 10 steps of
			 * at most two blocks (lanes 0-15 / 16-31, one sample each).  Per step: one prediction word
			 * (LDS offsets of three taps, weights, shift; fetched for all steps up front), the taps, the
			 * DC sums, one residual read, one write. */
			const uint64_t modes = (uint64_t)m.ipred[0] | ((uint64_t)m.ipred[1] << 32);
			uint64_t avs = 0;
#pragma unroll
			for (int blk = 0; blk < 16; ++blk) avs |= (uint64_t)avail4(blk, m.avail_luma) << (4 * blk);
			const int slot = t >> 4, px = t & 15;
			/* lane's prediction word of step s (0 for an idle lane) */
			auto word = [&](int s) -> uint32_t {
				const int by = max(0, (s - 2) >> 1) + slot, bx = s - 2 * by;
				const int blk = (by >> 1) * 8 + (bx >> 1) * 4 + (by & 1) * 2 + (bx & 1);
				const int mode = (int)((modes >> (4 * (blk & 15))) & 15);
				const int av = (int)((avs >> (4 * (blk & 15))) & 15);
				return (t < 32 && by <= min(3, s >> 1)) ? tabs->p4o[(av & 4) ? 0 : 1][mode][px] : 0u;
			};
			uint32_t wn = word(0);
			WSYNC();
			uint8_t *const L0 = &L[0][0];
#pragma unroll
			for (int s = 0; s < 10; ++s) {
				const uint32_t w = wn;
				if (s < 9) wn = word(s + 1); /* a step ahead: off the step's LDS round trip */
				const int by = max(0, (s - 2) >> 1) + slot, bx = s - 2 * by;
				if (t < 32 && by <= min(3, s >> 1)) {
					const int blk = (by >> 1) * 8 + (bx >> 1) * 4 + (by & 1) * 2 + (bx & 1);
					const int mode = (int)((modes >> (4 * blk)) & 15);
					const int av = (int)((avs >> (4 * blk)) & 15);
					const uint8_t *nb = L0 + (by * 4) * LW + bx * 4; /* the block's top-left neighbour */
					uint8_t *d = L0 + (by * 4 + 1 + (px >> 2)) * LW + bx * 4 + 1 + (px & 3);
					const int n0 = nb[w & 255], n1 = nb[(w >> 8) & 255], n2 = nb[(w >> 16) & 255];
					const int st = nb[1] + nb[2] + nb[3] + nb[4];
					const int sl = nb[LW] + nb[2 * LW] + nb[3 * LW] + nb[4 * LW];
					const int old = *d, res = R[blk * 16 + px];
					const int sh = (int)(w >> 30);
					const int pv = ((int)((w >> 24) & 3) * n0 + (int)((w >> 26) & 3) * n1 + (int)((w >> 28) & 3) * n2 + ((1 << sh) >> 1)) >> sh;
					/* DC: (avail & 3) picks the sum (pred4x4_dc family) */
					const int dv = ((av & 3) == 3) ? (st + sl + 4) >> 3 : ((av & 1) ? (sl + 2) >> 2 : ((av & 2) ? (st + 2) >> 2 : 128));
					const int req = d_req4(mode);
					/* a mode whose neighbours are missing leaves the sample as it was (the reference) */
					const int base = (mode == 2) ? dv : (((av & req) == req) ? pv : old);
					*d = (uint8_t)d_clip255(base + res);
				}
				WSYNC();
			}
		} else if (m.kind == M2R_MB_I8x8) {
			/* residual of all four 8x8 blocks first; per block: reference filtering, predict + add */
			/* per block: nonzero count and DC level (the SWAR DC-only quirk), in LDS: a register
			 * array indexed by the block loop would live in scratch */
			for (int b = 0; b < 4; ++b) {
				const int lv = ((m.nz >> (4 * b)) & 1) ? q[d_luma_off(m, 4 * b) + t] : 0;
				R[b * 64 + t] = lv * d_scale8(qp, t & 7, t >> 3);
				const int cnt = __popcll(__ballot(lv != 0));
				if (t == 0) {
					DC[b] = lv; /* lane 0 = coefficient 0 */
					DC[4 + b] = cnt;
				}
			}
			WSYNC();
			if (t < 32) {
				int v[8];
				int *p = &R[(t >> 3) * 64 + (t & 7) * 8];
				for (int k = 0; k < 8; ++k) v[k] = p[k];
				d_idct8_1d(v);
				for (int k = 0; k < 8; ++k) p[k] = v[k];
			}
			WSYNC();
			if (t < 32) {
				int v[8];
				int *p = &R[(t >> 3) * 64 + (t & 7)];
				for (int k = 0; k < 8; ++k) v[k] = p[k * 8];
				d_idct8_1d(v);
				for (int k = 0; k < 8; ++k) p[k * 8] = (v[k] + 32) >> 6;
			}
			WSYNC();
			for (int b = 0; b < 4; ++b) {
				const int ox = (b & 1) * 8, oy = (b >> 1) * 8;
				const int av = avail8(b, m.avail_luma);
				/* reference sample filtering (spec 8.3.2.2.1) */
				if (t < 25) {
					int hasL = av & 1, hasT = av & 2, hasTR = av & 4, hasTL = av & 8;
					int tl = L[oy][ox];
#define TP(i) ((i) < 8 ? (int)L[oy][1 + ox + (i)] : (hasTR ? (int)L[oy][1 + ox + (i)] : (int)L[oy][1 + ox + 7]))
#define LP(i) ((int)L[oy + 1 + (i)][ox])
					if (t < 16) {
						if (hasT) {
							int v;
							if (t == 0) v = hasTL ? (tl + 2 * TP(0) + TP(1) + 2) >> 2 : (3 * TP(0) + TP(1) + 2) >> 2;
							else if (t == 15) v = (TP(14) + 3 * TP(15) + 2) >> 2;
							else v = (TP(t - 1) + 2 * TP(t) + TP(t + 1) + 2) >> 2;
							F[t] = v;
						}
					} else if (t < 24) {
						int i = t - 16;
						if (hasL) {
							int v;
							if (i == 0) v = hasTL ? (tl + 2 * LP(0) + LP(1) + 2) >> 2 : (3 * LP(0) + LP(1) + 2) >> 2;
							else if (i == 7) v = (LP(6) + 3 * LP(7) + 2) >> 2;
							else v = (LP(i - 1) + 2 * LP(i) + LP(i + 1) + 2) >> 2;
							F[t] = v;
						}
					} else if (hasTL) {
						int v;
						if (hasT && hasL) v = (TP(0) + 2 * tl + LP(0) + 2) >> 2;
						else if (hasT) v = (3 * tl + TP(0) + 2) >> 2;
						else if (hasL) v = (3 * tl + LP(0) + 2) >> 2;
						else v = tl;
						F[24] = v;
					}
#undef TP
#undef LP
				}
				WSYNC();
				{
					const int mode = (m.ipred[0] >> (4 * b)) & 15;
					int v;
					if (mode == 2) {
						v = pred8_px(2, av, t & 7, t >> 3, F, F + 16, F[24]);
					} else {
						/* table-driven (intra_tables.h) over the filtered neighbours F */
						const uint32_t w = tabs->p8[mode][t];
						int nv[3];
#pragma unroll
						for (int k = 0; k < 3; ++k) nv[k] = F[(w >> (5 * k)) & 31];
						v = ((av & d_req8(mode)) == d_req8(mode)) ? ipred_taps(w, 5, nv) : -1;
					}
					uint8_t *d = &L[oy + 1 + (t >> 3)][1 + ox + (t & 7)];
					const int base = (v >= 0) ? v : *d;
					const int dcl = DC[b];
					if (DC[4 + b] == 1 && dcl != 0) *d = (uint8_t)d_swar(base, dcl * d_scale8(qp, 0, 0), t & 7, 8);
					else *d = (uint8_t)d_clip255(base + R[b * 64 + t]);
				}
				WSYNC();
			}
		} else {
			/* Intra16x16 (h264.cpp:4407-4555) */
			const int av = m.avail_luma, mode = m.pred_mode;
			if (t == 0 && mode == 3) {
				int Hh = 0, Vv = 0;
				for (int i = 0; i < 8; ++i) {
					Hh += (i + 1) * (L[0][1 + 8 + i] - L[0][1 + 6 - i]);
					Vv += (i + 1) * (L[1 + 8 + i][0] - L[1 + 6 - i][0]);
				}
				HV[0] = 16 * (L[16][0] + L[0][16]);
				HV[1] = (5 * Hh + 32) >> 6;
				HV[2] = (5 * Vv + 32) >> 6;
			}
			if (t == 1 && mode == 2) {
				int st = 0, sl = 0;
				for (int i = 0; i < 16; ++i) { st += L[0][1 + i]; sl += L[1 + i][0]; }
				HV[3] = ((av & 3) == 3) ? (st + sl + 16) >> 5 : ((av & 1) ? (sl + 8) >> 4 : ((av & 2) ? (st + 8) >> 4 : 128));
			}
			/* DC levels */
			if (t < 16) DC[t] = (m.nz & M2R_NZ_LUMA_DC) ? q[t] * d_scale4(qp, 0, 0) : 0;
			WSYNC();
			for (int k = t; k < 256; k += 64) {
				int px = k & 15, py = k >> 4, v = -1;
				if (mode == 0) { if (av & 2) v = L[0][1 + px]; }
				else if (mode == 1) { if (av & 1) v = L[1 + py][0]; }
				else if (mode == 2) v = HV[3];
				else v = d_clip255((HV[0] + HV[1] * (px - 7) + HV[2] * (py - 7) + 16) >> 5);
				R[k] = v;
			}
			WSYNC();
			for (int k = t; k < 256; k += 64) {
				int v = R[k];
				if (v >= 0) L[1 + (k >> 4)][1 + (k & 15)] = (uint8_t)v;
			}
			/* DC Hadamard: rows then columns, (x + 2) >> 2 */
			if (t < 4) {
				int *r = &DC[t * 4];
				int a0 = r[0] + r[1], a1 = r[0] - r[1], a2 = r[2] + r[3], a3 = r[2] - r[3];
				r[0] = a0 + a2; r[1] = a0 - a2; r[2] = a1 - a3; r[3] = a1 + a3;
			}
			WSYNC();
			if (t < 4) {
				int *r = &DC[t];
				int a0 = r[0] + r[4], a1 = r[0] - r[4], a2 = r[8] + r[12], a3 = r[8] - r[12];
				r[0] = (a0 + a2 + 2) >> 2; r[4] = (a0 - a2 + 2) >> 2; r[8] = (a1 - a3 + 2) >> 2; r[12] = (a1 + a3 + 2) >> 2;
			}
			WSYNC();
			if (m.cbp & 15) {
				/* AC blocks with coefficients: full transform with the DC inserted; others DC-only SWAR */
				for (int k = t; k < 256; k += 64) {
					int blk = k >> 4, pos = k & 15;
					int bx = d_blk_x(blk), by = d_blk_y(blk);
					int v = 0;
					if (pos == 0) v = DC[by * 4 + bx];
					else if (m.nz & (1u << blk)) v = q[d_luma_off(m, blk) + pos] * d_scale4(qp, pos & 3, pos >> 2);
					R[k] = v;
				}
				WSYNC();
				{
					int blk = t >> 2, row = t & 3;
					int *p = &R[blk * 16 + row * 4];
					int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
					d_idct4_1d(a0, a1, a2, a3);
					p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
				}
				WSYNC();
				{
					int blk = t >> 2, col = t & 3;
					int *p = &R[blk * 16 + col];
					int a0 = p[0], a1 = p[4], a2 = p[8], a3 = p[12];
					d_idct4_1d(a0, a1, a2, a3);
					p[0] = (a0 + 32) >> 6; p[4] = (a1 + 32) >> 6; p[8] = (a2 + 32) >> 6; p[12] = (a3 + 32) >> 6;
				}
				WSYNC();
				for (int k = t; k < 256; k += 64) {
					int blk = k >> 4, pos = k & 15;
					int bx = d_blk_x(blk), by = d_blk_y(blk);
					uint8_t *d = &L[1 + by * 4 + (pos >> 2)][1 + bx * 4 + (pos & 3)];
					if (m.nz & (1u << blk)) *d = (uint8_t)d_clip255(*d + R[k]);
					else *d = (uint8_t)d_swar(*d, DC[by * 4 + bx], pos & 3, 4);
				}
			} else if (m.nz & M2R_NZ_LUMA_DC) {
				for (int k = t; k < 256; k += 64) {
					int px = k & 15, py = k >> 4;
					uint8_t *d = &L[1 + py][1 + px];
					*d = (uint8_t)d_swar(*d, DC[(py >> 2) * 4 + (px >> 2)], px & 3, 4);
				}
			}
			WSYNC();
		}

		/* ---- chroma residual (residual_chroma, h264.cpp:2374-2461) */
		if (do_chroma && (m.cbp >> 4)) {
			int ccbp = m.cbp >> 4;
			for (int k = t; k < 128; k += 64) {
				int c = k >> 6, cx = k & 7, cy = (k >> 3) & 7;
				int cblk = (cy >> 2) * 2 + (cx >> 2), pos = (cy & 3) * 4 + (cx & 3);
				int v = 0;
				if (pos == 0) v = d_chroma_dc(m, q, c, cblk);
				else if (ccbp == 2 && (m.nz & M2R_NZ_CAC(c, cblk)))
					v = q[d_chroma_off(m, 19 + 4 * c + cblk) + pos] * d_scale4(c ? m.qpc[1] : m.qpc[0], cx & 3, cy & 3);
				R[256 + c * 64 + cy * 8 + cx] = v;
			}
			WSYNC();
			if (t < 32) {
				int comp = t >> 4, b = (t >> 2) & 3, row = t & 3;
				int *p = &R[256 + comp * 64 + ((b >> 1) * 4 + row) * 8 + (b & 1) * 4];
				int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
				d_idct4_1d(a0, a1, a2, a3);
				p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
			}
			WSYNC();
			if (t < 32) {
				int comp = t >> 4, b = (t >> 2) & 3, col = t & 3;
				int *p = &R[256 + comp * 64 + ((b >> 1) * 4) * 8 + (b & 1) * 4 + col];
				int a0 = p[0], a1 = p[8], a2 = p[16], a3 = p[24];
				d_idct4_1d(a0, a1, a2, a3);
				p[0] = (a0 + 32) >> 6; p[8] = (a1 + 32) >> 6; p[16] = (a2 + 32) >> 6; p[24] = (a3 + 32) >> 6;
			}
			WSYNC();
			for (int k = t; k < 128; k += 64) {
				int c = k >> 6, cx = k & 7, cy = (k >> 3) & 7;
				uint8_t *d = &C[c][1 + cy][1 + cx];
				*d = (uint8_t)d_clip255(*d + R[256 + c * 64 + cy * 8 + cx]);
			}
			WSYNC();
		}
	}
}

#ifdef M2DEC_INTRA_ROW_INLINE
#define M2DEC_INTRA_ROW_ATTR __attribute__((always_inline))
#else
#define M2DEC_INTRA_ROW_ATTR __attribute__((noinline))
#endif
__device__ M2DEC_INTRA_ROW_ATTR void intra_row(const int y, const int t, const int part, lds_u8 *lds, const int wave,
                          const m2r_mb_t *__restrict__ mbs, const int16_t *__restrict__ pool, uint8_t *cur, int W, int H, int Wmb,
                          uint8_t *hbi, const uint32_t tag, int *err)
{
	IntraLDS *const ctx = lds_ptr<IntraLDS>(lds) + wave; /* row blocks: 4 contexts, then the tables */
	const IntraTables *const tabs = (const IntraTables *)(lds_ptr<IntraLDS>(lds) + 4);
	const bool do_luma = part == 0, do_chroma = part != 0;
	uint8_t(&L)[17][LW] = ctx->L;
	uint8_t(&C)[2][9][9] = ctx->C;
	int(&R)[256 + 128] = ctx->R;
	int(&DC)[16] = ctx->DC;
	int(&F)[32] = ctx->F;
	int(&HV)[4] = ctx->HV;
	int16_t(&Q)[2][M2R_MB_COEF_MAX] = ctx->Q;
	uint8_t *chroma = cur + (size_t)W * H;
	int prev_x = -2;
	int qb = 0;
	const int y0 = y * 16;

	for (int xb = 0; xb < Wmb; xb += 64) {
		/* this chunk's records, one per lane; intra MBs of this row in [xb, xb + 64) and of the row above in [xb - 1, xb + 65) */
		const int xi = xb + t;
		MbWords mine;
#pragma unroll
		for (int i = 0; i < 8; ++i) mine.w[i] = 0;
		if (xi < Wmb) mine.m = mbs[y * Wmb + xi];
		unsigned long long cur_mask = __ballot(xi < Wmb && mine.m.kind != M2R_MB_INTER);
		unsigned long long up_mask = 0, up_lo = 0, up_hi = 0;
		if (y > 0) {
			up_mask = __ballot(xi < Wmb && mbs[(y - 1) * Wmb + xi].kind != M2R_MB_INTER);
			up_lo = (xb > 0) ? (mbs[(y - 1) * Wmb + xb - 1].kind != M2R_MB_INTER) : 0;
			up_hi = (xb + 64 < Wmb) ? (mbs[(y - 1) * Wmb + xb + 64].kind != M2R_MB_INTER) : 0;
		}
		auto up_intra = [&](int xx) -> bool {
			if (y == 0 || xx < 0 || xx >= Wmb) return false;
			int k = xx - xb;
			if (k < 0) return up_lo != 0;
			if (k >= 64) return up_hi != 0;
			return (up_mask >> k) & 1;
		};
		/* the row above's hand-off word this lane reads for intra MB xx (record mm), and whether it reads one:
		 * luma wave lanes 0-2 MB xx words 0-2, lanes 3-4 MB xx+1 words 0-1, lane 5 MB xx-1 word 2; chroma wave
		 * lanes 0-2 MB xx words 3-5, lane 3 MB xx-1 word 5.  Only the neighbours the MB's predictor may read:
		 * its avail bits (top 2, top-right 4, top-left 8) are slice-aware (get_availability,
		 * h264.cpp:9704-9715), so the first MB row of a slice waits for nothing of the slice above and each
		 * slice of an I picture runs its own intra wavefront (C5's 8 slices: 8 chains of Wmb + 2 (rows of the
		 * slice) steps instead of one of Wmb + 2 Hmb) */
		auto handoff_src = [&](int xx, const m2r_mb_t &mm, bool &mw) -> const uint8_t * {
			const int nw = do_luma ? 6 : 4;
			const int xs = (t < 3) ? xx : ((do_luma && t < 5) ? xx + 1 : xx - 1);
			const int wi = (t < 3) ? t : ((do_luma && t < 5) ? t - 3 : 2);
			const int av = do_luma ? mm.avail_luma : mm.avail_chroma;
			const int need = (t < 3) ? 2 : ((do_luma && t < 5) ? 4 : 8);
			mw = y > 0 && t < nw && xs >= 0 && xs < Wmb && (av & need) && up_intra(xs);
			return hbi + ((size_t)(y - 1) * Wmb + (mw ? xs : 0)) * HBI_BYTES + (do_luma ? 0 : 24) + wi * 8;
		};
		unsigned long long pv = 0; /* the hand-off word prefetched for intra MB pv_x */
		int pv_x = -1;
		if (cur_mask) {
			/* the chunk's first intra MB: stage its coefficients now (later ones are prefetched) */
			const m2r_mb_t m0 = lane_mb(mine, __builtin_ctzll(cur_mask));
			const int nq = d_mb_ncoef(m0);
			for (int k = t; k < nq; k += 64) Q[qb][k] = pool[m0.coef + k];
			WSYNC();
		}
		while (cur_mask) {
		const int lx = __builtin_ctzll(cur_mask);
		const int x = xb + lx;
		cur_mask &= cur_mask - 1;
		const m2r_mb_t m = lane_mb(mine, lx);
		const int16_t *q = Q[qb];
		/* prefetch the next intra MB's coefficients into registers; they land in Q[qb ^ 1] at the end */
		int16_t qv[7];
		int nqn = 0;
		/* ... and its upper neighbours' hand-off words (pv, for MB pv_x): issued before this MB's body, so that
		 * their round trip is hidden behind it when the row above is ahead (self-validating: a word without this
		 * picture's tag yet is polled again) */
		unsigned long long pv_next = 0;
		int pv_next_x = -1;
		if (cur_mask) {
			const m2r_mb_t mn = lane_mb(mine, __builtin_ctzll(cur_mask));
			nqn = d_mb_ncoef(mn);
#pragma unroll
			for (int i = 0; i < 7; ++i) qv[i] = (t + 64 * i < nqn) ? pool[mn.coef + t + 64 * i] : (int16_t)0;
			const int xn = xb + __builtin_ctzll(cur_mask);
			bool mw;
			const uint8_t *ps = handoff_src(xn, mn, mw);
			if (mw) pv_next = ld_sc1(ps);
			pv_next_x = xn;
		}
		const int x0 = x * 16;
		const int left_in_lds = (prev_x == x - 1);
		/* ---- gather the neighbourhood */
		if (left_in_lds) {
			if (do_luma && t < 17) L[t][0] = L[t][16];
			if (do_chroma && t < 18) { int c = t / 9, r = t % 9; C[c][r][0] = C[c][r][8]; }
		}
		WSYNC();
		if (y > 0) {
			/* the row above's hand-off words (self-validating: a word is this picture's once its tag is):
			 * luma wave lanes 0-2 MB x words 0-2, lanes 3-4 MB x+1 words 0-1, lane 5 MB x-1 word 2;
			 * chroma wave lanes 0-2 MB x words 3-5, lane 3 MB x-1 word 5 */
			const int wi = (t < 3) ? t : ((do_luma && t < 5) ? t - 3 : 2);
			bool mine_w;
			const uint8_t *src = handoff_src(x, m, mine_w);
			unsigned long long v = pv_x == x ? pv : 0; /* (prefetched during the previous MB) */
			unsigned spins = 0;
			for (bool first = pv_x == x;; first = false) {
				bool ok = true;
				if (mine_w) {
					if (!first) v = ld_sc1(src);
					ok = (uint32_t)(v >> 48) == tag;
				}
				if (__all(ok)) break;
				if (!first && !spin_ok(spins, err, 2)) break;
			}
			if (mine_w) {
#pragma unroll
				for (int b = 0; b < 6; ++b) {
					const uint8_t s8 = (uint8_t)(v >> (8 * b));
					const int j = wi * 6 + b; /* byte within the 16-byte bottom row */
					if (j < 16) {
						if (do_luma) {
							if (t < 3) L[0][1 + j] = s8;
							else if (t < 5) { if (j < 8) L[0][17 + j] = s8; }
							else if (j == 15) L[0][0] = s8;
						} else {
							if (t < 3) C[j & 1][0][1 + (j >> 1)] = s8;
							else if (j >= 14) C[j & 1][0][0] = s8;
						}
					}
				}
			}
		}
		if (x > 0 && !left_in_lds) {
			if (do_luma && t < 16) L[1 + t][0] = cur[(size_t)(y0 + t) * W + x0 - 1];
			if (do_chroma && t >= 16 && t < 32) { int k = t - 16; C[k & 1][1 + (k >> 1)][0] = chroma[(size_t)(y0 / 2 + (k >> 1)) * W + x0 - 2 + (k & 1)]; }
		}
		WSYNC();
		STAMPX(x, 0);

#ifdef M2DEC_DBG_INTRA
		const bool dbg_dump = x == 0 && y == 0 && do_luma && __builtin_amdgcn_readfirstlane(g_dbg[14]) != 12345;
		if (dbg_dump) {
			if (t < 8) g_dbg[t] = ((const int *)&m)[t];
			for (int k = t; k < M2R_MB_COEF_MAX; k += 64) g_dbg[16 + k] = q[k];
			for (int k = t; k < 17 * LW; k += 64) g_dbg[512 + k] = (&L[0][0])[k];
			if (t == 0) g_dbg[15] = qb;
		}
		WSYNC();
#endif
		intra_mb_body(m, q, t, do_luma, do_chroma, ctx, tabs);
#ifdef M2DEC_DBG_INTRA
		WSYNC();
		if (dbg_dump) {
			for (int k = t; k < 17 * LW; k += 64) g_dbg[1024 + k] = (&L[0][0])[k];
			for (int k = t; k < 384; k += 64) g_dbg[1536 + k] = R[k];
			if (t < 16) g_dbg[1936 + t] = DC[t];
			if (t < 4) g_dbg[1952 + t] = HV[t];
			if (t == 0) g_dbg[14] = 12345;
		}
		WSYNC();
#endif
		STAMPX(x, 3);
#ifdef M2DEC_DBG_ROWS
		if (x == 0 && t == 0) {
			const unsigned b = blockIdx.x & 255, wv = (unsigned)__builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6;
			g_dbg_rows[(b * 4 + wv) * 2] = (unsigned)y | ((unsigned)part << 8) | ((unsigned)wave << 12) | (0xabu << 24);
			g_dbg_rows[(b * 4 + wv) * 2 + 1] = (unsigned)(y0 & 0xffff) | ((unsigned)m.kind << 16) | ((m.coef & 0xff) << 24);
		}
#endif
		/* ---- write back and hand off the bottom rows */
		if (do_luma)
			for (int k = t; k < 256; k += 64) cur[(size_t)(y0 + (k >> 4)) * W + x0 + (k & 15)] = L[1 + (k >> 4)][1 + (k & 15)];
		else
			for (int k = t; k < 128; k += 64) {
				int cy = k >> 4, bx = k & 15;
				chroma[(size_t)(y0 / 2 + cy) * W + x0 + bx] = C[bx & 1][1 + cy][1 + (bx >> 1)];
			}
		if (t < 3) {
			/* hand-off words: 6 bottom-row bytes + the picture's 16-bit tag (no progress word, no drain) */
			unsigned long long v = (unsigned long long)tag << 48;
#pragma unroll
			for (int b = 0; b < 6; ++b) {
				const int j = t * 6 + b;
				if (j < 16) v |= (unsigned long long)(do_luma ? L[16][1 + j] : C[j & 1][8][1 + (j >> 1)]) << (8 * b);
			}
			st_sc1(hbi + ((size_t)y * Wmb + x) * HBI_BYTES + (do_luma ? 0 : 24) + t * 8, v);
		}
		STAMPX(x, 4);
		STAMP(y, 3, 16 + x, x);
		STAMPX(x, 5);
		/* the prefetched coefficients of the next intra MB */
		if (nqn) {
#pragma unroll
			for (int i = 0; i < 7; ++i)
				if (t + 64 * i < nqn) Q[qb ^ 1][t + 64 * i] = qv[i];
		}
		qb ^= 1;
		prev_x = x;
		pv = pv_next;
		pv_x = pv_next_x;
		WSYNC();
		}
	}
}

/* ======================================================================== inter workers */

/* MB (x, y)'s neighbour record is read by an intra MB: (x + 1, y) left, (x - 1 .. x + 1, y + 1) top */
__device__ __forceinline__ bool nb_needed(const m2r_mb_t *__restrict__ mbs, int x, int y, int Wmb, int Hmb)
{
	bool r = x + 1 < Wmb && mbs[y * Wmb + x + 1].kind != M2R_MB_INTER;
	if (y + 1 < Hmb)
		for (int d = -1; d <= 1; ++d)
			if (x + d >= 0 && x + d < Wmb && mbs[(y + 1) * Wmb + x + d].kind != M2R_MB_INTER) r = true;
	return r;
}

/* the neighbour record of MB (x, y) from the item's LDS segment (luma rows 0..15, interleaved chroma rows
 * 16..23, the MB at column (x & 7) * 16): lanes 0..7, one 8-byte write-through store each */
__device__ __forceinline__ void write_nb_record(uint8_t *hbp, int rs, int x, int y, const uint8_t *seg, int t)
{
	if (t < 8) {
		const uint8_t *mb = seg + (x & 7) * 16;
		unsigned long long v = 0;
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			int b;
			if (t < 2) b = mb[15 * SEG_ROW + 8 * t + i];                                   /* luma bottom row */
			else if (t < 4) b = mb[23 * SEG_ROW + 8 * (t - 2) + i];                        /* chroma bottom row */
			else if (t < 6) b = mb[(8 * (t - 4) + i) * SEG_ROW + 15];                      /* luma right column */
			else b = mb[(16 + 4 * (t - 6) + (i >> 1)) * SEG_ROW + 14 + (i & 1)];           /* chroma right column */
			v |= (unsigned long long)b << (8 * i);
		}
		st_sc1(hbp + ((size_t)y * rs + x) * HBP_BYTES + t * 8, v);
	}
}

/*
 * One intra / PCM MB of a P / B picture, inside an inter worker (all 256 lanes call): the unfiltered
 * neighbours come from the neighbour records of the MBs around it (sc1 loads; their work items are
 * done), the MB is reconstructed by intra_mb_body (wave 0 luma, wave 1 chroma) into the item's segment.
 */
/* LDS layout of an inter worker: one intra context, the prediction tables, the item's segment, and the
 * residual buffers of the four inter MBs in flight (one per wave) */
__device__ __forceinline__ IntraLDS *worker_ictx(lds_u8 *lds) { return lds_ptr<IntraLDS>(lds); }
__device__ __forceinline__ IntraTables *worker_tabs(lds_u8 *lds) { return (IntraTables *)(worker_ictx(lds) + 1); }
/* the item's reconstructed samples before they go out: 24 rows (16 luma, 8 interleaved chroma) of 8 MBs */
__device__ __forceinline__ uint8_t *worker_seg(lds_u8 *lds) { return (uint8_t *)(worker_tabs(lds) + 1); }
__device__ __forceinline__ InterRes *worker_res(lds_u8 *lds, int wave) { return (InterRes *)(worker_seg(lds) + 24 * SEG_ROW) + wave; }

__device__ __attribute__((noinline)) void intra_mb_wg(const int x, const int y, const m2r_mb_t m, const int16_t *__restrict__ pool, uint8_t *cur,
                            int W, int H, int Wmb, const uint8_t *hbp, int rs, lds_u8 *lds)
{
	IntraLDS *const ctx = worker_ictx(lds);
	const IntraTables *const tabs = worker_tabs(lds);
	uint8_t *const seg = worker_seg(lds);
	const int t = threadIdx.x;
	const int nq = d_mb_ncoef(m);
	for (int k = t; k < nq; k += blockDim.x) ctx->Q[0][k] = pool[m.coef + k];
	if (t < 11) {
		/* granule: 0,1 (x, y-1) luma bottom; 2 (x+1, y-1) luma bottom 0..7; 3 (x-1, y-1) luma bottom 8..15;
		 * 4,5 (x-1, y) luma right; 6,7 (x, y-1) chroma bottom; 8 (x-1, y-1) chroma bottom 8..15;
		 * 9,10 (x-1, y) chroma right */
		const int nx = (t == 2) ? x + 1 : ((t == 3 || t == 4 || t == 5 || t >= 8) ? x - 1 : x);
		const int ny = (t == 4 || t == 5 || t >= 9) ? y : y - 1;
		const int off = (t == 0 || t == 2) ? 0 : (t == 1 || t == 3) ? 8 : (t == 4) ? 32 : (t == 5) ? 40
		              : (t == 6) ? 16 : (t == 7 || t == 8) ? 24 : (t == 9) ? 48 : 56;
		if (nx >= 0 && nx < Wmb && ny >= 0) {
			const unsigned long long v = ld_sc1(hbp + ((size_t)ny * rs + nx) * HBP_BYTES + off);
#pragma unroll
			for (int i = 0; i < 8; ++i) {
				const uint8_t b = (uint8_t)(v >> (8 * i));
				if (t == 0) ctx->L[0][1 + i] = b;
				else if (t == 1) ctx->L[0][9 + i] = b;
				else if (t == 2) ctx->L[0][17 + i] = b;
				else if (t == 3) { if (i == 7) ctx->L[0][0] = b; }
				else if (t == 4) ctx->L[1 + i][0] = b;
				else if (t == 5) ctx->L[9 + i][0] = b;
				else if (t == 6) ctx->C[i & 1][0][1 + (i >> 1)] = b;
				else if (t == 7) ctx->C[i & 1][0][5 + (i >> 1)] = b;
				else if (t == 8) { if (i >= 6) ctx->C[i & 1][0][0] = b; }
				else if (t == 9) ctx->C[i & 1][1 + (i >> 1)][0] = b;
				else ctx->C[i & 1][5 + (i >> 1)][0] = b;
			}
		}
	}
	__syncthreads();
	const int w = t >> 6;
	if (w < 2) intra_mb_body(m, ctx->Q[0], t & 63, w == 0, w == 1, ctx, tabs);
	__syncthreads();
	{
		seg[(t >> 4) * SEG_ROW + (x & 7) * 16 + (t & 15)] = ctx->L[1 + (t >> 4)][1 + (t & 15)];
	}
	if (t < 128) {
		const int cy = t >> 4, bx = t & 15;
		seg[(16 + cy) * SEG_ROW + (x & 7) * 16 + bx] = ctx->C[bx & 1][1 + cy][1 + (bx >> 1)];
	}
}

/*
 * Inter MBs (and the intra MBs of P / B pictures) as a bounded persistent grid.  Work items are (MB
 * row, 8-MB segment) in raster order, dequeued from a per-launch counter.  Before its MBs, an item
 * waits until
 *   - every reference picture it reads has its final samples in all the MB rows and columns its
 *     motion vectors reach (rowflag[picture][row] = ROWFLAG(seq, columns final), raised by the
 *     deblocking storer as it writes; the columns are rounded up to whole 128-byte lines, so no
 *     partially final line is ever cached), and
 *   - if it holds intra MBs, the items holding their left / upper neighbours are done (their
 *     neighbour records are written; these items are earlier in the queue: no deadlock);
 * all polled with sc1 loads, then ONE agent acquire.  A picture's MC follows its references'
 * deblocking wavefront column by column, so consecutive anchor pictures overlap.  A finished item
 * raises its done flag, which the picture's deblocking loader streams on.  The grid is kept small (a
 * fraction of the CUs) so that spinning items can never keep the work they wait for off the device.
 */
/* (M2DEC_INTER_WORKER_NOINLINE: an out-of-line inter worker — r71: its MB loop spills more, 101 scratch
 * operations per MB and wave instead of 63, so it stays inlined) */
#ifdef M2DEC_INTER_WORKER_NOINLINE
#define M2DEC_INTER_WORKER_ATTR __attribute__((noinline))
#else
#define M2DEC_INTER_WORKER_ATTR
#endif
__device__ M2DEC_INTER_WORKER_ATTR void inter_worker(const PictureArgs &a, const SlotSeq &ss, uint8_t *smem)
{
	__shared__ int s_item, s_rmin, s_rmax, s_cmax, s_intra, s_rec;
	/* the item's MB records and the motion records of its inter MBs, staged once per item */
	__shared__ uint32_t s_mbw[8][sizeof(m2r_mb_t) / 4];
	__shared__ uint32_t s_itw[8][sizeof(m2r_inter_t) / 4];
	__shared__ unsigned int s_refs[2];
	const int t = threadIdx.x;
	const int W = a.W, H = a.H, Wmb = a.Wmb, Hmb = a.Hmb;
	const int nseg = NSEG(Wmb), nitems = Hmb * nseg, rs = nseg * 8;
	int *queue = a.scratch + SCR_QUEUE(Hmb), *inter_cnt = a.scratch + SCR_INTER(Hmb), *segdone = a.scratch + SCR_SEG(Hmb);
	const m2r_mb_t *__restrict__ mbs = a.mbs;
	uint8_t *cur = a.frames + (size_t)a.slot * a.fsz;
	/* intra MBs of this picture: an LDS context and the prediction tables */
	IntraTables *tabs = worker_tabs(LDS_ARG());
	const bool recs = a.n_intra != 0;
	if (recs) {
		for (int i = t; i < 2 * 9 * 16; i += blockDim.x) (&tabs->p4o[0][0][0])[i] = (&c_ipred4o[0][0][0])[i];
		for (int i = t; i < 9 * 64; i += blockDim.x) tabs->p8[i >> 6][i & 63] = c_ipred8[i >> 6][i & 63];
	}
	/* Single-lane work in this loop is done by the whole of wave 0 under a SCALAR branch, the one
	 * lane picked by value (atomic operand 0 on lanes 1..63).  An `if (t == 0)` here lets the
	 * compiler thread lanes 1..63 of wave 0 straight back to the next barrier while lane 0 is still
	 * dequeueing, which deadlocks the workgroup (seen on gfx950 with ROCm 7.2). */
	const bool wave0 = __builtin_amdgcn_readfirstlane(t) < 64;
	int nst_dbg = 0, nmb_dbg = 0;
	for (;;) {
		if (wave0) {
			const int v = __hip_atomic_fetch_add((gi32 *)queue, t == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			s_item = __builtin_amdgcn_readfirstlane(v);
			s_rmin = 1 << 30;
			s_rmax = -1;
			s_cmax = 0;
			s_intra = 0;
			s_rec = 0;
			s_refs[0] = s_refs[1] = 0;
		}
		__syncthreads();
		const int item = __builtin_amdgcn_readfirstlane(s_item);
		if (item >= nitems) break;
#ifndef M2DEC_NO_ITEM_LAUNDER
		/* (as in inter_mb: per-lane values re-derived per item instead of held across the item loop) */
		int t = threadIdx.x;
		asm volatile("" : "+v"(t));
#endif
		const int y = item / nseg, seg = item % nseg, x0 = seg * 8, x1 = min(x0 + 8, Wmb);
		STAMPI(96 + (blockIdx.x & 63), 0, nst_dbg & 255, item);
		/* ---- the item's records into LDS: MB records, then the motion records they point at */
		if (t < 8 * (int)(sizeof(m2r_mb_t) / 4)) {
			const int mb = t / (sizeof(m2r_mb_t) / 4), wd = t % (sizeof(m2r_mb_t) / 4);
			if (x0 + mb < x1) s_mbw[mb][wd] = ((const uint32_t *)&mbs[y * Wmb + x0 + mb])[wd];
		}
		__syncthreads();
		for (int k = t; k < 8 * (int)(sizeof(m2r_inter_t) / 4); k += blockDim.x) {
			const int mb = k / (sizeof(m2r_inter_t) / 4), wd = k % (sizeof(m2r_inter_t) / 4);
			const m2r_mb_t &mm = *(const m2r_mb_t *)s_mbw[mb];
			if (x0 + mb < x1 && mm.kind == M2R_MB_INTER) s_itw[mb][wd] = ((const uint32_t *)&a.inters[mm.inter])[wd];
		}
		__syncthreads();
		/* ---- vertical and rightward reach of this segment's motion into the references (8 lanes per MB;
		 * luma 6-tap window; the chroma window never reaches further), and its intra MBs */
		if (t < 64) {
			const int mbi = x0 + (t >> 3);
			int rmin = 1 << 30, rmax = -1, cmax = 0;
			unsigned int r0 = 0, r1 = 0;
			if (mbi < x1) {
				const m2r_mb_t &m = *(const m2r_mb_t *)s_mbw[mbi - x0];
				if (m.kind == M2R_MB_INTER) {
					const m2r_inter_t &it = *(const m2r_inter_t *)s_itw[mbi - x0];
					for (int k = (t & 7) * 4; k < (t & 7) * 4 + 4; ++k) {
						const int l = k >> 4, blk = k & 15;
						const int sl = it.slot[l][(blk >> 3) * 2 + ((blk & 3) >> 1)];
						if (sl < 0) continue;
						const int py = y * 16 + (blk >> 2) * 4 + (it.mv[l][blk][1] >> 2);
						const int top = py - 2, bot = py + 3 + 3;
						rmin = min(rmin, top < 0 ? 0 : min(top >> 4, Hmb - 1));
						rmax = max(rmax, bot < 0 ? 0 : min(bot >> 4, Hmb - 1));
						const int right = mbi * 16 + (blk & 3) * 4 + (it.mv[l][blk][0] >> 2) + 3 + 3;
						cmax = max(cmax, right < 0 ? 0 : min(right >> 4, Wmb - 1));
						if (sl < 32) r0 |= 1u << sl;
						else r1 |= 1u << (sl - 32);
					}
				} else if ((t & 7) == 0) {
					/* bit 0: an intra MB; 1: one at x0 (left / top-left in the previous items); 2: one at
					 * x1 - 1 (top-right in the next item of the row above) */
					atomicOr(&s_intra, 1 | (mbi == x0 ? 2 : 0) | (mbi == x1 - 1 ? 4 : 0));
				}
				/* this MB's neighbour record is read by an intra MB (lane 1 of the MB) */
				if (recs && (t & 7) == 1 && nb_needed(mbs, mbi, y, Wmb, Hmb)) atomicOr(&s_rec, 1 << (mbi - x0));
			}
			if (rmax >= 0) {
				atomicMin(&s_rmin, rmin);
				atomicMax(&s_rmax, rmax);
				atomicMax(&s_cmax, cmax);
				atomicOr(&s_refs[0], r0);
				atomicOr(&s_refs[1], r1);
			}
		}
		__syncthreads();
		const int rmin_u = __builtin_amdgcn_readfirstlane(s_rmin), rmax_u = __builtin_amdgcn_readfirstlane(s_rmax);
		const int intra_bits = __builtin_amdgcn_readfirstlane(s_intra);
		const bool has_intra = intra_bits != 0;
		const int rec_bits = __builtin_amdgcn_readfirstlane(s_rec);
		if (rmax_u >= 0 && wave0) {
			unsigned spins = 0;
#ifndef M2DEC_NO_REFWAIT
			if (rmax_u >= 0) {
				/* rows rmin .. rmax final up to the reach: their own stores and the next row's (rows 13..15)
				 * done.  Columns are whole 128-byte lines (8 MBs) when the stride allows, else whole rows:
				 * a line cached while partly unfinal could outlive the acquire below */
				const int rlast = min(rmax_u + 1, Hmb - 1);
				const int cmax_u = __builtin_amdgcn_readfirstlane(s_cmax);
				const int need = (W & 127) ? Wmb : min(Wmb, (cmax_u + 8) & ~7);
				for (int k = 0; k < 2; ++k) {
					unsigned int bits = __builtin_amdgcn_readfirstlane(s_refs[k]);
					while (bits) {
						const int sl = k * 32 + __builtin_ctz(bits);
						bits &= bits - 1;
						const int want = ss.s[sl];
						if (want <= 0) continue;
						/* entry (seq % ROWFLAG_N) only ever grows: a later picture's value also means "final" */
						const unsigned long long *fl = a.rowflag + (size_t)((want - 1) & (ROWFLAG_N - 1)) * Hmb;
						const unsigned long long wv = ROWFLAG(want - 1, need);
						for (int r0 = rmin_u; r0 <= rlast; r0 += 64) {
							const int r = r0 + t;
							for (;;) {
								const bool ok = (r > rlast) ||
								                __hip_atomic_load((gu64 *)&fl[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= wv;
								if (__all(ok)) break;
								if (!spin_ok(spins, a.err, 32)) break;
							}
						}
					}
				}
			}
#endif
			/* ALWAYS acquire, even when every flag was already set: this XCD's L2 may hold lines of
			 * rows 13..15 that the row's own deblock workgroup loaded before the row below filtered
			 * and rewrote them from another XCD */
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		}
		__syncthreads();
		STAMPI(96 + (blockIdx.x & 63), 1, nst_dbg & 255, item);
		/* inter MBs first (they never read this picture), then the intra MBs once the items holding their
		 * left / top-left / top / top-right neighbours are done (neighbour records, sc1 loads: no acquire) */
		for (int pass = 0; pass < (has_intra ? 2 : 1); ++pass) {
			if (pass == 1 && wave0) {
				unsigned spins = 0;
				int dep = -1;
				const bool want = (t == 1) || (t == 0 && (intra_bits & 2)) || (t == 2 && (intra_bits & 4));
				if (t < 3 && want && y > 0 && seg - 1 + t >= 0 && seg - 1 + t < nseg) dep = (y - 1) * nseg + seg - 1 + t;
				if (t == 3 && (intra_bits & 2) && seg > 0) dep = y * nseg + seg - 1;
				for (;;) {
					const bool ok = dep < 0 || __hip_atomic_load((gi32 *)&segdone[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
					if (__all(ok)) break;
					if (!spin_ok(spins, a.err, 64)) break;
				}
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keeps the record loads below the poll */
			}
			if (pass == 1) __syncthreads();
			if (pass == 0) {
				/* the inter MBs, one per wave: wave w takes x0 + w, x0 + w + 4 (no workgroup barrier per MB) */
				const int w = __builtin_amdgcn_readfirstlane(t) >> 6;
				for (int x = x0 + w; x < x1; x += 4) {
					const m2r_mb_t m = *(const m2r_mb_t *)s_mbw[x - x0];
					if (__builtin_amdgcn_readfirstlane(m.kind) != M2R_MB_INTER) continue;
					inter_mb(y * Wmb + x, m, *(const m2r_inter_t *)s_itw[x - x0], a.slices, a.pool, a.frames, a.fsz, W, H, Wmb,
					         worker_seg(LDS_ARG()), worker_res(LDS_ARG(), w), t & 63, nmb_dbg++);
					if ((rec_bits >> (x - x0)) & 1) {
						ISYNC();
						write_nb_record(a.hbp, rs, x, y, worker_seg(LDS_ARG()), t & 63);
					}
				}
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* the records are out before the barrier */
				__syncthreads();
				STAMPI(96 + (blockIdx.x & 63), 3, nst_dbg & 255, item);
				continue;
			}
			for (int x = x0; x < x1; ++x) {
				const m2r_mb_t m = mbs[y * Wmb + x];
				if (__builtin_amdgcn_readfirstlane(m.kind) == M2R_MB_INTER) continue;
				intra_mb_wg(x, y, m, a.pool, cur, W, H, Wmb, a.hbp, rs, LDS_ARG());
				if ((rec_bits >> (x - x0)) & 1) {
					__syncthreads();
					write_nb_record(a.hbp, rs, x, y, worker_seg(LDS_ARG()), t);
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				}
				__syncthreads();
			}
		}
		/* the item's samples out of LDS as whole 128-byte row pieces (8 MBs x 16 bytes, 16 bytes per lane; the
		 * byte stores of the MBs left one partially dirty line per MB row in whichever L2 they went to) */
		{
			const uint8_t *sg = worker_seg(LDS_ARG());
			const int nmb = x1 - x0;
			for (int k = t; k < 24 * 8; k += blockDim.x) {
				const int r = k >> 3, c = k & 7;
				if (c < nmb) {
					uint8_t *dst = r < 16 ? cur + (size_t)(y * 16 + r) * W + (x0 + c) * 16
					                      : cur + (size_t)W * H + (size_t)(y * 8 + r - 16) * W + (x0 + c) * 16;
					*(uint4 *)dst = *(const uint4 *)(sg + r * SEG_ROW + c * 16);
				}
			}
		}
		/* segment done: every wave drained, then ONE agent release, the row's counter and the item's flag */
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		if (wave0) {
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			__hip_atomic_fetch_add((gi32 *)&inter_cnt[y], t == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			__hip_atomic_fetch_or((gi32 *)&segdone[item], t == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		STAMPI(96 + (blockIdx.x & 63), 2, nst_dbg & 255, item);
		nst_dbg++;
	}
}

/* ======================================================================== k_deblock */

/*
 * In-loop deblocking (deblock_pb, h264.cpp:10540-10663) of TWO MB rows, A = yA and B = yA + 1, by
 * the four waves of the rows' workgroup:
 *   wave 0 (loader)   : copies MB after MB into a ring of DBK_RING MB slots in LDS: both rows' own
 *                       16 luma / 8 chroma rows from the frame (final inter + intra samples) and, below
 *                       row 0, the hand-off record of the row above A (its bottom 4 luma / 2 chroma
 *                       rows after that row's filtering; sc1 loads, G16 R1) once that row published it;
 *   wave 1 (filter A) / wave 3 (filter B): MB after MB in raster order, lanes 0..15 luma lines,
 *                       16..31 chroma lines; vertical edges with one line per lane, then horizontal
 *                       edges with one column per lane.  Row B's MB x waits (LDS word) until row A
 *                       finished MB x + 1: its top halo is row A's bottom lines in the same ring, so
 *                       the A -> B hand-off never leaves LDS, and the two filters run side by side;
 *   wave 2 (storer)   : writes every sample that became final to the frame, the hand-off records of
 *                       row B for the next workgroup (write-through sc1), drains, publishes progress,
 *                       frees the ring slots.
 * Ring lines: luma 0..3 halo (row above A, rows 12..15), 4..19 row A, 20..35 row B; chroma 0..1 halo,
 * 2..9 row A, 10..17 row B.  Ring columns wrap modulo DBK_RW.  Frame writes: rows 0..12 (chroma 0..6)
 * of an MB once its own row filtered it and its right neighbour, rows 13..15 (7) once the row below
 * filtered it.
 */
__device__ __forceinline__ int dbk_done012(int c, int Wmb) { return c >= Wmb ? Wmb : max(c - 1, 0); }

/* ---- boundary strengths, derived here from the MB and motion records (the host parser leaves
 * m2r_deblock_t.bs_v / bs_h at 0; bS is ~17 % of its cycles otherwise): store_strength_intra*
 * (h264.cpp:3086-3106, 4749-4755) for intra MBs; else per 4-sample segment 2 when either 4x4 block has
 * coefficients, else str_mv_calc* (h264.cpp:7119-7270) on the blocks' reference pictures (record slots,
 * one per picture) and vectors.  Same derivation as oracle/recon_oracle.c orc_bs. */
__device__ __forceinline__ int bs_nz(const m2r_mb_t &m, int bx, int by)
{
	const int r = by * 4 + bx;
	const int blk = ((r >> 3) << 3) | (((r >> 1) & 1) << 2) | ((r & 4) >> 1) | (r & 1); /* raster -> blkIdx */
	return (m.flags & M2R_FLAG_T8x8) ? (int)((m.nz >> (4 * (blk >> 2))) & 1) : (int)((m.nz >> blk) & 1);
}

__device__ __forceinline__ int bs_far(uint32_t a, uint32_t b)
{
	const int dx = (int)(int16_t)(a & 0xffff) - (int)(int16_t)(b & 0xffff);
	const int dy = (int)(int16_t)(a >> 16) - (int)(int16_t)(b >> 16);
	return (abs(dx) >= 4) | (abs(dy) >= 4);
}

__device__ int bs_motion(const m2r_inter_t *q, int qx, int qy, const m2r_inter_t *p, int px, int py)
{
	const int bq = (qy >> 1) * 2 + (qx >> 1), bp = (py >> 1) * 2 + (px >> 1);
	const int q0 = q->slot[0][bq], q1 = q->slot[1][bq], p0 = p->slot[0][bp], p1 = p->slot[1][bp];
	const uint32_t *qmv = (const uint32_t *)q->mv, *pmv = (const uint32_t *)p->mv;
	const uint32_t qm0 = qmv[qy * 4 + qx], qm1 = qmv[16 + qy * 4 + qx], pm0 = pmv[py * 4 + px], pm1 = pmv[16 + py * 4 + px];
	if ((p0 != q0 || p1 != q1) && (p1 != q0 || p0 != q1)) return 1;
	if (q0 >= 0 && q1 >= 0) {
		if (q0 == q1) return (bs_far(qm0, pm0) | bs_far(qm1, pm1)) & (bs_far(qm0, pm1) | bs_far(qm1, pm0));
		return q0 == p0 ? (bs_far(qm0, pm0) | bs_far(qm1, pm1)) : (bs_far(qm0, pm1) | bs_far(qm1, pm0));
	}
	if (q0 >= 0) return q0 == p0 ? bs_far(qm0, pm0) : bs_far(qm0, pm1);
	return q1 == p0 ? bs_far(qm1, pm0) : bs_far(qm1, pm1);
}

/* bS of MB (x, y), direction dir (0: vertical edges, 1: horizontal): byte e = edge, 2 bits per segment */
__device__ uint32_t bs_of(const m2r_mb_t *__restrict__ mbs, const m2r_inter_t *__restrict__ inters, int x, int y, int Wmb, int dir)
{
	const m2r_mb_t q = mbs[y * Wmb + x];
	if (q.kind != M2R_MB_INTER) return (q.kind == M2R_MB_PCM || q.kind == M2R_MB_I8x8) ? 0x00ff00ffu : 0xffffffffu;
	const m2r_inter_t *qi = &inters[q.inter];
	uint32_t str = 0;
	if (dir ? y > 0 : x > 0) {
		const m2r_mb_t p = mbs[dir ? (y - 1) * Wmb + x : y * Wmb + x - 1];
		if (p.kind != M2R_MB_INTER) {
			str = 0xaa; /* bS 2 on every segment; the BS4 flag makes it 4 */
		} else {
			const m2r_inter_t *pi = &inters[p.inter];
			for (int g = 0; g < 4; ++g) {
				const int qx = dir ? g : 0, qy = dir ? 0 : g, px = dir ? g : 3, py = dir ? 3 : g;
				const int v = (bs_nz(q, qx, qy) | bs_nz(p, px, py)) ? 2 : bs_motion(qi, qx, qy, pi, px, py);
				str |= (uint32_t)v << (2 * g);
			}
		}
	}
	for (int e = 1; e < 4; ++e) {
		if ((q.flags & M2R_FLAG_T8x8) && (e & 1)) continue;
		for (int g = 0; g < 4; ++g) {
			const int qx = dir ? g : e, qy = dir ? e : g, px = dir ? qx : qx - 1, py = dir ? qy - 1 : qy;
			const int v = (bs_nz(q, qx, qy) | bs_nz(q, px, py)) ? 2 : bs_motion(qi, qx, qy, qi, px, py);
			str |= (uint32_t)v << (8 * e + 2 * g);
		}
	}
	return str;
}

#ifdef M2DEC_DBK_NOINLINE
__attribute__((noinline))
#endif
__device__ void deblock_pair(const int yA, const bool hasB, uint8_t *smem, const m2r_deblock_t *__restrict__ dbk, uint8_t *cur,
                             int W, int H, int Wmb, int Hmb, uint8_t *hbd, int *progress, int *err,
                             unsigned long long *rowflag, int seq, const int *segdone,
                             const m2r_mb_t *__restrict__ mbs, const m2r_inter_t *__restrict__ inters)
{
	const int wave = threadIdx.x >> 6, t = threadIdx.x & 63;
	const int nthr = blockDim.x;
	constexpr int S = DBK_RW;                /* ring line: DBK_RING MB columns, wrapping */
	constexpr int M = DBK_RW - 1;
	uint8_t *RL = smem;                      /* 36 luma lines */
	uint8_t *RC = smem + 36 * S;             /* 18 chroma lines */
	m2r_deblock_t *rT = (m2r_deblock_t *)(smem + 54 * S); /* [Wmb] records of the row above A (A's own if yA == 0) */
	m2r_deblock_t *rA = rT + Wmb;            /* [Wmb] row A */
	m2r_deblock_t *rB = rA + Wmb;            /* [Wmb] row B */
	int *flags = (int *)(rB + Wmb);          /* [0] MBs loaded, [1] row A MBs filtered, [2] MBs stored, [3] row B MBs filtered */
	uint8_t *dummy = (uint8_t *)(flags + 4);  /* [64] per-lane sink for the filter's masked-off samples */
	uint8_t *chroma = cur + (size_t)W * H;
	const int yB = yA + 1;
	const bool lastA = !hasB;                /* row A is the picture's last row */
	const bool lastB = hasB && yB == Hmb - 1;

	__shared__ uint8_t s_alpha[52], s_beta[52], s_tc0[52][3];
	/* ---- prologue: the deblocking records and the tables into LDS */
	for (int i = threadIdx.x; i < 52; i += nthr) {
		s_alpha[i] = c_alpha[i];
		s_beta[i] = c_beta[i];
		s_tc0[i][0] = c_tc0[i][0];
		s_tc0[i][1] = c_tc0[i][1];
		s_tc0[i][2] = c_tc0[i][2];
	}
	for (int k = threadIdx.x; k < Wmb; k += nthr) {
		rA[k] = dbk[yA * Wmb + k];
		rT[k] = dbk[(yA > 0 ? yA - 1 : yA) * Wmb + k]; /* (a struct-valued ?: would go through scratch) */
		if (hasB) rB[k] = dbk[yB * Wmb + k];
	}
	if (threadIdx.x < 4) flags[threadIdx.x] = 0;
	__syncthreads();
	/* the rows' boundary strengths from the records: one (row, MB, direction) per lane */
	for (int k = threadIdx.x; k < (hasB ? 4 : 2) * Wmb; k += nthr) {
		const int r = k / (2 * Wmb), rem = k - r * 2 * Wmb, x = rem >> 1, dir = rem & 1;
		const uint32_t v = bs_of(mbs, inters, x, yA + r, Wmb, dir);
		m2r_deblock_t *rec = (r ? rB : rA) + x;
		if (dir) rec->bs_h = v;
		else rec->bs_v = v;
	}
	__syncthreads();

	/* the deblocking chain is the picture's critical path: let its waves win the SIMD arbitration
	 * over co-resident inter workers (filters highest) */
#ifndef M2DEC_DBK_PRIO_FILTER
#define M2DEC_DBK_PRIO_FILTER 3
#endif
#ifndef M2DEC_DBK_PRIO_OTHER
#define M2DEC_DBK_PRIO_OTHER 2
#endif
#ifndef M2DEC_DBK_PRIO_STORER
#define M2DEC_DBK_PRIO_STORER M2DEC_DBK_PRIO_OTHER
#endif
	/* s_setprio is a scalar instruction: the role must be a scalar (readfirstlane) value so that each
	 * s_setprio sits behind a scalar branch, not in an exec-masked block every wave executes */
	const int swave = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
	if (swave == 1 || swave == 3) __builtin_amdgcn_s_setprio(M2DEC_DBK_PRIO_FILTER);
	else if (swave == 2) __builtin_amdgcn_s_setprio(M2DEC_DBK_PRIO_STORER);
	else __builtin_amdgcn_s_setprio(M2DEC_DBK_PRIO_OTHER);
	if (wave == 0) {
		/* ---------------- loader: own samples run ahead as far as the ring allows (prep); only the
		 * hand-off record of the row above A waits for that row (got) */
		const int per = hasB ? 48 : 24; /* granules per MB: 16 luma + 8 chroma rows per row */
		int prep = 0, got = 0, nld = 0, ready = segdone ? 0 : Wmb;
		unsigned spins = 0;
		while (got < Wmb) {
			const int ring = min(Wmb, __hip_atomic_load(&flags[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) + DBK_RING);
			if (prep < ring && ready < ring) {
				/* P / B pictures: the MB columns of both rows whose work items are done (a prefix), then
				 * one agent acquire before their samples are read */
				const int nseg = NSEG(Wmb);
				int nr = Wmb;
				for (int r = 0; r < (hasB ? 2 : 1); ++r)
					for (int s0 = ready >> 3; s0 < nseg; s0 += 64) {
						const int sg = s0 + t;
						const bool done = sg >= nseg || __hip_atomic_load((gi32 *)&segdone[(yA + r) * nseg + sg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
						const unsigned long long nd = __ballot(!done);
						if (nd) {
							nr = min(nr, (s0 + __builtin_ctzll(nd)) * 8);
							break;
						}
					}
				if (nr > ready) {
					ready = nr;
					__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				}
			}
			const int target = min(ring, ready);
			if (prep < target) {
				const int ng = (target - prep) * per;
				for (int g0 = 0; g0 < ng; g0 += 64) {
					const int g = g0 + t;
					if (g < ng) {
						const int mb = prep + g / per, k = g % per;
						const int r = k >= 24, kk = k - 24 * r; /* row A / B, granule within the row */
						const int col = (mb & (DBK_RING - 1)) * 16;
						const int y0 = (yA + r) * 16, yc0 = (yA + r) * 8;
						if (kk < 16) *(uint4 *)(RL + (4 + 16 * r + kk) * S + col) = *(const uint4 *)(cur + (size_t)(y0 + kk) * W + mb * 16);
						else *(uint4 *)(RC + (2 + 8 * r + kk - 16) * S + col) = *(const uint4 *)(chroma + (size_t)(yc0 + kk - 16) * W + mb * 16);
					}
				}
				prep = target;
				if (yA == 0) {
					got = prep;
					if (t == 0) __hip_atomic_store(&flags[0], got, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
				}
				continue;
			}
			if (yA == 0) {
				if (!spin_ok(spins, err, 4)) return;
				continue;
			}
			const int lim = min(prep, __hip_atomic_load((gi32 *)&progress[yA - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
			if (lim <= got) {
				if (!spin_ok(spins, err, 4)) {
					/* give up (the launch is flagged bad): release the filter wave */
					if (t == 0) __hip_atomic_store(&flags[0], Wmb, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
					return;
				}
				continue;
			}
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			/* 12 hand-off granules per MB: 8 luma (rows 12..15 x 2 halves), 4 chroma (rows 6..7) */
			const int ng = (lim - got) * 12;
			for (int g0 = 0; g0 < ng; g0 += 64) {
				const int g = g0 + t;
				if (g < ng) {
					const int mb = got + g / 12, h = g % 12;
					const int col = (mb & (DBK_RING - 1)) * 16;
					const unsigned long long v = ld_sc1(hbd + ((size_t)(yA - 1) * Wmb + mb) * HBD_BYTES + h * 8);
					uint8_t *d = (h < 8) ? RL + (h >> 1) * S + col + (h & 1) * 8 : RC + ((h - 8) >> 1) * S + col + (h & 1) * 8;
					*(uint2 *)d = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
				}
			}
			got = lim;
			if (t == 0) __hip_atomic_store(&flags[0], got, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
			STAMP(yA, 0, nld, got);
			nld++;
		}
		return;
	}

	if (wave == 1 || wave == 3) {
		/* ---------------- filter (one row per wave): lanes 0..15 luma lines, 16..31 chroma lines (Cb
		 * 16..23, Cr 24..31), branch-free per edge.  A chroma line keeps its samples 0..3 / 4..7 at
		 * v[2..5] / v[10..13] so that its two edges sit where luma edges 0 and 2 do. */
		const bool rowB = wave == 3;
		if (rowB && !hasB) return;
		const m2r_deblock_t *rq = rowB ? rB : rA, *rt = rowB ? rA : rT;
		const int lumaL0 = rowB ? 20 : 4, chromaL0 = rowB ? 10 : 2; /* first own line of this row */
		int *done = &flags[rowB ? 3 : 1];
		const bool active = t < 32;
		const bool luma = t < 16;
		const int comp = (t >> 3) & 1;        /* chroma lanes */
		const int cl = t & 7;                 /* chroma line (row for dir 0, column for dir 1) */
		const int seg_l = (t & 15) >> 2, seg_c = cl >> 1;
		const int seg = luma ? seg_l : seg_c;
		uint8_t *const sink = dummy + t;
		/* bit offset of v[i] in its dword for the vertical edges, by i & 3: luma byte i & 3; chroma (Cb / Cr
		 * interleaved) byte 2 (i & 1) + comp */
		const int vsh[4] = {luma ? 0 : 8 * comp, luma ? 8 : 16 + 8 * comp, luma ? 16 : 8 * comp, luma ? 24 : 16 + 8 * comp};
		unsigned spins = 0;
		/* the last values seen of the loader's and row A's words: a word is polled again only when the value
		 * seen does not cover this MB (the acquire that returned it still orders the reads below) */
		int seen0 = 0, seen1 = 0;
		for (int x = 0; x < Wmb; ++x) {
			if (seen0 <= x)
				while ((seen0 = __hip_atomic_load(&flags[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) <= x) {
					if (!spin_ok(spins, err, 16)) break;
				}
			if (rowB && seen1 < min(x + 2, Wmb)) /* row A's MB x is final for us once A filtered MB x + 1 */
				while ((seen1 = __hip_atomic_load(&flags[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < min(x + 2, Wmb)) {
					if (!spin_ok(spins, err, 16)) break;
				}
			STAMP(yA + rowB, 1, x, x);
			STAMPD(yA + rowB, 0, x);
			const m2r_deblock_t q = rq[x];
			if (!(q.flags & M2R_DBK_OFF)) {
				const m2r_deblock_t pl = x > 0 ? rq[x - 1] : q, pt = rt[x];
				const int base = (x & (DBK_RING - 1)) * 16; /* ring column of the MB's first sample */
#pragma unroll
				for (int dir = 0; dir < 2; ++dir) {
					const uint32_t str = dir ? q.bs_h : q.bs_v;
					const int edge_flag = dir ? M2R_DBK_TOP : M2R_DBK_LEFT;
					const int bs4 = (q.flags & (dir ? M2R_DBK_TOP_BS4 : M2R_DBK_LEFT_BS4)) != 0;
					const bool e0 = (q.flags & edge_flag) && (str & 255);
					const int nqpy = dir ? pt.qpy : pl.qpy, nqc0 = dir ? pt.qpc[0] : pl.qpc[0], nqc1 = dir ? pt.qpc[1] : pl.qpc[1];
					const int qc = comp ? q.qpc[1] : q.qpc[0];
					const int nqc = comp ? nqc1 : nqc0;
					const int qp_edge0 = e0 ? (luma ? (q.qpy + nqpy + 1) >> 1 : (qc + nqc + 1) >> 1) : 0;
					const int qp_inner = luma ? q.qpy : qc;
					/* sample addressing: V: own line, columns from 4 left of the MB, wrapping in the ring;
					 * H: column t / byte column 2 cl + comp, lines from 4 (2) above the row */
					uint8_t *lb;
					int c0, cst;
					if (dir == 0) {
						lb = luma ? RL + (lumaL0 + t) * S : RC + (chromaL0 + cl) * S;
						c0 = base - 4 + (luma ? 0 : comp);
						cst = luma ? 1 : 2;
					} else {
						lb = luma ? RL + (lumaL0 - 4) * S + base + t : RC + (chromaL0 - 2) * S + base + 2 * cl + comp;
						c0 = 0;
						cst = S;
					}
#define DBK_ADDR(j) (dir == 0 ? lb + ((c0 + (j) * cst) & M) : lb + (j) * cst)
					/* branch-free sample access: a masked-off sample goes to the lane's dummy byte (an
					 * exec-masked load/store per sample would cost a branch each) */
					int v[20];
#ifndef M2DEC_DBK_BYTE_V
					if (dir == 0) {
						/* vertical edges: the line's 20 bytes from 4 left of the MB are 5 aligned dwords of the
						 * ring line (a chroma line's samples are every other byte of the first 4: v[2..5] /
						 * v[10..13] sit in the same dwords as the luma lanes' bytes 2..5 / 10..13) */
						uint32_t dw[5];
#pragma unroll
						for (int k = 0; k < 5; ++k) dw[k] = *(const uint32_t *)(lb + ((base - 4 + 4 * k) & M));
#pragma unroll
						for (int i = 0; i < 20; ++i) v[i] = (int)__builtin_amdgcn_ubfe(dw[i >> 2], (uint32_t)vsh[i & 3], 8);
					} else
#endif
#ifndef M2DEC_DBK_BYTE_H
					if (dir == 1) {
						/* horizontal edges: one byte per line at a fixed stride, so every load is an immediate
						 * offset from one of two per-lane bases (a chroma lane's v[2..5] / v[10..13] are its
						 * samples 0..3 / 4..7; its other v[] read in-bounds bytes it never uses) */
						const uint8_t *const blo = luma ? lb : lb - 2 * S, *const bhi = luma ? lb : lb - 6 * S;
#pragma unroll
						for (int i = 0; i < 20; ++i) v[i] = (i < 6 ? blo : bhi)[i * S];
					} else
#endif
#pragma unroll
					for (int i = 0; i < 20; ++i) {
						const int ci = (i < 6) ? i - 2 : i - 6; /* chroma sample index for v[i] */
						const bool cv = (i >= 2 && i <= 5) || (i >= 10 && i <= 13);
						const bool ok = active && (luma || cv);
						v[i] = *(ok ? DBK_ADDR(luma ? i : ci) : sink);
					}
#pragma unroll
					for (int e = 0; e < 4; ++e) {
						int bs = active ? (int)((str >> (8 * e + 2 * seg)) & 3) : 0;
						if (e == 0) bs = e0 ? (bs4 ? 4 : bs) : 0;
						if (!luma && (e & 1)) bs = 0;
						if (!__any(bs)) continue;
						const int qp = e ? qp_inner : qp_edge0;
						const int ia = min(max(qp + q.alpha_off, 0), 51), ib = min(max(qp + q.beta_off, 0), 51);
						const int A = s_alpha[ia], B = s_beta[ib];
						const int tc0l = s_tc0[ia][max(min(bs, 3) - 1, 0)]; /* unconditional load, then select */
						const int tc0 = bs ? tc0l : 0;
						const int at = 4 + 4 * e;
						const int p0 = v[at - 1], p1 = v[at - 2], p2 = v[at - 3], p3 = v[at - 4];
						const int q0 = v[at], q1 = v[at + 1], q2 = v[at + 2], q3 = v[at + 3];
						/* bitwise, not short-circuit: && here becomes exec-mask branches */
						const bool filt = (bs != 0) & (abs(p0 - q0) < A) & (abs(p1 - p0) < B) & (abs(q1 - q0) < B);
						const bool ap = abs(p2 - p0) < B, aq = abs(q2 - q0) < B;
						/* every candidate computed, then selected */
						/* bS < 4 */
						const int tc = tc0 + (luma ? (int)ap + (int)aq : 1);
						const int delta = d_clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
						const int avg = (p0 + q0 + 1) >> 1;
						const int w0 = d_clip255(p0 + delta), w1 = d_clip255(q0 - delta);
						const int wp1 = p1 + d_clip3(-tc0, tc0, (p2 + avg - (p1 << 1)) >> 1);
						const int wq1 = q1 + d_clip3(-tc0, tc0, (q2 + avg - (q1 << 1)) >> 1);
						/* bS == 4 */
						const bool small = abs(p0 - q0) < ((A >> 2) + 2);
						const bool sp = luma & ap & small, sq = luma & aq & small;
						const int a0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, b0 = (2 * p1 + p0 + q1 + 2) >> 2;
						const int a1 = (p2 + p1 + p0 + q0 + 2) >> 2, a2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
						const int c0_ = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, e0_ = (2 * q1 + q0 + p1 + 2) >> 2;
						const int c1 = (p0 + q0 + q1 + q2 + 2) >> 2, c2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
						/* bS 4 only on the MB edge (e == 0, unrolled): the inner edges skip the strong filter */
						const bool strong = (e == 0) && bs == 4;
						const int np0 = d_sel(strong, d_sel(sp, a0, b0), w0), nq0 = d_sel(strong, d_sel(sq, c0_, e0_), w1);
						const int np1 = d_sel(strong, d_sel(sp, a1, p1), d_sel(luma & ap, wp1, p1));
						const int nq1 = d_sel(strong, d_sel(sq, c1, q1), d_sel(luma & aq, wq1, q1));
						const int np2 = d_sel(strong & sp, a2, p2), nq2 = d_sel(strong & sq, c2, q2);
						v[at - 1] = d_sel(filt, np0, p0);
						v[at - 2] = d_sel(filt, np1, p1);
						v[at - 3] = d_sel(filt, np2, p2);
						v[at] = d_sel(filt, nq0, q0);
						v[at + 1] = d_sel(filt, nq1, q1);
						v[at + 2] = d_sel(filt, nq2, q2);
					}
					/* write back; at x == 0 the 4 columns left of the MB wrap onto a slot the loader may
					 * be filling, and edge 0 is off there anyway */
					const int i0 = (dir == 0 && x == 0) ? 4 : 1;
#ifndef M2DEC_DBK_BYTE_V
					if (dir == 0) {
						/* luma lines back as dwords (bytes 0 and 19 are p3 / q3, never changed); chroma lanes
						 * share dwords between Cb and Cr, so their 8 samples stay byte stores */
						if (luma) {
#pragma unroll
							for (int k = (x == 0 ? 1 : 0); k < 5; ++k)
								*(uint32_t *)(lb + ((base - 4 + 4 * k) & M)) =
								    (uint32_t)v[4 * k] | ((uint32_t)v[4 * k + 1] << 8) | ((uint32_t)v[4 * k + 2] << 16) | ((uint32_t)v[4 * k + 3] << 24);
						} else if (active) {
							/* (ring columns wrap at every 16th MB: c0 is negative there) */
#pragma unroll
							for (int i = 2; i < 14; ++i) {
								if (i > 5 && i < 10) continue;
								const int ci = (i < 6) ? i - 2 : i - 6;
								if (i >= i0) *DBK_ADDR(ci) = (uint8_t)v[i];
							}
						}
					} else
#endif
#ifndef M2DEC_DBK_BYTE_H
					if (dir == 1) {
						if (luma) {
#pragma unroll
							for (int i = 1; i < 19; ++i) lb[i * S] = (uint8_t)v[i];
						} else if (active) {
#pragma unroll
							for (int i = 2; i < 14; ++i) {
								if (i > 5 && i < 10) continue;
								lb[((i < 6) ? i - 2 : i - 6) * S] = (uint8_t)v[i];
							}
						}
					} else
#endif
#pragma unroll
					for (int i = 1; i < 19; ++i) {
						const int ci = (i < 6) ? i - 2 : i - 6;
						const bool cv = (i >= 2 && i <= 5) || (i >= 10 && i <= 13);
						const bool ok = i >= i0 && active && (luma || cv);
						*(ok ? DBK_ADDR(luma ? i : ci) : sink) = (uint8_t)v[i];
					}
#undef DBK_ADDR
					/* the next direction's reads are this wave's later LDS operations: performed in order */
					asm volatile("" ::: "memory");
					__builtin_amdgcn_wave_barrier();
					STAMPD(yA + rowB, 1 + dir, x);
				}
			}
			if (t == 0) __hip_atomic_store(done, x + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
		}
		STAMP(yA + rowB, 1, Wmb, Wmb);
		return;
	}

	/* ---------------- storer (wave 2) */
	{
		int dA = 0, dA13 = 0, dB = 0, dH = 0, nst = 0, pubA = 0, pubB = 0;
		unsigned spins = 0;
		const int y0A = yA * 16, yc0A = yA * 8, y0B = yB * 16, yc0B = yB * 8;
		/* frame stores go out in groups of 4 MBs (one 64-byte piece of each sample row, 16 bytes per lane,
		 * write-through): a final-MB count is rounded down to 4 except at the row end */
		auto g4 = [Wmb](int v) { return v >= Wmb ? Wmb : (v & ~(DBK_SG - 1)); };
		/* n MBs from m0 of `rows` sample rows: frame row fy0 + r <- ring line rl0 + r of plane `ring` */
		auto store_rows = [&](uint8_t *plane, int fy0, const uint8_t *ring, int rl0, int m0, int n, int rows) {
			for (int k = t; k < n * rows; k += 64) {
				const int r = k / n, mb = m0 + k - r * n;
				st128_sc1(plane + (size_t)(fy0 + r) * W + mb * 16, *(const uint4 *)(ring + (rl0 + r) * S + (mb & (DBK_RING - 1)) * 16));
			}
		};
		for (;;) {
			const int cA = __hip_atomic_load(&flags[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
			const int cB = hasB ? __hip_atomic_load(&flags[3], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
			const int tA = g4(dbk_done012(cA, Wmb));
			const int tA13 = g4(cB);             /* row B filtered MB m (so row A had MB m + 1 done) */
			const int tH = hasB ? dbk_done012(cB, Wmb) : 0;
			const int tB = g4(tH);
			if (tA <= dA && tA13 <= dA13 && tB <= dB && (lastB || tH <= dH)) {
				if ((hasB ? dB : dA) >= Wmb) break;
				if (!spin_ok(spins, err, 8)) {
					if (hasB && !lastB) signal_progress(&progress[yB], Wmb); /* release the next workgroup */
					break;
				}
				continue;
			}
			/* the next workgroup waits on row B's hand-off records (MB by MB): write them first, drain, publish */
			if (tH > dH && !lastB) {
				const int n = tH - dH;
				for (int g0 = 0; g0 < n * 12; g0 += 64) {
					const int g = g0 + t;
					if (g < n * 12) {
						const int mb = dH + g / 12, k = g % 12;
						const int col = (mb & (DBK_RING - 1)) * 16;
						const uint8_t *sp = (k < 8) ? RL + (32 + (k >> 1)) * S + col + (k & 1) * 8
						                            : RC + (16 + ((k - 8) >> 1)) * S + col + (k & 1) * 8;
						const uint2 v = *(const uint2 *)sp;
						st_sc1(hbd + ((size_t)yB * Wmb + mb) * HBD_BYTES + k * 8, ((unsigned long long)v.y << 32) | v.x);
					}
				}
				signal_progress(&progress[yB], tH);
				dH = tH;
			}
			/* row A: rows 0..12 (all 16 if A is the last row) and the row above's rows 13..15 */
			if (tA > dA) {
				const int n = tA - dA;
				store_rows(cur, y0A, RL, 4, dA, n, lastA ? 16 : 13);
				store_rows(chroma, yc0A, RC, 2, dA, n, lastA ? 8 : 7);
				if (yA > 0) {
					store_rows(cur, y0A - 3, RL, 1, dA, n, 3);
					store_rows(chroma, yc0A - 1, RC, 1, dA, n, 1);
				}
				dA = tA;
			}
			/* row A's rows 13..15 (chroma 7), final once row B filtered its top edge */
			if (tA13 > dA13) {
				const int n = tA13 - dA13;
				store_rows(cur, y0A + 13, RL, 17, dA13, n, 3);
				store_rows(chroma, yc0A + 7, RC, 9, dA13, n, 1);
				dA13 = tA13;
			}
			/* row B: rows 0..12 (all 16 if B is the last row) */
			if (tB > dB) {
				const int n = tB - dB;
				store_rows(cur, y0B, RL, 20, dB, n, lastB ? 16 : 13);
				store_rows(chroma, yc0B, RC, 10, dB, n, lastB ? 8 : 7);
				dB = tB;
			}
			/* the slots' LDS reads are done (their values fed the stores above): hand them back */
			if (t == 0) __hip_atomic_store(&flags[2], hasB ? dB : dA, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
			/* column progress for the MC of later pictures, whole 8-MB (128-byte) groups at a time: the
			 * frame stores above are write-through (sc1); drain them, then raise the rows' words.
			 * rowflag[yA]: A's rows 0..12 and the row above's rows 13..15 (both up to dA);
			 * rowflag[yB]: B's rows 0..12 (dB) and A's rows 13..15 (dA13) */
			{
				const int cA = dA >= Wmb ? Wmb : (dA & ~7);
				const int mB = min(dB, dA13);
				const int cB = hasB ? (mB >= Wmb ? Wmb : (mB & ~7)) : 0;
				if (cA > pubA || cB > pubB) {
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
					if (t == 0) {
						if (cA > pubA)
							__hip_atomic_store((gu64 *)&rowflag[(size_t)(seq & (ROWFLAG_N - 1)) * Hmb + yA], ROWFLAG(seq, cA), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						if (cB > pubB)
							__hip_atomic_store((gu64 *)&rowflag[(size_t)(seq & (ROWFLAG_N - 1)) * Hmb + yB], ROWFLAG(seq, cB), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					}
					pubA = max(pubA, cA);
					pubB = max(pubB, cB);
				}
			}
			STAMP(yA, 2, nst, hasB ? dB : dA);
			nst++;
		}
		/* every store of these rows is in: both rows complete (a stalled launch that broke out of the
		 * loop above still releases its waiters; the error word reports it) */
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		if (t == 0) {
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			__hip_atomic_store((gu64 *)&rowflag[(size_t)(seq & (ROWFLAG_N - 1)) * Hmb + yA], ROWFLAG(seq, Wmb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			if (hasB) __hip_atomic_store((gu64 *)&rowflag[(size_t)(seq & (ROWFLAG_N - 1)) * Hmb + yB], ROWFLAG(seq, Wmb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
	}
	/* the raised priority covers the deblocking chain only, not the caller's copy-out / next row pair */
	__builtin_amdgcn_s_setprio(0);
}


/* ======================================================================== k_picture */
/*
 * One launch per picture, all three stages overlapped row by row.  Workgroups [0, G) are persistent
 * inter workers (work items = 8-MB segments in raster order); workgroup G + g owns MB rows 2g, 2g+1:
 *   phase A: waits until every inter segment of its rows is stored (per-row counters, agent release /
 *            acquire), publishes the unfiltered bottom rows of their inter MBs (hand-off records read
 *            by the intra MBs of the row below), then reconstructs the intra / PCM MBs, one row per
 *            wave (2-MB-lag wavefront on the row above);
 *   phase B: deblocks both rows on waves 0..2 (loader / filter / storer, see deblock_pair) and
 *            finally flags the rows final for the motion compensation of later pictures.
 * Every wait points at a lower block index of the same launch or at an earlier launch, so FIFO
 * queues and in-order dispatch cannot deadlock; the host reserves every launch's workgroups from a
 * device-wide budget (SlotBudget, runtime.hip) so that all launches in flight fit on the device.
 */
/* batch launches: before writing its slot, wait until the earlier batch pictures that read the
 * slot's previous content have finished their motion compensation, and the previous content's
 * writer has finished all its rows (their counters live at lower block indices: no deadlock) */
__device__ void war_wait(const PictureArgs &a)
{
	if (__builtin_amdgcn_readfirstlane(threadIdx.x) < 64) { /* wave 0, scalar branch */
		const int t = threadIdx.x;
		const int rows_wg = (a.Hmb + 1) / 2 + (a.capture ? 1 : 0); /* capture: + the copy-out */
		unsigned spins = 0;
		for (;;) {
			bool ok = true;
			if (t < a.n_war) ok = __hip_atomic_load((gi32 *)&a.fin[2 * a.war[t]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.inter_workers;
			else if (t == a.n_war && a.war_writer >= 0)
				ok = __hip_atomic_load((gi32 *)&a.fin[2 * a.war_writer + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= rows_wg;
			if (__all(ok)) break;
			if (!spin_ok(spins, a.err, 128)) break;
		}
	}
	__syncthreads();
}

/* one pair of MB rows (yA, yA + 1) by the whole workgroup: the I-picture intra wavefront (phase A),
 * then deblocking (phase B), then the picture's row-pair counter (and the verification copy-out) */
__device__ __attribute__((noinline)) void row_pair(const PictureArgs *__restrict__ ap, const int yA, lds_u8 *lds)
{
	uint8_t *const smem = lds_ptr<uint8_t>(lds);
	const PictureArgs &a = *ap;
	const int t = threadIdx.x;
	const bool wave0 = __builtin_amdgcn_readfirstlane(t) < 64;
	const bool hasB = yA + 1 < a.Hmb;
	const int nrows = hasB ? 2 : 1;
	const int Wmb = a.Wmb;
	uint8_t *cur = a.frames + (size_t)a.slot * a.fsz;
	STAMP(yA, 3, 0, 1);
	if (!a.n_inter) {
		/* ---- I picture, phase A: intra / PCM MBs as a wavefront over the row workgroups: luma of rows A / B
		 * on waves 0 / 1, their chroma on waves 2 / 3, each wave with its own LDS context.  (P / B pictures:
		 * the inter workers reconstruct every MB, intra ones included, and the deblocking below streams
		 * on their per-item done flags.) */
		IntraTables *tabs = (IntraTables *)((IntraLDS *)smem + 4);
		for (int i = t; i < 2 * 9 * 16; i += blockDim.x) (&tabs->p4o[0][0][0])[i] = (&c_ipred4o[0][0][0])[i];
		for (int i = t; i < 9 * 64; i += blockDim.x) tabs->p8[i >> 6][i & 63] = c_ipred8[i >> 6][i & 63];
		__syncthreads();
		const int w = __builtin_amdgcn_readfirstlane(t) >> 6;
		const int r = w & 1, part = w >> 1;
		if (r < nrows) {
			__builtin_amdgcn_s_setprio(3); /* the intra wavefront is an I picture's critical path */
			intra_row(yA + r, t & 63, part, lds, w, a.mbs, a.pool, cur, a.W, a.H, Wmb, a.hbi,
			          (uint32_t)(a.seq % 65535) + 1, a.err);
			/* write the intra samples back out of this XCD's L2 now: rows 13..15 of an MB row are
			 * rewritten (filtered) by the row below's deblocking, possibly from another XCD, and a later
			 * write-back of our dirty unfiltered bytes would land on top of them */
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
			__builtin_amdgcn_s_setprio(0);
		}
	}
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__syncthreads();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
	STAMP(yA, 3, 3, 4);
	/* ---- phase B: deblocking (always: it also publishes the row flags) */
	deblock_pair(yA, hasB, smem, a.dbk, cur, a.W, a.H, Wmb, a.Hmb, a.hbd, a.scratch + SCR_DPROG(a.Hmb), a.err, a.rowflag, a.seq,
	             a.n_inter ? a.scratch + SCR_SEG(a.Hmb) : nullptr, a.mbs, a.inters);
	STAMP(yA, 3, 4, 5);
	if (a.fin) {
		/* the storer drained and released every frame store before its row flags */
		__shared__ int s_last;
		__syncthreads();
		if (wave0) { /* scalar branch, the lane picked by value (this may run inside a loop) */
			const int prev = __builtin_amdgcn_readfirstlane(
			    __hip_atomic_fetch_add((gi32 *)&a.fin[2 * a.pidx + 1], t == 0 ? 1 : 0, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT));
			s_last = a.capture && prev == (a.Hmb + 1) / 2 - 1;
			if (t == 0 && prev == (a.Hmb + 1) / 2 - 1) STAMPP(a.didx, 2);
		}
		__syncthreads();
		if (s_last) {
			/* verification mode: the last row workgroup copies the finished picture out, then
			 * releases the slot to later writers (their war_wait counts this copy) */
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
			const size_t n16 = (size_t)a.W * a.H * 3 / 2 / 16;
			const uint4 *src = (const uint4 *)cur;
			uint4 *dst = (uint4 *)a.capture;
			for (size_t i = t; i < n16; i += blockDim.x) dst[i] = src[i];
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			__syncthreads();
			if (wave0) __hip_atomic_fetch_add((gi32 *)&a.fin[2 * a.pidx + 1], t == 0 ? 1 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
		}
	}
}

/* block b of one picture (the picture's own block index in k_batch) */
__device__ __forceinline__ void picture_block(const PictureArgs &a, const int b, uint8_t *smem)
{
	if (b == 0 && threadIdx.x == 0) STAMPP(a.didx, 0);
	if (a.fin && (a.n_war || a.war_writer >= 0)) war_wait(a);
	if (b < a.inter_workers) {
		if (a.n_inter)
			inter_worker(a, a.ss, smem);
		if (a.fin) {
			/* every reference read of this worker has returned (its values were consumed) */
			__syncthreads();
			if (threadIdx.x == 0 && __hip_atomic_fetch_add((gi32 *)&a.fin[2 * a.pidx], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.inter_workers - 1)
				STAMPP(a.didx, 1);
		}
		return;
	}
	/* I picture: one workgroup per pair of rows (the intra wavefront needs them all resident).
	 * P / B picture: a.row_wgs workgroups take the row pairs in order from a queue (a pair's deblocking
	 * waits only for the pair above, taken earlier: no deadlock); the other row blocks leave at once.
	 * (One call site of row_pair: it is large.) */
	const int r = b - a.inter_workers;
	const bool queued = a.n_inter != 0;
	if (queued && r >= a.row_wgs) return;
	__shared__ int s_pair;
	const bool wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x) < 64;
	int *pq = a.scratch + SCR_QUEUE(a.Hmb) + 1;
	for (int k = 0;; ++k) {
		int pair = r;
		if (queued) {
			__syncthreads();
			if (wave0) s_pair = __builtin_amdgcn_readfirstlane(
			               __hip_atomic_fetch_add((gi32 *)pq, threadIdx.x == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
			__syncthreads();
			pair = __builtin_amdgcn_readfirstlane(s_pair);
		} else if (k) {
			break;
		}
		if (pair >= (a.Hmb + 1) / 2) break;
		row_pair(&a, 2 * pair, LDS_ARG());
	}
}

#ifndef M2DEC_MIN_BLOCKS
/* workgroups per CU = waves per SIMD: the VGPR budget (3: 168, 4: 128, 5: 96).  The pictures in flight
 * are bounded by the workgroup slots their waiting workers hold: 4 gives 1024 slots for +5-8 % (the extra
 * call-stack spills cost less); 5 spills the filter and intra chains (-25 %).  profiles/r25_occupancy.txt */
#define M2DEC_MIN_BLOCKS 4
#endif
__global__ __launch_bounds__(256, M2DEC_MIN_BLOCKS) void k_batch(const PictureArgs *pics, int bpp)
{
	const int p = blockIdx.x / bpp;
	picture_block(pics[p], blockIdx.x - p * bpp, g_lds);
}

/* the decode path's launch (up to BMAX pictures per launch, h264d_func): the blocks of k_batch that have
 * work, under its own name so that rocprofv3 reports the decode path and the trace replay separately.
 * Picture p owns blocks [blk0, blk0 + nblk) (increasing in p); a picture without inter MBs starts at its
 * row workgroups (no idle inter workers holding workgroup slots of the device-wide budget), a P / B
 * picture has only its row_wgs row workgroups. */
__global__ __launch_bounds__(256, M2DEC_MIN_BLOCKS) void k_picture(const PictureArgs *pics, int n)
{
	int p = 0;
	while (p + 1 < n && (int)blockIdx.x >= pics[p + 1].blk0) ++p;
	const PictureArgs &a = pics[p];
	const int b = (int)blockIdx.x - a.blk0;
	picture_block(a, a.n_inter ? b : b + a.inter_workers, g_lds);
}

size_t m2r_deblock_lds_bytes(int W, int Wmb)
{
	(void)W;
	const size_t dbk = (size_t)54 * DBK_RW + 3 * (size_t)Wmb * sizeof(m2r_deblock_t) + 16 + 64;
	const size_t intra = 4 * sizeof(IntraLDS) + sizeof(IntraTables);
	const size_t worker = sizeof(IntraLDS) + sizeof(IntraTables) + 24 * SEG_ROW + 4 * sizeof(InterRes);
	return std::max(dbk, std::max(intra, worker));
}

extern "C" int m2dec_amd_debug_stamps(unsigned long long *out, size_t n)
{
#ifdef M2DEC_STAMPS
	size_t bytes = sizeof(unsigned long long) * STAMP_ROWS * 4 * STAMP_EV;
	if (n * sizeof(unsigned long long) < bytes) return -1;
	CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost));
	return (int)(bytes / sizeof(unsigned long long));
#else
	(void)out;
	(void)n;
	return -1;
#endif
}

extern "C" int m2dec_amd_debug_pstamps(unsigned long long *out, size_t n)
{
#ifdef M2DEC_STAMPS
	if (n < 256 * 4) return -1;
	CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pstamps), sizeof(unsigned long long) * 256 * 4, 0, hipMemcpyDeviceToHost));
	return 256 * 4;
#else
	(void)out;
	(void)n;
	return -1;
#endif
}

extern "C" int m2dec_amd_debug_dstamps(unsigned long long *out, size_t n)
{
#if defined(M2DEC_STAMPS) && defined(M2DEC_STAMPD)
	if (n < 160 * 3 * 128) return -1;
	CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dstamps), sizeof(unsigned long long) * 160 * 3 * 128, 0, hipMemcpyDeviceToHost));
	return 160 * 3 * 128;
#else
	(void)out;
	(void)n;
	return -1;
#endif
}

extern "C" int m2dec_amd_debug_rows(unsigned *out, size_t n)
{
#ifdef M2DEC_DBG_ROWS
	if (n < 256 * 4 * 2) return -1;
	CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_rows), sizeof(unsigned) * 256 * 4 * 2, 0, hipMemcpyDeviceToHost));
	return 256 * 4 * 2;
#else
	(void)out;
	(void)n;
	return -1;
#endif
}

extern "C" int m2dec_amd_debug_intra(int *out, size_t n)
{
#ifdef M2DEC_DBG_INTRA
	if (n < 2048) return -1;
	CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(int) * 2048, 0, hipMemcpyDeviceToHost));
	return 2048;
#else
	(void)out;
	(void)n;
	return -1;
#endif
}

extern "C" int m2dec_amd_debug_stamps_clear(void)
{
#ifdef M2DEC_STAMPS
	static unsigned long long zero[STAMP_ROWS][4][STAMP_EV];
	CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice));
	return 0;
#else
	return -1;
#endif
}
