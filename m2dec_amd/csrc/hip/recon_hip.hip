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
#include "recon_kernels.h"
#include "m2dec_amd.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "m2dec_amd HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -1; } } while (0)

#define SPIN_LIMIT (1 << 24)

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

/* ======================================================================== k_inter */
__global__ __launch_bounds__(256) void k_inter(const m2r_mb_t *__restrict__ mbs, const m2r_inter_t *__restrict__ inters,
                                               const m2r_slice_t *__restrict__ slices, const int16_t *__restrict__ pool,
                                               uint8_t *frames, size_t fsz, int W, int H, int Wmb, int slot)
{
	const int addr = blockIdx.x;
	const m2r_mb_t m = mbs[addr];
	if (m.kind != M2R_MB_INTER) return;
	__shared__ int s_res[256 + 128];
	__shared__ int s_cnt[4];
	const int t = threadIdx.x;
	const int mbx = addr % Wmb, mby = addr / Wmb;
	const m2r_inter_t &it = inters[m.inter];
	const m2r_slice_t *sl = &slices[m.slice];
	uint8_t *cur = frames + (size_t)slot * fsz;
	const int CH = H >> 1;

	/* ---- luma prediction: one sample per thread */
	const int lx = t & 15, ly = t >> 4;
	const int lb = (ly >> 2) * 4 + (lx >> 2), lb8 = (ly >> 3) * 2 + (lx >> 3);
	int predl;
	{
		int v[2] = {0, 0};
		int use[2];
		for (int l = 0; l < 2; ++l) {
			int s = it.slot[l][lb8];
			use[l] = s >= 0;
			if (use[l]) {
				RefPlane r = {frames + (size_t)s * fsz, W, H};
				int mx = it.mv[l][lb][0], my = it.mv[l][lb][1];
				v[l] = luma_mc(r, mbx * 16 + lx + (mx >> 2), mby * 16 + ly + (my >> 2), mx & 3, my & 3);
			}
		}
		predl = combine(sl, it, lb8, 0, use[0], use[1], v[0], v[1]);
	}
	/* ---- chroma prediction: threads 0..127, one sample each */
	const int cc = (t >> 6) & 1, cx = t & 7, cy = (t >> 3) & 7;
	const int cb = (cy >> 1) * 4 + (cx >> 1), cb8 = (cy >> 2) * 2 + (cx >> 2);
	int predc = 0;
	if (t < 128) {
		int v[2] = {0, 0};
		int use[2];
		for (int l = 0; l < 2; ++l) {
			int s = it.slot[l][cb8];
			use[l] = s >= 0;
			if (use[l]) {
				int mx = it.mv[l][cb][0], my = it.mv[l][cb][1];
				v[l] = chroma_mc(frames + (size_t)s * fsz + (size_t)W * H, W, CH, cc, mbx * 8 + cx + (mx >> 3), mby * 8 + cy + (my >> 3), mx & 7, my & 7);
			}
		}
		predc = combine(sl, it, cb8, 1 + cc, use[0], use[1], v[0], v[1]);
	}

	uint8_t *dl = cur + (size_t)(mby * 16 + ly) * W + mbx * 16 + lx;
	uint8_t *dc = cur + (size_t)W * H + (size_t)(mby * 8 + cy) * W + mbx * 16 + cx * 2 + cc;
	if (m.cbp == 0) {
		*dl = (uint8_t)predl;
		if (t < 128) *dc = (uint8_t)predc;
		return;
	}

	/* ---- residual: dequantise into LDS */
	const int t8 = (m.flags & M2R_FLAG_T8x8) != 0;
	if (t < 4) s_cnt[t] = 0;
	__syncthreads();
	{
		int r = 0;
		if (t8) {
			int bit = 4 * lb8;
			if (m.nz & (1u << bit)) {
				int lv = pool[m.coef + d_luma_off(m, bit) + (ly & 7) * 8 + (lx & 7)];
				r = lv * d_scale8(m.qpy, lx & 7, ly & 7);
				if (lv) atomicAdd(&s_cnt[lb8], 1);
			}
		} else {
			int blk = c_rast2blk[lb];
			if (m.nz & (1u << blk)) r = pool[m.coef + d_luma_off(m, blk) + (ly & 3) * 4 + (lx & 3)] * d_scale4(m.qpy, lx & 3, ly & 3);
		}
		s_res[t] = r;
	}
	if (t < 128) {
		int ccbp = m.cbp >> 4;
		int cblk = (cy >> 2) * 2 + (cx >> 2);
		int pos = (cy & 3) * 4 + (cx & 3);
		int r = 0;
		if (ccbp) {
			if (pos == 0) {
				r = d_chroma_dc(m, pool, cc, cblk);
			} else if (ccbp == 2 && (m.nz & M2R_NZ_CAC(cc, cblk))) {
				int bit = 19 + 4 * cc + cblk;
				r = pool[m.coef + d_chroma_off(m, bit) + pos] * d_scale4(m.qpc[cc], cx & 3, cy & 3);
			}
		}
		s_res[256 + cc * 64 + cy * 8 + cx] = r;
	}
	__syncthreads();
	/* ---- row pass */
	if (t8) {
		if (t < 32) {
			int b8 = t >> 3, row = t & 7;
			int *p = &s_res[((b8 >> 1) * 8 + row) * 16 + (b8 & 1) * 8];
			int v[8];
			for (int k = 0; k < 8; ++k) v[k] = p[k];
			d_idct8_1d(v);
			for (int k = 0; k < 8; ++k) p[k] = v[k];
		}
	} else if (t < 64) {
		int b = t >> 2, row = t & 3;
		int *p = &s_res[((b >> 2) * 4 + row) * 16 + (b & 3) * 4];
		int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
	}
	if (t >= 128 && t < 160) {
		int k = t - 128, comp = k >> 4, b = (k >> 2) & 3, row = k & 3;
		int *p = &s_res[256 + comp * 64 + ((b >> 1) * 4 + row) * 8 + (b & 1) * 4];
		int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
	}
	__syncthreads();
	/* ---- column pass (+32 >> 6) */
	if (t8) {
		if (t < 32) {
			int b8 = t >> 3, col = t & 7;
			int *p = &s_res[((b8 >> 1) * 8) * 16 + (b8 & 1) * 8 + col];
			int v[8];
			for (int k = 0; k < 8; ++k) v[k] = p[k * 16];
			d_idct8_1d(v);
			for (int k = 0; k < 8; ++k) p[k * 16] = (v[k] + 32) >> 6;
		}
	} else if (t < 64) {
		int b = t >> 2, col = t & 3;
		int *p = &s_res[((b >> 2) * 4) * 16 + (b & 3) * 4 + col];
		int a0 = p[0], a1 = p[16], a2 = p[32], a3 = p[48];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = (a0 + 32) >> 6; p[16] = (a1 + 32) >> 6; p[32] = (a2 + 32) >> 6; p[48] = (a3 + 32) >> 6;
	}
	if (t >= 128 && t < 160) {
		int k = t - 128, comp = k >> 4, b = (k >> 2) & 3, col = k & 3;
		int *p = &s_res[256 + comp * 64 + ((b >> 1) * 4) * 8 + (b & 1) * 4 + col];
		int a0 = p[0], a1 = p[8], a2 = p[16], a3 = p[24];
		d_idct4_1d(a0, a1, a2, a3);
		p[0] = (a0 + 32) >> 6; p[8] = (a1 + 32) >> 6; p[16] = (a2 + 32) >> 6; p[24] = (a3 + 32) >> 6;
	}
	__syncthreads();
	/* ---- add */
	{
		int out;
		if (t8 && s_cnt[lb8] == 1 && (m.nz & (1u << (4 * lb8)))) {
			int lv0 = pool[m.coef + d_luma_off(m, 4 * lb8)];
			if (lv0 != 0) out = d_swar(predl, lv0 * d_scale8(m.qpy, 0, 0), lx & 7, 8);
			else out = d_clip255(predl + s_res[t]);
		} else {
			out = d_clip255(predl + s_res[t]);
		}
		*dl = (uint8_t)out;
	}
	if (t < 128) *dc = (uint8_t)d_clip255(predc + s_res[256 + cc * 64 + cy * 8 + cx]);
}

/* ======================================================================== wavefront hand-off */
__device__ __forceinline__ bool wait_progress(int *flag, int need, int *err)
{
	unsigned spins = 0;
	while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
		__builtin_amdgcn_s_sleep(1);
		if (++spins > SPIN_LIMIT) {
			atomicOr(err, 1);
			return false;
		}
	}
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	return true;
}

__device__ __forceinline__ void publish_progress(int *flag, int value)
{
	/* every storing wave drained + workgroup barrier happened before this call */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* ======================================================================== intra prediction (per sample) */
/* 4x4 (h264.cpp:2510-2997) on neighbours P[0..7] (top, top-right replicated when unavailable),
 * L[0..3] (left), tl; returns -1 where the reference writes nothing. */
__device__ int pred4_px(int mode, int avail, int x, int y, const int *P, const int *L, int tl)
{
#define PP(i) ((i) < 0 ? tl : P[i])
#define LL(i) ((i) < 0 ? tl : L[i])
	switch (mode) {
	case 0: return (avail & 2) ? P[x] : -1;
	case 1: return (avail & 1) ? L[y] : -1;
	case 2:
		if ((avail & 3) == 3) return (P[0] + P[1] + P[2] + P[3] + L[0] + L[1] + L[2] + L[3] + 4) >> 3;
		if (avail & 1) return (L[0] + L[1] + L[2] + L[3] + 2) >> 2;
		if (avail & 2) return (P[0] + P[1] + P[2] + P[3] + 2) >> 2;
		return 128;
	case 3:
		if (x == 3 && y == 3) return (P[6] + 3 * P[7] + 2) >> 2;
		return (P[x + y] + 2 * P[x + y + 1] + P[x + y + 2] + 2) >> 2;
	case 4:
		if ((avail & 3) != 3) return -1;
		if (x > y) return (PP(x - y - 2) + 2 * PP(x - y - 1) + P[x - y] + 2) >> 2;
		if (x < y) return (LL(y - x - 2) + 2 * LL(y - x - 1) + L[y - x] + 2) >> 2;
		return (P[0] + 2 * tl + L[0] + 2) >> 2;
	case 5: {
		if ((avail & 3) != 3) return -1;
		int z = 2 * x - y, i = x - (y >> 1);
		if (z >= 0 && !(z & 1)) return (PP(i - 1) + P[i] + 1) >> 1;
		if (z >= 0) return (PP(i - 2) + 2 * PP(i - 1) + P[i] + 2) >> 2;
		if (z == -1) return (L[0] + 2 * tl + P[0] + 2) >> 2;
		return (L[y - 1] + 2 * L[y - 2] + LL(y - 3) + 2) >> 2;
	}
	case 6: {
		if ((avail & 3) != 3) return -1;
		int z = 2 * y - x, i = y - (x >> 1);
		if (z >= 0 && !(z & 1)) return (LL(i - 1) + L[i] + 1) >> 1;
		if (z >= 0) return (LL(i - 2) + 2 * LL(i - 1) + L[i] + 2) >> 2;
		if (z == -1) return (L[0] + 2 * tl + P[0] + 2) >> 2;
		return (P[x - 1] + 2 * P[x - 2] + PP(x - 3) + 2) >> 2;
	}
	case 7: {
		int i = x + (y >> 1);
		if (!(y & 1)) return (P[i] + P[i + 1] + 1) >> 1;
		return (P[i] + 2 * P[i + 1] + P[i + 2] + 2) >> 2;
	}
	default: {
		if (!(avail & 1)) return -1;
		int z = x + 2 * y, i = y + (x >> 1);
		if (z > 5) return L[3];
		if (z == 5) return (L[2] + 3 * L[3] + 2) >> 2;
		if (!(z & 1)) return (L[i] + L[i + 1] + 1) >> 1;
		return (L[i] + 2 * L[i + 1] + L[i + 2] + 2) >> 2;
	}
	}
#undef PP
#undef LL
}

/* 8x8 on filtered neighbours pt[0..15], lf[0..7], tlf (spec 8.3.2.2; h264.cpp:3301-3929) */
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
#define LW 25 /* luma context row: [0] = x0 - 1, [1..24] = x0 .. x0 + 23 */

__global__ __launch_bounds__(64) void k_intra(const m2r_mb_t *__restrict__ mbs, const int16_t *__restrict__ pool,
                                              uint8_t *cur, int W, int H, int Wmb, int *progress, int *err)
{
	const int y = blockIdx.x;
	const int t = threadIdx.x;
	__shared__ uint8_t L[17][LW];   /* row 0: top neighbours; rows 1..16: MB rows; col 0: left neighbour */
	__shared__ uint8_t C[2][9][9];  /* per component: row 0 top (col 0 top-left), col 0 left */
	__shared__ int R[256 + 128];
	__shared__ int DC[16];
	__shared__ int F[32];           /* filtered 8x8 neighbours: [0..15] top, [16..23] left, [24] top-left */
	__shared__ int HV[4];
	int left_in_lds = 0;
	uint8_t *chroma = cur + (size_t)W * H;
	const int x_last = Wmb - 1;

	for (int x = 0; x < Wmb; ++x) {
		const m2r_mb_t m = mbs[y * Wmb + x];
		const int x0 = x * 16, y0 = y * 16;
		if (m.kind == M2R_MB_INTER) {
			left_in_lds = 0;
			continue;
		}
		if (y > 0) {
			if (t == 0) wait_progress(&progress[y - 1], min(x + 2, Wmb), err);
			__syncthreads();
		}
		/* ---- gather the neighbourhood */
		if (left_in_lds) {
			if (t < 17) L[t][0] = L[t][16];
			if (t < 18) { int c = t / 9, r = t % 9; C[c][r][0] = C[c][r][8]; }
		}
		__syncthreads();
		if (y > 0) {
			if (t < 24) {
				int xx = x0 + t;
				if (t < 16 || x < x_last) L[0][1 + t] = cur[(size_t)(y0 - 1) * W + xx];
			}
			if (t == 24 && x > 0 && !left_in_lds) L[0][0] = cur[(size_t)(y0 - 1) * W + x0 - 1];
			if (t >= 32 && t < 48) { int k = t - 32; C[k & 1][0][1 + (k >> 1)] = chroma[(size_t)(y0 / 2 - 1) * W + x0 + k]; }
			if (t == 48 && x > 0 && !left_in_lds) { C[0][0][0] = chroma[(size_t)(y0 / 2 - 1) * W + x0 - 2]; C[1][0][0] = chroma[(size_t)(y0 / 2 - 1) * W + x0 - 1]; }
		}
		if (x > 0 && !left_in_lds) {
			if (t < 16) L[1 + t][0] = cur[(size_t)(y0 + t) * W + x0 - 1];
			if (t >= 16 && t < 32) { int k = t - 16; C[k & 1][1 + (k >> 1)][0] = chroma[(size_t)(y0 / 2 + (k >> 1)) * W + x0 - 2 + (k & 1)]; }
		}
		__syncthreads();
		if (left_in_lds && y > 0) {
			/* the top-left sample moved with the left column copy only for row 0 of L; refresh it from the row above */
			if (t == 0) L[0][0] = cur[(size_t)(y0 - 1) * W + x0 - 1];
			if (t == 1) { C[0][0][0] = chroma[(size_t)(y0 / 2 - 1) * W + x0 - 2]; C[1][0][0] = chroma[(size_t)(y0 / 2 - 1) * W + x0 - 1]; }
			__syncthreads();
		}

		if (m.kind == M2R_MB_PCM) {
			const uint8_t *s = (const uint8_t *)(pool + m.coef);
			for (int k = t; k < 256; k += 64) L[1 + (k >> 4)][1 + (k & 15)] = s[k];
			for (int k = t; k < 128; k += 64) C[k >> 6][1 + ((k >> 3) & 7)][1 + (k & 7)] = s[256 + k];
			__syncthreads();
		} else {
			/* ---- chroma prediction (h264.cpp:4559-4706); thread t: sample (t & 7, t >> 3) of both components */
			{
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
			__syncthreads();
			for (int c = 0; c < 2; ++c) {
				int v = R[256 + c * 64 + t];
				if (v >= 0) C[c][1 + (t >> 3)][1 + (t & 7)] = (uint8_t)v;
			}
			__syncthreads();

			/* ---- luma */
			const int qp = m.qpy;
			if (m.kind == M2R_MB_I4x4) {
				for (int blk = 0; blk < 16; ++blk) {
					const int ox = c_blk_x[blk] * 4, oy = c_blk_y[blk] * 4;
					const int av = avail4(blk, m.avail_luma);
					const int coded = (m.nz >> blk) & 1;
					if (t < 16) {
						int P[8], Lf[4];
						for (int i = 0; i < 4; ++i) P[i] = L[oy][1 + ox + i];
						for (int i = 4; i < 8; ++i) P[i] = (av & 4) ? L[oy][1 + ox + i] : P[3];
						for (int i = 0; i < 4; ++i) Lf[i] = L[oy + 1 + i][ox];
						int mode = (m.ipred[blk >> 3] >> (4 * (blk & 7))) & 15;
						int v = pred4_px(mode, av, t & 3, t >> 2, P, Lf, L[oy][ox]);
						R[64 + t] = v;
						if (coded) R[t] = pool[m.coef + d_luma_off(m, blk) + t] * d_scale4(qp, t & 3, t >> 2);
					}
					__syncthreads();
					if (t < 16) {
						int v = R[64 + t];
						if (v >= 0) L[oy + 1 + (t >> 2)][1 + ox + (t & 3)] = (uint8_t)v;
					}
					if (coded) {
						if (t < 4) {
							int *p = &R[t * 4];
							int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
							d_idct4_1d(a0, a1, a2, a3);
							p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
						}
						__syncthreads();
						if (t < 4) {
							int *p = &R[t];
							int a0 = p[0], a1 = p[4], a2 = p[8], a3 = p[12];
							d_idct4_1d(a0, a1, a2, a3);
							p[0] = (a0 + 32) >> 6; p[4] = (a1 + 32) >> 6; p[8] = (a2 + 32) >> 6; p[12] = (a3 + 32) >> 6;
						}
						__syncthreads();
						if (t < 16) {
							uint8_t *d = &L[oy + 1 + (t >> 2)][1 + ox + (t & 3)];
							*d = (uint8_t)d_clip255(*d + R[t]);
						}
					}
					__syncthreads();
				}
			} else if (m.kind == M2R_MB_I8x8) {
				for (int b = 0; b < 4; ++b) {
					const int ox = (b & 1) * 8, oy = (b >> 1) * 8;
					const int av = avail8(b, m.avail_luma);
					const int coded = (m.nz >> (4 * b)) & 1;
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
					if (coded) {
						int lv = pool[m.coef + d_luma_off(m, 4 * b) + t];
						R[t] = lv * d_scale8(qp, t & 7, t >> 3);
						R[128 + t] = (lv != 0);
						if (t == 0) DC[0] = lv;
					}
					__syncthreads();
					{
						int mode = (m.ipred[0] >> (4 * b)) & 15;
						int v = pred8_px(mode, av, t & 7, t >> 3, F, F + 16, F[24]);
						if (v >= 0) L[oy + 1 + (t >> 3)][1 + ox + (t & 7)] = (uint8_t)v;
					}
					if (coded) {
						if (t < 8) {
							int v[8];
							int *p = &R[t * 8];
							for (int k = 0; k < 8; ++k) v[k] = p[k];
							d_idct8_1d(v);
							for (int k = 0; k < 8; ++k) p[k] = v[k];
						}
						if (t == 8) {
							int n = 0;
							for (int k = 0; k < 64; ++k) n += R[128 + k];
							HV[0] = n;
						}
						__syncthreads();
						if (t < 8) {
							int v[8];
							int *p = &R[t];
							for (int k = 0; k < 8; ++k) v[k] = p[k * 8];
							d_idct8_1d(v);
							for (int k = 0; k < 8; ++k) p[k * 8] = (v[k] + 32) >> 6;
						}
						__syncthreads();
						{
							uint8_t *d = &L[oy + 1 + (t >> 3)][1 + ox + (t & 7)];
							if (HV[0] == 1 && DC[0] != 0) *d = (uint8_t)d_swar(*d, DC[0] * d_scale8(qp, 0, 0), t & 7, 8);
							else *d = (uint8_t)d_clip255(*d + R[t]);
						}
					}
					__syncthreads();
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
				if (t < 16) DC[t] = (m.nz & M2R_NZ_LUMA_DC) ? pool[m.coef + t] * d_scale4(qp, 0, 0) : 0;
				__syncthreads();
				for (int k = t; k < 256; k += 64) {
					int px = k & 15, py = k >> 4, v = -1;
					if (mode == 0) { if (av & 2) v = L[0][1 + px]; }
					else if (mode == 1) { if (av & 1) v = L[1 + py][0]; }
					else if (mode == 2) v = HV[3];
					else v = d_clip255((HV[0] + HV[1] * (px - 7) + HV[2] * (py - 7) + 16) >> 5);
					R[k] = v;
				}
				__syncthreads();
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
				__syncthreads();
				if (t < 4) {
					int *r = &DC[t];
					int a0 = r[0] + r[4], a1 = r[0] - r[4], a2 = r[8] + r[12], a3 = r[8] - r[12];
					r[0] = (a0 + a2 + 2) >> 2; r[4] = (a0 - a2 + 2) >> 2; r[8] = (a1 - a3 + 2) >> 2; r[12] = (a1 + a3 + 2) >> 2;
				}
				__syncthreads();
				if (m.cbp & 15) {
					/* AC blocks with coefficients: full transform with the DC inserted; others DC-only SWAR */
					for (int k = t; k < 256; k += 64) {
						int blk = k >> 4, pos = k & 15;
						int bx = c_blk_x[blk], by = c_blk_y[blk];
						int v = 0;
						if (pos == 0) v = DC[by * 4 + bx];
						else if (m.nz & (1u << blk)) v = pool[m.coef + d_luma_off(m, blk) + pos] * d_scale4(qp, pos & 3, pos >> 2);
						R[k] = v;
					}
					__syncthreads();
					{
						int blk = t >> 2, row = t & 3;
						int *p = &R[blk * 16 + row * 4];
						int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
						d_idct4_1d(a0, a1, a2, a3);
						p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
					}
					__syncthreads();
					{
						int blk = t >> 2, col = t & 3;
						int *p = &R[blk * 16 + col];
						int a0 = p[0], a1 = p[4], a2 = p[8], a3 = p[12];
						d_idct4_1d(a0, a1, a2, a3);
						p[0] = (a0 + 32) >> 6; p[4] = (a1 + 32) >> 6; p[8] = (a2 + 32) >> 6; p[12] = (a3 + 32) >> 6;
					}
					__syncthreads();
					for (int k = t; k < 256; k += 64) {
						int blk = k >> 4, pos = k & 15;
						int bx = c_blk_x[blk], by = c_blk_y[blk];
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
				__syncthreads();
			}

			/* ---- chroma residual (residual_chroma, h264.cpp:2374-2461) */
			if (m.cbp >> 4) {
				int ccbp = m.cbp >> 4;
				for (int k = t; k < 128; k += 64) {
					int c = k >> 6, cx = k & 7, cy = (k >> 3) & 7;
					int cblk = (cy >> 2) * 2 + (cx >> 2), pos = (cy & 3) * 4 + (cx & 3);
					int v = 0;
					if (pos == 0) v = d_chroma_dc(m, pool, c, cblk);
					else if (ccbp == 2 && (m.nz & M2R_NZ_CAC(c, cblk)))
						v = pool[m.coef + d_chroma_off(m, 19 + 4 * c + cblk) + pos] * d_scale4(m.qpc[c], cx & 3, cy & 3);
					R[256 + c * 64 + cy * 8 + cx] = v;
				}
				__syncthreads();
				if (t < 32) {
					int comp = t >> 4, b = (t >> 2) & 3, row = t & 3;
					int *p = &R[256 + comp * 64 + ((b >> 1) * 4 + row) * 8 + (b & 1) * 4];
					int a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
					d_idct4_1d(a0, a1, a2, a3);
					p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3;
				}
				__syncthreads();
				if (t < 32) {
					int comp = t >> 4, b = (t >> 2) & 3, col = t & 3;
					int *p = &R[256 + comp * 64 + ((b >> 1) * 4) * 8 + (b & 1) * 4 + col];
					int a0 = p[0], a1 = p[8], a2 = p[16], a3 = p[24];
					d_idct4_1d(a0, a1, a2, a3);
					p[0] = (a0 + 32) >> 6; p[8] = (a1 + 32) >> 6; p[16] = (a2 + 32) >> 6; p[24] = (a3 + 32) >> 6;
				}
				__syncthreads();
				for (int k = t; k < 128; k += 64) {
					int c = k >> 6, cx = k & 7, cy = (k >> 3) & 7;
					uint8_t *d = &C[c][1 + cy][1 + cx];
					*d = (uint8_t)d_clip255(*d + R[256 + c * 64 + cy * 8 + cx]);
				}
				__syncthreads();
			}
		}

		/* ---- write back and publish */
		for (int k = t; k < 256; k += 64) cur[(size_t)(y0 + (k >> 4)) * W + x0 + (k & 15)] = L[1 + (k >> 4)][1 + (k & 15)];
		for (int k = t; k < 128; k += 64) {
			int cy = k >> 4, bx = k & 15;
			chroma[(size_t)(y0 / 2 + cy) * W + x0 + bx] = C[bx & 1][1 + cy][1 + (bx >> 1)];
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		if (t == 0) publish_progress(&progress[y], x + 1);
		left_in_lds = 1;
		/* keep this MB's right column (col 16 / chroma col 8) for the next MB's left neighbours */
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (t == 0) publish_progress(&progress[y], Wmb);
}

/* ======================================================================== k_deblock */
/* filter one line across an edge: q0 at s[0], p0 at s[-d] (spec 8.7.2.3 / 8.7.2.4) */
__device__ __forceinline__ void filter_line(uint8_t *s, int d, int bs, int alpha, int beta, int ia, int luma)
{
	int p0 = s[-d], p1 = s[-2 * d], q0 = s[0], q1 = s[d];
	if (!(abs(p0 - q0) < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta)) return;
	if (bs < 4) {
		int tc0 = c_tc0[ia][bs - 1], tc, delta;
		if (luma) {
			int p2 = s[-3 * d], q2 = s[2 * d];
			int ap = abs(p2 - p0) < beta, aq = abs(q2 - q0) < beta;
			tc = tc0 + ap + aq;
			if (ap) s[-2 * d] = (uint8_t)(p1 + d_clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
			if (aq) s[d] = (uint8_t)(q1 + d_clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
		} else {
			tc = tc0 + 1;
		}
		delta = d_clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
		s[-d] = (uint8_t)d_clip255(p0 + delta);
		s[0] = (uint8_t)d_clip255(q0 - delta);
	} else if (luma) {
		int p2 = s[-3 * d], q2 = s[2 * d], p3 = s[-4 * d], q3 = s[3 * d];
		int small = abs(p0 - q0) < ((alpha >> 2) + 2);
		if (abs(p2 - p0) < beta && small) {
			s[-d] = (uint8_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
			s[-2 * d] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
			s[-3 * d] = (uint8_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
		} else {
			s[-d] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
		}
		if (abs(q2 - q0) < beta && small) {
			s[0] = (uint8_t)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
			s[d] = (uint8_t)((p0 + q0 + q1 + q2 + 2) >> 2);
			s[2 * d] = (uint8_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
		} else {
			s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
		}
	} else {
		s[-d] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
		s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
	}
}

__device__ __forceinline__ int ab_idx(int qp, int off)
{
	return min(max(qp + off, 0), 51);
}

#define TLW 20 /* luma tile: rows y0-4 .. y0+15, cols x0-4 .. x0+15 */
#define TCW 20 /* chroma tile: rows y0/2-2 .. y0/2+7, bytes x0-4 .. x0+15 */

__global__ __launch_bounds__(64) void k_deblock(const m2r_deblock_t *__restrict__ dbk, uint8_t *cur, int W, int H, int Wmb,
                                                int *progress, int *err)
{
	const int y = blockIdx.x;
	const int t = threadIdx.x;
	__shared__ uint8_t T[20][TLW];
	__shared__ uint8_t TC[10][TCW];
	uint8_t *chroma = cur + (size_t)W * H;
	const int y0 = y * 16, yc0 = y * 8;

	for (int x = 0; x < Wmb; ++x) {
		const int x0 = x * 16;
		const m2r_deblock_t q = dbk[y * Wmb + x];
		if (y > 0) {
			if (t == 0) wait_progress(&progress[y - 1], min(x + 2, Wmb), err);
			__syncthreads();
		}
		/* left halo from the previous tile (already final w.r.t. this workgroup's writes) */
		if (x > 0) {
			if (t < 20) { for (int i = 0; i < 4; ++i) T[t][i] = T[t][16 + i]; }
			else if (t < 30) { int r = t - 20; for (int i = 0; i < 4; ++i) TC[r][i] = TC[r][16 + i]; }
		}
		__syncthreads();
		/* top halo (row above, other workgroup) and the MB itself */
		for (int k = t; k < 20 * 16; k += 64) {
			int r = k >> 4, c = k & 15;
			if (r >= 4 || y > 0) T[r][4 + c] = cur[(size_t)(y0 - 4 + r) * W + x0 + c];
		}
		for (int k = t; k < 10 * 16; k += 64) {
			int r = k >> 4, c = k & 15;
			if (r >= 2 || y > 0) TC[r][4 + c] = chroma[(size_t)(yc0 - 2 + r) * W + x0 + c];
		}
		__syncthreads();

		if (!(q.flags & M2R_DBK_OFF)) {
			for (int dir = 0; dir < 2; ++dir) {
				const uint32_t str = dir ? q.bs_h : q.bs_v;
				const int edge_flag = dir ? M2R_DBK_TOP : M2R_DBK_LEFT;
				const int bs4_flag = dir ? M2R_DBK_TOP_BS4 : M2R_DBK_LEFT_BS4;
				int qpn = q.qpy, qpcn0 = q.qpc[0], qpcn1 = q.qpc[1];
				if ((q.flags & edge_flag) && (str & 255)) {
					const m2r_deblock_t p = dir ? dbk[(y - 1) * Wmb + x] : dbk[y * Wmb + x - 1];
					qpn = (q.qpy + p.qpy + 1) >> 1;
					qpcn0 = (q.qpc[0] + p.qpc[0] + 1) >> 1;
					qpcn1 = (q.qpc[1] + p.qpc[1] + 1) >> 1;
				}
				for (int e = 0; e < 4; ++e) {
					uint32_t s = (str >> (8 * e)) & 255;
					int bs4 = 0;
					if (e == 0) {
						if (!((q.flags & edge_flag) && s)) continue;
						bs4 = (q.flags & bs4_flag) != 0;
					} else if (!s) {
						continue;
					}
					int ql = e ? q.qpy : qpn;
					if (t < 16) {
						int bs = bs4 ? 4 : (int)((s >> ((t >> 2) * 2)) & 3);
						if (bs) {
							int ia = ab_idx(ql, q.alpha_off), ib = ab_idx(ql, q.beta_off);
							uint8_t *pt = dir ? &T[4 + 4 * e][4 + t] : &T[4 + t][4 + 4 * e];
							filter_line(pt, dir ? TLW : 1, bs, c_alpha[ia], c_beta[ib], ia, 1);
						}
					} else if (t < 32 && (e == 0 || e == 2)) {
						int k = t - 16, comp = k >> 3, line = k & 7;
						int bs = bs4 ? 4 : (int)((s >> ((line >> 1) * 2)) & 3);
						if (bs) {
							int qc = e ? q.qpc[comp] : (comp ? qpcn1 : qpcn0);
							int ia = ab_idx(qc, q.alpha_off), ib = ab_idx(qc, q.beta_off);
							uint8_t *pt = dir ? &TC[2 + 2 * e][4 + line * 2 + comp] : &TC[2 + line][4 + 4 * e + comp];
							filter_line(pt, dir ? TCW : 2, bs, c_alpha[ia], c_beta[ib], ia, 0);
						}
					}
					__syncthreads();
				}
			}
		}
		/* write back: top rows y0-3..y0-1 (cols x0..x0+15) and the MB incl. left cols x0-3..x0-1 */
		for (int k = t; k < 19 * 19; k += 64) {
			int r = 1 + k / 19, c = 1 + k % 19;
			if (r < 4 && c < 4) continue;
			if (r < 4 && y == 0) continue;
			if (c < 4 && x == 0) continue;
			cur[(size_t)(y0 - 4 + r) * W + x0 - 4 + c] = T[r][c];
		}
		for (int k = t; k < 9 * 18; k += 64) {
			int r = 1 + k / 18, c = 2 + k % 18;
			if (r < 2 && c < 4) continue;
			if (r < 2 && y == 0) continue;
			if (c < 4 && x == 0) continue;
			chroma[(size_t)(yc0 - 2 + r) * W + x0 - 4 + c] = TC[r][c];
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		if (t == 0) publish_progress(&progress[y], x + 1);
	}
}

/* ======================================================================== host back end */
namespace {

struct Arena {
	m2r_picture_t pic;
	uint8_t *host = nullptr, *dev = nullptr;
	size_t size = 0, off_mb = 0, off_dbk = 0, off_slice = 0, off_inter = 0, off_coef = 0;
	hipEvent_t uploaded = nullptr;
	bool pending = false;
};

struct HipBackend {
	int dev = 0;
	hipStream_t stream = nullptr;
	int W = 0, H = 0, Wmb = 0, Hmb = 0, nframes = 0;
	size_t fsz = 0;
	uint8_t *d_frames = nullptr;
	m2d_frame_t frames[64];
	void *reg[64][2];
	hipEvent_t slot_ev[64];
	bool slot_pending[64];
	Arena ar[3];
	int next = 0;
	int *d_prog = nullptr; /* [2][Hmb] */
	int *d_err = nullptr;
	hipEvent_t ev[4][6]; /* timing ring: picture k uses ev[k % 4] */
	bool ev_pending[4];
	int ev_next = 0;
	m2dec_amd_hip_timing_t tm;
	bool timing = true;
};

/* accumulate the kernel times of timing-ring entry k (blocks until that picture finished) */
static void flush_timing(HipBackend *b, int k)
{
	if (!b->ev_pending[k]) return;
	hipEvent_t *e = b->ev[k];
	float ms;
	(void)hipEventSynchronize(e[5]);
	if (hipEventElapsedTime(&ms, e[0], e[1]) == hipSuccess) b->tm.h2d_us += ms * 1e3;
	if (hipEventElapsedTime(&ms, e[1], e[2]) == hipSuccess) b->tm.inter_us += ms * 1e3;
	if (hipEventElapsedTime(&ms, e[2], e[3]) == hipSuccess) b->tm.intra_us += ms * 1e3;
	if (hipEventElapsedTime(&ms, e[3], e[4]) == hipSuccess) b->tm.deblock_us += ms * 1e3;
	if (hipEventElapsedTime(&ms, e[4], e[5]) == hipSuccess) b->tm.d2h_us += ms * 1e3;
	b->ev_pending[k] = false;
}

struct RecPtrs {
	const m2r_mb_t *mb;
	const m2r_deblock_t *dbk;
	const m2r_slice_t *sl;
	const m2r_inter_t *it;
	const int16_t *coef;
};

struct Geometry {
	uint8_t *frames;
	size_t fsz;
	int W, H, Wmb, Hmb;
	int *prog; /* [2][Hmb] */
	int *err;
};

/* Enqueue one picture (k_inter -> k_intra -> k_deblock) on stream s.  ev (optional) receives
 * three records: after k_inter, after k_intra, after k_deblock. */
static int launch_picture(hipStream_t s, const Geometry &g, const RecPtrs &r, int slot, int n_inter, int n_intra,
                          int deblock, hipEvent_t *ev, m2dec_amd_hip_timing_t *tm)
{
	uint8_t *cur = g.frames + (size_t)slot * g.fsz;
	const int n = g.Wmb * g.Hmb;
	if (n_inter) {
		hipLaunchKernelGGL(k_inter, dim3(n), dim3(256), 0, s, r.mb, r.it, r.sl, r.coef, g.frames, g.fsz, g.W, g.H, g.Wmb, slot);
		CHECK(hipGetLastError());
		tm->inter_launches++;
	}
	if (ev) CHECK(hipEventRecord(ev[0], s));
	if (n_intra) {
		CHECK(hipMemsetAsync(g.prog, 0, sizeof(int) * g.Hmb, s));
		hipLaunchKernelGGL(k_intra, dim3(g.Hmb), dim3(64), 0, s, r.mb, r.coef, cur, g.W, g.H, g.Wmb, g.prog, g.err);
		CHECK(hipGetLastError());
		tm->intra_launches++;
	}
	if (ev) CHECK(hipEventRecord(ev[1], s));
	if (deblock) {
		CHECK(hipMemsetAsync(g.prog + g.Hmb, 0, sizeof(int) * g.Hmb, s));
		hipLaunchKernelGGL(k_deblock, dim3(g.Hmb), dim3(64), 0, s, r.dbk, cur, g.W, g.H, g.Wmb, g.prog + g.Hmb, g.err);
		CHECK(hipGetLastError());
		tm->deblock_launches++;
	}
	if (ev) CHECK(hipEventRecord(ev[2], s));
	return 0;
}

static const int kSlicesCap = 64;

static void unregister_frames(HipBackend *b)
{
	for (int i = 0; i < 64; ++i)
		for (int k = 0; k < 2; ++k)
			if (b->reg[i][k]) {
				(void)hipHostUnregister(b->reg[i][k]);
				b->reg[i][k] = nullptr;
			}
}

static int be_set_frames(void *self, int n, const m2d_frame_t *frames, int width, int height)
{
	HipBackend *b = (HipBackend *)self;
	CHECK(hipSetDevice(b->dev));
	CHECK(hipStreamSynchronize(b->stream));
	unregister_frames(b);
	if (n > 64) n = 64;
	memcpy(b->frames, frames, sizeof(m2d_frame_t) * (size_t)n);
	size_t fsz = ((size_t)width * height * 3 / 2 + 4095) & ~(size_t)4095;
	if (b->d_frames && (fsz != b->fsz || n > b->nframes)) {
		(void)hipFree(b->d_frames);
		b->d_frames = nullptr;
	}
	if (!b->d_frames) {
		CHECK(hipMalloc(&b->d_frames, fsz * (size_t)n));
		CHECK(hipMemset(b->d_frames, 0, fsz * (size_t)n));
	}
	if (b->d_prog && height / 16 != b->Hmb) {
		(void)hipFree(b->d_prog);
		b->d_prog = nullptr;
	}
	b->W = width;
	b->H = height;
	b->Wmb = width / 16;
	b->Hmb = height / 16;
	b->fsz = fsz;
	b->nframes = n;
	if (!b->d_prog) CHECK(hipMalloc(&b->d_prog, sizeof(int) * 2 * (size_t)b->Hmb));
	size_t ls = (size_t)width * height, cs = ls / 2;
	for (int i = 0; i < n; ++i) {
		b->slot_pending[i] = false;
		if (b->frames[i].chroma == b->frames[i].luma + ls) {
			if (hipHostRegister(b->frames[i].luma, ls + cs, hipHostRegisterDefault) == hipSuccess) b->reg[i][0] = b->frames[i].luma;
		} else {
			if (hipHostRegister(b->frames[i].luma, ls, hipHostRegisterDefault) == hipSuccess) b->reg[i][0] = b->frames[i].luma;
			if (hipHostRegister(b->frames[i].chroma, cs, hipHostRegisterDefault) == hipSuccess) b->reg[i][1] = b->frames[i].chroma;
		}
		(void)hipGetLastError();
	}
	return 0;
}

static int arena_alloc(Arena &a, int wm, int hm)
{
	size_t n = (size_t)wm * hm;
	size_t off = 0;
	auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
	a.off_mb = off; off = al(off + n * sizeof(m2r_mb_t));
	a.off_dbk = off; off = al(off + n * sizeof(m2r_deblock_t));
	a.off_slice = off; off = al(off + kSlicesCap * sizeof(m2r_slice_t));
	a.off_inter = off; off = al(off + n * sizeof(m2r_inter_t));
	a.off_coef = off; off = al(off + n * 416 * sizeof(int16_t));
	if (a.size < off) {
		if (a.host) (void)hipHostFree(a.host);
		if (a.dev) (void)hipFree(a.dev);
		a.host = nullptr;
		a.dev = nullptr;
		CHECK(hipHostMalloc(&a.host, off, hipHostMallocDefault));
		CHECK(hipMalloc(&a.dev, off));
		a.size = off;
	}
	if (!a.uploaded) CHECK(hipEventCreateWithFlags(&a.uploaded, hipEventDisableTiming));
	m2r_picture_t &p = a.pic;
	memset(&p, 0, sizeof(p));
	p.width_mbs = wm;
	p.height_mbs = hm;
	p.mb = (m2r_mb_t *)(a.host + a.off_mb);
	p.dbk = (m2r_deblock_t *)(a.host + a.off_dbk);
	p.slice = (m2r_slice_t *)(a.host + a.off_slice);
	p.inter = (m2r_inter_t *)(a.host + a.off_inter);
	p.coef = (int16_t *)(a.host + a.off_coef);
	p.cap_slices = kSlicesCap;
	p.cap_inter = (int)n;
	p.cap_coef = (int)(n * 416);
	return 0;
}

static m2r_picture_t *be_acquire(void *self, int wm, int hm)
{
	HipBackend *b = (HipBackend *)self;
	Arena &a = b->ar[b->next];
	b->next = (b->next + 1) % 3;
	if (a.pending) {
		if (hipEventSynchronize(a.uploaded) != hipSuccess) return nullptr;
		a.pending = false;
	}
	if (arena_alloc(a, wm, hm) < 0) return nullptr;
	return &a.pic;
}

static int64_t ref_bytes_of(const m2r_picture_t *pic)
{
	/* algorithmic MC input: one reference byte per predicted sample per list */
	int64_t s = 0;
	for (int i = 0; i < pic->n_inter; ++i)
		for (int l = 0; l < 2; ++l)
			for (int b8 = 0; b8 < 4; ++b8)
				if (pic->inter[i].slot[l][b8] >= 0) s += 64 + 32;
	return s;
}

static int be_submit(void *self, m2r_picture_t *pic)
{
	HipBackend *b = (HipBackend *)self;
	Arena *a = nullptr;
	for (auto &x : b->ar)
		if (&x.pic == pic) a = &x;
	if (!a) return -1;
	const int n = pic->width_mbs * pic->height_mbs;
	if (pic->width_mbs != b->Wmb || pic->height_mbs != b->Hmb || pic->slot < 0 || pic->slot >= b->nframes) return -1;
	CHECK(hipSetDevice(b->dev));
	hipStream_t s = b->stream;
	size_t rec_bytes = n * (sizeof(m2r_mb_t) + sizeof(m2r_deblock_t)) + pic->n_slices * sizeof(m2r_slice_t) +
	                   pic->n_inter * sizeof(m2r_inter_t) + pic->n_coef * sizeof(int16_t);
	hipEvent_t *ev = b->ev[b->ev_next];
	if (b->timing) {
		flush_timing(b, b->ev_next);
		CHECK(hipEventRecord(ev[0], s));
	}
	CHECK(hipMemcpyAsync(a->dev + a->off_mb, a->host + a->off_mb, a->off_slice - a->off_mb, hipMemcpyHostToDevice, s));
	if (pic->n_slices) CHECK(hipMemcpyAsync(a->dev + a->off_slice, a->host + a->off_slice, pic->n_slices * sizeof(m2r_slice_t), hipMemcpyHostToDevice, s));
	if (pic->n_inter) CHECK(hipMemcpyAsync(a->dev + a->off_inter, a->host + a->off_inter, pic->n_inter * sizeof(m2r_inter_t), hipMemcpyHostToDevice, s));
	if (pic->n_coef) CHECK(hipMemcpyAsync(a->dev + a->off_coef, a->host + a->off_coef, pic->n_coef * sizeof(int16_t), hipMemcpyHostToDevice, s));
	CHECK(hipEventRecord(a->uploaded, s));
	a->pending = true;
	if (b->timing) CHECK(hipEventRecord(ev[1], s));
	RecPtrs rp;
	rp.mb = (const m2r_mb_t *)(a->dev + a->off_mb);
	rp.dbk = (const m2r_deblock_t *)(a->dev + a->off_dbk);
	rp.sl = (const m2r_slice_t *)(a->dev + a->off_slice);
	rp.it = (const m2r_inter_t *)(a->dev + a->off_inter);
	rp.coef = (const int16_t *)(a->dev + a->off_coef);
	uint8_t *cur = b->d_frames + (size_t)pic->slot * b->fsz;
	Geometry gm{b->d_frames, b->fsz, b->W, b->H, b->Wmb, b->Hmb, b->d_prog, b->d_err};
	if (launch_picture(s, gm, rp, pic->slot, pic->n_inter, pic->n_intra, pic->deblock, b->timing ? ev + 2 : nullptr, &b->tm) < 0) return -1;
	const m2d_frame_t &f = b->frames[pic->slot];
	size_t ls = (size_t)b->W * b->H;
	CHECK(hipMemcpyAsync(f.luma, cur, ls, hipMemcpyDeviceToHost, s));
	CHECK(hipMemcpyAsync(f.chroma, cur + ls, ls / 2, hipMemcpyDeviceToHost, s));
	CHECK(hipEventRecord(b->slot_ev[pic->slot], s));
	b->slot_pending[pic->slot] = true;
	if (b->timing) {
		CHECK(hipEventRecord(ev[5], s));
		b->ev_pending[b->ev_next] = true;
		b->ev_next = (b->ev_next + 1) % 4;
	}
	b->tm.pictures++;
	b->tm.record_bytes += (int64_t)rec_bytes;
	b->tm.ref_bytes += ref_bytes_of(pic);
	b->tm.frame_bytes += (int64_t)(ls * 3 / 2);
	return 0;
}

static int be_sync(void *self, int slot)
{
	HipBackend *b = (HipBackend *)self;
	if (slot < 0 || slot >= 64) return -1;
	if (b->slot_pending[slot]) {
		CHECK(hipEventSynchronize(b->slot_ev[slot]));
		b->slot_pending[slot] = false;
		int err = 0;
		CHECK(hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost));
		if (err) {
			fprintf(stderr, "m2dec_amd: wavefront hand-off timed out (err=%d)\n", err);
			return -1;
		}
	}
	return 0;
}

static void be_destroy(void *self)
{
	HipBackend *b = (HipBackend *)self;
	(void)hipSetDevice(b->dev);
	(void)hipStreamSynchronize(b->stream);
	unregister_frames(b);
	for (auto &a : b->ar) {
		if (a.host) (void)hipHostFree(a.host);
		if (a.dev) (void)hipFree(a.dev);
		if (a.uploaded) (void)hipEventDestroy(a.uploaded);
	}
	for (int i = 0; i < 64; ++i) (void)hipEventDestroy(b->slot_ev[i]);
	for (int k = 0; k < 4; ++k)
		for (int i = 0; i < 6; ++i) (void)hipEventDestroy(b->ev[k][i]);
	if (b->d_frames) (void)hipFree(b->d_frames);
	if (b->d_prog) (void)hipFree(b->d_prog);
	if (b->d_err) (void)hipFree(b->d_err);
	(void)hipStreamDestroy(b->stream);
	delete b;
}

} // namespace

extern "C" int m2dec_amd_hip_available(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n > 0;
}

extern "C" int m2dec_amd_hip_backend_create(m2r_backend_t *out, int device)
{
	if (!m2dec_amd_hip_available()) return -1;
	HipBackend *b = new HipBackend();
	memset(&b->tm, 0, sizeof(b->tm));
	memset(b->reg, 0, sizeof(b->reg));
	memset(b->slot_pending, 0, sizeof(b->slot_pending));
	b->dev = device;
	CHECK(hipSetDevice(device));
	CHECK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
	for (int i = 0; i < 64; ++i) CHECK(hipEventCreateWithFlags(&b->slot_ev[i], hipEventDisableTiming));
	for (int k = 0; k < 4; ++k) {
		b->ev_pending[k] = false;
		for (int i = 0; i < 6; ++i) CHECK(hipEventCreate(&b->ev[k][i]));
	}
	CHECK(hipMalloc(&b->d_err, sizeof(int)));
	CHECK(hipMemset(b->d_err, 0, sizeof(int)));
	const char *tm = getenv("M2DEC_AMD_TIMING");
	b->timing = tm ? atoi(tm) != 0 : true;
	out->self = b;
	out->set_frames = be_set_frames;
	out->acquire = be_acquire;
	out->submit = be_submit;
	out->sync_frame = be_sync;
	out->destroy = be_destroy;
	return 0;
}

extern "C" int m2dec_amd_hip_backend_timing(const m2r_backend_t *be, m2dec_amd_hip_timing_t *out)
{
	if (!be || !be->self || !out) return -1;
	HipBackend *b = (HipBackend *)be->self;
	for (int k = 0; k < 4; ++k) flush_timing(b, k);
	*out = b->tm;
	return 0;
}

/* ======================================================================== trace replay */
struct m2dec_amd_hip_replay {
	int dev = 0;
	hipStream_t stream = nullptr;
	int W = 0, H = 0, Wmb = 0, Hmb = 0, nslots = 0, npics = 0;
	int crop[4] = {0, 0, 0, 0};
	size_t fsz = 0;
	uint8_t *d_frames = nullptr, *d_rec = nullptr;
	int *d_prog = nullptr, *d_err = nullptr;
	m2dec_amd_trace_pic_t *pics = nullptr;
	/* timing: 4 events per enqueued picture (start, after inter, after intra, after deblock) */
	hipEvent_t *ev = nullptr;
	int ev_cap = 0, ev_used = 0;
	m2dec_amd_hip_timing_t tm;
};

static void replay_free(m2dec_amd_hip_replay_t *r)
{
	(void)hipSetDevice(r->dev);
	if (r->stream) (void)hipStreamSynchronize(r->stream);
	for (int i = 0; i < r->ev_cap; ++i) (void)hipEventDestroy(r->ev[i]);
	free(r->ev);
	free(r->pics);
	if (r->d_frames) (void)hipFree(r->d_frames);
	if (r->d_rec) (void)hipFree(r->d_rec);
	if (r->d_prog) (void)hipFree(r->d_prog);
	if (r->d_err) (void)hipFree(r->d_err);
	if (r->stream) (void)hipStreamDestroy(r->stream);
	delete r;
}

extern "C" int m2dec_amd_hip_replay_create(const m2dec_amd_trace_t *t, int device, m2dec_amd_hip_replay_t **out)
{
	int npics, W, H, nslots, nout;
	size_t len;
	if (!t || !out || !m2dec_amd_hip_available()) return -1;
	if (m2dec_amd_trace_info(t, &npics, &W, &H, &nslots, &nout) < 0 || npics <= 0 || W <= 0 || H <= 0) return -1;
	const uint8_t *rec = m2dec_amd_trace_records(t, &len);
	const m2dec_amd_trace_pic_t *pics = m2dec_amd_trace_pictures(t);
	for (int i = 0; i < npics; ++i)
		if (pics[i].slot < 0 || pics[i].slot >= nslots || pics[i].width_mbs != W / 16 || pics[i].height_mbs != H / 16) return -1;
	m2dec_amd_hip_replay_t *r = new m2dec_amd_hip_replay_t();
	memset(&r->tm, 0, sizeof(r->tm));
	r->dev = device;
	r->W = W;
	r->H = H;
	r->Wmb = W / 16;
	r->Hmb = H / 16;
	r->nslots = nslots;
	r->npics = npics;
	m2dec_amd_trace_crop(t, r->crop);
	r->fsz = ((size_t)W * H * 3 / 2 + 4095) & ~(size_t)4095;
	r->pics = (m2dec_amd_trace_pic_t *)malloc(sizeof(*pics) * (size_t)npics);
	memcpy(r->pics, pics, sizeof(*pics) * (size_t)npics);
#define RCHECK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "m2dec_amd replay: %s failed\n", #x); replay_free(r); return -1; } } while (0)
	RCHECK(hipSetDevice(device));
	RCHECK(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
	RCHECK(hipMalloc(&r->d_frames, r->fsz * (size_t)nslots));
	RCHECK(hipMemset(r->d_frames, 0, r->fsz * (size_t)nslots));
	RCHECK(hipMalloc(&r->d_rec, len));
	RCHECK(hipMemcpy(r->d_rec, rec, len, hipMemcpyHostToDevice));
	RCHECK(hipMalloc(&r->d_prog, sizeof(int) * 2 * (size_t)r->Hmb));
	RCHECK(hipMalloc(&r->d_err, sizeof(int)));
	RCHECK(hipMemset(r->d_err, 0, sizeof(int)));
#undef RCHECK
	*out = r;
	return 0;
}

static int replay_enqueue(m2dec_amd_hip_replay_t *r, int i, bool timed)
{
	const m2dec_amd_trace_pic_t &p = r->pics[i];
	RecPtrs rp;
	rp.mb = (const m2r_mb_t *)(r->d_rec + p.off_mb);
	rp.dbk = (const m2r_deblock_t *)(r->d_rec + p.off_dbk);
	rp.sl = (const m2r_slice_t *)(r->d_rec + p.off_slice);
	rp.it = (const m2r_inter_t *)(r->d_rec + p.off_inter);
	rp.coef = (const int16_t *)(r->d_rec + p.off_coef);
	Geometry gm{r->d_frames, r->fsz, r->W, r->H, r->Wmb, r->Hmb, r->d_prog, r->d_err};
	hipEvent_t *ev = nullptr;
	if (timed) {
		if (r->ev_used + 4 > r->ev_cap) {
			int nc = r->ev_cap ? r->ev_cap * 2 : 1024;
			hipEvent_t *ne = (hipEvent_t *)realloc(r->ev, sizeof(hipEvent_t) * (size_t)nc);
			if (!ne) return -1;
			r->ev = ne;
			for (int k = r->ev_cap; k < nc; ++k) CHECK(hipEventCreate(&r->ev[k]));
			r->ev_cap = nc;
		}
		ev = r->ev + r->ev_used;
		r->ev_used += 4;
		CHECK(hipEventRecord(ev[0], r->stream));
	}
	if (launch_picture(r->stream, gm, rp, p.slot, p.n_inter, p.n_intra, p.deblock, ev ? ev + 1 : nullptr, &r->tm) < 0) return -1;
	r->tm.pictures++;
	r->tm.record_bytes += p.record_bytes;
	r->tm.ref_bytes += p.ref_bytes;
	r->tm.frame_bytes += p.frame_bytes;
	return 0;
}

extern "C" int m2dec_amd_hip_replay_run(m2dec_amd_hip_replay_t *r, int passes)
{
	if (!r) return -1;
	CHECK(hipSetDevice(r->dev));
	for (int k = 0; k < passes; ++k)
		for (int i = 0; i < r->npics; ++i)
			if (replay_enqueue(r, i, true) < 0) return -1;
	return 0;
}

extern "C" int m2dec_amd_hip_replay_sync(m2dec_amd_hip_replay_t *r)
{
	int err = 0;
	if (!r) return -1;
	CHECK(hipSetDevice(r->dev));
	CHECK(hipStreamSynchronize(r->stream));
	CHECK(hipMemcpy(&err, r->d_err, sizeof(int), hipMemcpyDeviceToHost));
	if (err) {
		fprintf(stderr, "m2dec_amd replay: wavefront hand-off timed out (err=%d)\n", err);
		return -1;
	}
	return 0;
}

extern "C" int m2dec_amd_hip_replay_timing(m2dec_amd_hip_replay_t *r, m2dec_amd_hip_timing_t *out, int reset)
{
	if (!r || !out) return -1;
	CHECK(hipSetDevice(r->dev));
	for (int i = 0; i + 4 <= r->ev_used; i += 4) {
		float ms;
		hipEvent_t *e = r->ev + i;
		CHECK(hipEventSynchronize(e[3]));
		if (hipEventElapsedTime(&ms, e[0], e[1]) == hipSuccess) r->tm.inter_us += ms * 1e3;
		if (hipEventElapsedTime(&ms, e[1], e[2]) == hipSuccess) r->tm.intra_us += ms * 1e3;
		if (hipEventElapsedTime(&ms, e[2], e[3]) == hipSuccess) r->tm.deblock_us += ms * 1e3;
	}
	r->ev_used = 0;
	*out = r->tm;
	if (reset) memset(&r->tm, 0, sizeof(r->tm));
	return 0;
}

extern "C" int m2dec_amd_hip_replay_md5(m2dec_amd_hip_replay_t *r, char *md5s)
{
	if (!r || !md5s) return -1;
	size_t ls = (size_t)r->W * r->H;
	uint8_t *host = (uint8_t *)malloc(ls * 3 / 2);
	if (!host) return -1;
	CHECK(hipSetDevice(r->dev));
	for (int i = 0; i < r->npics; ++i) {
		if (replay_enqueue(r, i, false) < 0 || m2dec_amd_hip_replay_sync(r) < 0) {
			free(host);
			return -1;
		}
		if (hipMemcpy(host, r->d_frames + (size_t)r->pics[i].slot * r->fsz, ls * 3 / 2, hipMemcpyDeviceToHost) != hipSuccess) {
			free(host);
			return -1;
		}
		m2d_frame_t f;
		memset(&f, 0, sizeof(f));
		f.luma = host;
		f.chroma = host + ls;
		f.width = (int16_t)r->W;
		f.height = (int16_t)r->H;
		for (int k = 0; k < 4; ++k) f.crop[k] = (int16_t)r->crop[k];
		m2dec_amd_frame_md5(&f, md5s + 35 * (size_t)i);
	}
	free(host);
	return 0;
}

extern "C" void m2dec_amd_hip_replay_destroy(m2dec_amd_hip_replay_t *r)
{
	if (r) replay_free(r);
}
