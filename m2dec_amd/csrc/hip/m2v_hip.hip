/*
 * gfx950 reconstruction of MPEG-1/2 pictures (m2d_func with m2dec_amd_m2v_use_gpu): the records of
 * one picture (include/m2d_recon.h m2v_mb_t, made by m2dec_amd/csrc/host/mpeg2_dec.c) in, the
 * picture's NV12 samples in its device frame out.
 *
 * k_m2v: one 64-lane wave per macroblock — MPEG-2 has no prediction inside a picture, so every MB
 * of a picture is independent and a picture is one launch of n_mbs waves:
 *   1. prediction into LDS (384 bytes: 16x16 luma + 8 rows of 16 interleaved CbCr bytes), 6
 *      samples per lane: half-sample bilinear (motioncomp.cpp: copy, (a+b+1)>>1, (a+b+c+d+2)>>2),
 *      frame or field prediction, forward / backward / both averaged (a+b+1)>>1, chroma vectors
 *      halved toward zero (motioncomp.cpp:499-505);
 *   2. the coded blocks' coefficients into LDS, the integer Chen-Wang IDCT (idct.cpp:35-40, 69-236
 *      rows, 286-358 columns) as 48 row / column lanes, the result stored (intra) or added to the
 *      prediction (inter) with CLIP255C saturation (idct.cpp:364-422), luma placed per dct_type;
 *   3. the MB written out as whole 16-byte rows.
 * Reads of the reference frames are clamped to the frame (the reference has no bound: a conformant
 * stream never leaves it).  The bound is HBM: ~1.5 W H bytes written per picture plus 1.5 W H read per
 * prediction direction, and the records.
 *
 * Frames reach the caller only inside peek / get (m2v_hip_sync): device frame -> the context's
 * pinned staging buffer (asynchronous, behind the picture's kernel) -> the caller's frame, on the
 * caller's thread — the same ownership rule as the H.264 back end (runtime.hip).
 */
#include <hip/hip_runtime.h>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "m2d_recon.h"
#include "mpeg2_dec.h"

#define M2V_CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "m2dec_amd HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -1; } } while (0)

namespace {

struct M2vArgs {
	const m2v_mb_t *mb;
	const int16_t *coef;
	uint8_t *frames;    /* [slots] x fsz, NV12, stride W */
	size_t fsz;
	int W, H;
	int cur, fwd, bwd, copy;
	int n_mbs;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* one prediction sample of plane p (stride, w x h, gap bytes between horizontal neighbours) */
__device__ __forceinline__ int mc_px(const uint8_t *p, int stride, int w, int h, int gap, int x, int y, int hx, int hy)
{
	const int xa = clampi(x, 0, w - 1), ya = clampi(y, 0, h - 1);
	const int xb = clampi(x + gap * hx, 0, w - 1), yb = clampi(y + hy, 0, h - 1);
	const int a = p[ya * stride + xa], b = p[ya * stride + xb], c = p[yb * stride + xa], d = p[yb * stride + xb];
	if (hx && hy) return (a + b + c + d + 2) >> 2;
	if (hx) return (a + b + 1) >> 1;
	if (hy) return (a + c + 1) >> 1;
	return a;
}

/* prediction sample s (0..255 luma raster, 256..383 chroma bytes) of direction dir from ref */
__device__ int pred_sample(const uint8_t *ref, const M2vArgs &a, const m2v_mb_t &r, int dir, int s, bool zero_mv)
{
	const int W = a.W, H = a.H;
	const bool field = !zero_mv && (r.flags & M2V_REC_FIELD);
	if (s < 256) {
		const int i = s & 15, j = s >> 4;
		const int part = field ? (j & 1) : 0;
		const int mvx = zero_mv ? 0 : r.mv[dir][part][0], mvy = zero_mv ? 0 : r.mv[dir][part][1];
		if (field) {
			const int sel = (r.field_sel >> (2 * dir + part)) & 1;
			return mc_px(ref + sel * W, 2 * W, W, H / 2, 1, r.mbx * 16 + i + (mvx >> 1), r.mby * 8 + (j >> 1) + (mvy >> 1),
			             mvx & 1, mvy & 1);
		}
		return mc_px(ref, W, W, H, 1, r.mbx * 16 + i + (mvx >> 1), r.mby * 16 + j + (mvy >> 1), mvx & 1, mvy & 1);
	}
	{
		const uint8_t *cp = ref + (size_t)W * H;
		const int t = s - 256, i = t & 15, j = t >> 4;
		const int part = field ? (j & 1) : 0;
		const int mvx = zero_mv ? 0 : r.mv[dir][part][0], mvy = zero_mv ? 0 : r.mv[dir][part][1];
		const int cx = mvx / 2, cy = mvy / 2;
		if (field) {
			const int sel = (r.field_sel >> (2 * dir + part)) & 1;
			return mc_px(cp + sel * W, 2 * W, W, H / 4, 2, r.mbx * 16 + i + 2 * (cx >> 1), r.mby * 4 + (j >> 1) + (cy >> 1),
			             cx & 1, cy & 1);
		}
		return mc_px(cp, W, W, H / 2, 2, r.mbx * 16 + i + 2 * (cx >> 1), r.mby * 8 + j + (cy >> 1), cx & 1, cy & 1);
	}
}

#define W1 2841
#define W2 2676
#define W3 2408
#define W5 1609
#define W6 1108
#define W7 565

/* idct.cpp:69-236: one row in place (int16) */
__device__ __forceinline__ void idct_row(int16_t *s)
{
	const int s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3], s4 = s[4], s5 = s[5], s6 = s[6], s7 = s[7];
	const int a0 = s0 * 2048 + 128, a1 = s4 * 2048;
	int e0 = a0 - a1, e1 = a0 + a1;
	const int o4 = W7 * (s1 + s7) + (W1 - W7) * s1;
	const int o5 = W7 * (s1 + s7) - (W1 + W7) * s7;
	const int o6 = W3 * (s5 + s3) - (W3 - W5) * s5;
	const int o7 = W3 * (s5 + s3) - (W3 + W5) * s3;
	const int p4 = o4 - o6, p6 = o4 + o6, p5 = o5 - o7, p7 = o5 + o7;
	const int q5 = ((p4 + p5) * 181 + 128) >> 8;
	const int q4 = ((p4 - p5) * 181 + 128) >> 8;
	int x2 = W6 * (s2 + s6) - (W2 + W6) * s6;
	int x3 = W6 * (s2 + s6) + (W2 - W6) * s2;
	int t = e0;
	e0 = e0 - x2;
	x2 = t + x2;
	t = e1;
	e1 = e1 - x3;
	x3 = t + x3;
	s[0] = (int16_t)((x3 + p6) >> 8);
	s[1] = (int16_t)((x2 + q5) >> 8);
	s[2] = (int16_t)((e0 + q4) >> 8);
	s[3] = (int16_t)((e1 + p7) >> 8);
	s[4] = (int16_t)((e1 - p7) >> 8);
	s[5] = (int16_t)((e0 - q4) >> 8);
	s[6] = (int16_t)((x2 - q5) >> 8);
	s[7] = (int16_t)((x3 - p6) >> 8);
}

/* idct.cpp:286-358: one column, the 8 outputs (x + 8192) >> 14 */
__device__ __forceinline__ void idct_col(const int16_t *c, int v[8])
{
	const int s0 = c[0], s1 = c[8], s2 = c[16], s3 = c[24], s4 = c[32], s5 = c[40], s6 = c[48], s7 = c[56];
	int x8 = W3 * (s5 + s3) + 4;
	const int x6a = (x8 - (W3 - W5) * s5) >> 3, x7a = (x8 - (W3 + W5) * s3) >> 3;
	x8 = W7 * (s1 + s7) + 4;
	const int x4a = (x8 + (W1 - W7) * s1) >> 3, x5a = (x8 - (W1 + W7) * s7) >> 3;
	int x1 = W6 * (s2 + s6) + 4;
	const int x2 = (x1 - (W2 + W6) * s6) >> 3, x3 = (x1 + (W2 - W6) * s2) >> 3;
	x1 = x4a + x6a;
	const int x4 = x4a - x6a, x6 = x5a + x7a, x5 = x5a - x7a;
	int x0 = s0 * 256 + 8192;
	const int x7 = s4 * 256;
	x8 = x0 + x7;
	x0 = x0 - x7;
	const int y7 = x8 + x3, y8 = x8 - x3, y3 = x0 + x2, y0 = x0 - x2;
	const int z2 = ((x4 + x5) * 181 + 128) >> 8, z4 = ((x4 - x5) * 181 + 128) >> 8;
	v[0] = (y7 + x1) >> 14;
	v[1] = (y3 + z2) >> 14;
	v[2] = (y0 + z4) >> 14;
	v[3] = (y8 + x6) >> 14;
	v[4] = (y8 - x6) >> 14;
	v[5] = (y0 - z4) >> 14;
	v[6] = (y3 - z2) >> 14;
	v[7] = (y7 - x1) >> 14;
}

__global__ __launch_bounds__(64) void k_m2v(const M2vArgs *args)
{
	const M2vArgs a = *args;
	const int k = blockIdx.x, lane = threadIdx.x;
	__shared__ uint8_t pred[384];
	__shared__ int16_t coef[6][64];
	if (k >= a.n_mbs) return;
	const m2v_mb_t r = a.mb[k];
	if (!r.flags) return;
	const bool copy = (r.flags & M2V_REC_COPY) != 0;
	if (copy && (a.copy < 0 || a.copy == a.cur)) return; /* (in place: nothing to do) */
	uint8_t *cur = a.frames + (size_t)a.cur * a.fsz;
	const int W = a.W;
	/* 1. prediction */
	{
		const uint8_t *f = copy ? a.frames + (size_t)a.copy * a.fsz
		                        : a.frames + (size_t)(a.fwd < 0 ? a.cur : a.fwd) * a.fsz;
		const uint8_t *b = a.frames + (size_t)(a.bwd < 0 ? a.cur : a.bwd) * a.fsz;
		for (int s = lane; s < 384; s += 64) {
			int v = 0;
			if (copy) {
				v = pred_sample(f, a, r, 0, s, true);
			} else if (!(r.flags & M2V_REC_INTRA)) {
				const bool fw = r.flags & M2V_REC_FWD, bw = r.flags & M2V_REC_BWD;
				if (fw) v = pred_sample(f, a, r, 0, s, false);
				if (bw) {
					const int vb = pred_sample(b, a, r, 1, s, false);
					v = fw ? (v + vb + 1) >> 1 : vb;
				}
			}
			pred[s] = (uint8_t)v;
		}
	}
	/* 2. residual */
	if (!copy && r.cbp) {
		/* coefficients of the coded blocks (in block order in the pool) */
		{
			int base = 0;
			for (int i = 0; i < 6; ++i) {
				if (!(r.cbp & (1 << (5 - i)))) continue;
				coef[i][lane] = a.coef[r.coef + base + lane];
				base += 64;
			}
		}
		__syncthreads();
		if (lane < 48) {
			const int i = lane >> 3, row = lane & 7;
			if (r.cbp & (1 << (5 - i))) idct_row(&coef[i][row * 8]);
		}
		__syncthreads();
		if (lane < 48) {
			const int i = lane >> 3, col = lane & 7;
			if (r.cbp & (1 << (5 - i))) {
				const bool add = !(r.flags & M2V_REC_INTRA), fld = (r.flags & M2V_REC_DCT_FIELD) != 0;
				int v[8];
				idct_col(&coef[i][col], v);
				for (int y = 0; y < 8; ++y) {
					int idx;
					if (i < 4) { /* LUMA_BLOCK_OFFSET (mpeg2.cpp:1120) */
						const int row = fld ? ((i >> 1) + 2 * y) : ((i >> 1) * 8 + y);
						idx = row * 16 + (i & 1) * 8 + col;
					} else {
						idx = 256 + y * 16 + 2 * col + (i - 4);
					}
					const int t = add ? pred[idx] + v[y] : v[y];
					pred[idx] = (uint8_t)clampi(t, 0, 255); /* CLIP255C */
				}
			}
		}
	}
	__syncthreads();
	/* 3. out: 24 rows of 16 bytes, one 16-bit pair per lane per step */
	for (int s = lane; s < 192; s += 64) {
		const int row = s >> 3, off = (s & 7) * 2;
		uint8_t *d = row < 16 ? cur + (size_t)(r.mby * 16 + row) * W + r.mbx * 16 + off
		                      : cur + (size_t)W * a.H + (size_t)(r.mby * 8 + row - 16) * W + r.mbx * 16 + off;
		const int p = row * 16 + off;
		*(uint16_t *)d = (uint16_t)(pred[p] | (pred[p + 1] << 8));
	}
}

struct M2vGpu {
	int dev = 0;
	hipStream_t st = nullptr;
	int W = 0, H = 0, n = 0;
	size_t fsz = 0;
	uint8_t *frames = nullptr;
	m2d_frame_t caller[M2V_MAX_FRAMES];
	uint8_t *stg[M2V_MAX_FRAMES] = {};
	hipEvent_t ev[M2V_MAX_FRAMES] = {};
	bool pend[M2V_MAX_FRAMES] = {};
	/* two record arenas (pinned host + device) used in turn; `used` fires when a launch is done with one */
	struct Arena {
		uint8_t *host = nullptr, *dev = nullptr;
		size_t size = 0;
		M2vArgs *args = nullptr;
		hipEvent_t used = nullptr;
		hipEvent_t t0 = nullptr, t1 = nullptr; /* timing: around the launch that used this arena last */
		bool timed = false;
	} ar[2];
	int next = 0;
};

/* Process-wide kernel timing of the MPEG-2 back end (bench.py end_to_end_m2v): HIP-event time of the
 * k_m2v launches and SURVEY.md §8d algorithmic bytes of their pictures (F_write 1.5 W H, the records and
 * coefficients read, one reference byte per predicted sample per direction). */
struct M2vTiming {
	std::mutex mu;
	double kernel_us = 0;
	int64_t pictures = 0, bytes = 0;
} g_m2v_tm;

void arena_account(M2vGpu::Arena &a)
{
	float ms = 0;
	if (!a.timed) return;
	a.timed = false;
	if (hipEventElapsedTime(&ms, a.t0, a.t1) != hipSuccess) return;
	std::lock_guard<std::mutex> lk(g_m2v_tm.mu);
	g_m2v_tm.kernel_us += ms * 1e3;
}

int arena_fit(M2vGpu *g, M2vGpu::Arena &a, size_t need)
{
	if (a.size >= need) return 0;
	if (a.host) (void)hipHostFree(a.host);
	if (a.dev) (void)hipFree(a.dev);
	a.host = a.dev = nullptr;
	M2V_CHECK(hipHostMalloc((void **)&a.host, need, hipHostMallocDefault));
	M2V_CHECK(hipMalloc((void **)&a.dev, need));
	a.size = need;
	(void)g;
	return 0;
}

} // namespace

extern "C" void *m2v_hip_create(int device)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return nullptr;
	M2vGpu *g = new M2vGpu();
	g->dev = device;
	if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking) != hipSuccess) {
		delete g;
		return nullptr;
	}
	for (int i = 0; i < M2V_MAX_FRAMES; ++i) (void)hipEventCreateWithFlags(&g->ev[i], hipEventDisableTiming);
	for (auto &a : g->ar) {
		(void)hipEventCreateWithFlags(&a.used, hipEventDisableTiming);
		(void)hipEventCreate(&a.t0);
		(void)hipEventCreate(&a.t1);
		(void)hipMalloc((void **)&a.args, sizeof(M2vArgs));
	}
	return g;
}

extern "C" int m2v_hip_set_frames(void *p, int n, const m2d_frame_t *frames, int width, int height)
{
	M2vGpu *g = (M2vGpu *)p;
	if (!g || n <= 0 || n > M2V_MAX_FRAMES || width <= 0 || height <= 0) return -1;
	M2V_CHECK(hipSetDevice(g->dev));
	M2V_CHECK(hipStreamSynchronize(g->st));
	const size_t fsz = ((size_t)width * height * 3 / 2 + 4095) & ~(size_t)4095;
	if (!g->frames || fsz != g->fsz || n > g->n) {
		if (g->frames) (void)hipFree(g->frames);
		g->frames = nullptr;
		M2V_CHECK(hipMalloc((void **)&g->frames, fsz * (size_t)n));
		M2V_CHECK(hipMemset(g->frames, 0, fsz * (size_t)n));
	}
	for (int i = 0; i < M2V_MAX_FRAMES; ++i) {
		if (g->stg[i] && ((size_t)width * height * 3 / 2 != (size_t)g->W * g->H * 3 / 2 || i >= n)) {
			(void)hipHostFree(g->stg[i]);
			g->stg[i] = nullptr;
		}
		g->pend[i] = false; /* (frames handed to a new set_frames start unwritten, as in the reference) */
	}
	g->fsz = fsz;
	g->n = n;
	g->W = width;
	g->H = height;
	memcpy(g->caller, frames, sizeof(m2d_frame_t) * (size_t)n);
	return 0;
}

extern "C" int m2v_hip_submit(void *p, const m2v_picture_t *pic)
{
	M2vGpu *g = (M2vGpu *)p;
	if (!g || !g->frames || pic->width != g->W || pic->height != g->H || pic->cur < 0 || pic->cur >= g->n ||
	    pic->fwd >= g->n || pic->bwd >= g->n || pic->copy >= g->n || pic->n_mbs != (g->W / 16) * (g->H / 16))
		return -1;
	for (int i = 0; i < pic->n_mbs; ++i) /* (a record's coefficients must lie inside the pool) */
		if (pic->mb[i].cbp && (int64_t)pic->mb[i].coef + 64 * __builtin_popcount(pic->mb[i].cbp & 63) > (int64_t)pic->n_coef)
			return -1;
	M2V_CHECK(hipSetDevice(g->dev));
	M2vGpu::Arena &a = g->ar[g->next];
	g->next ^= 1;
	M2V_CHECK(hipEventSynchronize(a.used)); /* the launch before last is done with this arena */
	arena_account(a);
	const size_t rb = sizeof(m2v_mb_t) * (size_t)pic->n_mbs, cb = sizeof(int16_t) * (size_t)pic->n_coef;
	if (arena_fit(g, a, rb + cb + 256) < 0) return -1;
	memcpy(a.host, pic->mb, rb);
	memcpy(a.host + rb, pic->coef, cb);
	M2vArgs h;
	h.mb = (const m2v_mb_t *)a.dev;
	h.coef = (const int16_t *)(a.dev + rb);
	h.frames = g->frames;
	h.fsz = g->fsz;
	h.W = g->W;
	h.H = g->H;
	h.cur = pic->cur;
	h.fwd = pic->fwd;
	h.bwd = pic->bwd;
	h.copy = pic->copy;
	h.n_mbs = pic->n_mbs;
	M2V_CHECK(hipMemcpyAsync(a.dev, a.host, rb + cb, hipMemcpyHostToDevice, g->st));
	M2V_CHECK(hipMemcpyAsync(a.args, &h, sizeof(h), hipMemcpyHostToDevice, g->st));
	M2V_CHECK(hipEventRecord(a.t0, g->st));
	hipLaunchKernelGGL(k_m2v, dim3(pic->n_mbs), dim3(64), 0, g->st, (const M2vArgs *)a.args);
	M2V_CHECK(hipGetLastError());
	M2V_CHECK(hipEventRecord(a.t1, g->st));
	M2V_CHECK(hipEventRecord(a.used, g->st));
	a.timed = true;
	{
		int64_t refb = 0;
		for (int i = 0; i < pic->n_mbs; ++i) {
			const unsigned f = pic->mb[i].flags;
			refb += 384 * (((f & M2V_REC_FWD) != 0) + ((f & M2V_REC_BWD) != 0) + ((f & M2V_REC_COPY) != 0));
		}
		std::lock_guard<std::mutex> lk(g_m2v_tm.mu);
		g_m2v_tm.pictures++;
		g_m2v_tm.bytes += (int64_t)(rb + cb) + refb + (int64_t)g->W * g->H * 3 / 2;
	}
	/* the picture to its staging buffer, behind the kernel */
	const int c = pic->cur;
	const size_t bytes = (size_t)g->W * g->H * 3 / 2;
	if (!g->stg[c]) M2V_CHECK(hipHostMalloc((void **)&g->stg[c], bytes, hipHostMallocDefault));
	M2V_CHECK(hipMemcpyAsync(g->stg[c], g->frames + (size_t)c * g->fsz, bytes, hipMemcpyDeviceToHost, g->st));
	M2V_CHECK(hipEventRecord(g->ev[c], g->st));
	g->pend[c] = true;
	return 0;
}

/* the picture of `slot` into the caller's frame, on the caller's thread */
extern "C" int m2v_hip_sync(void *p, int slot)
{
	M2vGpu *g = (M2vGpu *)p;
	if (!g || slot < 0 || slot >= M2V_MAX_FRAMES) return -1;
	if (!g->pend[slot]) return 0;
	M2V_CHECK(hipEventSynchronize(g->ev[slot]));
	const size_t ls = (size_t)g->W * g->H;
	memcpy(g->caller[slot].luma, g->stg[slot], ls);
	memcpy(g->caller[slot].chroma, g->stg[slot] + ls, ls / 2);
	g->pend[slot] = false;
	return 0;
}

extern "C" void m2v_hip_destroy(void *p)
{
	M2vGpu *g = (M2vGpu *)p;
	if (!g) return;
	(void)hipSetDevice(g->dev);
	(void)hipStreamSynchronize(g->st);
	for (auto &a : g->ar) {
		arena_account(a);
		if (a.t0) (void)hipEventDestroy(a.t0);
		if (a.t1) (void)hipEventDestroy(a.t1);
		if (a.host) (void)hipHostFree(a.host);
		if (a.dev) (void)hipFree(a.dev);
		if (a.args) (void)hipFree(a.args);
		if (a.used) (void)hipEventDestroy(a.used);
	}
	for (int i = 0; i < M2V_MAX_FRAMES; ++i) {
		if (g->stg[i]) (void)hipHostFree(g->stg[i]);
		if (g->ev[i]) (void)hipEventDestroy(g->ev[i]);
	}
	if (g->frames) (void)hipFree(g->frames);
	(void)hipStreamDestroy(g->st);
	delete g;
}

/* kernel time and algorithmic bytes of the k_m2v launches since the last reset (destroyed back ends
 * included; a live one's last two launches are counted when their arenas are reused or it is destroyed) */
extern "C" int m2dec_amd_m2v_hip_timing(double *kernel_us, int64_t *pictures, int64_t *bytes, int reset)
{
	std::lock_guard<std::mutex> lk(g_m2v_tm.mu);
	if (kernel_us) *kernel_us = g_m2v_tm.kernel_us;
	if (pictures) *pictures = g_m2v_tm.pictures;
	if (bytes) *bytes = g_m2v_tm.bytes;
	if (reset) {
		g_m2v_tm.kernel_us = 0;
		g_m2v_tm.pictures = g_m2v_tm.bytes = 0;
	}
	return 0;
}
