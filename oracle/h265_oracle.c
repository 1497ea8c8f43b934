/*
 * TEST INFRASTRUCTURE ONLY — the CPU oracle of the H.265 reconstruction.  Only tests/, smoke() and
 * bench.py's cpu_baseline leg load it; the product path (libm2dec_amd.so) never links it.
 *
 * A plain-C restatement of the reference decoder's reconstruction of an intra picture over the records
 * of include/m2d_recon.h (h265r_*), as an h265r_backend_t writing straight into the caller's frames:
 *   - intra prediction (h265.cpp:2297-2913): reference-sample substitution, [1 2 1] / strong (bilinear)
 *     smoothing, planar, DC with its edge filters, the 33 angular modes with the mode 10 / 26 edge
 *     filters, chroma without filtering — spec 8.4.4.2, to which the reference's code is equal;
 *   - the residual (h265.cpp:1693-2167, h265_x86.cpp): the 2-D inverse DCT / DST with the int16 clip
 *     after each stage, transform skip ((c + 16) >> 5), and the reference's DC-only shortcut
 *     acNxNtransform_dconly<N, 7> (m2d.h:306-341): (dc + 64) >> 7 added to every sample — NOT the
 *     two-stage rounding of the full transform (a reference quirk);
 *   - deblocking (h265.cpp:4125-4384) over the picture, vertical edges first: the luma tc QP clipped to
 *     51 instead of 53 (deblocking_edge_luma_block, a reference quirk), chroma only on bS 2 edges;
 *   - SAO (h265.cpp:4386-4729) on the deblocked picture: band offset without the band-table wrap of
 *     the spec (sao_bo_block, a reference quirk), edge offset skipping samples whose neighbour lies
 *     outside the picture.
 *   - motion compensation of P / B pictures (h265.cpp:3132-3595), before the picture's transform blocks:
 *     luma with the 8-tap quarter-sample filters and clamped reference positions (the reference's
 *     fir1 / fir2 / fir3 and its 1-D / 2-D paths, whose integers equal spec 8.5.3.3.3.1), chroma with
 *     the reference's packed two-component uint64 arithmetic restated literally (interp_chroma*: Cb in
 *     the high half, Cr in the low half behind a 0x80000000 guard and the & ~0xf8000000 mask, which
 *     does not hold a negative horizontal Cr sum apart from the Cb half — kept as it is), default
 *     weighted bi-prediction (store_pix<0> into int16, then add_store_pix);
 * Every CLIP255C argument outside the reference table's domain [-256, 767] (m2d.cpp:157-289) and
 * every DC-only term the reference's byte-wise SWAR add would corrupt (|dc| > 255) is counted:
 * golden streams must have none.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "m2d.h"
#include "m2d_recon.h"

static uint64_t g_violations;

uint64_t h265_oracle_violations(int reset)
{
	const uint64_t v = g_violations;
	if (reset) g_violations = 0;
	return v;
}

static inline int clip255c(int v)
{
	if (v < -256 || v > 767) g_violations++;
	return v < 0 ? 0 : (v > 255 ? 255 : v);
}

static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int16_t sat16(int v) { return (int16_t)clip3(-32768, 32767, v); }

/* ------------------------------------------------------------------ transforms */
static int mat32[32][32];
static const int dst4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};

/* the DCT matrices (spec 8.6.4.2, eq. 8-315): T_N[k][n] = 64 sqrt(2) cos((2n + 1) k pi / 2N) as tabulated */
static void build_mat(void)
{
	static const int c[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
	                          61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
	for (int k = 0; k < 32; ++k)
		for (int n = 0; n < 32; ++n) {
			int m = ((2 * n + 1) * k) % 128, sign = 1;
			if (m > 64) m = 128 - m;
			if (m > 32) {
				m = 64 - m;
				sign = -1;
			}
			mat32[k][n] = sign * c[m];
		}
}

/* T_N[k][n] = T_32[k * 32 / N][n] */
static inline int tm(int log2, int k, int n) { return mat32[k << (5 - log2)][n]; }

/* residual of one block: r[y * n + x] */
static void residual(const int16_t *d, int log2, int kind, int *r)
{
	const int n = 1 << log2;
	if (kind == H265R_RES_NONE) {
		memset(r, 0, sizeof(int) * (size_t)(n * n));
		return;
	}
	if (kind == H265R_RES_SKIP) {
		for (int i = 0; i < n * n; ++i) r[i] = (d[i] + 16) >> 5;
		return;
	}
	if (kind == H265R_RES_DC) {
		const int dc = (d[0] + 64) >> 7;
		if (dc > 255 || dc < -255) g_violations++;
		for (int i = 0; i < n * n; ++i) r[i] = dc;
		return;
	}
	{
		int g[32 * 32];
		const int dstm = kind == H265R_RES_DST;
		/* columns (vertical frequencies j), then rows */
		for (int x = 0; x < n; ++x)
			for (int y = 0; y < n; ++y) {
				int e = 0;
				for (int j = 0; j < n; ++j) e += (dstm ? dst4[j][y] : tm(log2, j, y)) * d[j * n + x];
				g[y * n + x] = sat16((e + 64) >> 7);
			}
		for (int y = 0; y < n; ++y)
			for (int x = 0; x < n; ++x) {
				int e = 0;
				for (int j = 0; j < n; ++j) e += (dstm ? dst4[j][x] : tm(log2, j, x)) * g[y * n + j];
				r[y * n + x] = sat16((e + 2048) >> 12);
			}
	}
}

/* ------------------------------------------------------------------ intra prediction (8.4.4.2) */
typedef struct {
	uint8_t *base;  /* plane origin (chroma: the component's first byte) */
	int stride, step;
} plane_t;

#define PX(pl, x, y) ((pl)->base[(size_t)(y) * (size_t)(pl)->stride + (size_t)(x) * (size_t)(pl)->step])

static void intra_pred(const plane_t *pl, int x0, int y0, int log2, int mode, int at, int al, int luma, int strong_en, int *pred)
{
	const int n = 1 << log2;
	int ref[2][65]; /* [0]: left column p[-1][-1 + i], [1]: top row p[-1 + i][-1]; index 0 = corner */
	int avl[2][65];
	const int top_ok = at > 0, left_ok = al > 0;
	/* availability */
	avl[0][0] = avl[1][0] = top_ok && left_ok;
	for (int i = 1; i <= 2 * n; ++i) {
		avl[0][i] = left_ok && (i - 1) < al;
		avl[1][i] = top_ok && (i - 1) < at;
		ref[0][i] = avl[0][i] ? PX(pl, x0 - 1, y0 + i - 1) : 0;
		ref[1][i] = avl[1][i] ? PX(pl, x0 + i - 1, y0 - 1) : 0;
	}
	ref[0][0] = ref[1][0] = avl[0][0] ? PX(pl, x0 - 1, y0 - 1) : 0;
	/* substitution (8.4.4.2.2): order p[-1][2n-1] .. p[-1][-1], p[0][-1] .. p[2n-1][-1] */
	{
		int seq[129], ok[129], cnt = 0, any = 0;
		for (int i = 2 * n; i >= 1; --i) {
			seq[cnt] = ref[0][i];
			ok[cnt++] = avl[0][i];
		}
		seq[cnt] = ref[0][0];
		ok[cnt++] = avl[0][0];
		for (int i = 1; i <= 2 * n; ++i) {
			seq[cnt] = ref[1][i];
			ok[cnt++] = avl[1][i];
		}
		for (int i = 0; i < cnt; ++i) any |= ok[i];
		if (!any) {
			for (int i = 0; i < cnt; ++i) seq[i] = 128;
		} else {
			if (!ok[0]) {
				for (int i = 1; i < cnt; ++i)
					if (ok[i]) {
						seq[0] = seq[i];
						break;
					}
			}
			for (int i = 1; i < cnt; ++i)
				if (!ok[i]) seq[i] = seq[i - 1];
		}
		/* filtering (8.4.4.2.3): luma only */
		if (luma && mode != 1 && n != 4) {
			const int dist = abs(mode - 26) < abs(mode - 10) ? abs(mode - 26) : abs(mode - 10);
			const int thres = n == 8 ? 7 : (n == 16 ? 1 : 0);
			if (mode == 0 || dist > thres) {
				int f[129];
				const int last = cnt - 1; /* seq[0] = p[-1][2n-1], seq[2n] = corner, seq[last] = p[2n-1][-1] */
				const int corner = 2 * n;
				const int bl = seq[0], tr = seq[last], c = seq[corner];
				if (strong_en && n == 32 && abs(c + tr - 2 * seq[corner + n]) < 8 && abs(c + bl - 2 * seq[corner - n]) < 8) {
					for (int i = 0; i <= last; ++i) f[i] = seq[i];
					for (int y = 0; y <= 62; ++y) f[corner - 1 - y] = ((63 - y) * c + (y + 1) * bl + 32) >> 6;
					for (int xx = 0; xx <= 62; ++xx) f[corner + 1 + xx] = ((63 - xx) * c + (xx + 1) * tr + 32) >> 6;
				} else {
					f[0] = seq[0];
					f[last] = seq[last];
					for (int i = 1; i < last; ++i) f[i] = (seq[i - 1] + 2 * seq[i] + seq[i + 1] + 2) >> 2;
				}
				memcpy(seq, f, sizeof(int) * (size_t)cnt);
			}
		}
		for (int i = 2 * n; i >= 1; --i) ref[0][i] = seq[2 * n - i];
		ref[0][0] = ref[1][0] = seq[2 * n];
		for (int i = 1; i <= 2 * n; ++i) ref[1][i] = seq[2 * n + i];
	}
#define L(y) ref[0][(y) + 1] /* p[-1][y], y >= -1 */
#define T(x) ref[1][(x) + 1] /* p[x][-1], x >= -1 */
	if (mode == 0) {
		for (int y = 0; y < n; ++y)
			for (int x = 0; x < n; ++x)
				pred[y * n + x] = ((n - 1 - x) * L(y) + (x + 1) * T(n) + (n - 1 - y) * T(x) + (y + 1) * L(n) + n) >> (log2 + 1);
		return;
	}
	if (mode == 1) {
		int s = n;
		for (int i = 0; i < n; ++i) s += T(i) + L(i);
		const int dc = s >> (log2 + 1);
		for (int i = 0; i < n * n; ++i) pred[i] = dc;
		if (luma && n < 32) {
			pred[0] = (L(0) + 2 * dc + T(0) + 2) >> 2;
			for (int x = 1; x < n; ++x) pred[x] = (T(x) + 3 * dc + 2) >> 2;
			for (int y = 1; y < n; ++y) pred[y * n] = (L(y) + 3 * dc + 2) >> 2;
		}
		return;
	}
	{
		static const int ang[35] = {0,  0,  32, 26, 21, 17, 13, 9,  5,  2,   0,   -2,  -5,  -9,  -13, -17, -21, -26,
		                            -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
		static const int inv[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482, -390, -315,
		                            -256, -315, -390, -482, -630, -910, -1638, -4096, 0, 0, 0, 0, 0, 0, 0, 0, 0};
		const int a = ang[mode];
		int rr[3 * 64 + 1], *r = rr + 64; /* r[-n .. 2n] */
		const int vert = mode >= 18;
		for (int i = 0; i <= 2 * n; ++i) r[i] = vert ? T(i - 1) : L(i - 1);
		if (a < 0 && ((n * a) >> 5) < -1)
			for (int xx = (n * a) >> 5; xx <= -1; ++xx) r[xx] = vert ? L(-1 + ((xx * inv[mode] + 128) >> 8)) : T(-1 + ((xx * inv[mode] + 128) >> 8));
		for (int y = 0; y < n; ++y)
			for (int x = 0; x < n; ++x) {
				const int p = vert ? y : x, q = vert ? x : y;
				const int idx = ((p + 1) * a) >> 5, fr = ((p + 1) * a) & 31;
				const int v = fr ? ((32 - fr) * r[q + idx + 1] + fr * r[q + idx + 2] + 16) >> 5 : r[q + idx + 1];
				pred[y * n + x] = v;
			}
		if (luma && n < 32) {
			if (mode == 26)
				for (int y = 0; y < n; ++y) pred[y * n] = clip255c(T(0) + ((L(y) - L(-1)) >> 1));
			if (mode == 10)
				for (int x = 0; x < n; ++x) pred[x] = clip255c(L(0) + ((T(x) - T(-1)) >> 1));
		}
	}
#undef L
#undef T
}

/* ------------------------------------------------------------------ deblocking (8.7.2) */
static const uint8_t beta_tab[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                     8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                     34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
static const uint8_t tc_tab[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

/* one luma edge segment of 4 lines: s points at q0 of line 0; xs = step across the edge, ls = step along */
static void luma_edge(uint8_t *s, int xs, int ls, int bs, int qp, int beta_off, int tc_off)
{
	const int bq = clip3(0, 51, qp + beta_off);
	const int tq = clip3(0, 51, qp + 2 * (bs - 1) + tc_off); /* reference: clipped to 51 */
	const int beta = beta_tab[bq], tc = tc_tab[tq];
#define P(i, k) s[(k) * ls - ((i) + 1) * xs]
#define Q(i, k) s[(k) * ls + (i) * xs]
	const int dp0 = abs(P(2, 0) - 2 * P(1, 0) + P(0, 0)), dp3 = abs(P(2, 3) - 2 * P(1, 3) + P(0, 3));
	const int dq0 = abs(Q(2, 0) - 2 * Q(1, 0) + Q(0, 0)), dq3 = abs(Q(2, 3) - 2 * Q(1, 3) + Q(0, 3));
	const int d = dp0 + dq0 + dp3 + dq3;
	if (!(d < beta)) return;
	{
		int strong = 1;
		for (int k = 0; k < 4; k += 3) {
			const int dpq = 2 * ((k ? dp3 : dp0) + (k ? dq3 : dq0));
			if (!(dpq < (beta >> 2) && abs(P(3, k) - P(0, k)) + abs(Q(0, k) - Q(3, k)) < (beta >> 3) &&
			      abs(P(0, k) - Q(0, k)) < ((5 * tc + 1) >> 1)))
				strong = 0;
		}
		const int dep = (dp0 + dp3) < ((beta + (beta >> 1)) >> 3), deq = (dq0 + dq3) < ((beta + (beta >> 1)) >> 3);
		for (int k = 0; k < 4; ++k) {
			const int p0 = P(0, k), p1 = P(1, k), p2 = P(2, k), p3 = P(3, k);
			const int q0 = Q(0, k), q1 = Q(1, k), q2 = Q(2, k), q3 = Q(3, k);
			if (strong) {
				const int t2 = 2 * tc;
				P(0, k) = (uint8_t)clip3(p0 - t2, p0 + t2, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
				P(1, k) = (uint8_t)clip3(p1 - t2, p1 + t2, (p2 + p1 + p0 + q0 + 2) >> 2);
				P(2, k) = (uint8_t)clip3(p2 - t2, p2 + t2, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
				Q(0, k) = (uint8_t)clip3(q0 - t2, q0 + t2, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
				Q(1, k) = (uint8_t)clip3(q1 - t2, q1 + t2, (p0 + q0 + q1 + q2 + 2) >> 2);
				Q(2, k) = (uint8_t)clip3(q2 - t2, q2 + t2, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
			} else {
				int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
				if (abs(delta) < tc * 10) {
					delta = clip3(-tc, tc, delta);
					P(0, k) = (uint8_t)clip255c(p0 + delta);
					Q(0, k) = (uint8_t)clip255c(q0 - delta);
					if (dep) P(1, k) = (uint8_t)clip255c(p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1));
					if (deq) Q(1, k) = (uint8_t)clip255c(q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1));
				}
			}
		}
	}
#undef P
#undef Q
}

static int qpc_deb(int qpi)
{
	/* qpi_to_qpc_deb (h265.cpp:4279-4288) */
	if (qpi < 30) return qpi;
	if (qpi >= 43) return qpi - 6;
	static const int8_t t[13] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37};
	return t[qpi - 30];
}

/* one chroma component, 2 lines: s at q0 of line 0 */
static void chroma_edge(uint8_t *s, int xs, int ls, int qp, int qp_off, int tc_off)
{
	const int q = clip3(0, 53, qpc_deb(qp + qp_off) + 2 + tc_off);
	const int tc = tc_tab[q];
	if (q < 16) return;
	for (int k = 0; k < 2; ++k) {
		uint8_t *l = s + k * ls;
		const int p1 = l[-2 * xs], p0 = l[-xs], q0 = l[0], q1 = l[xs];
		const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
		if (delta) {
			l[-xs] = (uint8_t)clip255c(p0 + delta);
			l[0] = (uint8_t)clip255c(q0 - delta);
		}
	}
}

static void deblock(const h265r_picture_t *pic, uint8_t *luma, uint8_t *chroma)
{
	const int W = pic->width, H = pic->height;
	for (int dir = 0; dir < 2; ++dir) {
		const uint8_t *bs = dir ? pic->bs_h : pic->bs_v;
		const int rows = dir ? H / 8 : H / 4, cols = dir ? W / 4 : W / 8;
		for (int j = 0; j < rows; ++j)
			for (int i = 0; i < cols; ++i) {
				const int v = bs[(size_t)j * (size_t)cols + (size_t)i], b = v & 3, qp = v >> 2;
				if (!b) continue;
				const int ex = dir ? 4 * i : 8 * i, ey = dir ? 8 * j : 4 * j; /* luma edge segment origin (q side) */
				if (dir == 0) luma_edge(luma + (size_t)ey * (size_t)W + (size_t)ex, 1, W, b, qp, pic->beta_offset, pic->tc_offset);
				else luma_edge(luma + (size_t)ey * (size_t)W + (size_t)ex, W, 1, b, qp, pic->beta_offset, pic->tc_offset);
				if (b == 2 && ((dir == 0 ? ex : ey) & 15) == 0) {
					/* chroma: the 2 chroma lines of this luma segment, both components */
					const int cx = ex >> 1, cy = ey >> 1;
					for (int c = 0; c < 2; ++c) {
						uint8_t *s = chroma + (size_t)cy * (size_t)W + (size_t)(2 * cx + c);
						const int off = c ? pic->cr_qp_offset : pic->cb_qp_offset;
						if (dir == 0) chroma_edge(s, 2, W, qp, off, pic->tc_offset);
						else chroma_edge(s, W, 2, qp, off, pic->tc_offset);
					}
				}
			}
	}
}

/* ------------------------------------------------------------------ SAO (8.7.3) */
static void sao(const h265r_picture_t *pic, uint8_t *luma, uint8_t *chroma)
{
	const int W = pic->width, H = pic->height, ctb = 1 << pic->ctb_log2;
	const int cols = (pic->pic_w + ctb - 1) / ctb, rows = (pic->pic_h + ctb - 1) / ctb;
	uint8_t *copy = (uint8_t *)malloc((size_t)W * (size_t)H * 3 / 2);
	if (!copy) return;
	memcpy(copy, luma, (size_t)W * (size_t)H);
	memcpy(copy + (size_t)W * (size_t)H, chroma, (size_t)W * (size_t)H / 2);
	static const int dx[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}}, dy[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
	for (int cy = 0; cy < rows; ++cy)
		for (int cx = 0; cx < cols; ++cx) {
			const h265r_sao_t *sa = &pic->sao[(size_t)cy * (size_t)cols + (size_t)cx];
			for (int ci = 0; ci < 3; ++ci) {
				if (!sa->type[ci] || (ci == 0 ? !(pic->flags & H265R_PIC_SAO_LUMA) : !(pic->flags & H265R_PIC_SAO_CHROMA))) continue;
				const int sub = ci ? 1 : 0, cs = ctb >> sub;
				const int pw = pic->pic_w >> sub, ph = pic->pic_h >> sub;
				const uint8_t *src = ci ? copy + (size_t)W * (size_t)H + (ci - 1) : copy;
				uint8_t *dst = ci ? chroma + (ci - 1) : luma;
				const int step = ci ? 2 : 1;
				for (int y = cy * cs; y < (cy + 1) * cs && y < ph; ++y)
					for (int x = cx * cs; x < (cx + 1) * cs && x < pw; ++x) {
						const int v = src[(size_t)y * (size_t)W + (size_t)x * (size_t)step];
						int o = 0;
						if (sa->type[ci] == 1) {
							const int k = (v >> 3) - sa->band[ci];
							if (k >= 0 && k < 4) o = sa->off[ci][k];
						} else {
							const int e = sa->eo[ci];
							const int ax = x + dx[e][0], ay = y + dy[e][0], bx = x + dx[e][1], by = y + dy[e][1];
							if (ax < 0 || ay < 0 || bx < 0 || by < 0 || ax >= pw || bx >= pw || ay >= ph || by >= ph) continue;
							const int a = src[(size_t)ay * (size_t)W + (size_t)ax * (size_t)step];
							const int b = src[(size_t)by * (size_t)W + (size_t)bx * (size_t)step];
							const int ei = 2 + (v > a) - (v < a) + (v > b) - (v < b);
							static const int cat[5] = {1, 2, 0, 3, 4};
							if (cat[ei]) o = sa->off[ci][cat[ei] - 1];
						}
						dst[(size_t)y * (size_t)W + (size_t)x * (size_t)step] = (uint8_t)clip3(0, 255, v + o);
					}
			}
		}
	free(copy);
}

/* ------------------------------------------------------------------ motion compensation (h265.cpp:3132-3595) */
/* luma filters by quarter-sample phase over positions -3..4 (fir1 / fir2 / fir3 with their window offsets) */
static const int luma_fir[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                   {-1, 4, -10, 58, 17, -5, 1, 0},
                                   {-1, 4, -11, 40, 40, -11, 4, -1},
                                   {0, 1, -5, 17, 58, -10, 4, -1}};
static const int chroma_fir[8][4] = {{0, 64, 0, 0},  {2, 58, 10, 2}, {4, 54, 16, 2}, {6, 46, 28, 4},
                                     {4, 36, 36, 4}, {4, 28, 46, 6}, {2, 16, 54, 4}, {2, 10, 58, 2}};

static inline int clampx(int v, int m) { return v < 0 ? 0 : (v >= m ? m - 1 : v); } /* CLAMPX (h265.cpp:3158) */

/* the value and shift one luma sample of one list hands the reference's Store functor (interp_luma,
 * h265.cpp:3388-3446): integer position << 12 with the full shift; 1-D filtered with shift - 6; 2-D: the
 * horizontal sums as int16, then the vertical sum with the full shift */
static int mc_luma(const uint8_t *ref, int W, int pw, int ph, int x, int y, int fx, int fy, int full, int *shift)
{
#define RS(xx, yy) ((int)ref[(size_t)clampx(yy, ph) * (size_t)W + (size_t)clampx(xx, pw)])
	int v = 0;
	if (!fx && !fy) {
		*shift = full;
		return RS(x, y) << 12;
	}
	if (!fy) {
		for (int k = 0; k < 8; ++k) v += luma_fir[fx][k] * RS(x - 3 + k, y);
		*shift = full - 6;
		return v;
	}
	if (!fx) {
		for (int k = 0; k < 8; ++k) v += luma_fir[fy][k] * RS(x, y - 3 + k);
		*shift = full - 6;
		return v;
	}
	for (int r = 0; r < 8; ++r) {
		int h = 0;
		for (int k = 0; k < 8; ++k) h += luma_fir[fx][k] * RS(x - 3 + k, y - 3 + r);
		v += luma_fir[fy][r] * (int16_t)h;
	}
	*shift = full;
	return v;
#undef RS
}

/* load2pix(umv) + interp_chroma1hline_base (h265.cpp:3448-3490): one row's horizontal sums, packed */
static uint64_t chroma_h(const uint8_t *ch, int W, int cw, int chh, int x, int y, int fx)
{
	const uint8_t *row = ch + (size_t)clampx(y, chh) * (size_t)W;
	uint64_t a[4];
	for (int k = 0; k < 4; ++k) {
		const int p = clampx(x - 1 + k, cw) * 2;
		a[k] = ((uint64_t)row[p] << 32) | row[p + 1];
	}
	const uint64_t c0 = (uint64_t)chroma_fir[fx][0], c1 = (uint64_t)chroma_fir[fx][1], c2 = (uint64_t)chroma_fir[fx][2],
	               c3 = (uint64_t)chroma_fir[fx][3];
	return (((c1 * a[1] + c2 * a[2]) | 0x80000000ull) - (c0 * a[0] + c3 * a[3])) & ~0xf8000000ull;
}

/* interp_chroma1hline_vert_base (h265.cpp:3493-3511): the Cb and Cr values of one position */
static void mc_chroma(const uint8_t *ch, int W, int cw, int chh, int x, int y, int fx, int fy, int v[2])
{
	const uint64_t h0 = chroma_h(ch, W, cw, chh, x, y - 1, fx), h1 = chroma_h(ch, W, cw, chh, x, y, fx);
	const uint64_t h2 = chroma_h(ch, W, cw, chh, x, y + 1, fx), h3 = chroma_h(ch, W, cw, chh, x, y + 2, fx);
	const uint64_t k0 = (uint64_t)chroma_fir[fy][0], k1 = (uint64_t)chroma_fir[fy][1], k2 = (uint64_t)chroma_fir[fy][2],
	               k3 = (uint64_t)chroma_fir[fy][3];
	const uint64_t w = ((h1 * k1 + h2 * k2) | 0x80000000ull) - (h0 * k0 + h3 * k3);
	v[0] = (int32_t)(uint32_t)(w >> 32);
	v[1] = (int32_t)((uint32_t)w ^ 0x80000000u);
}

/* store_pix<1> / store_pix<0> / add_store_pix (h265.cpp:3160-3178), with the int wrap of the reference's adds */
static inline uint8_t st_uni(int val, int shift) { return (uint8_t)clampx((int)((unsigned)val + (1u << (shift - 1))) >> shift, 256); }
static inline int16_t st_bi0(int val, int shift) { return (int16_t)(val >> shift); }
static inline uint8_t st_bi1(int16_t d, int val, int shift) { return (uint8_t)clampx((int)((unsigned)d + (unsigned)(val >> shift) + 64u) >> 7, 256); }

/* merge_pred / pred_amvp_l0 / pred_amvp_l1 (h265.cpp:3572-3595, 3868-3903) for every prediction block */
static void mc_picture(const h265r_picture_t *pic, const m2d_frame_t *frames, int nframes, uint8_t *luma, uint8_t *chroma)
{
	const int W = pic->width, pw = pic->pic_w, ph = pic->pic_h;
	static int16_t tl[64 * 64], tc[64 * 64];
	for (int i = 0; i < pic->n_pu; ++i) {
		const h265r_pu_t *u = &pic->pu[i];
		const int bi = u->ref[0] >= 0 && u->ref[1] >= 0;
		int first = 1;
		for (int l = 0; l < 2; ++l) {
			if (u->ref[l] < 0 || u->ref[l] >= nframes) continue;
			const uint8_t *rl = frames[u->ref[l]].luma, *rc = frames[u->ref[l]].chroma;
			const int mvx = u->mv[l][0], mvy = u->mv[l][1], full = bi ? 6 : 12;
			{
				const int xi = u->x + (mvx >> 2), yi = u->y + (mvy >> 2), fx = mvx & 3, fy = mvy & 3;
				for (int y = 0; y < u->h; ++y)
					for (int x = 0; x < u->w; ++x) {
						int sh;
						const int v = mc_luma(rl, W, pw, ph, xi + x, yi + y, fx, fy, full, &sh);
						uint8_t *o = &luma[(size_t)(u->y + y) * (size_t)W + (size_t)(u->x + x)];
						if (!bi) *o = st_uni(v, sh);
						else if (first) tl[y * 64 + x] = st_bi0(v, sh);
						else *o = st_bi1(tl[y * 64 + x], v, sh);
					}
			}
			{
				const int xi = (u->x >> 1) + (mvx >> 3), yi = (u->y >> 1) + (mvy >> 3), fx = mvx & 7, fy = mvy & 7;
				for (int y = 0; y < u->h / 2; ++y)
					for (int x = 0; x < u->w / 2; ++x) {
						int v[2];
						mc_chroma(rc, W, pw >> 1, ph >> 1, xi + x, yi + y, fx, fy, v);
						for (int c = 0; c < 2; ++c) {
							uint8_t *o = &chroma[(size_t)((u->y >> 1) + y) * (size_t)W + (size_t)(u->x + 2 * x + c)];
							if (!bi) *o = st_uni(v[c], full);
							else if (first) tc[y * 64 + 2 * x + c] = st_bi0(v[c], full);
							else *o = st_bi1(tc[y * 64 + 2 * x + c], v[c], full);
						}
					}
			}
			first = 0;
		}
	}
}

/* ------------------------------------------------------------------ the block dependency graph (analysis) */
static int64_t g_chain[2]; /* the longest chain of blocks (the GPU kernel's critical path), blocks */

int64_t h265_oracle_chain(int which) { return g_chain[which & 1]; }

static void chain_depth(const h265r_picture_t *pic)
{
	int *lv = (int *)calloc((size_t)pic->n_tu + 1, sizeof(int));
	int best = 0;
	if (!lv) return;
	for (int i = 0; i < pic->n_tu; ++i) {
		const h265r_tu_t *t = &pic->tu[i];
		const int n = 1 << t->log2;
		const int at = t->avail_top > 2 * n ? 2 * n : t->avail_top, al = t->avail_left > 2 * n ? 2 * n : t->avail_left;
		const int mw = t->plane ? pic->width / 8 : pic->width / 4;
		const int32_t *map = pic->map + (t->plane ? (size_t)(pic->width / 4) * (size_t)(pic->height / 4) : 0);
		int m = 0;
		for (int k = 0; at > 0 && k < (at + 3) / 4; ++k) {
			const int j = map[(size_t)((t->y >> 2) - 1) * (size_t)mw + (size_t)((t->x >> 2) + k)];
			if (j >= 0 && j < i && lv[j] > m) m = lv[j];
		}
		for (int k = 0; al > 0 && k < (al + 3) / 4; ++k) {
			const int j = map[(size_t)((t->y >> 2) + k) * (size_t)mw + (size_t)((t->x >> 2) - 1)];
			if (j >= 0 && j < i && lv[j] > m) m = lv[j];
		}
		lv[i] = m + 1;
		if (lv[i] > best) best = lv[i];
	}
	g_chain[0] = best;
	g_chain[1] = pic->n_tu;
	free(lv);
}

/* ------------------------------------------------------------------ the picture */
void h265_oracle_recon_picture(const h265r_picture_t *pic, const m2d_frame_t *frames, int nframes)
{
	static int built;
	if (!built) {
		build_mat();
		built = 1;
	}
	if (pic->slot < 0 || pic->slot >= nframes) return;
	uint8_t *luma = frames[pic->slot].luma, *chroma = frames[pic->slot].chroma;
	const int W = pic->width;
	chain_depth(pic);
	if (pic->n_pu) mc_picture(pic, frames, nframes, luma, chroma);
	int pred[32 * 32], res[32 * 32];
	for (int i = 0; i < pic->n_tu; ++i) {
		const h265r_tu_t *t = &pic->tu[i];
		const int n = 1 << t->log2;
		const int ncomp = t->plane ? 2 : 1;
		for (int c = 0; c < ncomp; ++c) {
			plane_t pl;
			pl.base = t->plane ? chroma + c : luma;
			pl.stride = W;
			pl.step = t->plane ? 2 : 1;
			if (t->flags & H265R_TU_PRED) intra_pred(&pl, t->x, t->y, t->log2, t->mode, t->avail_top, t->avail_left, !t->plane, t->strong, pred);
			else
				for (int k = 0; k < n * n; ++k) pred[k] = PX(&pl, t->x + (k % n), t->y + k / n);
			residual(t->res[c] ? pic->coef + t->coef[c] : NULL, t->log2, t->res[c], res);
			for (int y = 0; y < n; ++y)
				for (int x = 0; x < n; ++x) PX(&pl, t->x + x, t->y + y) = (uint8_t)clip255c(pred[y * n + x] + res[y * n + x]);
		}
	}
	if (pic->flags & H265R_PIC_DEBLOCK) deblock(pic, luma, chroma);
	if (pic->flags & (H265R_PIC_SAO_LUMA | H265R_PIC_SAO_CHROMA)) sao(pic, luma, chroma);
}

/* ------------------------------------------------------------------ as an h265r_backend_t */
typedef struct {
	m2d_frame_t frames[H265R_MAX_FRAMES];
	int n;
} oracle265_t;

static int o_set_frames(void *self, int n, const m2d_frame_t *frames, int w, int h)
{
	oracle265_t *o = (oracle265_t *)self;
	(void)w;
	(void)h;
	if (n < 1 || n > H265R_MAX_FRAMES) return -1;
	memcpy(o->frames, frames, sizeof(m2d_frame_t) * (size_t)n);
	o->n = n;
	return 0;
}

static int o_submit(void *self, const h265r_picture_t *pic)
{
	oracle265_t *o = (oracle265_t *)self;
	h265_oracle_recon_picture(pic, o->frames, o->n);
	return 0;
}

static int o_sync(void *self, int slot)
{
	(void)self;
	(void)slot;
	return 0;
}

static void o_destroy(void *self) { free(self); }

int h265_oracle_backend_create(h265r_backend_t *out)
{
	oracle265_t *o = (oracle265_t *)calloc(1, sizeof(oracle265_t));
	if (!o || !out) {
		free(o);
		return -1;
	}
	out->self = o;
	out->set_frames = o_set_frames;
	out->submit = o_submit;
	out->sync_frame = o_sync;
	out->destroy = o_destroy;
	out->stage = NULL;
	return 0;
}
