/*
 * Synthetic H.264 stream generator (test and benchmark input; not part of the decoder).
 *
 * Written from ITU-T H.264 (05/2003+) clauses 7.3 (syntax), 8.4.1.3 (motion vector prediction),
 * 8.3.1.1 / 8.3.2.1 (intra mode prediction) and 9.2 / 9.3 (CAVLC / CABAC binarisations and context
 * selection).  See gen.h for the approach and SURVEY.md Appendix A for the constraints kept here:
 *   - no plane prediction unless params.planar (CLIP255C domain, A#2: streams with planar are kept
 *     only where the oracle reports no out-of-domain CLIP255C argument);
 *   - per-block residual bounded so that prediction + residual stays in [-256, 767] and DC-only
 *     adds stay within +-255 (A#2, A#17);
 *   - scaling lists only in the SPS, in the reference's 6 + 8 list layout, and only with
 *     params.scaling (the reference parses and ignores them; PPS lists desynchronise it, A#4); deblocking idc 2 only with params.idc2 (A#6);
 *     beta offset >= alpha offset (A#7);
 *   - constrained intra prediction only with params.cip: modes are chosen from the spec's masked
 *     availability (every inter neighbour, top-left included, is unavailable), so the streams are
 *     conforming; the decoder reproduces the reference's own masks (A#8); only legal intra modes (A#9);
 *   - moderate explicit weights (A#1, A#16); CABAC only for 8x8 transforms;
 *   - in transform-8x8 mode B_8x8 uses only 8x8 sub-partitions.
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gen.h"
#include "h264_spec_tables.h"

/* ------------------------------------------------------------------ RNG (xorshift64*) */
static uint64_t rs = 88172645463325252ull;
static uint32_t rnd(void)
{
	rs ^= rs >> 12;
	rs ^= rs << 25;
	rs ^= rs >> 27;
	return (uint32_t)((rs * 2685821657736338717ull) >> 32);
}
static int rr(int lo, int hi) { return lo + (int)(rnd() % (uint32_t)(hi - lo + 1)); }
static int pct(int p) { return (int)(rnd() % 100u) < p; }
static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }
static int iabs(int a) { return a < 0 ? -a : a; }
static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* ------------------------------------------------------------------ scans and block geometry */
static const uint8_t zz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
static const uint8_t zz8[64] = {0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
                                41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22,
                                15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
static const uint8_t blk_x[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static const uint8_t blk_y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
static int blkidx(int x, int y) { return (y >> 1) * 8 + (x >> 1) * 4 + (y & 1) * 2 + (x & 1); }

/* largest dequantisation factor of any position (4x4: normAdjust row max; 8x8 likewise) */
static const int max4[6] = {16, 18, 20, 23, 25, 29};
static const int dc4[6] = {10, 11, 13, 14, 16, 18};
static const int max8[6] = {32, 35, 42, 45, 51, 58};
static int scale4max(int qp) { return max4[qp % 6] << (qp / 6); }
static int scale4dc(int qp) { return dc4[qp % 6] << (qp / 6); }
static int scale8max(int qp)
{
	int s = qp / 6 - 2;
	return s >= 0 ? max8[qp % 6] << s : max8[qp % 6] >> -s;
}
#define RES_BUDGET (180 * 64) /* sum |dequantised coefficient| bound giving |residual| <= ~180 */

/* ------------------------------------------------------------------ macroblock state */
typedef struct {
	int slice;        /* picture-unique slice id, -1 = not coded yet */
	uint8_t intra, pcm, skip, i16, inxn, t8x8, direct16;
	uint8_t cbp, cmode, qpd_nz;
	int8_t ipm[16];   /* per raster 4x4 (I4x4 / I8x8 replicated) */
	uint8_t nnz[16];  /* luma total_coeff per raster 4x4 */
	uint8_t nnzc[2][4];
	uint8_t cdc[2], ldc;
	int8_t ref[2][4]; /* per 8x8 raster; -1 = list not used */
	uint8_t dir8;     /* direct-predicted 8x8 blocks */
	int16_t mv[2][16][2];
	int16_t mvd[2][16][2];
} gmb_t;

/* syntax of one macroblock as chosen, emitted by the CABAC or CAVLC writer */
enum { K_I4, K_I8, K_I16, K_PCM, K_INTER, K_SKIP };
typedef struct {
	int kind;
	int mbtype;          /* P: 0..3, B: 0..22 (B_Direct_16x16 = 0); I16: 1..24 */
	int sub[4];          /* sub_mb_type */
	int npart;
	int part_x[4], part_y[4], part_w[4], part_h[4], part_pred[4]; /* pred bit0 L0, bit1 L1 */
	int ref[2][4];       /* per partition (or 8x8 for 8x8 MBs) */
	int mvd[2][16][2];   /* per (sub)partition in emission order */
	int nmvd[2];
	int mvd_x[2][16], mvd_y[2][16], mvd_w[2][16], mvd_h[2][16];
	int ipm_flag[16], ipm_rem[16];
	int i16_pred;
	int t8x8;
	int qpd;
	int16_t ldc[16];
	int16_t luma[16][16];  /* per blkIdx, scan order (I16 AC at 1..15) */
	int16_t luma8[4][64];  /* per 8x8, scan order */
	int16_t cdc[2][4];
	int16_t cac[2][4][16]; /* scan order, AC at 1..15 */
	uint8_t pcm[384];
} mbsyn_t;

typedef struct {
	const params_t *p;
	int mbw, mbh, nmb;
	gmb_t *mb;
	int slice_type; /* 0 P, 1 B, 2 I */
	int slice_id;
	int qp;
	int l0n, l1n;
	int direct_spatial;
	int prev_qpd_nz;
	cenc_t ce;
	bw_t *w;
	int cur, mbx, mby;
	/* motion */
	int poc;
	int ref_poc[2][32];
	int ref_lt[2][32];      /* the list entry is a long-term reference */
	int gv[2];
	int16_t *region; /* per 4x4-MB region velocity (qpel / frame) */
	int rw, rh;
	/* direct prediction of B pictures (8.4.1.2) */
	const struct gcol *col; /* co-located store of RefPicList1[0] */
	int dsf[32];            /* DistScaleFactor per L0 index */
	int taint;              /* a direct block's motion is not defined by the spec: later MVs inexact */
} gctx_t;

/* co-located motion of a reference picture (8.4.1.2.1).  Anchors are I / P pictures, so the
 * co-located block's motion is its L0 motion (or intra: ref -1). */
typedef struct gcol {
	int8_t ref[4];      /* refIdxCol per 8x8 */
	int ref_poc[4];     /* POC of the picture it names */
	int16_t mv[16][2];  /* mvCol per raster 4x4 */
} gcol_t;

static gmb_t *nbmb(gctx_t *g, int x, int y, int *bx, int *by)
{
	int mx = g->mbx, my = g->mby;
	gmb_t *n;
	if (y >= 0 && x >= 4) return NULL;
	if (y < 0) {
		my--;
		*by = 3;
	} else {
		*by = y;
	}
	if (x < 0) {
		mx--;
		*bx = 3;
	} else if (x >= 4) {
		mx++;
		*bx = 0;
	} else {
		*bx = x;
	}
	if (mx == g->mbx && my == g->mby) return &g->mb[g->cur];
	if (mx < 0 || my < 0 || mx >= g->mbw) return NULL;
	n = &g->mb[my * g->mbw + mx];
	return (n->slice == g->slice_id) ? n : NULL;
}

/* ------------------------------------------------------------------ motion (believed field) */
typedef struct {
	int avail, ref;
	int mv[2];
} nbm_t;

static void nb_motion(gctx_t *g, int lx, int x, int y, nbm_t *o)
{
	int bx, by;
	gmb_t *n = nbmb(g, x, y, &bx, &by);
	if (!n) {
		o->avail = 0;
		o->ref = -1;
		o->mv[0] = o->mv[1] = 0;
		return;
	}
	o->avail = 1;
	o->ref = n->ref[lx][(by >> 1) * 2 + (bx >> 1)];
	o->mv[0] = n->mv[lx][by * 4 + bx][0];
	o->mv[1] = n->mv[lx][by * 4 + bx][1];
	if (o->ref < 0) o->mv[0] = o->mv[1] = 0;
}

static void nb_c(gctx_t *g, int lx, int x, int y, int w, nbm_t *o)
{
	int cx = x + w, cy = y - 1, ok;
	if (cy < 0) ok = 1;
	else ok = (cx < 4) && blkidx(cx, cy) < blkidx(x, y);
	if (ok) {
		nb_motion(g, lx, cx, cy, o);
		if (o->avail) return;
	}
	nb_motion(g, lx, x - 1, y - 1, o);
}

static int median3(int a, int b, int c) { return imax(imin(a, b), imin(imax(a, b), c)); }

/* shape: 0 generic, 1 16x8 top, 2 16x8 bottom, 3 8x16 left, 4 8x16 right (8.4.1.3) */
static void mvpred(gctx_t *g, int lx, int x, int y, int w, int ref, int shape, int out[2])
{
	nbm_t A, B, C;
	int n;
	nb_motion(g, lx, x - 1, y, &A);
	nb_motion(g, lx, x, y - 1, &B);
	nb_c(g, lx, x, y, w, &C);
	if (shape == 1 && B.ref == ref) { out[0] = B.mv[0]; out[1] = B.mv[1]; return; }
	if (shape == 2 && A.ref == ref) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
	if (shape == 3 && A.ref == ref) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
	if (shape == 4 && C.ref == ref) { out[0] = C.mv[0]; out[1] = C.mv[1]; return; }
	if (!B.avail && !C.avail && A.avail) {
		B = A;
		C = A;
	}
	n = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
	if (n == 1) {
		const nbm_t *s = (A.ref == ref) ? &A : ((B.ref == ref) ? &B : &C);
		out[0] = s->mv[0];
		out[1] = s->mv[1];
		return;
	}
	out[0] = median3(A.mv[0], B.mv[0], C.mv[0]);
	out[1] = median3(A.mv[1], B.mv[1], C.mv[1]);
}

static void pskip_mv(gctx_t *g, int out[2])
{
	nbm_t A, B;
	nb_motion(g, 0, -1, 0, &A);
	nb_motion(g, 0, 0, -1, &B);
	if (!A.avail || !B.avail || (A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) ||
	    (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0)) {
		out[0] = out[1] = 0;
		return;
	}
	mvpred(g, 0, 0, 0, 4, 0, 0, out);
}

/* target motion vector (quarter-pel) of a block referencing POC ref_poc */
static void target_mv(gctx_t *g, int x4, int y4, int ref_poc, int out[2])
{
	int d = g->poc - ref_poc; /* in POC units (2 per frame) */
	int rx = imin(g->rw - 1, (g->mbx * 4 + x4) / 16), ry = imin(g->rh - 1, (g->mby * 4 + y4) / 16);
	const int16_t *rv = &g->region[(ry * g->rw + rx) * 2];
	int lim = g->p->mv_px * 4;
	for (int c = 0; c < 2; ++c) {
		int v = (g->gv[c] + rv[c]) * d / 2 + rr(-3, 3);
		out[c] = clampi(v, -lim, lim);
	}
}

/* ------------------------------------------------------------------ residual generation */
/* fill `n` scan positions [first, first+n) of lv with a sparse random block whose
 * sum |level * scale| stays within budget; returns the sum used */
static int gen_levels(int16_t *lv, int first, int n, int scale, int budget, int density)
{
	int k, sum = 0;
	memset(lv, 0, sizeof(int16_t) * (size_t)(first + n));
	k = 1 + (int)(rnd() % (uint32_t)imax(1, density));
	k = imin(k, n);
	for (int i = 0; i < k; ++i) {
		int pos, mag, r = (int)(rnd() % 100u);
		/* low-frequency bias */
		pos = (int)(rnd() % (uint32_t)n);
		if (pct(60)) pos = (int)(rnd() % (uint32_t)imin(n, 6));
		mag = (r < 70) ? 1 : (r < 85 ? 2 : (r < 95 ? rr(3, 6) : rr(7, 40)));
		while (mag > 0 && sum + mag * scale > budget) mag--;
		if (mag == 0) break;
		if (lv[first + pos] != 0) continue;
		lv[first + pos] = (int16_t)(pct(50) ? -mag : mag);
		sum += mag * scale;
	}
	/* guarantee a non-empty block (the caller asked for a coded block) */
	{
		int any = 0;
		for (int i = first; i < first + n; ++i) any |= lv[i];
		if (!any) {
			lv[first] = (int16_t)(pct(50) ? -1 : 1);
			sum += scale;
		}
	}
	return sum;
}

static int nz_count(const int16_t *lv, int first, int n)
{
	int c = 0;
	for (int i = first; i < first + n; ++i) c += lv[i] != 0;
	return c;
}

/* ------------------------------------------------------------------ CABAC syntax writers */
static void ce_bin(gctx_t *g, int ctx, int b) { cenc_decision(&g->ce, ctx, b); }

static void cabac_ueg(gctx_t *g, int v, int k)
{
	while (v >= (1 << k)) {
		cenc_bypass(&g->ce, 1);
		v -= 1 << k;
		k++;
	}
	cenc_bypass(&g->ce, 0);
	while (k--) cenc_bypass(&g->ce, (v >> k) & 1);
}

static const int16_t sig_base[5] = {105 + 0, 105 + 15, 105 + 29, 105 + 44, 105 + 47};
static const int16_t last_base[5] = {166 + 0, 166 + 15, 166 + 29, 166 + 44, 166 + 47};
static const int16_t abs_base[5] = {227 + 0, 227 + 10, 227 + 20, 227 + 30, 227 + 39};
static const int16_t cbf_base[5] = {85 + 0, 85 + 4, 85 + 8, 85 + 12, 85 + 16};

/* lv: coefficients in scan order, `num` entries starting at lv[0] */
static void cabac_block(gctx_t *g, int cat, const int16_t *lv, int num)
{
	int last = -1, gt1 = 0, eq1 = 0;
	for (int i = 0; i < num; ++i)
		if (lv[i]) last = i;
	if (cat == 5) {
		for (int i = 0; i < 63; ++i) {
			int sig = lv[i] != 0;
			ce_bin(g, 402 + h264_sig8x8_frame[i], sig);
			if (sig) {
				ce_bin(g, 417 + h264_last8x8[i], i == last);
				if (i == last) break;
			}
		}
	} else {
		for (int i = 0; i < num - 1; ++i) {
			int sig = lv[i] != 0;
			ce_bin(g, sig_base[cat] + i, sig);
			if (sig) {
				ce_bin(g, last_base[cat] + i, i == last);
				if (i == last) break;
			}
		}
	}
	{
		int ab = (cat == 5) ? 426 : abs_base[cat];
		for (int i = last; i >= 0; --i) {
			int a, v = lv[i];
			if (!v) continue;
			a = iabs(v) - 1;
			ce_bin(g, ab + ((gt1 != 0) ? 0 : imin(4, 1 + eq1)), a > 0);
			if (a > 0) {
				int ctx2 = ab + 5 + imin(4 - (cat == 3), gt1);
				int k;
				for (k = 1; k < 14 && k < a; ++k) ce_bin(g, ctx2, 1);
				if (a < 14) ce_bin(g, ctx2, 0);
				else cabac_ueg(g, a - 14, 0);
				gt1++;
			} else {
				eq1++;
			}
			cenc_bypass(&g->ce, v < 0);
		}
	}
}

/* coded_block_flag neighbour condition (9.3.3.1.1.9) */
static int cbf_cond_luma(gctx_t *g, int x, int y, int cat, int cur_intra)
{
	int bx, by;
	gmb_t *n = nbmb(g, x, y, &bx, &by);
	if (!n) return cur_intra;
	if (n->pcm) return 1;
	if (cat == 0) return n->i16 ? n->ldc : 0;
	if (n->skip) return 0;
	if (!((n->cbp >> ((by >> 1) * 2 + (bx >> 1))) & 1)) return 0;
	if (n->t8x8) return 1;
	return n->nnz[by * 4 + bx] != 0;
}

static gmb_t *nbc(gctx_t *g, int x, int y, int *bx, int *by)
{
	/* chroma 2x2 block grid: map to the luma neighbour MB selection */
	int lx = x < 0 ? -1 : x * 2, ly = y < 0 ? -1 : y * 2;
	gmb_t *n = nbmb(g, lx, ly, bx, by);
	*bx = x < 0 ? 1 : x;
	*by = y < 0 ? 1 : y;
	return n;
}

static int cbf_cond_chroma(gctx_t *g, int c, int x, int y, int dc, int cur_intra)
{
	int bx, by;
	gmb_t *n = nbc(g, x, y, &bx, &by);
	if (!n) return cur_intra;
	if (n->pcm) return 1;
	if (n->skip) return 0;
	if (dc) return ((n->cbp >> 4) != 0) ? n->cdc[c] : 0;
	return ((n->cbp >> 4) == 2) ? (n->nnzc[c][by * 2 + bx] != 0) : 0;
}

/* ------------------------------------------------------------------ CAVLC block writer (9.2) */
static void put_vlc(bw_t *w, const h264_vlc_code_t *t, int value)
{
	for (; t->value >= 0; ++t)
		if (t->value == value) {
			bw_bits(w, t->code, t->len);
			return;
		}
	fprintf(stderr, "h264gen: no VLC code for value %d\n", value);
	exit(2);
}

static int cavlc_block(bw_t *w, const int16_t *lv, int num, int nc)
{
	int lev[16], runs[16], total = 0, t1 = 0, last = -1, tz, sl;
	int tab = (nc < 0) ? 4 : (nc >= 8 ? 3 : (nc >= 4 ? 2 : (nc >= 2 ? 1 : 0)));
	for (int i = num - 1; i >= 0; --i) {
		if (lv[i]) {
			if (last < 0) last = i;
			lev[total] = lv[i];
			/* zeros below this coefficient until the next nonzero */
			runs[total] = 0;
			for (int j = i - 1; j >= 0 && !lv[j]; --j) runs[total]++;
			total++;
		}
	}
	for (int i = 0; i < total && i < 3; ++i) {
		if (iabs(lev[i]) == 1) t1++;
		else break;
	}
	put_vlc(w, h264_coeff_token_tab[tab], (t1 << 5) | total);
	if (!total) return 0;
	for (int i = 0; i < t1; ++i) bw_bit(w, lev[i] < 0);
	sl = (total > 10 && t1 < 3) ? 1 : 0;
	for (int i = t1; i < total; ++i) {
		int level = lev[i];
		int code = level > 0 ? 2 * level - 2 : -2 * level - 1;
		if (i == t1 && t1 < 3) code -= 2;
		if (sl == 0) {
			if (code < 14) {
				bw_bits(w, 1, code + 1);
			} else if (code < 30) {
				bw_bits(w, 1, 15);
				bw_bits(w, (uint32_t)(code - 14), 4);
			} else {
				bw_bits(w, 1, 16);
				bw_bits(w, (uint32_t)(code - 30), 12);
			}
		} else {
			if ((code >> sl) < 15) {
				bw_bits(w, 1, (code >> sl) + 1);
				bw_bits(w, (uint32_t)(code & ((1 << sl) - 1)), sl);
			} else {
				bw_bits(w, 1, 16);
				bw_bits(w, (uint32_t)(code - (15 << sl)), 12);
			}
		}
		if (sl == 0) sl = 1;
		if (iabs(level) > (3 << (sl - 1)) && sl < 6) sl++;
	}
	tz = last + 1 - total;
	if (total < num) {
		if (num == 4) {
			/* chroma DC 2x2 (Table 9-9a) */
			if (total == 1) {
				static const char *c1[4] = {"1", "01", "001", "000"};
				for (const char *s = c1[tz]; *s; ++s) bw_bit(w, *s == '1');
			} else if (total == 2) {
				static const char *c2[3] = {"1", "01", "00"};
				for (const char *s = c2[tz]; *s; ++s) bw_bit(w, *s == '1');
			} else {
				bw_bit(w, tz == 0);
			}
		} else {
			put_vlc(w, h264_total_zeros_tab[total], tz);
		}
	}
	{
		int left = tz;
		for (int i = 0; i < total - 1 && left > 0; ++i) {
			put_vlc(w, h264_run_before_tab[imin(left, 7)], runs[i]);
			left -= runs[i];
		}
	}
	return total;
}

static int nc_luma(gctx_t *g, int x, int y)
{
	int bx, by, na = -1, nb = -1;
	gmb_t *a = nbmb(g, x - 1, y, &bx, &by);
	if (a) na = a->pcm ? 16 : (a->skip ? 0 : a->nnz[by * 4 + bx]);
	gmb_t *b = nbmb(g, x, y - 1, &bx, &by);
	if (b) nb = b->pcm ? 16 : (b->skip ? 0 : b->nnz[by * 4 + bx]);
	if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
	if (na >= 0) return na;
	if (nb >= 0) return nb;
	return 0;
}

static int nc_chroma(gctx_t *g, int c, int x, int y)
{
	int bx, by, na = -1, nb = -1;
	gmb_t *a = nbc(g, x - 1, y, &bx, &by);
	if (a) na = a->pcm ? 16 : (a->skip ? 0 : a->nnzc[c][by * 2 + bx]);
	gmb_t *b = nbc(g, x, y - 1, &bx, &by);
	if (b) nb = b->pcm ? 16 : (b->skip ? 0 : b->nnzc[c][by * 2 + bx]);
	if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
	if (na >= 0) return na;
	if (nb >= 0) return nb;
	return 0;
}

/* ------------------------------------------------------------------ intra mode choice */
/* neighbour available for intra prediction: with constrained_intra_pred an inter neighbour is not
 * (8.3.1.2 / 8.3.1.1 dcPredModePredictedFlag) */
static gmb_t *ipnb(gctx_t *g, int x, int y, int *bx, int *by)
{
	gmb_t *n = nbmb(g, x, y, bx, by);
	if (n && g->p->cip && !n->intra) return NULL;
	return n;
}

static int pred_ipm(gctx_t *g, int x, int y)
{
	int ax, ay, bx, by, ma, mb;
	gmb_t *a = ipnb(g, x - 1, y, &ax, &ay), *b = ipnb(g, x, y - 1, &bx, &by);
	if (!a || !b) return 2;
	ma = a->inxn ? a->ipm[ay * 4 + ax] : 2;
	mb = b->inxn ? b->ipm[by * 4 + bx] : 2;
	return imin(ma, mb);
}

static int pick_mode9(int L, int T, int TL)
{
	int modes[9], n = 0;
	modes[n++] = 2;
	if (T) { modes[n++] = 0; modes[n++] = 3; modes[n++] = 7; }
	if (L) { modes[n++] = 1; modes[n++] = 8; }
	if (L && T && TL) { modes[n++] = 4; modes[n++] = 5; modes[n++] = 6; }
	return modes[rnd() % (uint32_t)n];
}

/* ------------------------------------------------------------------ macroblock decision */
static void choose_residual(gctx_t *g, mbsyn_t *s, gmb_t *m, int qp)
{
	int qpc[2];
	static const int8_t lut[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
	int dens = 1 + g->p->coef_pct / 12;
	for (int c = 0; c < 2; ++c) {
		int q = clampi(qp, 0, 51);
		qpc[c] = q < 30 ? q : lut[q - 30];
	}
	memset(m->nnz, 0, sizeof(m->nnz));
	memset(m->nnzc, 0, sizeof(m->nnzc));
	m->cdc[0] = m->cdc[1] = 0;
	m->ldc = 0;
	if (s->kind == K_I16) {
		int dcsum = 0;
		/* luma DC: hadamard output <= sum|f| * scale / 4 ; keep it under half the budget */
		if (pct(70)) {
			dcsum = gen_levels(s->ldc, 0, 16, scale4dc(qp), RES_BUDGET * 2, dens);
			m->ldc = 1;
		} else {
			memset(s->ldc, 0, sizeof(s->ldc));
		}
		(void)dcsum;
		if (m->cbp & 15) {
			for (int b = 0; b < 16; ++b) {
				int x = blk_x[b], y = blk_y[b];
				if (pct(g->p->coef_pct)) {
					gen_levels(s->luma[b], 1, 15, scale4max(qp), RES_BUDGET / 2, dens);
				} else {
					memset(s->luma[b], 0, sizeof(s->luma[b]));
				}
				m->nnz[y * 4 + x] = (uint8_t)nz_count(s->luma[b], 1, 15);
			}
		}
	} else {
		for (int b8 = 0; b8 < 4; ++b8) {
			if (!((m->cbp >> b8) & 1)) continue;
			if (s->t8x8 && g->p->quirks && pct(15)) {
				/* one DC coefficient: the reference's SWAR DC-only add (h264.cpp:4072-4080, m2d.h:306-336)
				 * adjusting by 200..255 */
				static const int n0[6] = {20, 22, 26, 28, 32, 36};
				const int sc = qp >= 12 ? n0[qp % 6] << (qp / 6 - 2) : n0[qp % 6] >> (2 - qp / 6), t = rr(200, 255);
				int level = imax(1, (t * 64 + sc / 2) / sc);
				while (level > 1 && ((level * sc + 32) >> 6) > 255) level--;
				memset(s->luma8[b8], 0, sizeof(s->luma8[b8]));
				s->luma8[b8][0] = (int16_t)(pct(50) ? -level : level);
				for (int k = 0; k < 4; ++k) {
					int b = b8 * 4 + k;
					m->nnz[blk_y[b] * 4 + blk_x[b]] = 1;
				}
			} else if (s->t8x8) {
				gen_levels(s->luma8[b8], 0, 64, scale8max(qp), RES_BUDGET * 64 / 144, dens + 2);
				for (int k = 0; k < 4; ++k) {
					int b = b8 * 4 + k;
					m->nnz[blk_y[b] * 4 + blk_x[b]] = (uint8_t)nz_count(s->luma8[b8], 0, 64);
				}
			} else {
				int any = 0;
				for (int k = 0; k < 4; ++k) {
					int b = b8 * 4 + k;
					if (g->p->quirks && pct(12)) {
						/* DC-only block whose DC-only add (m2d.h:306-336) adjusts by 200..255 */
						static const int n0[6] = {10, 11, 13, 14, 16, 18};
						const int sc = n0[qp % 6] << (qp / 6), t = rr(200, 255);
						int level = imax(1, (t * 64 + sc / 2) / sc);
						while (level > 1 && ((level * sc + 32) >> 6) > 255) level--;
						memset(s->luma[b], 0, sizeof(s->luma[b]));
						s->luma[b][0] = (int16_t)(pct(50) ? -level : level);
						any = 1;
					} else if (pct(g->p->coef_pct) || (k == 3 && !any)) {
						gen_levels(s->luma[b], 0, 16, scale4max(qp), RES_BUDGET, dens);
						any = 1;
					} else {
						memset(s->luma[b], 0, sizeof(s->luma[b]));
					}
					m->nnz[blk_y[b] * 4 + blk_x[b]] = (uint8_t)nz_count(s->luma[b], 0, 16);
				}
			}
		}
	}
	if ((m->cbp >> 4) >= 1) {
		for (int c = 0; c < 2; ++c) {
			if (pct(75)) {
				gen_levels(s->cdc[c], 0, 4, scale4dc(qpc[c]), RES_BUDGET, 2);
				m->cdc[c] = 1;
			} else {
				memset(s->cdc[c], 0, sizeof(s->cdc[c]));
			}
		}
	}
	if ((m->cbp >> 4) == 2) {
		for (int c = 0; c < 2; ++c)
			for (int b = 0; b < 4; ++b) {
				if (pct(g->p->coef_pct) || (c == 1 && b == 3)) gen_levels(s->cac[c][b], 1, 15, scale4max(qpc[c]), RES_BUDGET / 2, dens);
				else memset(s->cac[c][b], 0, sizeof(s->cac[c][b]));
				m->nnzc[c][b] = (uint8_t)nz_count(s->cac[c][b], 1, 15);
			}
	}
}

static void choose_intra(gctx_t *g, mbsyn_t *s, gmb_t *m)
{
	int r = (int)(rnd() % 100u);
	int bx, by;
	int L, T;
	m->intra = 1;
	L = ipnb(g, -1, 0, &bx, &by) != NULL;
	T = ipnb(g, 0, -1, &bx, &by) != NULL;
	for (int lx = 0; lx < 2; ++lx)
		for (int k = 0; k < 4; ++k) m->ref[lx][k] = -1;
	if ((int)(rnd() % 1000u) < g->p->pcm_permille) {
		s->kind = K_PCM;
		m->pcm = 1;
		m->cbp = 0x2f;
		for (int i = 0; i < 384; ++i) s->pcm[i] = (uint8_t)rr(16, 235);
		memset(m->nnz, 16, sizeof(m->nnz));
		memset(m->nnzc, 16, sizeof(m->nnzc));
		m->cdc[0] = m->cdc[1] = m->ldc = 1;
		return;
	}
	if (r < g->p->i4_pct + (g->p->t8x8 ? g->p->i8_pct : 0)) {
		int t8 = g->p->t8x8 && r >= g->p->i4_pct;
		m->inxn = 1;
		m->t8x8 = (uint8_t)t8;
		s->t8x8 = t8;
		s->kind = t8 ? K_I8 : K_I4;
		if (t8) {
			for (int b8 = 0; b8 < 4; ++b8) {
				int x = (b8 & 1) * 2, y = (b8 >> 1) * 2;
				int l = ipnb(g, x - 1, y, &bx, &by) != NULL, t = ipnb(g, x, y - 1, &bx, &by) != NULL;
				int tl = ipnb(g, x - 1, y - 1, &bx, &by) != NULL;
				int pred = pred_ipm(g, x, y), mode = pick_mode9(l, t, tl);
				s->ipm_flag[b8] = (mode == pred);
				s->ipm_rem[b8] = mode < pred ? mode : mode - 1;
				for (int k = 0; k < 4; ++k) m->ipm[(y + (k >> 1)) * 4 + x + (k & 1)] = (int8_t)mode;
			}
		} else {
			for (int b = 0; b < 16; ++b) {
				int x = blk_x[b], y = blk_y[b];
				int l = ipnb(g, x - 1, y, &bx, &by) != NULL, t = ipnb(g, x, y - 1, &bx, &by) != NULL;
				int tl = ipnb(g, x - 1, y - 1, &bx, &by) != NULL;
				int pred = pred_ipm(g, x, y), mode = pick_mode9(l, t, tl);
				s->ipm_flag[b] = (mode == pred);
				s->ipm_rem[b] = mode < pred ? mode : mode - 1;
				m->ipm[y * 4 + x] = (int8_t)mode;
			}
		}
		m->cbp = (uint8_t)((pct(g->p->coef_pct + 20) ? rr(1, 15) : 0) | (rr(0, 2) << 4));
	} else {
		int modes[4], n = 0, lc;
		int TL = ipnb(g, -1, -1, &bx, &by) != NULL;
		s->kind = K_I16;
		m->i16 = 1;
		modes[n++] = 2;
		if (T) modes[n++] = 0;
		if (L) modes[n++] = 1;
		if (L && T && TL && g->p->planar) modes[n++] = 3;
		s->i16_pred = modes[rnd() % (uint32_t)n];
		lc = pct(g->p->coef_pct) ? 15 : 0;
		m->cbp = (uint8_t)(lc | (rr(0, 2) << 4));
		s->mbtype = 1 + s->i16_pred + 4 * (m->cbp >> 4) + (lc ? 12 : 0);
	}
	{
		int modes[4], n = 0;
		int TL = ipnb(g, -1, -1, &bx, &by) != NULL;
		modes[n++] = 0;
		if (L) modes[n++] = 1;
		if (T) modes[n++] = 2;
		if (L && T && TL && g->p->planar) modes[n++] = 3;
		m->cmode = (uint8_t)modes[rnd() % (uint32_t)n];
	}
}

/* P/B partition tables */
static const int b_pred16[23][2] = {
	{0, 0}, {1, 0}, {2, 0}, {3, 0},             /* direct, L0, L1, Bi (16x16) */
	{1, 1}, {1, 1}, {2, 2}, {2, 2}, {1, 2}, {1, 2}, {2, 1}, {2, 1}, {1, 3}, {1, 3},
	{2, 3}, {2, 3}, {3, 1}, {3, 1}, {3, 2}, {3, 2}, {3, 3}, {3, 3}, {0, 0}};
/* B sub types: pred flags and partition shape (0 8x8, 1 8x4, 2 4x8, 3 4x4) */
static const int b_sub_pred[13] = {0, 1, 2, 3, 1, 1, 2, 2, 3, 3, 1, 2, 3};
static const int b_sub_shape[13] = {0, 0, 0, 0, 1, 2, 1, 2, 1, 2, 3, 3, 3};

static void set_motion(gctx_t *g, gmb_t *m, mbsyn_t *s, int lx, int x, int y, int w, int h, int ref, int shape)
{
	int mvp[2], t[2], rp = g->ref_poc[lx][ref];
	int k = s->nmvd[lx]++;
	mvpred(g, lx, x, y, w, ref, shape, mvp);
	target_mv(g, x, y, rp, t);
	s->mvd[lx][k][0] = t[0] - mvp[0];
	s->mvd[lx][k][1] = t[1] - mvp[1];
	s->mvd_x[lx][k] = x;
	s->mvd_y[lx][k] = y;
	s->mvd_w[lx][k] = w;
	s->mvd_h[lx][k] = h;
	for (int yy = y; yy < y + h; ++yy)
		for (int xx = x; xx < x + w; ++xx) {
			m->mv[lx][yy * 4 + xx][0] = (int16_t)t[0];
			m->mv[lx][yy * 4 + xx][1] = (int16_t)t[1];
			m->mvd[lx][yy * 4 + xx][0] = (int16_t)s->mvd[lx][k][0];
			m->mvd[lx][yy * 4 + xx][1] = (int16_t)s->mvd[lx][k][1];
		}
}

/* Direct motion of 8x8 block b8 of a B macroblock, restated from the spec (ITU-T H.264 8.4.1.2)
 * so that the dump's B-picture motion checks the parser's derivation (h264.cpp:8325-8387 spatial,
 * :1247-1277 + temporal_direct_block temporal).  direct_8x8_inference_flag is 1 in every stream
 * (write_sps), so the co-located vector is the corner 4x4 of the 8x8 block.
 *  - spatial (8.4.1.2.2): per list refIdx = MinPositive over the MB neighbours A, B, C (C falling
 *    back to D), mv = the 16x16 prediction for that refIdx; both refIdx < 0 -> refs 0 / 0, mvs 0;
 *    a list with refIdx 0 gets a zero mv where colZeroFlag (L1[0] short-term, refIdxCol 0,
 *    |mvCol| <= 1 in both components) holds;
 *  - temporal (8.4.1.2.3): refIdxL0 = the lowest L0 index naming refIdxCol's picture (0 for an
 *    intra co-located block), refIdxL1 = 0, mvL0 = (DistScaleFactor * mvCol + 128) >> 8,
 *    mvL1 = mvL0 - mvCol.  A co-located picture absent from L0 (not in a conforming stream, and
 *    never produced by these presets) taints the rest of the picture instead of guessing. */
static void direct_motion(gctx_t *g, gmb_t *m, int b8)
{
	const gcol_t *col = &g->col[g->cur];
	const int16_t *mc = col->mv[(b8 >> 1) * 12 + (b8 & 1) * 3];
	int x0 = (b8 & 1) * 2, y0 = (b8 >> 1) * 2;
	int ref[2], mv[2][2];
	if (g->direct_spatial) {
		/* colZeroFlag needs RefPicList1[0] short-term (8.4.1.2.2; h264.cpp:8507, 9960) */
		int colzero = !g->ref_lt[1][0] && col->ref[b8] == 0 && mc[0] >= -1 && mc[0] <= 1 && mc[1] >= -1 && mc[1] <= 1;
		for (int lx = 0; lx < 2; ++lx) {
			nbm_t A, B, C;
			unsigned r;
			nb_motion(g, lx, -1, 0, &A);
			nb_motion(g, lx, 0, -1, &B);
			nb_c(g, lx, 0, 0, 4, &C);
			r = (unsigned)A.ref < (unsigned)B.ref ? (unsigned)A.ref : (unsigned)B.ref;
			r = r < (unsigned)C.ref ? r : (unsigned)C.ref;
			ref[lx] = (int)r;
			mv[lx][0] = mv[lx][1] = 0;
			if (ref[lx] >= 0) mvpred(g, lx, 0, 0, 4, ref[lx], 0, mv[lx]);
		}
		if (ref[0] < 0 && ref[1] < 0) {
			ref[0] = ref[1] = 0;
		} else {
			for (int lx = 0; lx < 2; ++lx)
				if (ref[lx] < 0 || (ref[lx] == 0 && colzero)) mv[lx][0] = mv[lx][1] = 0;
		}
	} else {
		ref[1] = 0;
		if (col->ref[b8] < 0) {
			ref[0] = 0;
			mv[0][0] = mv[0][1] = mv[1][0] = mv[1][1] = 0;
		} else {
			int k = 0;
			while (k < g->l0n && g->ref_poc[0][k] != col->ref_poc[b8]) ++k;
			if (k >= g->l0n) {
				g->taint = 1;
				k = 0;
			}
			ref[0] = k;
			if (g->ref_lt[0][k]) {
				/* RefPicList0[refIdxL0] long-term: the spec takes mvL0 = mvCol, mvL1 = 0 (8.4.1.2.3); the
				 * reference gives both lists a zero vector (temporal_direct_block, h264.cpp:10049-10054) */
				mv[0][0] = mv[0][1] = mv[1][0] = mv[1][1] = 0;
			} else {
				for (int c = 0; c < 2; ++c) {
					mv[0][c] = (g->dsf[k] * mc[c] + 128) >> 8;
					mv[1][c] = mv[0][c] - mc[c];
				}
			}
		}
	}
	for (int lx = 0; lx < 2; ++lx) {
		m->ref[lx][b8] = (int8_t)ref[lx];
		for (int yy = y0; yy < y0 + 2; ++yy)
			for (int xx = x0; xx < x0 + 2; ++xx) {
				m->mv[lx][yy * 4 + xx][0] = (int16_t)mv[lx][0];
				m->mv[lx][yy * 4 + xx][1] = (int16_t)mv[lx][1];
				m->mvd[lx][yy * 4 + xx][0] = m->mvd[lx][yy * 4 + xx][1] = 0;
			}
	}
}

static int pick_ref(int n)
{
	if (n <= 1) return 0;
	return pct(70) ? 0 : rr(1, n - 1);
}

static void choose_inter(gctx_t *g, mbsyn_t *s, gmb_t *m)
{
	int is_b = g->slice_type == 1;
	int r = (int)(rnd() % 100u);
	s->kind = K_INTER;
	for (int lx = 0; lx < 2; ++lx)
		for (int k = 0; k < 4; ++k) m->ref[lx][k] = -1;
	s->nmvd[0] = s->nmvd[1] = 0;
	if (is_b && r < 15) {
		/* B_Direct_16x16 */
		s->mbtype = 0;
		m->direct16 = 1;
		m->dir8 = 15;
		for (int b8 = 0; b8 < 4; ++b8) direct_motion(g, m, b8);
	} else if (r < 100 - g->p->sub8x8_pct) {
		int shape = (r < 55) ? 0 : (r < 55 + (45 - g->p->sub8x8_pct) / 2 ? 1 : 2); /* 16x16, 16x8, 8x16 */
		int np = shape ? 2 : 1;
		int pred[2];
		if (is_b) {
			int t;
			if (shape == 0) t = rr(1, 3);
			else t = 4 + rr(0, 8) * 2 + (shape == 2);
			s->mbtype = t;
			pred[0] = b_pred16[t][0];
			pred[1] = b_pred16[t][1];
			if (shape == 0) pred[1] = 0;
		} else {
			s->mbtype = shape;
			pred[0] = pred[1] = 1;
		}
		s->npart = np;
		for (int p = 0; p < np; ++p) {
			s->part_x[p] = (shape == 2) ? p * 2 : 0;
			s->part_y[p] = (shape == 1) ? p * 2 : 0;
			s->part_w[p] = (shape == 2) ? 2 : 4;
			s->part_h[p] = (shape == 1) ? 2 : 4;
			s->part_pred[p] = pred[p];
			for (int lx = 0; lx < 2; ++lx) {
				int ref = ((pred[p] >> lx) & 1) ? pick_ref(lx ? g->l1n : g->l0n) : -1;
				s->ref[lx][p] = ref;
				for (int k = 0; k < 4; ++k) {
					int kx = (k & 1) * 2, ky = (k >> 1) * 2;
					if (kx >= s->part_x[p] && kx < s->part_x[p] + s->part_w[p] && ky >= s->part_y[p] &&
					    ky < s->part_y[p] + s->part_h[p])
						m->ref[lx][k] = (int8_t)ref;
				}
			}
		}
		/* motion in syntax order: all L0 partitions, then L1 (mvp of partition 1 sees partition 0) */
		for (int lx = 0; lx < 2; ++lx)
			for (int p = 0; p < np; ++p) {
				int sh;
				if (s->ref[lx][p] < 0) continue;
				sh = (shape == 0) ? 0 : (shape == 1 ? 1 + p : 3 + p);
				set_motion(g, m, s, lx, s->part_x[p], s->part_y[p], s->part_w[p], s->part_h[p], s->ref[lx][p], sh);
			}
	} else {
		/* 8x8 */
		s->mbtype = is_b ? 22 : 3;
		for (int b8 = 0; b8 < 4; ++b8) {
			int st;
			if (is_b) {
				if (g->p->t8x8) st = rr(0, 3);
				else st = rr(0, 12);
			} else {
				st = pct(50) ? 0 : rr(1, 3);
			}
			s->sub[b8] = st;
		}
		for (int b8 = 0; b8 < 4; ++b8) {
			int pf = is_b ? b_sub_pred[s->sub[b8]] : 1;
			for (int lx = 0; lx < 2; ++lx) {
				int ref = -1;
				if (is_b && s->sub[b8] == 0) ref = -1;
				else if ((pf >> lx) & 1) ref = pick_ref(lx ? g->l1n : g->l0n);
				s->ref[lx][b8] = ref;
				m->ref[lx][b8] = (int8_t)ref;
			}
			if (is_b && s->sub[b8] == 0) {
				m->dir8 |= (uint8_t)(1 << b8);
				direct_motion(g, m, b8);
			}
		}
		for (int lx = 0; lx < 2; ++lx)
			for (int b8 = 0; b8 < 4; ++b8) {
				int x0 = (b8 & 1) * 2, y0 = (b8 >> 1) * 2;
				int shp = is_b ? b_sub_shape[s->sub[b8]] : s->sub[b8];
				if (s->ref[lx][b8] < 0) continue;
				if (shp == 0) set_motion(g, m, s, lx, x0, y0, 2, 2, s->ref[lx][b8], 0);
				else if (shp == 1) {
					set_motion(g, m, s, lx, x0, y0, 2, 1, s->ref[lx][b8], 0);
					set_motion(g, m, s, lx, x0, y0 + 1, 2, 1, s->ref[lx][b8], 0);
				} else if (shp == 2) {
					set_motion(g, m, s, lx, x0, y0, 1, 2, s->ref[lx][b8], 0);
					set_motion(g, m, s, lx, x0 + 1, y0, 1, 2, s->ref[lx][b8], 0);
				} else {
					for (int k = 0; k < 4; ++k)
						set_motion(g, m, s, lx, x0 + (k & 1), y0 + (k >> 1), 1, 1, s->ref[lx][b8], 0);
				}
			}
	}
	m->cbp = (uint8_t)((pct(g->p->coef_pct + 10) ? rr(1, 15) : 0) | ((pct(50) ? rr(1, 2) : 0) << 4));
	/* transform size: spec 7.3.5 condition (reference quirks kept out of reach, see file header) */
	s->t8x8 = 0;
	if (g->p->t8x8 && (m->cbp & 15)) {
		int ok = 1;
		if ((is_b && s->mbtype == 22) || (!is_b && s->mbtype == 3)) {
			for (int b8 = 0; b8 < 4; ++b8) {
				int shp = is_b ? b_sub_shape[s->sub[b8]] : s->sub[b8];
				if (shp != 0) ok = 0;
			}
		}
		if (ok && pct(50)) s->t8x8 = 1;
	}
	m->t8x8 = (uint8_t)s->t8x8;
}

/* ------------------------------------------------------------------ macroblock writers */
static void write_mb_cabac(gctx_t *g, mbsyn_t *s, gmb_t *m)
{
	int bx, by;
	gmb_t *A = nbmb(g, -1, 0, &bx, &by), *B = nbmb(g, 0, -1, &bx, &by);
	int is_i = g->slice_type == 2, is_b = g->slice_type == 1;
	int intra = (s->kind <= K_PCM);
	/* mb_type */
	if (intra) {
		int base;
		if (is_i) {
			int inc = (A && !A->inxn) + (B && !B->inxn);
			ce_bin(g, 3 + inc, s->kind != K_I4 && s->kind != K_I8);
			base = 5; /* bins 2.. use 3+3.. */
		} else {
			if (is_b) {
				int inc = (A && !A->direct16) + (B && !B->direct16);
				static const int pre[6] = {1, 1, 1, 1, 0, 1};
				ce_bin(g, 27 + inc, 1);
				ce_bin(g, 27 + 3, 1);
				ce_bin(g, 27 + 4, pre[2]);
				for (int i = 3; i < 6; ++i) ce_bin(g, 27 + 5, pre[i]);
				base = 32;
			} else {
				ce_bin(g, 14, 1);
				base = 17;
			}
			ce_bin(g, base, s->kind != K_I4 && s->kind != K_I8);
		}
		if (s->kind != K_I4 && s->kind != K_I8) {
			cenc_terminate(&g->ce, s->kind == K_PCM);
			if (s->kind == K_PCM) {
				while (!bw_aligned(g->w)) bw_bit(g->w, 0);
				for (int i = 0; i < 384; ++i) bw_bits(g->w, s->pcm[i], 8);
				cenc_start(&g->ce, g->w);
				return;
			}
			{
				int lc = (m->cbp & 15) != 0, cc = m->cbp >> 4, pm = s->i16_pred;
				ce_bin(g, base + 1, lc);
				ce_bin(g, base + 2, cc != 0);
				if (cc) ce_bin(g, base + 2 + is_i, cc == 2);
				ce_bin(g, base + 3 + is_i, pm >> 1);
				ce_bin(g, base + 3 + 2 * is_i, pm & 1);
			}
		}
	} else if (is_b) {
		int inc = (A && !A->direct16) + (B && !B->direct16);
		int t = s->mbtype;
		if (t == 0) {
			ce_bin(g, 27 + inc, 0);
		} else if (t <= 2) {
			ce_bin(g, 27 + inc, 1);
			ce_bin(g, 27 + 3, 0);
			ce_bin(g, 27 + 5, t - 1);
		} else {
			int bits, nb;
			ce_bin(g, 27 + inc, 1);
			ce_bin(g, 27 + 3, 1);
			if (t <= 10) { bits = t - 3; nb = 4; }
			else if (t == 11) { bits = 14; nb = 4; }
			else if (t == 22) { bits = 15; nb = 4; }
			else { bits = t + 4; nb = 5; }
			for (int i = nb - 1; i >= 0; --i) ce_bin(g, (i == nb - 1) ? 27 + 4 : 27 + 5, (bits >> i) & 1);
		}
	} else {
		static const int pbins[4][3] = {{0, 0, 0}, {0, 1, 1}, {0, 1, 0}, {0, 0, 1}};
		const int *b = pbins[s->mbtype];
		ce_bin(g, 14, b[0]);
		ce_bin(g, 15, b[1]);
		ce_bin(g, b[1] ? 17 : 16, b[2]);
	}

	if (s->kind == K_I4 || s->kind == K_I8) {
		if (g->p->t8x8) ce_bin(g, 399 + (A && A->t8x8) + (B && B->t8x8), s->kind == K_I8);
		for (int i = 0; i < (s->kind == K_I8 ? 4 : 16); ++i) {
			ce_bin(g, 68, s->ipm_flag[i]);
			if (!s->ipm_flag[i])
				for (int k = 0; k < 3; ++k) ce_bin(g, 69, (s->ipm_rem[i] >> k) & 1);
		}
	}
	if (intra) {
		int inc = (A && A->intra && !A->pcm && A->cmode) + (B && B->intra && !B->pcm && B->cmode);
		int cm = m->cmode;
		ce_bin(g, 64 + inc, cm != 0);
		if (cm) {
			ce_bin(g, 67, cm > 1);
			if (cm > 1) ce_bin(g, 67, cm > 2);
		}
	} else {
		int is8 = (is_b && s->mbtype == 22) || (!is_b && s->mbtype == 3);
		if (is8) {
			for (int b8 = 0; b8 < 4; ++b8) {
				int st = s->sub[b8];
				if (!is_b) {
					static const int pb[4][3] = {{1, 0, 0}, {0, 0, 0}, {0, 1, 1}, {0, 1, 0}};
					ce_bin(g, 21, pb[st][0]);
					if (st) {
						ce_bin(g, 22, pb[st][1]);
						if (st >= 2) ce_bin(g, 23, pb[st][2]);
					}
				} else {
					ce_bin(g, 36, st != 0);
					if (st == 0) continue;
					if (st <= 2) {
						ce_bin(g, 37, 0);
						ce_bin(g, 39, st - 1);
					} else {
						ce_bin(g, 37, 1);
						if (st >= 11) {
							ce_bin(g, 38, 1);
							ce_bin(g, 39, 1);
							ce_bin(g, 39, st - 11);
						} else if (st >= 7) {
							ce_bin(g, 38, 1);
							ce_bin(g, 39, 0);
							ce_bin(g, 39, ((st - 7) >> 1) & 1);
							ce_bin(g, 39, (st - 7) & 1);
						} else {
							ce_bin(g, 38, 0);
							ce_bin(g, 39, ((st - 3) >> 1) & 1);
							ce_bin(g, 39, (st - 3) & 1);
						}
					}
				}
			}
		}
		/* ref_idx */
		for (int lx = 0; lx < 2; ++lx) {
			int nact = lx ? g->l1n : g->l0n;
			int np = is8 ? 4 : s->npart;
			if (nact <= 1) continue;
			for (int p = 0; p < np; ++p) {
				int ref = s->ref[lx][p], x, y, inc = 0, ax, ay;
				gmb_t *n;
				if (ref < 0) continue;
				if (is8) { x = (p & 1) * 2; y = (p >> 1) * 2; }
				else { x = s->part_x[p]; y = s->part_y[p]; }
				n = nbmb(g, x - 1, y, &ax, &ay);
				if (n) {
					int k = (ay >> 1) * 2 + (ax >> 1);
					if (!((n->dir8 >> k) & 1) && !n->skip && n->ref[lx][k] > 0) inc += 1;
				}
				n = nbmb(g, x, y - 1, &ax, &ay);
				if (n) {
					int k = (ay >> 1) * 2 + (ax >> 1);
					if (!((n->dir8 >> k) & 1) && !n->skip && n->ref[lx][k] > 0) inc += 2;
				}
				for (int k = 0; k < ref; ++k) {
					ce_bin(g, 54 + inc, 1);
					inc = (k == 0) ? 4 : 5;
				}
				ce_bin(g, 54 + inc, 0);
			}
		}
		/* mvd: neighbour mvd sums need the mvd of earlier partitions of this MB, so restore them in
		 * emission order from a shadow copy */
		{
			int16_t saved[2][16][2];
			memcpy(saved, m->mvd, sizeof(saved));
			memset(m->mvd, 0, sizeof(m->mvd));
			for (int lx = 0; lx < 2; ++lx)
				for (int k = 0; k < s->nmvd[lx]; ++k) {
					int x = s->mvd_x[lx][k], y = s->mvd_y[lx][k], ax, ay;
					int sum[2] = {0, 0};
					gmb_t *n = nbmb(g, x - 1, y, &ax, &ay);
					if (n) { sum[0] += iabs(n->mvd[lx][ay * 4 + ax][0]); sum[1] += iabs(n->mvd[lx][ay * 4 + ax][1]); }
					n = nbmb(g, x, y - 1, &ax, &ay);
					if (n) { sum[0] += iabs(n->mvd[lx][ay * 4 + ax][0]); sum[1] += iabs(n->mvd[lx][ay * 4 + ax][1]); }
					for (int c = 0; c < 2; ++c) {
						int v = s->mvd[lx][k][c], a = iabs(v), base = c ? 47 : 40;
						int inc = sum[c] < 3 ? 0 : (sum[c] <= 32 ? 1 : 2);
						ce_bin(g, base + inc, a != 0);
						if (a) {
							int ctx = base + 3, j;
							for (j = 1; j < 9 && j < a; ++j) {
								ce_bin(g, ctx, 1);
								if (ctx < base + 6) ctx++;
							}
							if (a < 9) ce_bin(g, ctx, 0);
							else cabac_ueg(g, a - 9, 3);
							cenc_bypass(&g->ce, v < 0);
						}
					}
					for (int yy = y; yy < y + s->mvd_h[lx][k]; ++yy)
						for (int xx = x; xx < x + s->mvd_w[lx][k]; ++xx) {
							m->mvd[lx][yy * 4 + xx][0] = (int16_t)s->mvd[lx][k][0];
							m->mvd[lx][yy * 4 + xx][1] = (int16_t)s->mvd[lx][k][1];
						}
				}
			(void)saved;
		}
	}
	/* coded_block_pattern */
	if (s->kind != K_I16) {
		int ca = A ? (A->pcm ? 0x2f : (A->skip ? 0 : A->cbp)) : 0x0f;
		int cb = B ? (B->pcm ? 0x2f : (B->skip ? 0 : B->cbp)) : 0x0f;
		int cbp = m->cbp, inc;
		if (!A) ca = 0x0f;
		if (!B) cb = 0x0f;
		/* luma bits: left neighbour 8x8 of b8 0 is A's b8 1, etc. */
		inc = !(ca & 2) + 2 * !(cb & 4);
		ce_bin(g, 73 + inc, cbp & 1);
		inc = !(cbp & 1) + 2 * !(cb & 8);
		ce_bin(g, 73 + inc, (cbp >> 1) & 1);
		inc = !(ca & 8) + 2 * !(cbp & 1);
		ce_bin(g, 73 + inc, (cbp >> 2) & 1);
		inc = !(cbp & 4) + 2 * !(cbp & 2);
		ce_bin(g, 73 + inc, (cbp >> 3) & 1);
		{
			int a4 = A ? ((A->pcm ? 0x2f : (A->skip ? 0 : A->cbp)) >> 4) : 0;
			int b4 = B ? ((B->pcm ? 0x2f : (B->skip ? 0 : B->cbp)) >> 4) : 0;
			int cc = cbp >> 4;
			ce_bin(g, 77 + (a4 != 0) + 2 * (b4 != 0), cc != 0);
			if (cc) ce_bin(g, 77 + 4 + (a4 == 2) + 2 * (b4 == 2), cc == 2);
		}
		if (s->kind == K_INTER && (cbp & 15) && g->p->t8x8) {
			int is8 = (is_b && s->mbtype == 22) || (!is_b && s->mbtype == 3);
			int present = 1;
			if (is8) {
				for (int b8 = 0; b8 < 4; ++b8) {
					int shp = is_b ? b_sub_shape[s->sub[b8]] : s->sub[b8];
					if (shp != 0) present = 0;
				}
			}
			if (present) ce_bin(g, 399 + (A && A->t8x8) + (B && B->t8x8), s->t8x8);
		}
	}
	/* mb_qp_delta + residual */
	if (m->cbp || s->kind == K_I16) {
		int v = s->qpd, k = v > 0 ? 2 * v - 1 : -2 * v;
		ce_bin(g, 60 + (g->prev_qpd_nz != 0), k != 0);
		if (k) {
			for (int j = 1; j < k; ++j) ce_bin(g, j == 1 ? 62 : 63, 1);
			ce_bin(g, k == 1 ? 62 : 63, 0);
		}
		g->prev_qpd_nz = v != 0;
		m->qpd_nz = (uint8_t)(v != 0);
		/* luma */
		if (s->kind == K_I16) {
			int inc = cbf_cond_luma(g, -1, 0, 0, 1) + 2 * cbf_cond_luma(g, 0, -1, 0, 1);
			int nz = nz_count(s->ldc, 0, 16);
			ce_bin(g, cbf_base[0] + inc, nz != 0);
			if (nz) cabac_block(g, 0, s->ldc, 16);
			if (m->cbp & 15)
				for (int b = 0; b < 16; ++b) {
					int x = blk_x[b], y = blk_y[b];
					int n2 = m->nnz[y * 4 + x];
					/* temporarily hide this and later blocks from the neighbour lookup */
					inc = cbf_cond_luma(g, x - 1, y, 1, 1) + 2 * cbf_cond_luma(g, x, y - 1, 1, 1);
					ce_bin(g, cbf_base[1] + inc, n2 != 0);
					if (n2) cabac_block(g, 1, s->luma[b] + 1, 15);
				}
		} else {
			for (int b8 = 0; b8 < 4; ++b8) {
				if (!((m->cbp >> b8) & 1)) continue;
				if (s->t8x8) {
					cabac_block(g, 5, s->luma8[b8], 64);
					continue;
				}
				for (int k = 0; k < 4; ++k) {
					int b = b8 * 4 + k, x = blk_x[b], y = blk_y[b];
					int n2 = m->nnz[y * 4 + x];
					int inc = cbf_cond_luma(g, x - 1, y, 2, intra) + 2 * cbf_cond_luma(g, x, y - 1, 2, intra);
					ce_bin(g, cbf_base[2] + inc, n2 != 0);
					if (n2) cabac_block(g, 2, s->luma[b], 16);
				}
			}
		}
		if (m->cbp >> 4) {
			for (int c = 0; c < 2; ++c) {
				int inc = cbf_cond_chroma(g, c, -1, 0, 1, intra) + 2 * cbf_cond_chroma(g, c, 0, -1, 1, intra);
				int nz = nz_count(s->cdc[c], 0, 4);
				ce_bin(g, cbf_base[3] + inc, nz != 0);
				if (nz) cabac_block(g, 3, s->cdc[c], 4);
			}
			if ((m->cbp >> 4) == 2)
				for (int c = 0; c < 2; ++c)
					for (int b = 0; b < 4; ++b) {
						int x = b & 1, y = b >> 1;
						int inc = cbf_cond_chroma(g, c, x - 1, y, 0, intra) + 2 * cbf_cond_chroma(g, c, x, y - 1, 0, intra);
						int n2 = m->nnzc[c][b];
						ce_bin(g, cbf_base[4] + inc, n2 != 0);
						if (n2) cabac_block(g, 4, s->cac[c][b] + 1, 15);
					}
		}
	} else {
		g->prev_qpd_nz = 0;
	}
}

static void write_mb_cavlc(gctx_t *g, mbsyn_t *s, gmb_t *m)
{
	bw_t *w = g->w;
	int is_i = g->slice_type == 2, is_b = g->slice_type == 1;
	int intra = s->kind <= K_PCM;
	int off = is_i ? 0 : (is_b ? 23 : 5);
	if (intra) {
		int t = (s->kind == K_I4 || s->kind == K_I8) ? 0 : (s->kind == K_PCM ? 25 : s->mbtype);
		bw_ue(w, (uint32_t)(t + off));
		if (s->kind == K_PCM) {
			while (!bw_aligned(w)) bw_bit(w, 0);
			for (int i = 0; i < 384; ++i) bw_bits(w, s->pcm[i], 8);
			return;
		}
	} else {
		bw_ue(w, (uint32_t)s->mbtype);
	}
	if (s->kind == K_I4) {
		for (int i = 0; i < 16; ++i) {
			bw_bit(w, s->ipm_flag[i]);
			if (!s->ipm_flag[i]) bw_bits(w, (uint32_t)s->ipm_rem[i], 3);
		}
	}
	if (intra) {
		bw_ue(w, m->cmode);
	} else {
		int is8 = (is_b && s->mbtype == 22) || (!is_b && s->mbtype == 3);
		int np = is8 ? 4 : s->npart;
		if (is8)
			for (int b8 = 0; b8 < 4; ++b8) bw_ue(w, (uint32_t)s->sub[b8]);
		for (int lx = 0; lx < 2; ++lx) {
			int nact = lx ? g->l1n : g->l0n;
			if (nact <= 1) continue;
			for (int p = 0; p < np; ++p)
				if (s->ref[lx][p] >= 0) bw_te(w, s->ref[lx][p], nact - 1);
		}
		for (int lx = 0; lx < 2; ++lx)
			for (int k = 0; k < s->nmvd[lx]; ++k) {
				bw_se(w, s->mvd[lx][k][0]);
				bw_se(w, s->mvd[lx][k][1]);
			}
	}
	if (s->kind != K_I16) {
		int v = -1;
		for (int i = 0; i < 48; ++i)
			if (h264_me_cbp[intra ? 0 : 1][i] == m->cbp) v = i;
		bw_ue(w, (uint32_t)v);
	}
	if (m->cbp || s->kind == K_I16) {
		bw_se(w, s->qpd);
		if (s->kind == K_I16) {
			cavlc_block(w, s->ldc, 16, nc_luma(g, 0, 0));
			if (m->cbp & 15)
				for (int b = 0; b < 16; ++b) cavlc_block(w, s->luma[b] + 1, 15, nc_luma(g, blk_x[b], blk_y[b]));
		} else {
			for (int b8 = 0; b8 < 4; ++b8) {
				if (!((m->cbp >> b8) & 1)) continue;
				for (int k = 0; k < 4; ++k) {
					int b = b8 * 4 + k;
					cavlc_block(w, s->luma[b], 16, nc_luma(g, blk_x[b], blk_y[b]));
				}
			}
		}
		if (m->cbp >> 4) {
			for (int c = 0; c < 2; ++c) cavlc_block(w, s->cdc[c], 4, -1);
			if ((m->cbp >> 4) == 2)
				for (int c = 0; c < 2; ++c)
					for (int b = 0; b < 4; ++b) cavlc_block(w, s->cac[c][b] + 1, 15, nc_chroma(g, c, b & 1, b >> 1));
		}
	}
}

/* ------------------------------------------------------------------ headers */
/* SPS scaling lists (7.3.2.1.1.1) in the layout the reference reads: 6 4x4 lists, then 8 (not 2)
 * 8x8 lists for chroma_format_idc 1 (h264.cpp:280-296) — a spec layout would desynchronise it.
 * Each list is present with p = 1/2 and is either the "use default" escape (first delta makes
 * nextScale 0) or a random walk of delta_scale values, sometimes ended early by a nextScale of 0.
 * The reference discards the lists (flat dequant), so the output equals the same stream without. */
static uint32_t sl_rnd(uint64_t *x)
{
	/* own generator: the lists do not perturb the main RNG, so a stream with lists and the same
	 * stream without them carry identical slice data (tests compare their outputs) */
	*x ^= *x >> 12;
	*x ^= *x << 25;
	*x ^= *x >> 27;
	return (uint32_t)((*x * 2685821657736338717ull) >> 32);
}

static void write_scaling_lists(bw_t *r, uint64_t seed)
{
	uint64_t st = seed * 0x9e3779b97f4a7c15ull + 1;
#define rnd() sl_rnd(&st)
	for (int i = 0; i < 6 + 8; ++i) {
		int size = i < 6 ? 16 : 64, last = 8, next = 8;
		int present = (rnd() & 1) != 0;
		bw_bit(r, present);
		if (!present) continue;
		if (rnd() % 4u == 0) {
			bw_se(r, -8); /* nextScale = 0 at j = 0: useDefaultScalingMatrixFlag */
			continue;
		}
		for (int j = 0; j < size && next; ++j) {
			int target = (j > 4 && rnd() % 16u == 0) ? 0 : 4 + (int)(rnd() % 60u);
			int d = target - last;
			if (d > 127) d -= 256;
			if (d < -128) d += 256;
			bw_se(r, d);
			next = (last + d + 256) % 256;
			last = next ? next : last;
		}
	}
#undef rnd
}

static void write_sps(const params_t *p, bw_t *out, int log2_fn, int log2_poc, int poc1_cycle)
{
	bw_t r;
	bw_init(&r);
	bw_bits(&r, (uint32_t)p->profile, 8);
	bw_bits(&r, 0, 8);
	bw_bits(&r, (uint32_t)p->level, 8);
	bw_ue(&r, 0);
	if (p->profile >= 100) {
		bw_ue(&r, 1); /* chroma_format_idc */
		bw_ue(&r, 0);
		bw_ue(&r, 0);
		bw_bit(&r, 0);
		bw_bit(&r, p->scaling != 0); /* seq_scaling_matrix_present_flag */
		if (p->scaling) write_scaling_lists(&r, p->seed);
	}
	bw_ue(&r, (uint32_t)(log2_fn - 4));
	bw_ue(&r, (uint32_t)p->poc_type);
	if (p->poc_type == 0) {
		bw_ue(&r, (uint32_t)(log2_poc - 4));
	} else if (p->poc_type == 1) {
		bw_bit(&r, 0);  /* delta_pic_order_always_zero_flag */
		bw_se(&r, 0);   /* offset_for_non_ref_pic */
		bw_se(&r, 0);   /* offset_for_top_to_bottom_field */
		bw_ue(&r, (uint32_t)poc1_cycle);
		for (int i = 0; i < poc1_cycle; ++i) bw_se(&r, 1); /* offset_for_ref_frame[i] */
	}
	bw_ue(&r, (uint32_t)p->num_ref_frames);
	bw_bit(&r, 0);
	bw_ue(&r, (uint32_t)(p->width / 16 - 1));
	bw_ue(&r, (uint32_t)(p->height / 16 - 1));
	bw_bit(&r, 1); /* frame_mbs_only */
	bw_bit(&r, 1); /* direct_8x8_inference */
	bw_bit(&r, p->crop_bottom > 0);
	if (p->crop_bottom > 0) {
		bw_ue(&r, 0);
		bw_ue(&r, 0);
		bw_ue(&r, 0);
		bw_ue(&r, (uint32_t)(p->crop_bottom / 2));
	}
	bw_bit(&r, 0); /* vui */
	bw_trailing(&r);
	nal_emit(out, 3, 7, &r);
	free(r.b);
}

static void write_pps(const params_t *p, bw_t *out, int cqp_off)
{
	bw_t r;
	bw_init(&r);
	bw_ue(&r, 0);
	bw_ue(&r, 0);
	bw_bit(&r, p->cabac);
	bw_bit(&r, 0);
	bw_ue(&r, 0);
	bw_ue(&r, (uint32_t)(p->l0_active - 1));
	bw_ue(&r, (uint32_t)(p->l1_active - 1));
	bw_bit(&r, p->wp_p);
	bw_bits(&r, (uint32_t)p->wp_b, 2);
	bw_se(&r, 0); /* pic_init_qp 26 */
	bw_se(&r, 0);
	bw_se(&r, cqp_off);
	bw_bit(&r, 1); /* deblocking_filter_control_present */
	bw_bit(&r, p->cip); /* constrained_intra_pred */
	bw_bit(&r, 0);
	if (p->profile >= 100) {
		bw_bit(&r, p->t8x8);
		bw_bit(&r, 0);
		bw_se(&r, cqp_off);
	}
	bw_trailing(&r);
	nal_emit(out, 3, 8, &r);
	free(r.b);
}

/* ------------------------------------------------------------------ picture / stream */
typedef struct {
	int disp, type, idr, ref; /* type 0 P 1 B 2 I */
	int mmco5;                /* a P picture whose marking is MMCO 5 (all references unused, POC / frame_num reset) */
} picdesc_t;

/* ------------------------------------------------------------------ reference pictures
 * The generator restates the spec's reference-picture machinery (8.2.4 list initialisation and
 * modification, 8.2.5 marking) and only writes streams on which the reference decoder agrees with it;
 * where the reference deviates from the spec in a way a stream can reach, it follows the reference and
 * says so (B lists order long-term pictures by POC, h264.cpp:10929-10935 — the generator keeps
 * LongTermFrameIdx order equal to POC order, so both orders agree; no L1 swap when L1 == L0,
 * h264.cpp:10985; zero vectors for temporal direct from a long-term reference, h264.cpp:10049-10054;
 * POC type 1 of the IDR, h264.cpp:1183-1185). */
typedef struct {
	int disp, poc, frame_num;
	int long_term, lt_idx; /* long-term reference (LongTermFrameIdx) */
	int store;             /* its co-located store (gen_stream's pool) */
} dpbref_t;

typedef struct {
	dpbref_t e[16];
	int n;
	int max_lt_idx; /* MaxLongTermFrameIdx; -1: "no long-term frame indices" */
} gdpb_t;

/* DistScaleFactor (8.4.1.2.3) */
static int dist_scale(int poc0, int poc1, int cur)
{
	int td = clampi(poc1 - poc0, -128, 127), tb = clampi(cur - poc0, -128, 127), tx;
	if (td == 0) return 256; /* mvL0 = mvCol, mvL1 = 0 */
	tx = (16384 + abs(td / 2)) / td;
	return clampi((tb * tx + 32) >> 6, -1024, 1023);
}

/* FrameNumWrap / PicNum of a short-term frame (8.2.4.1) */
static int pic_num(const dpbref_t *r, int cur_fn, int max_fn) { return r->frame_num > cur_fn ? r->frame_num - max_fn : r->frame_num; }

static void sort_by(dpbref_t *v, int n, int (*before)(const dpbref_t *, const dpbref_t *, int, int), int a, int b)
{
	for (int i = 1; i < n; ++i) {
		dpbref_t t = v[i];
		int j = i - 1;
		while (j >= 0 && before(&t, &v[j], a, b)) {
			v[j + 1] = v[j];
			j--;
		}
		v[j + 1] = t;
	}
}
static int p_before(const dpbref_t *l, const dpbref_t *r, int cur_fn, int max_fn)
{
	if (l->long_term != r->long_term) return !l->long_term;
	if (l->long_term) return l->lt_idx < r->lt_idx;                         /* ascending LongTermPicNum */
	return pic_num(l, cur_fn, max_fn) > pic_num(r, cur_fn, max_fn);          /* descending PicNum */
}
static int b0_before(const dpbref_t *l, const dpbref_t *r, int cur, int unused)
{
	(void)unused;
	if (l->long_term != r->long_term) return !l->long_term;
	if (l->long_term) return l->poc < r->poc; /* (reference: by POC; LongTermFrameIdx order kept equal) */
	if ((l->poc < cur) != (r->poc < cur)) return l->poc < cur;
	return l->poc < cur ? l->poc > r->poc : l->poc < r->poc;
}
static int b1_before(const dpbref_t *l, const dpbref_t *r, int cur, int unused)
{
	(void)unused;
	if (l->long_term != r->long_term) return !l->long_term;
	if (l->long_term) return l->poc < r->poc;
	if ((l->poc > cur) != (r->poc > cur)) return l->poc > cur;
	return l->poc > cur ? l->poc < r->poc : l->poc > r->poc;
}

/* one ref_pic_list_modification operation (8.2.4.3) */
typedef struct {
	int idc, val;
} lmod_t;

static int same_pic(const dpbref_t *a, const dpbref_t *b) { return a->long_term == b->long_term && a->disp == b->disp; }

/* choose up to 3 modifications of list `l` (n entries, `act` active) over the DPB, write them to `ops` and
 * apply them (8.2.4.3.1 / 8.2.4.3.2); distinct targets (the reference's list arrays then stay
 * permutations, h264.cpp:1640-1650).  Returns the number of operations. */
static int choose_modification(const gdpb_t *dpb, dpbref_t *l, int n, int act, int cur_fn, int max_fn, lmod_t *ops)
{
	int nops = 1 + (int)(rnd() % 3u), k = 0, pred = cur_fn;
	int used[16] = {0};
	if (nops > act) nops = act;
	for (int idx = 0; idx < nops; ++idx) {
		int cand[16], nc = 0;
		for (int i = 0; i < dpb->n; ++i)
			if (!used[i]) cand[nc++] = i;
		if (!nc) break;
		const int t = cand[rnd() % (unsigned)nc];
		const dpbref_t *tg = &dpb->e[t];
		used[t] = 1;
		if (tg->long_term) {
			ops[k].idc = 2;
			ops[k].val = tg->lt_idx;
		} else {
			const int pn = pic_num(tg, cur_fn, max_fn);
			if (pn < pred) {
				ops[k].idc = 0;
				ops[k].val = pred - pn - 1; /* abs_diff_pic_num_minus1 */
			} else {
				ops[k].idc = 1;
				ops[k].val = pn - pred - 1;
			}
			pred = pn;
		}
		k++;
		/* insert at idx, shift, drop the later copy (the list is temporarily n + 1 long) */
		{
			dpbref_t tmp[17];
			int m = 0;
			for (int i = 0; i < idx; ++i) tmp[m++] = l[i];
			tmp[m++] = *tg;
			for (int i = idx; i < n; ++i)
				if (!same_pic(&l[i], tg)) tmp[m++] = l[i];
			for (int i = 0; i < n && i < m; ++i) l[i] = tmp[i];
		}
	}
	return k;
}

static void write_modification(bw_t *r, const lmod_t *ops, int n)
{
	bw_bit(r, n > 0);
	if (!n) return;
	for (int i = 0; i < n; ++i) {
		bw_ue(r, (uint32_t)ops[i].idc);
		bw_ue(r, (uint32_t)ops[i].val);
	}
	bw_ue(r, 3);
}

/* adaptive marking operation (8.2.5.4) */
typedef struct {
	int op, a1, a2;
} mmco_t;

static int count_kind(const gdpb_t *d, int lt)
{
	int c = 0;
	for (int i = 0; i < d->n; ++i) c += d->e[i].long_term == lt;
	return c;
}
static void dpb_remove(gdpb_t *d, int i) { d->e[i] = d->e[--d->n]; }

/* a LongTermFrameIdx for a picture of POC `poc` such that LongTermFrameIdx order equals POC order among the
 * long-term frames (other than `skip`), or -1 */
static int lt_idx_for(const gdpb_t *d, int poc, int skip)
{
	int cand[16], nc = 0;
	for (int L = 0; L <= d->max_lt_idx; ++L) {
		int ok = 1;
		for (int i = 0; i < d->n && ok; ++i) {
			const dpbref_t *e = &d->e[i];
			if (i == skip || !e->long_term) continue;
			if (e->lt_idx == L) ok = 0; /* (never replace: the reference's MMCO 6 would keep both) */
			else if ((e->lt_idx < L) != (e->poc < poc)) ok = 0;
		}
		if (ok) cand[nc++] = L;
	}
	return nc ? cand[rnd() % (unsigned)nc] : -1;
}

/* choose the adaptive marking of the current (reference, non-IDR) picture and apply it to the DPB; the
 * current picture itself is added by the caller (unless it became long-term: *cur_lt >= 0) */
static int choose_mmco(const params_t *p, gdpb_t *d, int cur_fn, int max_fn, int cur_poc, mmco_t *ops, int *cur_lt)
{
	int k = 0;
	*cur_lt = -1;
	const int max_lt = imax(0, p->num_ref_frames - 2); /* keep a short-term frame beside the current one */
	if (p->long_term && d->max_lt_idx < 0 && pct(70)) {
		ops[k++] = (mmco_t){4, 2, 0}; /* MaxLongTermFrameIdx = 1 */
		d->max_lt_idx = 1;
	}
	for (int step = 0; step < 3; ++step) {
		const int r = (int)(rnd() % 100u);
		if (p->long_term && d->max_lt_idx >= 0 && r < 30 && count_kind(d, 1) < max_lt && count_kind(d, 0) > 1) {
			/* MMCO 3: a short-term frame (not the newest) becomes long-term */
			int cand[16], nc = 0;
			for (int i = 0; i < d->n; ++i)
				if (!d->e[i].long_term) cand[nc++] = i;
			const int i = cand[rnd() % (unsigned)nc];
			const int L = lt_idx_for(d, d->e[i].poc, i);
			if (L < 0) continue;
			ops[k++] = (mmco_t){3, cur_fn - pic_num(&d->e[i], cur_fn, max_fn) - 1, L};
			d->e[i].long_term = 1;
			d->e[i].lt_idx = L;
		} else if (r < 45 && count_kind(d, 1) > 0) {
			/* MMCO 2: a long-term frame unused */
			int cand[16], nc = 0;
			for (int i = 0; i < d->n; ++i)
				if (d->e[i].long_term) cand[nc++] = i;
			const int i = cand[rnd() % (unsigned)nc];
			ops[k++] = (mmco_t){2, d->e[i].lt_idx, 0};
			dpb_remove(d, i);
		} else if (r < 75 && count_kind(d, 0) > 1) {
			/* MMCO 1: a short-term frame unused */
			int cand[16], nc = 0;
			for (int i = 0; i < d->n; ++i)
				if (!d->e[i].long_term) cand[nc++] = i;
			const int i = cand[rnd() % (unsigned)nc];
			ops[k++] = (mmco_t){1, cur_fn - pic_num(&d->e[i], cur_fn, max_fn) - 1, 0};
			dpb_remove(d, i);
		} else if (p->long_term && d->max_lt_idx >= 0 && r < 90 && d->max_lt_idx >= 1 && count_kind(d, 1) > 0 && pct(30)) {
			/* MMCO 4: MaxLongTermFrameIdx = 0 (long-term frames with index 1 unused) */
			ops[k++] = (mmco_t){4, 1, 0};
			d->max_lt_idx = 0;
			for (int i = d->n - 1; i >= 0; --i)
				if (d->e[i].long_term && d->e[i].lt_idx > 0) dpb_remove(d, i);
		}
	}
	/* room for the current picture: spec marking has no sliding window after adaptive ops */
	while (d->n + 1 > p->num_ref_frames) {
		int oldest = -1;
		for (int i = 0; i < d->n; ++i)
			if (!d->e[i].long_term && (oldest < 0 || pic_num(&d->e[i], cur_fn, max_fn) < pic_num(&d->e[oldest], cur_fn, max_fn)))
				oldest = i;
		if (oldest < 0) { /* only long-term frames: drop one */
			ops[k++] = (mmco_t){2, d->e[0].lt_idx, 0};
			dpb_remove(d, 0);
			continue;
		}
		ops[k++] = (mmco_t){1, cur_fn - pic_num(&d->e[oldest], cur_fn, max_fn) - 1, 0};
		dpb_remove(d, oldest);
	}
	/* MMCO 6: the current picture long-term (last, as the reference applies it where it stands) */
	if (p->long_term && d->max_lt_idx >= 0 && count_kind(d, 1) < max_lt && pct(25)) {
		const int L = lt_idx_for(d, cur_poc, -1);
		if (L >= 0) {
			ops[k++] = (mmco_t){6, L, 0};
			*cur_lt = L;
		}
	}
	return k;
}

static void write_marking(bw_t *r, const picdesc_t *pd, int lt_idr, const mmco_t *ops, int n)
{
	if (pd->idr) {
		bw_bit(r, 0); /* no_output_of_prior_pics */
		bw_bit(r, lt_idr);
		return;
	}
	bw_bit(r, n > 0); /* adaptive_ref_pic_marking_mode_flag */
	if (!n) return;
	for (int i = 0; i < n; ++i) {
		bw_ue(r, (uint32_t)ops[i].op);
		if (ops[i].op == 1 || ops[i].op == 2 || ops[i].op == 4 || ops[i].op == 6) bw_ue(r, (uint32_t)ops[i].a1);
		if (ops[i].op == 3) {
			bw_ue(r, (uint32_t)ops[i].a1);
			bw_ue(r, (uint32_t)ops[i].a2);
		}
	}
	bw_ue(r, 0);
}

static void write_pred_weight_table(gctx_t *g, bw_t *r, int nl)
{
	int ld = rr(4, 5), cd = rr(4, 5); /* weights <= 48: bi sums stay inside int16 (Appendix A #1) */
	const int q = g->p->quirks;
	if (q) { /* denominator 7: absent weights default to 128, stored as int8 -128 (A#16) */
		ld = pct(50) ? 7 : 6;
		cd = pct(50) ? 7 : 6;
	}
	bw_ue(r, (uint32_t)ld);
	bw_ue(r, (uint32_t)cd);
	for (int lx = 0; lx < nl; ++lx) {
		int n = lx ? g->l1n : g->l0n;
		for (int i = 0; i < n; ++i) {
			int f = pct(q ? 60 : 70);
			bw_bit(r, f);
			if (f) {
				/* quirks: weights near 127 overflow the SSE2 int16 sum of a bright bi-pair (A#1) */
				bw_se(r, q ? rr(96, 127) : rr((1 << ld) / 2, (1 << ld) * 3 / 2));
				bw_se(r, q ? rr(0, 40) : rr(-20, 20));
			}
			f = pct(50);
			bw_bit(r, f);
			if (f)
				for (int c = 0; c < 2; ++c) {
					bw_se(r, q ? rr(96, 127) : rr((1 << cd) / 2, (1 << cd) * 3 / 2));
					bw_se(r, q ? rr(0, 20) : rr(-12, 12));
				}
		}
	}
}

int gen_stream(const params_t *p, bw_t *out, FILE *dump, FILE *refdump)
{
	gctx_t G, *g = &G;
	picdesc_t *order;
	const int log2_fn = p->log2_fn ? p->log2_fn : 8, log2_poc = 10, max_fn = 1 << log2_fn;
	int n = 0;
	gdpb_t dpb;
	gcol_t *store[17];
	int last_ref_fn = 0, idr_count = 0, cqp_off;
	int poc_base = 0;                      /* display index of the last IDR / MMCO 5 picture */
	int prev_fn = 0, fn_offset = 0;        /* POC types 1 / 2: previous picture's frame_num, FrameNumOffset */
	int poc1_cycle = 1;                    /* POC type 1: num_ref_frames_in_pic_order_cnt_cycle (offsets 1) */
	bw_t r;
	mbsyn_t *syn = (mbsyn_t *)calloc(1, sizeof(mbsyn_t));

	memset(g, 0, sizeof(*g));
	memset(&dpb, 0, sizeof(dpb));
	dpb.max_lt_idx = -1;
	rs = p->seed * 0x9E3779B97F4A7C15ull + 0x1234567ull;
	if (!rs) rs = 1;
	for (int i = 0; i < 8; ++i) rnd();
	g->p = p;
	g->mbw = p->width / 16;
	g->mbh = p->height / 16;
	g->nmb = g->mbw * g->mbh;
	g->mb = (gmb_t *)calloc((size_t)g->nmb, sizeof(gmb_t));
	g->rw = (g->mbw + 3) / 4;
	g->rh = (g->mbh + 3) / 4;
	g->region = (int16_t *)calloc((size_t)(g->rw * g->rh * 2), sizeof(int16_t));
	for (int i = 0; i < 17; ++i) store[i] = (gcol_t *)calloc((size_t)g->nmb, sizeof(gcol_t));
	bw_init(&r);
	if (p->poc_type == 1) poc1_cycle = 1 + (int)(p->seed % 3u);

	/* coding order */
	order = (picdesc_t *)calloc((size_t)p->frames, sizeof(picdesc_t));
	{
		int d = 0, prev_nonref = 0;
		int step = p->bframes + 1;
		while (d < p->frames) {
			if (d == 0) {
				order[n++] = (picdesc_t){0, 2, 1, 1, 0};
				d = 1;
				continue;
			}
			/* anchor at the end of the next group, then the B pictures before it */
			{
				int a = imin(d + step - 1, p->frames - 1);
				int is_i = (p->gop > 0 && a % p->gop == 0);
				int is_idr = is_i && p->idr_period > 0 && a % p->idr_period == 0;
				int is_m5 = !is_i && p->mmco5 > 0 && a % p->mmco5 == 0;
				if (is_idr || is_m5) {
					/* no B picture may reference across an IDR / MMCO 5 picture: emit the Bs first as P */
					for (int b = d; b < a; ++b) order[n++] = (picdesc_t){b, 0, 0, 1, 0};
					order[n++] = (picdesc_t){a, is_idr ? 2 : 0, is_idr, 1, is_m5};
					prev_nonref = 0;
				} else {
					/* IPPP: some P pictures non-reference (never two in a row, never right after an IDR) */
					int ref = 1;
					if (step == 1 && !is_i && p->nonref_pct && !prev_nonref && n > 1 && pct(p->nonref_pct)) ref = 0;
					prev_nonref = !ref;
					order[n++] = (picdesc_t){a, is_i ? 2 : 0, 0, ref, 0};
					for (int b = d; b < a; ++b) order[n++] = (picdesc_t){b, 1, 0, 0, 0};
				}
				d = a + 1;
			}
		}
	}

	cqp_off = rr(-2, 2);
	write_sps(p, out, log2_fn, log2_poc, poc1_cycle);
	write_pps(p, out, cqp_off);

	for (int pi = 0; pi < n; ++pi) {
		picdesc_t pd = order[pi];
		int frame_num, poc, delta_poc0 = 0, lt_idr = 0;
		int nsl = imax(1, p->slices), rows_per = (g->mbh + nsl - 1) / nsl;
		lmod_t mods[2][4];
		int nmods[2] = {0, 0};
		mmco_t mmco[16];
		int nmmco = 0, cur_lt = -1, td_ok = 1;
		if (pd.idr) {
			dpb.n = 0;
			dpb.max_lt_idx = -1;
			frame_num = 0;
			idr_count++;
			poc_base = pd.disp;
		} else {
			frame_num = (last_ref_fn + 1) % max_fn;
		}
		/* POC (8.2.1) */
		if (pd.idr) fn_offset = 0;
		else if (prev_fn > frame_num) fn_offset += max_fn;
		if (p->poc_type == 2) {
			poc = 2 * (fn_offset + frame_num) - (pd.ref ? 0 : 1);
		} else {
			poc = 2 * (pd.disp - poc_base);
			if (p->poc_type == 1) {
				/* expectedPicOrderCnt with offset_for_ref_frame[i] = 1 (= absFrameNum), offset_for_non_ref_pic 0;
				 * absFrameNum 0: the reference takes offset_for_ref_frame[0] (h264.cpp:1183-1185) */
				int abs_fn = fn_offset + frame_num;
				if (!pd.ref && abs_fn > 0) abs_fn--;
				const int expected = abs_fn > 0 ? abs_fn : 1;
				delta_poc0 = poc - expected;
			}
		}
		prev_fn = frame_num;
		g->poc = poc;
		/* motion field for this picture */
		{
			int v = imax(1, p->mv_px * 4 / 6);
			g->gv[0] = rr(-v, v);
			g->gv[1] = rr(-v / 2, v / 2);
			for (int i = 0; i < g->rw * g->rh * 2; ++i) g->region[i] = (int16_t)rr(-v / 2, v / 2);
		}
		/* reference lists (8.2.4.2, then the modifications of 8.2.4.3) */
		{
			dpbref_t l0[16], l1[16];
			int n0 = 0, n1 = 0;
			for (int i = 0; i < dpb.n; ++i) l0[n0++] = l1[n1++] = dpb.e[i];
			if (pd.type == 0) {
				sort_by(l0, n0, p_before, frame_num, max_fn);
				n1 = 0;
			} else if (pd.type == 1) {
				sort_by(l0, n0, b0_before, poc, 0);
				sort_by(l1, n1, b1_before, poc, 0);
				/* (L1 == L0 with more than one entry: the spec swaps L1[0] / L1[1]; the reference never does,
				 * h264.cpp:10985 — the generator follows the reference) */
			} else {
				n0 = n1 = 0;
			}
			g->l0n = imin(p->l0_active, n0);
			g->l1n = imin(p->l1_active, n1);
			if (pd.type == 1 && (g->l0n == 0 || g->l1n == 0)) pd.type = 0;
			if (pd.type == 0 && g->l0n == 0) pd.type = 2;
			if (pd.type == 0) {
				sort_by(l0, n0, p_before, frame_num, max_fn);
				n1 = 0;
				g->l1n = 0;
			}
			if (pd.type != 2 && p->reorder_pct && pct(p->reorder_pct)) nmods[0] = choose_modification(&dpb, l0, n0, g->l0n, frame_num, max_fn, mods[0]);
			if (pd.type == 1 && p->reorder_pct && pct(p->reorder_pct)) nmods[1] = choose_modification(&dpb, l1, n1, g->l1n, frame_num, max_fn, mods[1]);
			g->taint = 0;
			for (int i = 0; i < g->l0n; ++i) {
				g->ref_poc[0][i] = l0[i].poc;
				g->ref_lt[0][i] = l0[i].long_term;
			}
			for (int i = 0; i < g->l1n; ++i) {
				g->ref_poc[1][i] = l1[i].poc;
				g->ref_lt[1][i] = l1[i].long_term;
			}
			td_ok = 1;
			if (pd.type == 1) {
				g->col = store[l1[0].store];
				for (int i = 0; i < g->l0n; ++i) g->dsf[i] = dist_scale(l0[i].poc, l1[0].poc, poc);
				/* temporal direct needs every picture the co-located blocks reference in the active L0
				 * (MapColToList0, 8.4.1.2.3); marking (MMCO 1 / 5, the sliding window) or list modification can
				 * leave one out — spec-undefined, and the reference maps it through its marked list array
				 * (h264.cpp:10962-10968): such pictures use spatial direct */
				for (int a = 0; a < g->nmb && td_ok; ++a)
					for (int b8 = 0; b8 < 4 && td_ok; ++b8) {
						int k = 0;
						if (g->col[a].ref[b8] < 0) continue;
						while (k < g->l0n && g->ref_poc[0][k] != g->col[a].ref_poc[b8]) ++k;
						td_ok = k < g->l0n;
					}
			}
		}
		/* marking of this picture (syntax in every slice header; applied after the picture) */
		if (pd.ref && pd.idr) {
			lt_idr = p->long_term && pct(30);
		} else if (pd.ref && pd.mmco5) {
			mmco[nmmco++] = (mmco_t){5, 0, 0};
		} else if (pd.ref && p->mmco_pct && pct(p->mmco_pct)) {
			gdpb_t after = dpb;
			nmmco = choose_mmco(p, &after, frame_num, max_fn, poc, mmco, &cur_lt);
			if (nmmco) dpb = after;
		}
		for (int i = 0; i < g->nmb; ++i) g->mb[i].slice = -1;

		for (int sl = 0; sl < nsl; ++sl) {
			int first = sl * rows_per * g->mbw, last = imin(g->nmb, (sl + 1) * rows_per * g->mbw);
			int slice_qp = rr(p->qp_min, p->qp_max);
			int didc = 0, aoff = 0, boff = 0, cinit = rr(0, 2);
			int skip_run = 0;
			if (first >= g->nmb) break;
			g->slice_type = pd.type;
			g->slice_id = pi * 256 + sl;
			g->qp = slice_qp;
			g->prev_qpd_nz = 0;
			g->direct_spatial = (p->direct == 2) ? pct(50) : p->direct;
			if (!td_ok) g->direct_spatial = 1;
			if (p->deblock) {
				int r2 = (int)(rnd() % 100u);
				didc = (r2 < 10) ? 1 : ((p->idc2 && r2 < 40) ? 2 : 0);
				aoff = rr(-3, 3);
				boff = rr(aoff, 3);
			}
			if (refdump) {
				gen_refdump_t rd;
				memset(&rd, 0, sizeof(rd));
				rd.pic = pi;
				rd.first_mb = first;
				rd.slice_type = pd.type;
				rd.poc = poc;
				rd.n[0] = pd.type != 2 ? g->l0n : 0;
				rd.n[1] = pd.type == 1 ? g->l1n : 0;
				for (int lx = 0; lx < 2; ++lx)
					for (int i = 0; i < rd.n[lx]; ++i) {
						rd.poc_l[lx][i] = g->ref_poc[lx][i];
						rd.lt[lx][i] = (int8_t)g->ref_lt[lx][i];
					}
				fwrite(&rd, sizeof(rd), 1, refdump);
			}
			bw_reset(&r);
			bw_ue(&r, (uint32_t)first);
			bw_ue(&r, (uint32_t)(pd.type == 2 ? 7 : (pd.type == 1 ? 6 : 5)));
			bw_ue(&r, 0);
			bw_bits(&r, (uint32_t)frame_num, log2_fn);
			if (pd.idr) bw_ue(&r, (uint32_t)(idr_count & 1));
			if (p->poc_type == 0) bw_bits(&r, (uint32_t)(poc & ((1 << log2_poc) - 1)), log2_poc);
			else if (p->poc_type == 1) bw_se(&r, delta_poc0);
			if (pd.type == 1) bw_bit(&r, g->direct_spatial);
			if (pd.type != 2) {
				bw_bit(&r, 1); /* num_ref_idx_active_override */
				bw_ue(&r, (uint32_t)(g->l0n - 1));
				if (pd.type == 1) bw_ue(&r, (uint32_t)(g->l1n - 1));
				write_modification(&r, mods[0], nmods[0]);
				if (pd.type == 1) write_modification(&r, mods[1], nmods[1]);
			}
			if ((p->wp_p && pd.type == 0) || (p->wp_b == 1 && pd.type == 1)) write_pred_weight_table(g, &r, pd.type == 1 ? 2 : 1);
			if (pd.ref) write_marking(&r, &pd, lt_idr, mmco, nmmco);
			if (p->cabac && pd.type != 2) bw_ue(&r, (uint32_t)cinit);
			bw_se(&r, slice_qp - 26);
			bw_ue(&r, (uint32_t)didc);
			if (didc != 1) {
				bw_se(&r, aoff);
				bw_se(&r, boff);
			}
			g->w = &r;
			if (p->cabac) {
				while (!bw_aligned(&r)) bw_bit(&r, 1);
				cenc_init_ctx(&g->ce, pd.type == 2, cinit, slice_qp);
				cenc_start(&g->ce, &r);
			}
			for (int a = first; a < last; ++a) {
				gmb_t *m = &g->mb[a];
				mbsyn_t *s = syn;
				int skip = 0;
				g->cur = a;
				g->mbx = a % g->mbw;
				g->mby = a / g->mbw;
				memset(m, 0, sizeof(*m));
				memset(m->ipm, -1, sizeof(m->ipm));
				m->slice = g->slice_id;
				memset(s, 0, offsetof(mbsyn_t, ldc));
				if (pd.type != 2 && pct(p->p_skip_pct)) {
					skip = 1;
					m->skip = 1;
					s->kind = K_SKIP;
					if (pd.type == 0) {
						int mv[2];
						pskip_mv(g, mv);
						for (int k = 0; k < 4; ++k) {
							m->ref[0][k] = 0;
							m->ref[1][k] = -1;
						}
						for (int k = 0; k < 16; ++k) {
							m->mv[0][k][0] = (int16_t)mv[0];
							m->mv[0][k][1] = (int16_t)mv[1];
						}
					} else {
						m->direct16 = 1;
						m->dir8 = 15;
						for (int b8 = 0; b8 < 4; ++b8) direct_motion(g, m, b8);
					}
				} else if (pd.type == 2 || pct(p->p_intra_pct)) {
					choose_intra(g, s, m);
				} else {
					choose_inter(g, s, m);
				}
				if (!skip && s->kind != K_PCM) {
					if (m->cbp || s->kind == K_I16) {
						int nq = clampi(g->qp + rr(-2, 2), p->qp_min, p->qp_max);
						s->qpd = nq - g->qp;
						g->qp = nq;
					}
					choose_residual(g, s, m, g->qp);
				}
				if (dump) {
					gen_dump_t dd;
					memset(&dd, 0, sizeof(dd));
					dd.pic = pi;
					dd.mbaddr = a;
					dd.kind = (uint8_t)s->kind;
					dd.cbp = m->cbp;
					dd.qp = (int8_t)g->qp;
					dd.t8x8 = (uint8_t)(s->kind == K_I8 || (s->kind == K_INTER && s->t8x8));
					dd.exact_mv = !g->taint;
					dd.dir8 = m->dir8;
					dd.i16_pred = (uint8_t)s->i16_pred;
					dd.cmode = m->cmode;
					if (s->kind == K_I4)
						for (int b = 0; b < 16; ++b) dd.ipm[b] = m->ipm[blk_y[b] * 4 + blk_x[b]];
					if (s->kind == K_I8)
						for (int b8 = 0; b8 < 4; ++b8) dd.ipm[b8] = m->ipm[(b8 >> 1) * 8 + (b8 & 1) * 2];
					for (int lx = 0; lx < 2; ++lx)
						for (int k = 0; k < 4; ++k) dd.ref[lx][k] = m->ref[lx][k];
					memcpy(dd.mv, m->mv, sizeof(dd.mv));
					if (!skip && s->kind != K_PCM) {
						if (s->kind == K_I16) {
							for (int i = 0; i < 16; ++i) dd.ldc[zz4[i]] = s->ldc[i];
							if (m->cbp & 15)
								for (int b = 0; b < 16; ++b)
									for (int i = 1; i < 16; ++i) dd.luma[b * 16 + zz4[i]] = s->luma[b][i];
						} else {
							for (int b8 = 0; b8 < 4; ++b8) {
								if (!((m->cbp >> b8) & 1)) continue;
								if (dd.t8x8) {
									for (int i = 0; i < 64; ++i) dd.luma[b8 * 64 + zz8[i]] = s->luma8[b8][i];
								} else {
									for (int k = 0; k < 4; ++k)
										for (int i = 0; i < 16; ++i) dd.luma[(b8 * 4 + k) * 16 + zz4[i]] = s->luma[b8 * 4 + k][i];
								}
							}
						}
						if (m->cbp >> 4)
							for (int c = 0; c < 2; ++c)
								for (int i = 0; i < 4; ++i) dd.cdc[c][i] = s->cdc[c][i];
						if ((m->cbp >> 4) == 2)
							for (int c = 0; c < 2; ++c)
								for (int b = 0; b < 4; ++b)
									for (int i = 1; i < 16; ++i) dd.cac[c][b][zz4[i]] = s->cac[c][b][i];
					}
					fwrite(&dd, sizeof(dd), 1, dump);
				}
				if (p->cabac) {
					if (pd.type != 2) {
						int bx, by;
						gmb_t *A = nbmb(g, -1, 0, &bx, &by), *B = nbmb(g, 0, -1, &bx, &by);
						int inc = (A && !A->skip) + (B && !B->skip);
						ce_bin(g, (pd.type == 1 ? 24 : 11) + inc, skip);
					}
					if (!skip) write_mb_cabac(g, s, m);
					else g->prev_qpd_nz = 0;
					if (s->kind == K_PCM) g->prev_qpd_nz = 0;
					cenc_terminate(&g->ce, a == last - 1);
				} else {
					if (skip) {
						skip_run++;
					} else {
						if (pd.type != 2) bw_ue(&r, (uint32_t)skip_run);
						skip_run = 0;
						write_mb_cavlc(g, s, m);
					}
				}
			}
			if (!p->cabac) {
				if (skip_run) bw_ue(&r, (uint32_t)skip_run);
				bw_trailing(&r);
			} else {
				while (!bw_aligned(&r)) bw_bit(&r, 0);
			}
			nal_emit(out, pd.ref ? 2 : 0, pd.idr ? 5 : 1, &r);
		}
		/* reference marking (8.2.5): IDR, MMCO 5, adaptive (applied above), or the sliding window */
		if (pd.ref) {
			int used[17] = {0}, st = 0;
			dpbref_t cur;
			if (pd.mmco5) {
				dpb.n = 0;
				dpb.max_lt_idx = -1;
			} else if (!pd.idr && !nmmco && dpb.n == p->num_ref_frames) {
				int oldest = -1;
				for (int i = 0; i < dpb.n; ++i)
					if (!dpb.e[i].long_term && (oldest < 0 || pic_num(&dpb.e[i], frame_num, max_fn) < pic_num(&dpb.e[oldest], frame_num, max_fn)))
						oldest = i;
				if (oldest >= 0) dpb_remove(&dpb, oldest);
			}
			/* the picture's co-located store: L0 motion (anchors are I / P) or intra */
			for (int i = 0; i < dpb.n; ++i) used[dpb.e[i].store] = 1;
			while (used[st]) ++st;
			for (int a = 0; a < g->nmb; ++a) {
				const gmb_t *m = &g->mb[a];
				gcol_t *c = &store[st][a];
				for (int b8 = 0; b8 < 4; ++b8) {
					c->ref[b8] = m->ref[0][b8];
					c->ref_poc[b8] = m->ref[0][b8] >= 0 ? g->ref_poc[0][m->ref[0][b8]] : 0;
				}
				for (int k = 0; k < 16; ++k) {
					int on = m->ref[0][(k >> 3) * 2 + ((k & 3) >> 1)] >= 0;
					c->mv[k][0] = on ? m->mv[0][k][0] : 0;
					c->mv[k][1] = on ? m->mv[0][k][1] : 0;
				}
			}
			cur = (dpbref_t){pd.disp, poc, frame_num, 0, 0, st};
			if (pd.idr && lt_idr) {
				cur.long_term = 1; /* LongTermFrameIdx 0, MaxLongTermFrameIdx 0 */
				dpb.max_lt_idx = 0;
			}
			if (cur_lt >= 0) {
				cur.long_term = 1;
				cur.lt_idx = cur_lt;
			}
			if (pd.mmco5) {
				/* after MMCO 5 the picture counts as frame_num 0, POC 0 (8.2.1), and later POCs restart from it */
				cur.frame_num = 0;
				cur.poc = 0;
				poc_base = pd.disp;
				fn_offset = 0;
				prev_fn = 0;
			}
			dpb.e[dpb.n++] = cur;
			last_ref_fn = cur.frame_num;
		}
	}
	free(r.b);
	free(order);
	free(g->mb);
	free(g->region);
	for (int i = 0; i < 17; ++i) free(store[i]);
	free(syn);
	return n;
}
