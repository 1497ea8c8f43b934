/*
 * H.264 macroblock layer for the m2dec_amd host parser: CABAC / CAVLC entropy decoding, motion
 * vector prediction (incl. P_Skip, spatial and temporal direct), deblocking boundary strengths,
 * and emission of the reconstruction records (include/m2d_recon.h).
 *
 * The parse is semantically the reference's (h264.cpp:1739-2110 CAVLC, 11052-12055 CABAC,
 * 6651-10127 motion, 7119-9390 bS), restated around a per-macroblock neighbour store instead of
 * the reference's fused parse+recon.  Reconstruction itself is NOT done here: every sample
 * operation is deferred to the back end through the records.
 */
#include <stdio.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <unistd.h>
#include <time.h>
#include "h264_dec.h"

/* blkIdx -> 4x4 position (spec 6.4.3) and inverse */
static const uint8_t blk_x[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static const uint8_t blk_y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
static const uint8_t rast2blk[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
/* frame zig-zag scans, raster index = y * N + x (spec 8.5.6) */
static const uint8_t zz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
static const uint8_t zz8[64] = {
	0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
	12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
	35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
	58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iabs(int a) { return a < 0 ? -a : a; }
static inline int median3(int a, int b, int c) { return imax(imin(a, b), imin(imax(a, b), c)); }

/* ================================================================== CABAC engine (9.3.1.2, 9.3.3.2) */
static void cab_build(void);
static pthread_once_t cab_once;

static void cabac_init_ctx(h264_cabac_t *c, int qp, int idc)
{
	pthread_once(&cab_once, cab_build);
	const int8_t (*mn)[2] = h264_cabac_init_mn[idc];
	for (int i = 0; i < H264_NUM_CTX; ++i) {
		int pre = ((mn[i][0] * qp) >> 4) + mn[i][1];
		if (pre < 1) pre = 1;
		if (pre > 126) pre = 126;
		c->ctx[i] = (pre <= 63) ? (uint8_t)((63 - pre) << 1) : (uint8_t)(((pre - 64) << 1) | 1);
	}
}

/* Engine state lives in h264_cabac_eng_t; the eng_* primitives take it apart from the context
 * bytes so that a caller holding a local copy keeps value/range/bits in registers (a store to a
 * uint8_t context may alias anything reachable through a pointer). */
static inline void eng_refill(h264_cabac_eng_t *e)
{
	if (e->bits >= 16) return;
	if (__builtin_expect(e->p + 4 <= e->end, 1)) {
		/* value < range << bits < 2^25 here: a 32-bit look-ahead keeps it under 2^57 */
		uint32_t w = ((uint32_t)e->p[0] << 24) | ((uint32_t)e->p[1] << 16) | ((uint32_t)e->p[2] << 8) | e->p[3];
		e->p += 4;
		e->value = (e->value << 32) | w;
		e->bits += 32;
		return;
	}
	while (e->bits < 24) {
		uint32_t byte = (e->p < e->end) ? *e->p : 0;
		e->p++;
		e->value = (e->value << 8) | byte;
		e->bits += 8;
	}
}

static void cabac_start(h264_cabac_t *c, const uint8_t *p, const uint8_t *end)
{
	h264_cabac_eng_t *e = &c->e;
	e->p = p;
	e->end = end;
	e->value = 0;
	e->bits = -9;
	e->range = 510;
	while (e->bits < 16) { /* the 9-bit codIOffset plus look-ahead */
		uint32_t byte = (e->p < e->end) ? *e->p : 0;
		e->p++;
		e->value = (e->value << 8) | byte;
		e->bits += 8;
	}
}

/* bit position (spec bitstream pointer) relative to the start of the engine's data */
static inline size_t cabac_bitpos(const h264_cabac_t *c, const uint8_t *start)
{
	return (size_t)(c->e.p - start) * 8 - (size_t)c->e.bits;
}

/* next context byte after a bin: cab_next[(lps << 7) | ctx] (9.3.3.2.1.1 transitions) */
static uint8_t cab_next[256];
static pthread_once_t cab_once = PTHREAD_ONCE_INIT;

static void cab_build(void)
{
	for (int s = 0; s < 128; ++s) {
		const int state = s >> 1, mps = s & 1;
		cab_next[s] = (uint8_t)(((state + (state < 62)) << 1) | mps);
		cab_next[128 | s] = (uint8_t)((h264_trans_idx_lps[state] << 1) | (mps ^ (state == 0)));
	}
}

/* branch-free on the MPS/LPS outcome, which is unpredictable for residual bins; the context state in and out
 * through *st (a run of bins of one context keeps it in a register: no store-to-load forwarding per bin) */
static inline int eng_decide(h264_cabac_eng_t *e, uint32_t *st)
{
	const uint32_t s = *st;
	const uint32_t lps = h264_range_lps[s >> 1][(e->range >> 6) & 3];
	uint32_t range = e->range - lps;
	const uint64_t scaled = (uint64_t)range << e->bits;
	const uint32_t is_lps = e->value >= scaled;
	const uint64_t m = (uint64_t)0 - is_lps;
	e->value -= scaled & m;
	range ^= (range ^ lps) & (uint32_t)m;
	*st = cab_next[(is_lps << 7) | s];
	{
		const int n = __builtin_clz(range) - 23;
		e->range = range << n;
		e->bits -= n;
		eng_refill(e);
	}
	return (int)((s & 1) ^ is_lps);
}

static inline int eng_decision(h264_cabac_eng_t *e, uint8_t *ctx, int ctxidx)
{
	uint32_t st = ctx[ctxidx];
	const int bin = eng_decide(e, &st);
	ctx[ctxidx] = (uint8_t)st;
	return bin;
}

/* branch-free: bypass bins (signs, suffixes) are coin flips to a branch predictor */
static inline int eng_bypass(h264_cabac_eng_t *e)
{
	e->bits -= 1;
	{
		const uint64_t scaled = (uint64_t)e->range << e->bits;
		const uint64_t ge = e->value >= scaled;
		e->value -= scaled & ((uint64_t)0 - ge);
		eng_refill(e); /* keeps the invariant value < range << bits */
		return (int)ge;
	}
}

/* v negated when the next bypass bin (a sign) is 1, without a branch */
static inline int eng_bypass_sign(h264_cabac_eng_t *e, int v)
{
	const int s = eng_bypass(e);
	return (v ^ -s) + s;
}

/* k <= 16 bypass bins at once, MSB first: k steps of the bypass compare-subtract are one long division
 * of value by range << (bits - k) (value < range << bits bounds the quotient by 2^k) */
static inline uint32_t eng_bypass_bits(h264_cabac_eng_t *e, int k)
{
	e->bits -= k;
	{
		const uint64_t scaled = (uint64_t)e->range << e->bits;
		const uint64_t q = e->value / scaled;
		e->value -= q * scaled;
		eng_refill(e);
		return (uint32_t)q;
	}
}

/* a unary run of bypass 1s ended by a 0 (Exp-Golomb prefix), at most 16 bins: the number of 1s, the 0
 * consumed; -1 (nothing consumed) if no 0 within 16 bins */
static inline int eng_bypass_ones(h264_cabac_eng_t *e)
{
	const uint64_t scaled = (uint64_t)e->range << (e->bits - 16);
	const uint32_t q = (uint32_t)(e->value / scaled); /* the next 16 bins, not consumed yet */
	const int ones = __builtin_clz(~(q << 16) | 1u);  /* leading 1s of the 16-bit window */
	if (ones >= 16) return -1;
	{
		/* consume ones + 1 bins: the quotient's top (ones + 1) bits */
		const int n = ones + 1;
		e->bits -= n;
		e->value -= (uint64_t)(q >> (16 - n)) * ((uint64_t)e->range << e->bits);
		eng_refill(e);
	}
	return ones;
}

static inline int cabac_decision(h264_cabac_t *c, int ctxidx)
{
	return eng_decision(&c->e, c->ctx, ctxidx);
}

static inline int cabac_bypass(h264_cabac_t *c)
{
	return eng_bypass(&c->e);
}

static inline int cabac_terminate(h264_cabac_t *c)
{
	h264_cabac_eng_t *e = &c->e;
	uint32_t range = e->range - 2;
	uint64_t scaled = (uint64_t)range << e->bits;
	if (e->value >= scaled) {
		e->range = range;
		return 1;
	}
	if (range < 256) {
		e->range = range << 1;
		e->bits -= 1;
		eng_refill(e);
	} else {
		e->range = range;
	}
	return 0;
}

/* ================================================================== CAVLC VLC tables */
typedef struct {
	uint16_t *lut; /* [1 << bits] = (value << 5) | len, len 0 = invalid */
	int bits;
} vlc_lut_t;

static vlc_lut_t ct_lut[5], tz_lut[16], rb_lut[8];
static pthread_once_t vlc_once = PTHREAD_ONCE_INIT; /* decoder contexts may run on several threads */

static void build_lut(vlc_lut_t *t, const h264_vlc_code_t *codes, int bits)
{
	t->bits = bits;
	t->lut = (uint16_t *)calloc((size_t)1 << bits, sizeof(uint16_t));
	for (; codes->value >= 0; ++codes) {
		int shift = bits - codes->len;
		uint32_t base = codes->code << shift;
		for (uint32_t k = 0; k < (1u << shift); ++k)
			t->lut[base + k] = (uint16_t)((codes->value << 5) | codes->len);
	}
}

static void vlc_build(void)
{
	for (int i = 0; i < 5; ++i) build_lut(&ct_lut[i], h264_coeff_token_tab[i], 16);
	for (int i = 1; i < 16; ++i) build_lut(&tz_lut[i], h264_total_zeros_tab[i], 9);
	for (int i = 1; i < 8; ++i) build_lut(&rb_lut[i], h264_run_before_tab[i], 11);
}

static void vlc_init(void)
{
	pthread_once(&vlc_once, vlc_build);
}

static inline int vlc_read(h264_bits_t *b, const vlc_lut_t *t)
{
	uint32_t e = t->lut[hb_show(b, t->bits)];
	hb_skip(b, e & 31);
	return (int)(e >> 5);
}

/* ================================================================== slice-level state */
typedef struct {
	h264_dec_t *d;
	h264_slice_t *sh;
	const h264_pps_t *pps;
	const h264_sps_t *sps;
	int cabac;
	int slice_type;
	int qp;
	int prev_qp_delta;      /* last decoded mb_qp_delta in the slice (ctxIdxInc of mb_qp_delta) */
	int chroma_qp[2];
	int firstline;          /* reference get_availability counter (h264.cpp:9704) */
	int t8x8_mode;
	int8_t skip_dsf_dummy;
	/* current MB */
	int addr, mbx, mby, avail;
	h264_mbinfo_t *cur, *A, *B, *C, *D;
	m2r_mb_t *rec;
	m2r_deblock_t *dbk;
	int16_t *coef;          /* next free coefficient slot of the picture pool */
	/* spatial direct cache of the current MB */
	int direct_ready;
	int8_t dref[2];
	int16_t dmv[2][2];
} slice_ctx_t;

static int qpc_of(int qpy, int off)
{
	static const int8_t lut[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
	int q = qpy + off;
	if (q <= 0) return 0;
	if (q >= 30) return lut[imin(q, 51) - 30];
	return q;
}

static void set_qp(slice_ctx_t *s, int qp)
{
	if (qp < 0) qp += 52;
	else if (52 <= qp) qp -= 52;
	s->qp = qp;
	s->chroma_qp[0] = qpc_of(qp, s->pps->chroma_qp_index[0]);
	s->chroma_qp[1] = qpc_of(qp, s->pps->chroma_qp_index[1]);
}

/* ================================================================== neighbours */
/* neighbouring 4x4 block of (x, y) in units of 4x4 relative to the current MB (x,y may be -1 / 4) */
static inline const h264_mbinfo_t *nb_mb(const slice_ctx_t *s, int x, int y, int *bx, int *by)
{
	*bx = 0;
	*by = 0;
	if (y < 0) {
		*by = 3;
		if (x < 0) { *bx = 3; return s->D; }
		if (x < 4) { *bx = x; return s->B; }
		*bx = 0;
		return s->C;
	}
	if (x < 0) {
		*bx = 3;
		*by = y;
		return s->A;
	}
	if (x < 4) {
		*bx = x;
		*by = y;
		return s->cur;
	}
	return NULL;
}

/* ================================================================== coefficient pool */
static inline int16_t *coef_alloc(slice_ctx_t *s, int n)
{
	int16_t *p = s->coef;
	memset(p, 0, (size_t)n * sizeof(int16_t));
	s->coef += n;
	return p;
}

/* ================================================================== CABAC residual (9.3.3.1.1.9, 9.3.3.1.3) */
static const int16_t sig_base[5] = {105 + 0, 105 + 15, 105 + 29, 105 + 44, 105 + 47};
static const int16_t last_base[5] = {166 + 0, 166 + 15, 166 + 29, 166 + 44, 166 + 47};
static const int16_t abs_base[5] = {227 + 0, 227 + 10, 227 + 20, 227 + 30, 227 + 39};

/* decode one block; writes levels at raster positions out[scan[i]]; returns number of nonzero */
static int cabac_block(h264_cabac_t *c, int cat, int16_t *out)
{
	h264_cabac_eng_t e = c->e;
	uint8_t *ctx = c->ctx;
	int map[64];
	int n = 0, i, num;
	const uint8_t *scan;
	int first = 0;
	int sbase, lbase, abase;
	int gt1 = 0, eq1 = 0;

	if (cat == 5) {
		num = 64;
		for (i = 0; i < 63; ++i) {
			if (eng_decision(&e, ctx, 402 + h264_sig8x8_frame[i])) {
				map[n++] = i;
				if (eng_decision(&e, ctx, 417 + h264_last8x8[i])) goto done;
			}
		}
		map[n++] = 63;
		goto done;
	}
	num = (cat == 3) ? 4 : ((cat == 1 || cat == 4) ? 15 : 16);
	sbase = sig_base[cat];
	lbase = last_base[cat];
	for (i = 0; i < num - 1; ++i) {
		if (eng_decision(&e, ctx, sbase + i)) {
			map[n++] = i;
			if (eng_decision(&e, ctx, lbase + i)) goto done;
		}
	}
	map[n++] = num - 1;
done:
	if (cat == 5) {
		scan = zz8;
		abase = 426;
	} else if (cat == 3) {
		scan = NULL;
		abase = abs_base[3];
	} else {
		scan = zz4;
		abase = abs_base[cat];
		first = (cat == 1 || cat == 4) ? 1 : 0;
	}
	for (int k = n - 1; k >= 0; --k) {
		int ctxinc = (gt1 != 0) ? 0 : imin(4, 1 + eq1);
		int lvl;
		if (!eng_decision(&e, ctx, abase + ctxinc)) {
			lvl = 1;
			eq1++;
		} else {
			const int ctx2 = abase + 5 + imin(4 - (cat == 3), gt1);
			uint32_t st = ctx[ctx2];
			lvl = 2;
			while (lvl < 15 && eng_decide(&e, &st)) lvl++;
			ctx[ctx2] = (uint8_t)st;
			if (lvl == 15) {
				/* UEG0 suffix (9.3.2.3): unary prefix and k fixed bits in batches */
				int k2 = 0;
				const int ones = eng_bypass_ones(&e);
				if (ones >= 0) {
					lvl += (1 << ones) - 1;
					if (ones) lvl += (int)eng_bypass_bits(&e, ones);
				} else {
					while (eng_bypass(&e)) {
						lvl += 1 << k2;
						k2++;
						if (k2 > 24) break;
					}
					while (k2-- > 0) lvl += eng_bypass(&e) << k2;
				}
			}
			gt1++;
		}
		lvl = eng_bypass_sign(&e, lvl);
		{
			int pos = map[k] + first;
			out[scan ? scan[pos] : pos] = (int16_t)lvl;
		}
	}
	(void)num;
	c->e = e;
	return n;
}

/* coded_block_flag ctxIdxInc from neighbour MBs / current MB (9.3.3.1.1.9) */
static inline int cbf_cond(const slice_ctx_t *s, const h264_mbinfo_t *n, int bit)
{
	if (!n) return s->cur->type < MBT_IPCM ? 1 : 0; /* unavailable: intra -> 1, inter -> 0 */
	if (n->type == MBT_IPCM) return 1;
	return (int)((n->cbf >> bit) & 1);
}

static int cabac_cbf_luma(slice_ctx_t *s, int blk, int cat)
{
	int x = blk_x[blk], y = blk_y[blk], bx, by;
	const h264_mbinfo_t *a = nb_mb(s, x - 1, y, &bx, &by);
	int ia = rast2blk[by * 4 + bx];
	const h264_mbinfo_t *b = nb_mb(s, x, y - 1, &bx, &by);
	int ib = rast2blk[by * 4 + bx];
	int inc = cbf_cond(s, a, ia) + 2 * cbf_cond(s, b, ib);
	return cabac_decision(&s->d->cabac, 85 + cat * 4 + inc);
}

/* ================================================================== CAVLC residual (9.2) */
static int cavlc_nc_luma(const slice_ctx_t *s, int blk)
{
	int x = blk_x[blk], y = blk_y[blk], bx, by;
	int na = -1, nb = -1;
	const h264_mbinfo_t *a = nb_mb(s, x - 1, y, &bx, &by);
	if (a) na = (a->type == MBT_IPCM) ? 16 : a->nnz[rast2blk[by * 4 + bx]];
	const h264_mbinfo_t *b = nb_mb(s, x, y - 1, &bx, &by);
	if (b) nb = (b->type == MBT_IPCM) ? 16 : b->nnz[rast2blk[by * 4 + bx]];
	if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
	if (na >= 0) return na;
	if (nb >= 0) return nb;
	return 0;
}

static int cavlc_nc_chroma(const slice_ctx_t *s, int c, int blk)
{
	int x = blk & 1, y = blk >> 1;
	int na = -1, nb = -1;
	if (x > 0) na = s->cur->nnzc[c * 4 + blk - 1];
	else if (s->A) na = (s->A->type == MBT_IPCM) ? 16 : s->A->nnzc[c * 4 + y * 2 + 1];
	if (y > 0) nb = s->cur->nnzc[c * 4 + blk - 2];
	else if (s->B) nb = (s->B->type == MBT_IPCM) ? 16 : s->B->nnzc[c * 4 + 2 + x];
	if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
	if (na >= 0) return na;
	if (nb >= 0) return nb;
	return 0;
}

/* cat: 0 luma DC, 1 luma AC, 2 luma 4x4, 3 chroma DC, 4 chroma AC ; returns TotalCoeff (-1 error) */
static int cavlc_block(h264_bits_t *b, int cat, int nc, int16_t *out)
{
	int level[16], run[16];
	int max = (cat == 3) ? 4 : ((cat == 1 || cat == 4) ? 15 : 16);
	int tab = (cat == 3) ? 4 : (nc >= 8 ? 3 : (nc >= 4 ? 2 : (nc >= 2 ? 1 : 0)));
	int v = vlc_read(b, &ct_lut[tab]);
	int total = v & 31, t1 = v >> 5;
	int suffix, zeros, i;
	if (total == 0) return 0;
	if (total > max) return -1;
	for (i = 0; i < t1; ++i) level[i] = hb_get1(b) ? -1 : 1;
	suffix = (total > 10 && t1 < 3) ? 1 : 0;
	for (; i < total; ++i) {
		int prefix = 0, code, size;
		while (prefix < 32 && !hb_get1(b)) prefix++;
		code = imin(15, prefix) << suffix;
		if (suffix > 0 || prefix >= 14) {
			size = (prefix == 14 && suffix == 0) ? 4 : (prefix >= 15 ? prefix - 3 : suffix);
			if (size > 0) code += (int)hb_get(b, size);
		}
		if (prefix >= 15 && suffix == 0) code += 15;
		if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
		if (i == t1 && t1 < 3) code += 2;
		level[i] = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
		if (suffix == 0) suffix = 1;
		if (iabs(level[i]) > (3 << (suffix - 1)) && suffix < 6) suffix++;
	}
	if (total < max) {
		if (cat == 3) {
			if (hb_get1(b)) zeros = 0;
			else if (total == 1) zeros = hb_get1(b) ? 1 : 3 - (int)hb_get1(b);
			else if (total == 2) zeros = 2 - (int)hb_get1(b);
			else zeros = 1;
		} else {
			zeros = vlc_read(b, &tz_lut[total]);
		}
	} else {
		zeros = 0;
	}
	for (i = 0; i < total - 1; ++i) {
		int r = 0;
		if (zeros > 0) r = vlc_read(b, &rb_lut[imin(zeros, 7)]);
		if (r > zeros) return -1; /* run_before beyond the zeros left: damaged data */
		run[i] = r;
		zeros -= r;
	}
	run[total - 1] = zeros;
	{
		int pos = -1;
		int first = (cat == 1 || cat == 4) ? 1 : 0;
		for (i = total - 1; i >= 0; --i) {
			int sc;
			pos += run[i] + 1;
			if (pos >= max) return -1;
			sc = pos + first;
			out[(cat == 3) ? sc : zz4[sc]] = (int16_t)level[i];
		}
	}
	return total;
}

/* ================================================================== motion vector prediction (8.4.1.3) */
typedef struct {
	int avail;
	int ref;
	int16_t mv[2];
} nbmv_t;

static inline void nb_motion(const slice_ctx_t *s, int lx, int x, int y, nbmv_t *o)
{
	int bx, by;
	const h264_mbinfo_t *n = nb_mb(s, x, y, &bx, &by);
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
}

/* C neighbour with the in-MB decoding order rule; falls back to D */
static void nb_c(const slice_ctx_t *s, int lx, int x, int y, int w, nbmv_t *o)
{
	int cx = x + w, cy = y - 1;
	int ok;
	if (cy < 0) {
		ok = (cx < 4) ? (s->B != NULL) : (cx == 4 && s->C != NULL);
	} else if (cx >= 4) {
		ok = 0;
	} else {
		ok = rast2blk[cy * 4 + cx] < rast2blk[y * 4 + x];
	}
	if (ok) {
		nb_motion(s, lx, cx, cy, o);
	} else {
		nb_motion(s, lx, x - 1, y - 1, o);
	}
}

/* shape: 0 generic median, 1 16x8 top, 2 16x8 bottom, 3 8x16 left, 4 8x16 right */
static void mvp(const slice_ctx_t *s, int lx, int x, int y, int w, int ref, int shape, int16_t out[2])
{
	nbmv_t a, b, c;
	nb_motion(s, lx, x - 1, y, &a);
	nb_motion(s, lx, x, y - 1, &b);
	nb_c(s, lx, x, y, w, &c);
	if (shape == 1 && b.ref == ref) { out[0] = b.mv[0]; out[1] = b.mv[1]; return; }
	if (shape == 2 && a.ref == ref) { out[0] = a.mv[0]; out[1] = a.mv[1]; return; }
	if (shape == 3 && a.ref == ref) { out[0] = a.mv[0]; out[1] = a.mv[1]; return; }
	if (shape == 4 && c.ref == ref) { out[0] = c.mv[0]; out[1] = c.mv[1]; return; }
	if (!b.avail && !c.avail && a.avail) {
		b = a;
		c = a;
	}
	{
		int m = (a.ref == ref) + (b.ref == ref) * 2 + (c.ref == ref) * 4;
		if (m == 1) { out[0] = a.mv[0]; out[1] = a.mv[1]; }
		else if (m == 2) { out[0] = b.mv[0]; out[1] = b.mv[1]; }
		else if (m == 4) { out[0] = c.mv[0]; out[1] = c.mv[1]; }
		else {
			out[0] = (int16_t)median3(a.mv[0], b.mv[0], c.mv[0]);
			out[1] = (int16_t)median3(a.mv[1], b.mv[1], c.mv[1]);
		}
	}
}

static void fill_mv(h264_mbinfo_t *m, int lx, int x, int y, int w, int h, int mx, int my)
{
	for (int j = y; j < y + h; ++j)
		for (int i = x; i < x + w; ++i) {
			m->mv[lx][j * 4 + i][0] = (int16_t)mx;
			m->mv[lx][j * 4 + i][1] = (int16_t)my;
		}
}

static void fill_mvd(h264_mbinfo_t *m, int lx, int x, int y, int w, int h, int dx, int dy)
{
	uint8_t ax = (uint8_t)imin(iabs(dx), 255), ay = (uint8_t)imin(iabs(dy), 255);
	for (int j = y; j < y + h; ++j)
		for (int i = x; i < x + w; ++i) {
			m->mvd[lx][j * 4 + i][0] = ax;
			m->mvd[lx][j * 4 + i][1] = ay;
		}
}

/* P_Skip (8.4.1.1) */
static void pskip_mv(const slice_ctx_t *s, int16_t out[2])
{
	nbmv_t a, b;
	nb_motion(s, 0, -1, 0, &a);
	nb_motion(s, 0, 0, -1, &b);
	if (!a.avail || !b.avail || (a.ref == 0 && a.mv[0] == 0 && a.mv[1] == 0) || (b.ref == 0 && b.mv[0] == 0 && b.mv[1] == 0)) {
		out[0] = out[1] = 0;
		return;
	}
	mvp(s, 0, 0, 0, 4, 0, 0, out);
}

/* ------------------------------------------------------------------ direct prediction */
/* spatial refs/mv of the whole MB (b_direct_ref_mv_calc + b_skip_ref_mv, h264.cpp:8325-8387) */
static void spatial_ref_mv(slice_ctx_t *s)
{
	if (s->direct_ready) return;
	for (int lx = 0; lx < 2; ++lx) {
		nbmv_t a, b, c;
		unsigned r;
		int ref;
		nb_motion(s, lx, -1, 0, &a);
		nb_motion(s, lx, 0, -1, &b);
		nb_c(s, lx, 0, 0, 4, &c);
		{
			unsigned ua = (unsigned)a.ref, ub = (unsigned)b.ref, uc = (unsigned)c.ref;
			r = ua < ub ? ua : ub;
			r = r < uc ? r : uc;
		}
		ref = (int)r;
		s->dref[lx] = (int8_t)ref;
		if (ref < 0) {
			s->dmv[lx][0] = s->dmv[lx][1] = 0;
		} else if (a.ref == ref && b.ref != ref && c.ref != ref) {
			s->dmv[lx][0] = a.mv[0]; s->dmv[lx][1] = a.mv[1];
		} else if (a.ref != ref && b.ref == ref && c.ref != ref) {
			s->dmv[lx][0] = b.mv[0]; s->dmv[lx][1] = b.mv[1];
		} else if (a.ref != ref && b.ref != ref && c.ref == ref) {
			s->dmv[lx][0] = c.mv[0]; s->dmv[lx][1] = c.mv[1];
		} else {
			s->dmv[lx][0] = (int16_t)median3(a.mv[0], b.mv[0], c.mv[0]);
			s->dmv[lx][1] = (int16_t)median3(a.mv[1], b.mv[1], c.mv[1]);
		}
	}
	s->direct_ready = 1;
}

/* thread time spent waiting in col_wait, process-wide (M2DEC_AMD_ASYNC_STATS) */
static long long g_col_spin_ns;
long long h264_col_spin_ns(void) { return __atomic_load_n(&g_col_spin_ns, __ATOMIC_RELAXED); }

static long long mono_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

/* the co-located MB of the current one is stored: wait for the parse writing it (row pipelining) */
static void col_wait(slice_ctx_t *s)
{
	h264_dec_t *d = s->d;
	long long t0 = 0;
	for (int spins = 0;; ++spins) {
		const int v = __atomic_load_n(d->col_sub, __ATOMIC_ACQUIRE);
		if (v < 0 || v > s->addr) {
			if (spins) __atomic_fetch_add(&g_col_spin_ns, mono_ns() - t0, __ATOMIC_RELAXED);
			if (v < 0) { /* that parse failed: this picture fails too (job_run) */
				d->col_sub_fail = 1;
				d->col_sub_ok = 1 << 30;
			} else {
				d->col_sub_ok = v;
			}
			return;
		}
		if (!spins) t0 = mono_ns();
		if (spins < 64) __builtin_ia32_pause();
		else sched_yield(); /* (the writer may be waiting for a CPU) */
	}
}

/* derive direct motion of 8x8 partition b8 into cur (pred_direct8x8_spatial_dec / temporal_direct_block) */
static void direct_8x8(slice_ctx_t *s, int b8)
{
	h264_dec_t *d = s->d;
	if (d->col_sub && s->addr >= d->col_sub_ok) col_wait(s);
	h264_mbinfo_t *m = s->cur;
	const h264_ref_t *l1 = &d->refs[1][0];
	const h264_colmb_t *col = &d->colpic[l1->col].mb[s->addr];
	int inference = s->sps->direct_8x8_inference_flag;
	int x0 = (b8 & 1) * 2, y0 = (b8 >> 1) * 2;

	if (s->sh->direct_spatial) {
		spatial_ref_mv(s);
		if (s->dref[0] < 0 && s->dref[1] < 0) {
			m->ref[0][b8] = 0;
			m->ref[1][b8] = 0;
			fill_mv(m, 0, x0, y0, 2, 2, 0, 0);
			fill_mv(m, 1, x0, y0, 2, 2, 0, 0);
			return;
		}
		m->ref[0][b8] = s->dref[0];
		m->ref[1][b8] = s->dref[1];
		for (int j = 0; j < 2; ++j) {
			for (int i = 0; i < 2; ++i) {
				int bx = x0 + i, by = y0 + j;
				int cx = inference ? (b8 & 1) * 3 : bx;
				int cy = inference ? (b8 >> 1) * 3 : by;
				const int16_t *mc = col->mv[cy * 4 + cx];
				int colzero = (l1->in_use == REF_SHORT) && (col->ref[b8] == 0) &&
				              (unsigned)(mc[0] + 1) <= 2u && (unsigned)(mc[1] + 1) <= 2u;
				for (int lx = 0; lx < 2; ++lx) {
					int mx = s->dmv[lx][0], my = s->dmv[lx][1];
					if (s->dref[lx] < 0 || (s->dref[lx] == 0 && colzero)) mx = my = 0;
					m->mv[lx][by * 4 + bx][0] = (int16_t)mx;
					m->mv[lx][by * 4 + bx][1] = (int16_t)my;
				}
			}
		}
	} else {
		int map_idx = col->ref[b8];
		int ref = (0 <= map_idx) ? d->map_col_to_list0[map_idx] : 0;
		m->ref[0][b8] = (int8_t)ref;
		m->ref[1][b8] = 0;
		if (0 <= map_idx && ref >= 0 && d->refs[0][ref].in_use == REF_LONG) h264_hit(H264_HIT_TD_LT);
		if (0 <= map_idx && ref >= 0 && d->refs[0][ref].in_use != REF_LONG) {
			int scale = d->dist_scale[ref];
			for (int j = 0; j < 2; ++j) {
				for (int i = 0; i < 2; ++i) {
					int bx = x0 + i, by = y0 + j;
					int cx = inference ? (b8 & 1) * 3 : bx;
					int cy = inference ? (b8 >> 1) * 3 : by;
					const int16_t *mc = col->mv[cy * 4 + cx];
					for (int c = 0; c < 2; ++c) {
						int t = (mc[c] * scale + 128) >> 8;
						m->mv[0][by * 4 + bx][c] = (int16_t)t;
						m->mv[1][by * 4 + bx][c] = (int16_t)(t - mc[c]);
					}
				}
			}
		} else {
			fill_mv(m, 0, x0, y0, 2, 2, 0, 0);
			fill_mv(m, 1, x0, y0, 2, 2, 0, 0);
		}
	}
}

/* ================================================================== syntax elements */
static int read_mb_skip(slice_ctx_t *s)
{
	int inc = (s->A && !s->A->skip) + (s->B && !s->B->skip);
	return cabac_decision(&s->d->cabac, (s->slice_type == 0 ? 11 : 24) + inc);
}

static int cabac_mb_type_i(slice_ctx_t *s, int ctx, int is_i)
{
	h264_cabac_t *c = &s->d->cabac;
	int t;
	if (is_i) {
		int inc = (s->B && s->B->type != MBT_INxN) + (s->A && s->A->type != MBT_INxN);
		if (!cabac_decision(c, ctx + inc)) return 0;
		ctx = 5;
	} else if (!cabac_decision(c, ctx)) {
		return 0;
	}
	if (cabac_terminate(c)) return 25;
	t = cabac_decision(c, ctx + 1) * 12 + 1;
	if (cabac_decision(c, ctx + 2)) t += cabac_decision(c, ctx + 2 + is_i) * 4 + 4;
	t += cabac_decision(c, ctx + 3 + is_i) * 2;
	t += cabac_decision(c, ctx + 3 + is_i * 2);
	return t;
}

/* returns the unified mb type (adjust_mb_type, h264.cpp:9689-9703) */
static int read_mb_type(slice_ctx_t *s)
{
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		if (s->slice_type == 2) return cabac_mb_type_i(s, 3, 1);
		if (s->slice_type == 0) {
			if (cabac_decision(c, 14)) return cabac_mb_type_i(s, 17, 0);
			if (cabac_decision(c, 15)) return 26 + (cabac_decision(c, 17) ? 1 : 2);
			return 26 + (cabac_decision(c, 16) ? 3 : 0);
		} else {
			int inc = (s->A && s->A->type != MBT_SKIP) + (s->B && s->B->type != MBT_SKIP);
			int mode;
			if (!cabac_decision(c, 27 + inc)) return 31;
			if (!cabac_decision(c, 27 + 3)) return 31 + 1 + cabac_decision(c, 27 + 5);
			mode = cabac_decision(c, 27 + 4) * 8;
			mode += cabac_decision(c, 27 + 5) * 4;
			mode += cabac_decision(c, 27 + 5) * 2;
			mode += cabac_decision(c, 27 + 5);
			if (mode < 8) return 31 + mode + 3;
			if (mode < 13) return 31 + mode * 2 + cabac_decision(c, 27 + 5) - 4;
			if (mode == 13) return cabac_mb_type_i(s, 32, 0);
			if (mode == 14) return 31 + 11;
			return 31 + 22;
		}
	} else {
		uint32_t t = hb_ue(&s->d->bs);
		if (s->slice_type == 2) return (t <= 25) ? (int)t : -1;
		if (s->slice_type == 0) {
			if (t > 30) return -1;
			return (t < 5) ? (int)t + 26 : (int)t - 5;
		}
		if (t > 48) return -1;
		return (t < 23) ? (int)t + 31 : (int)t - 23;
	}
}

static int read_ipred(slice_ctx_t *s, int pred)
{
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		if (!cabac_decision(c, 68)) {
			int rem = cabac_decision(c, 69);
			rem += cabac_decision(c, 69) * 2;
			rem += cabac_decision(c, 69) * 4;
			return (rem < pred) ? rem : rem + 1;
		}
		return pred;
	} else {
		h264_bits_t *b = &s->d->bs;
		if (!hb_get1(b)) {
			int rem = (int)hb_get(b, 3);
			return (rem < pred) ? rem : rem + 1;
		}
		return pred;
	}
}

static int read_chroma_mode(slice_ctx_t *s)
{
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		int inc = (s->A && s->A->type < MBT_IPCM && s->A->cpm) + (s->B && s->B->type < MBT_IPCM && s->B->cpm);
		int m = cabac_decision(c, 64 + inc);
		if (m) {
			while (m < 3 && cabac_decision(c, 67)) m++;
		}
		return m;
	} else {
		uint32_t m = hb_ue(&s->d->bs);
		return m <= 3 ? (int)m : 0;
	}
}

static int read_cbp(slice_ctx_t *s, int intra)
{
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		int ca = s->A ? s->A->cbp : 0x0f;
		int cb = s->B ? s->B->cbp : 0x0f;
		int cbp, inc;
		if (s->A && s->A->type == MBT_IPCM) ca = 0x2f;
		if (s->B && s->B->type == MBT_IPCM) cb = 0x2f;
		inc = (!(ca & 2)) + (!(cb & 4)) * 2;
		cbp = cabac_decision(c, 73 + inc);
		inc = !(cbp & 1) + (!(cb & 8)) * 2;
		cbp += cabac_decision(c, 73 + inc) * 2;
		inc = (!(ca & 8)) + !(cbp & 1) * 2;
		cbp += cabac_decision(c, 73 + inc) * 4;
		inc = !(cbp & 4) + !(cbp & 2) * 2;
		cbp += cabac_decision(c, 73 + inc) * 8;
		ca >>= 4;
		cb >>= 4;
		inc = (ca != 0) + (cb != 0) * 2;
		if (cabac_decision(c, 77 + inc)) {
			inc = (ca >> 1) + (cb & 2);
			cbp += cabac_decision(c, 77 + 4 + inc) * 16 + 16;
		}
		return cbp;
	} else {
		uint32_t v = hb_ue(&s->d->bs);
		if (v > 47) return -1;
		return h264_me_cbp[intra ? 0 : 1][v];
	}
}

static int read_qp_delta(slice_ctx_t *s)
{
	int dq;
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		dq = cabac_decision(c, 60 + (s->prev_qp_delta != 0));
		if (dq) {
			int k = 1, ctx = 62;
			while (k < 53 && cabac_decision(c, ctx)) {
				k++;
				ctx = 63;
			}
			dq = ((k & 1) ? (k + 1) : -k) >> 1;
		}
	} else {
		dq = hb_se(&s->d->bs);
		dq = imax(-26, imin(25, dq));
	}
	s->prev_qp_delta = dq;
	return dq;
}

static int read_t8x8_flag(slice_ctx_t *s)
{
	if (s->cabac) {
		int inc = (s->B && s->B->t8x8) + (s->A && s->A->t8x8);
		return cabac_decision(&s->d->cabac, 399 + inc);
	}
	return (int)hb_get1(&s->d->bs);
}

static int read_ref_idx(slice_ctx_t *s, int lx, int b8, int num_active)
{
	if (num_active <= 1) return 0;
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		int x = (b8 & 1) * 2, y = (b8 >> 1) * 2, bx, by, inc = 0, k = 0;
		const h264_mbinfo_t *n = nb_mb(s, x - 1, y, &bx, &by);
		int nb8;
		if (n) {
			nb8 = (by >> 1) * 2 + (bx >> 1);
			if (!((n->direct >> nb8) & 1) && n->ref[lx][nb8] > 0 && !(n->type == MBT_SKIP && n->skip)) inc += 1;
		}
		n = nb_mb(s, x, y - 1, &bx, &by);
		if (n) {
			nb8 = (by >> 1) * 2 + (bx >> 1);
			if (!((n->direct >> nb8) & 1) && n->ref[lx][nb8] > 0 && !(n->type == MBT_SKIP && n->skip)) inc += 2;
		}
		while (cabac_decision(c, 54 + inc)) {
			inc = (inc >> 2) + 4;
			k++;
			if (k > 32) break;
		}
		return k;
	} else {
		h264_bits_t *b = &s->d->bs;
		if (num_active == 2) return hb_get1(b) ^ 1;
		{
			uint32_t v = hb_ue(b);
			return (v <= (uint32_t)(num_active - 1)) ? (int)v : num_active - 1;
		}
	}
}

static int cabac_mvd(h264_cabac_t *c, int base, int sum)
{
	h264_cabac_eng_t e;
	uint8_t *ctx = c->ctx;
	const int inc = (sum < 3) ? 0 : (sum <= 32 ? 1 : 2);
	int mvd, ci;
	if (!cabac_decision(c, base + inc)) return 0;
	e = c->e;
	mvd = 1;
	/* prefix bins 2..4 on contexts base + 3..5, bins 5..9 all on base + 6 (its state kept in a register) */
	for (ci = base + 3; ci < base + 6; ++ci) {
		if (!eng_decision(&e, ctx, ci)) goto sign;
		mvd++;
	}
	{
		uint32_t st = ctx[base + 6];
		int more;
		while ((more = eng_decide(&e, &st)) && ++mvd < 9)
			;
		ctx[base + 6] = (uint8_t)st;
		if (more) {
			/* mvd 9: UEG3 suffix, a unary prefix of bypass 1s, then k fixed bits, in batches (9.3.2.3) */
			int k = 3;
			const int ones = eng_bypass_ones(&e);
			if (ones >= 0 && ones <= 13) {
				mvd += ((1 << ones) - 1) << 3; /* sum of 1 << (3 + i), i < ones */
				k = 3 + ones;
				mvd += (int)eng_bypass_bits(&e, k);
			} else {
				while (eng_bypass(&e)) {
					mvd += 1 << k;
					k++;
					if (k > 24) break;
				}
				while (k-- > 0) mvd += eng_bypass(&e) << k;
			}
		}
	}
sign:
	mvd = eng_bypass_sign(&e, mvd);
	c->e = e;
	return mvd;
}

static void read_mvd(slice_ctx_t *s, int lx, int x, int y, int out[2])
{
	if (s->cabac) {
		int bx, by, sx = 0, sy = 0;
		const h264_mbinfo_t *n = nb_mb(s, x - 1, y, &bx, &by);
		if (n) { sx += n->mvd[lx][by * 4 + bx][0]; sy += n->mvd[lx][by * 4 + bx][1]; }
		n = nb_mb(s, x, y - 1, &bx, &by);
		if (n) { sx += n->mvd[lx][by * 4 + bx][0]; sy += n->mvd[lx][by * 4 + bx][1]; }
		out[0] = cabac_mvd(&s->d->cabac, 40, sx);
		out[1] = cabac_mvd(&s->d->cabac, 47, sy);
	} else {
		out[0] = hb_se(&s->d->bs);
		out[1] = hb_se(&s->d->bs);
	}
}

static int read_sub_mb_type(slice_ctx_t *s)
{
	if (s->cabac) {
		h264_cabac_t *c = &s->d->cabac;
		if (s->slice_type == 0) {
			if (cabac_decision(c, 21)) return 0;
			if (!cabac_decision(c, 22)) return 1;
			return cabac_decision(c, 23) ? 2 : 3;
		} else {
			int t;
			if (!cabac_decision(c, 36)) return 0;
			if (!cabac_decision(c, 37)) return 1 + cabac_decision(c, 39);
			if (cabac_decision(c, 38)) {
				if (cabac_decision(c, 39)) return 11 + cabac_decision(c, 39);
				t = 7;
			} else {
				t = 3;
			}
			t += cabac_decision(c, 39) * 2;
			return t + cabac_decision(c, 39);
		}
	} else {
		uint32_t v = hb_ue(&s->d->bs);
		if (s->slice_type == 0) return v <= 3 ? (int)v : -1;
		return v <= 12 ? (int)v : -1;
	}
}

/* ================================================================== residual (7.3.5.3) */
static void record_nnz_luma(h264_mbinfo_t *m, int blk, int n)
{
	m->nnz[blk] = (uint8_t)imin(n, 15);
}

/* luma residual of a non-I16 MB: 4x4 or 8x8 blocks */
static int residual_luma(slice_ctx_t *s, int cbp, int t8x8, uint32_t *nz)
{
	h264_mbinfo_t *m = s->cur;
	for (int b8 = 0; b8 < 4; ++b8) {
		if (!((cbp >> b8) & 1)) continue;
		if (t8x8) {
			int16_t *blk;
			int n;
			if (!s->cabac) return -1; /* CAVLC 8x8 is not supported (the reference mis-parses it) */
			blk = coef_alloc(s, 64);
			n = cabac_block(&s->d->cabac, 5, blk);
			m->cbf |= 0xfu << (b8 * 4);
			for (int k = 0; k < 4; ++k) record_nnz_luma(m, b8 * 4 + k, n);
			*nz |= M2R_NZ_LUMA(b8 * 4);
		} else {
			for (int k = 0; k < 4; ++k) {
				int blk = b8 * 4 + k;
				int16_t *out = s->coef;
				int n;
				memset(out, 0, 16 * sizeof(int16_t));
				if (s->cabac) {
					if (!cabac_cbf_luma(s, blk, 2)) { record_nnz_luma(m, blk, 0); continue; }
					m->cbf |= 1u << blk;
					n = cabac_block(&s->d->cabac, 2, out);
				} else {
					n = cavlc_block(&s->d->bs, 2, cavlc_nc_luma(s, blk), out);
					if (n < 0) return -1;
				}
				record_nnz_luma(m, blk, n);
				if (n) {
					s->coef += 16;
					*nz |= M2R_NZ_LUMA(blk);
				}
			}
		}
	}
	return 0;
}

static int residual_luma16(slice_ctx_t *s, int cbp, uint32_t *nz)
{
	h264_mbinfo_t *m = s->cur;
	int16_t *dc = s->coef;
	int n;
	memset(dc, 0, 16 * sizeof(int16_t));
	if (s->cabac) {
		int a = s->A ? (s->A->type == MBT_IPCM ? 1 : (int)((s->A->cbf >> 16) & 1)) : 1;
		int b = s->B ? (s->B->type == MBT_IPCM ? 1 : (int)((s->B->cbf >> 16) & 1)) : 1;
		n = 0;
		if (cabac_decision(&s->d->cabac, 85 + 0 + a + 2 * b)) {
			m->cbf |= 1u << 16;
			n = cabac_block(&s->d->cabac, 0, dc);
		}
	} else {
		n = cavlc_block(&s->d->bs, 0, cavlc_nc_luma(s, 0), dc);
		if (n < 0) return -1;
	}
	if (n) {
		s->coef += 16;
		*nz |= M2R_NZ_LUMA_DC;
	}
	if (cbp & 15) {
		for (int blk = 0; blk < 16; ++blk) {
			int16_t *out = s->coef;
			memset(out, 0, 16 * sizeof(int16_t));
			if (s->cabac) {
				if (!cabac_cbf_luma(s, blk, 1)) { record_nnz_luma(m, blk, 0); continue; }
				m->cbf |= 1u << blk;
				n = cabac_block(&s->d->cabac, 1, out);
			} else {
				n = cavlc_block(&s->d->bs, 1, cavlc_nc_luma(s, blk), out);
				if (n < 0) return -1;
			}
			record_nnz_luma(m, blk, n);
			if (n) {
				s->coef += 16;
				*nz |= M2R_NZ_LUMA(blk);
			}
		}
	}
	return 0;
}

static int residual_chroma(slice_ctx_t *s, int cbp, uint32_t *nz)
{
	h264_mbinfo_t *m = s->cur;
	int ccbp = cbp >> 4;
	if (!ccbp) return 0;
	for (int c = 0; c < 2; ++c) {
		int16_t *dc = s->coef;
		int n;
		memset(dc, 0, 4 * sizeof(int16_t));
		if (s->cabac) {
			int a = s->A ? (s->A->type == MBT_IPCM ? 1 : (int)((s->A->cbf >> (17 + c)) & 1)) : (m->type < MBT_IPCM);
			int b = s->B ? (s->B->type == MBT_IPCM ? 1 : (int)((s->B->cbf >> (17 + c)) & 1)) : (m->type < MBT_IPCM);
			n = 0;
			if (cabac_decision(&s->d->cabac, 85 + 12 + a + 2 * b)) {
				m->cbf |= 1u << (17 + c);
				n = cabac_block(&s->d->cabac, 3, dc);
			}
		} else {
			n = cavlc_block(&s->d->bs, 3, -1, dc);
			if (n < 0) return -1;
		}
		if (n) {
			s->coef += 4;
			*nz |= M2R_NZ_CDC(c);
		}
	}
	if (ccbp & 2) {
		for (int c = 0; c < 2; ++c) {
			for (int blk = 0; blk < 4; ++blk) {
				int16_t *out = s->coef;
				int n;
				memset(out, 0, 16 * sizeof(int16_t));
				if (s->cabac) {
					int x = blk & 1, y = blk >> 1;
					int bit = 19 + c * 4 + blk;
					int a, b;
					if (x) a = (int)((m->cbf >> (bit - 1)) & 1);
					else a = s->A ? (s->A->type == MBT_IPCM ? 1 : (int)((s->A->cbf >> (19 + c * 4 + y * 2 + 1)) & 1)) : (m->type < MBT_IPCM);
					if (y) b = (int)((m->cbf >> (bit - 2)) & 1);
					else b = s->B ? (s->B->type == MBT_IPCM ? 1 : (int)((s->B->cbf >> (19 + c * 4 + 2 + x)) & 1)) : (m->type < MBT_IPCM);
					if (!cabac_decision(&s->d->cabac, 85 + 16 + a + 2 * b)) { m->nnzc[c * 4 + blk] = 0; continue; }
					m->cbf |= 1u << bit;
					n = cabac_block(&s->d->cabac, 4, out);
				} else {
					n = cavlc_block(&s->d->bs, 4, cavlc_nc_chroma(s, c, blk), out);
					if (n < 0) return -1;
				}
				m->nnzc[c * 4 + blk] = (uint8_t)imin(n, 15);
				if (n) {
					s->coef += 16;
					*nz |= M2R_NZ_CAC(c, blk);
				}
			}
		}
	}
	return 0;
}

/* ================================================================== deblocking strengths */
static inline int is_intra_type(int t) { return t >= 0 && t <= MBT_IPCM; }

/* the BS4 flags of the current MB's deblock record: bS 4 on an MB edge with an intra MB on either side
 * (store_strength_intra*, h264.cpp:3086-3106, 4749-4755).  The strengths themselves (bs_v / bs_h) are
 * derived by the back end from the MB and motion records (recon_hip.hip bs_of, the oracle's orc_bs):
 * the parser leaves them 0. */
static void bs_strength(slice_ctx_t *s)
{
	h264_mbinfo_t *q = s->cur;
	m2r_deblock_t *db = s->dbk;
	uint8_t flags = 0;
	if (is_intra_type(q->type)) {
		flags = M2R_DBK_LEFT_BS4 | M2R_DBK_TOP_BS4;
	} else {
		for (int dir = 0; dir < 2; ++dir) {
			const h264_mbinfo_t *p = NULL;
			if (dir == 0 && s->mbx != 0) p = &s->d->mbi[s->addr - 1];
			if (dir == 1 && s->mby != 0) p = &s->d->mbi[s->addr - s->d->mb_w];
			if (p && (int)(p - s->d->mbi) < s->d->par_first_mb) p = NULL; /* h264_fix_bs, once that slice is parsed */
			if (p && is_intra_type(p->type)) flags |= dir ? M2R_DBK_TOP_BS4 : M2R_DBK_LEFT_BS4;
		}
	}
	db->bs_v = 0;
	db->bs_h = 0;
	db->flags = flags;
}

/* slice-parallel parse: an MB whose left or top neighbour lies in an earlier slice gets its bS again
 * once every slice of the picture is parsed */
void h264_fix_bs(h264_dec_t *d, int addr)
{
	slice_ctx_t s;
	memset(&s, 0, sizeof(s));
	s.d = d;
	s.addr = addr;
	s.mbx = addr % d->mb_w;
	s.mby = addr / d->mb_w;
	s.cur = &d->mbi[addr];
	s.dbk = &d->pic->dbk[addr];
	bs_strength(&s);
}

static void compute_bs(slice_ctx_t *s)
{
	const h264_mbinfo_t *q = s->cur;
	m2r_deblock_t *db = s->dbk;
	bs_strength(s);
	if (q->type == MBT_IPCM) {
		/* I_PCM deblock qp quirk (h264.cpp:4749-4751, Appendix A #5) */
		db->qpy = 0;
		db->qpc[0] = (int8_t)(s->chroma_qp[0] - s->qp);
		db->qpc[1] = (int8_t)(s->chroma_qp[1] - s->qp);
	} else {
		db->qpy = (int8_t)s->qp;
		db->qpc[0] = (int8_t)s->chroma_qp[0];
		db->qpc[1] = (int8_t)s->chroma_qp[1];
	}
}

/* ================================================================== co-located store */
static void store_col(slice_ctx_t *s)
{
	h264_colmb_t *col = &s->d->colpic[s->d->curr_col].mb[s->addr];
	const h264_mbinfo_t *m = s->cur;
	for (int b8 = 0; b8 < 4; ++b8) {
		int lx = (m->ref[0][b8] >= 0) ? 0 : 1;
		int x0 = (b8 & 1) * 2, y0 = (b8 >> 1) * 2;
		col->ref[b8] = m->ref[lx][b8];
		for (int j = 0; j < 2; ++j)
			for (int i = 0; i < 2; ++i) {
				int r = (y0 + j) * 4 + x0 + i;
				col->mv[r][0] = m->mv[lx][r][0];
				col->mv[r][1] = m->mv[lx][r][1];
			}
	}
	/* (single-slice pictures store in raster order: MBs [0, addr] are stored) */
	if (s->d->col_pub) {
		__atomic_store_n(s->d->col_pub, s->addr + 1, __ATOMIC_RELEASE);
		if (s->d->col_pub_delay_us && s->mbx == s->d->mb_w - 1) usleep((useconds_t)s->d->col_pub_delay_us);
	}
}

/* ================================================================== record emission */
static void emit_inter(slice_ctx_t *s)
{
	m2r_picture_t *pic = s->d->pic;
	m2r_inter_t *it = &pic->inter[pic->n_inter];
	const h264_mbinfo_t *m = s->cur;
	s->rec->inter = (uint32_t)pic->n_inter;
	pic->n_inter++;
	memcpy(it->mv, m->mv, sizeof(it->mv));
	for (int lx = 0; lx < 2; ++lx)
		for (int b8 = 0; b8 < 4; ++b8) {
			it->slot[lx][b8] = (int8_t)m->fidx[lx][b8];
			it->refidx[lx][b8] = m->ref[lx][b8];
		}
}

static void finish_mb_common(slice_ctx_t *s)
{
	h264_mbinfo_t *m = s->cur;
	/* frame identities of the references (bS, records) */
	for (int lx = 0; lx < 2; ++lx)
		for (int b8 = 0; b8 < 4; ++b8) {
			int r = m->ref[lx][b8];
			m->fidx[lx][b8] = (int16_t)((r >= 0) ? s->d->refs[lx][r].frame_idx : -1);
		}
	compute_bs(s);
	store_col(s);
	s->rec->qpy = (int8_t)s->qp;
	s->rec->qpc[0] = (int8_t)s->chroma_qp[0];
	s->rec->qpc[1] = (int8_t)s->chroma_qp[1];
	s->rec->slice = (uint16_t)s->d->slice_rec;
	if (s->rec->kind == M2R_MB_INTER) emit_inter(s);
	else s->d->pic->n_intra++;
}

static void init_mb(slice_ctx_t *s)
{
	h264_dec_t *d = s->d;
	int w = d->mb_w;
	h264_mbinfo_t *m = &d->mbi[s->addr];
	int fl = s->firstline;
	s->mbx = s->addr % w;
	s->mby = s->addr / w;
	/* get_availability, h264.cpp:9704-9715 */
	s->avail = ((s->mbx != 0 && fl < 0) * 8) | ((s->mbx != w - 1 && fl <= 1) * 4) | ((fl <= 0) * 2) | (s->mbx != 0 && fl != w);
	s->cur = m;
	s->A = (s->avail & 1) ? m - 1 : NULL;
	s->B = (s->avail & 2) ? m - w : NULL;
	s->C = (s->avail & 4) ? m - w + 1 : NULL;
	s->D = (s->avail & 8) ? m - w - 1 : NULL;
	s->rec = &d->pic->mb[s->addr];
	s->dbk = &d->pic->dbk[s->addr];
	memset(s->rec, 0, sizeof(*s->rec));
	s->rec->coef = (uint32_t)(s->coef - d->pic->coef);
	s->direct_ready = 0;
	d->mbs_coded += m->slice < 0;
	m->slice = (int16_t)d->slice_num;
	m->skip = 0;
	m->t8x8 = 0;
	m->cbp = 0;
	m->cpm = 0;
	m->direct = 0;
	m->cbf = 0;
	memset(m->nnz, 0, sizeof(m->nnz));
	memset(m->nnzc, 0, sizeof(m->nnzc));
	memset(m->ipred, 2, sizeof(m->ipred));
	memset(m->ref, -1, sizeof(m->ref));
	memset(m->mv, 0, sizeof(m->mv));
	memset(m->mvd, 0, sizeof(m->mvd));
}

/* ================================================================== macroblock types */
static int decode_skip(slice_ctx_t *s)
{
	h264_mbinfo_t *m = s->cur;
	m->type = MBT_SKIP;
	m->skip = 1;
	s->rec->kind = M2R_MB_INTER;
	s->prev_qp_delta = 0;
	if (s->slice_type == 0) {
		int16_t mv[2];
		pskip_mv(s, mv);
		for (int b8 = 0; b8 < 4; ++b8) m->ref[0][b8] = 0;
		fill_mv(m, 0, 0, 0, 4, 4, mv[0], mv[1]);
	} else {
		m->direct = 0xf;
		for (int b8 = 0; b8 < 4; ++b8) direct_8x8(s, b8);
	}
	finish_mb_common(s);
	return 0;
}

static int decode_pcm(slice_ctx_t *s)
{
	h264_dec_t *d = s->d;
	h264_mbinfo_t *m = s->cur;
	uint8_t *dst;
	const uint8_t *src;
	m->type = MBT_IPCM;
	m->cbp = 0x2f;
	m->cbf = 0x7ffffff;
	memset(m->nnz, 16, sizeof(m->nnz));
	memset(m->nnzc, 16, sizeof(m->nnzc));
	s->rec->kind = M2R_MB_PCM;
	s->prev_qp_delta = 0;
	dst = (uint8_t *)coef_alloc(s, 192);
	if (s->cabac) {
		/* 9.3.1.2: samples start at the byte boundary after the bits the engine consumed */
		size_t pos = (cabac_bitpos(&d->cabac, d->cabac_start) + 7) >> 3;
		src = d->cabac_start + pos;
		if (src + 384 > d->cabac.e.end) return -1;
		memcpy(dst, src, 384);
		cabac_start(&d->cabac, src + 384, d->cabac.e.end);
	} else {
		h264_bits_t *b = &d->bs;
		int mis = b->bits & 7;
		hb_skip(b, mis);
		for (int i = 0; i < 384; ++i) dst[i] = (uint8_t)hb_get(b, 8);
	}
	finish_mb_common(s);
	return 0;
}

static int decode_intra(slice_ctx_t *s, int type)
{
	h264_dec_t *d = s->d;
	h264_mbinfo_t *m = s->cur;
	m2r_mb_t *r = s->rec;
	int avail_intra = s->avail;
	int cbp, cm;
	uint32_t nz = 0;
	m->type = (int8_t)type;
	if (s->pps->constrained_intra_pred_flag) {
		/* h264.cpp:3271-3273: mask inter neighbours */
		const h264_mbinfo_t *w = d->mbi + s->addr;
		int mw = d->mb_w;
		int mask = 0;
		if ((s->avail & 4) && w[-mw + 1].type > MBT_IPCM) mask |= 4;
		if ((s->avail & 2) && w[-mw].type > MBT_IPCM) mask |= 2;
		if ((s->avail & 1) && w[-1].type > MBT_IPCM) mask |= 1;
		avail_intra &= ~mask;
	}
	if (type == MBT_INxN) {
		int t8 = s->t8x8_mode ? read_t8x8_flag(s) : 0;
		uint32_t ip[2] = {0, 0};
		m->t8x8 = (uint8_t)t8;
		/* predicted modes (8.3.1.1 / 8.3.2.1); DC (2) when a neighbour is unavailable */
		for (int blk = 0; blk < 16; blk += t8 ? 4 : 1) {
			int x = blk_x[blk], y = blk_y[blk], bx, by, ma, mb, pred, mode;
			const h264_mbinfo_t *a = nb_mb(s, x - 1, y, &bx, &by);
			int ia = rast2blk[by * 4 + bx];
			const h264_mbinfo_t *b = nb_mb(s, x, y - 1, &bx, &by);
			int ib = rast2blk[by * 4 + bx];
			int a_ok = (a == m) || (a && (avail_intra & 1));
			int b_ok = (b == m) || (b && (avail_intra & 2));
			if (!a_ok || !b_ok) {
				pred = 2;
			} else {
				if (t8 && a != m && a->type == MBT_INxN && !a->t8x8) ia = (ia & ~3) | 1;
				if (t8 && b != m && b->type == MBT_INxN && !b->t8x8) ib = (ib & ~3) | 2;
				ma = (a->type == MBT_INxN) ? a->ipred[ia] : 2;
				mb = (b->type == MBT_INxN) ? b->ipred[ib] : 2;
				pred = imin(ma, mb);
			}
			mode = read_ipred(s, pred);
			if (t8) {
				for (int k = 0; k < 4; ++k) m->ipred[blk + k] = (int8_t)mode;
				ip[0] |= (uint32_t)mode << (4 * (blk >> 2));
			} else {
				m->ipred[blk] = (int8_t)mode;
				ip[blk >> 3] |= (uint32_t)mode << (4 * (blk & 7));
			}
		}
		r->ipred[0] = ip[0];
		r->ipred[1] = ip[1];
		cm = read_chroma_mode(s);
		cbp = read_cbp(s, 1);
		if (cbp < 0) return -1;
		if (cbp) {
			int dq = read_qp_delta(s);
			if (dq) set_qp(s, s->qp + dq);
		} else {
			s->prev_qp_delta = 0;
		}
		m->cbp = (uint8_t)cbp;
		if (residual_luma(s, cbp, t8, &nz) < 0) return -1;
		r->kind = t8 ? M2R_MB_I8x8 : M2R_MB_I4x4;
		r->flags = t8 ? M2R_FLAG_T8x8 : 0;
		/* luma_intra4x4_pred gets the unmasked avail (h264.cpp:3290-3292, Appendix A #8) */
		r->avail_luma = (uint8_t)((!t8 && !(cbp & 15)) ? s->avail : avail_intra);
	} else {
		int it = type - 1;
		r->pred_mode = (uint8_t)(it & 3);
		cbp = ((it >> 2) % 3) << 4;
		if (it >= 12) cbp |= 15;
		cm = read_chroma_mode(s);
		{
			int dq = read_qp_delta(s);
			if (dq) set_qp(s, s->qp + dq);
		}
		m->cbp = (uint8_t)cbp;
		if (residual_luma16(s, cbp, &nz) < 0) return -1;
		r->kind = M2R_MB_I16x16;
		r->avail_luma = (uint8_t)avail_intra;
	}
	m->cpm = (uint8_t)cm;
	r->chroma_mode = (uint8_t)cm;
	r->avail_chroma = (uint8_t)avail_intra;
	r->cbp = (uint8_t)cbp;
	if (residual_chroma(s, cbp, &nz) < 0) return -1;
	r->nz = nz;
	finish_mb_common(s);
	return 0;
}

/* partition prediction flags of B 16x16/16x8/8x16 types (reference mb_decode[].cbp, h264.cpp:9589-9680) */
static const uint8_t b_predmap[22] = {
	1, 2, 3, 0x3, 0x3, 0xc, 0xc, 0x9, 0x9, 0x6, 0x6, 0xb, 0xb, 0xe, 0xe, 0x7, 0x7, 0xd, 0xd, 0xf, 0xf, 0};
/* sub_mb_ref_map_b: pred flags of B sub types (h264vld.h:476) */
static const int8_t b_sub_pred[13] = {-1, 1, 2, 3, 1, 1, 2, 2, 3, 3, 1, 2, 3};
static const int8_t b_sub_shape[13] = {0, 0, 0, 0, 1, 2, 1, 2, 1, 2, 3, 3, 3};

static int decode_residual_inter(slice_ctx_t *s, int allow_t8)
{
	h264_mbinfo_t *m = s->cur;
	m2r_mb_t *r = s->rec;
	uint32_t nz = 0;
	int cbp = read_cbp(s, 0);
	int t8 = 0;
	if (cbp < 0) return -1;
	m->cbp = (uint8_t)cbp;
	if (cbp) {
		int dq;
		if (allow_t8 && s->t8x8_mode && (cbp & 15) && s->cabac) t8 = read_t8x8_flag(s);
		m->t8x8 = (uint8_t)t8;
		dq = read_qp_delta(s);
		if (dq) set_qp(s, s->qp + dq);
		if (residual_luma(s, cbp, t8, &nz) < 0) return -1;
		if (residual_chroma(s, cbp, &nz) < 0) return -1;
	} else {
		s->prev_qp_delta = 0;
	}
	r->kind = M2R_MB_INTER;
	r->cbp = (uint8_t)cbp;
	r->flags = t8 ? M2R_FLAG_T8x8 : 0;
	r->nz = nz;
	return 0;
}

static int decode_inter(slice_ctx_t *s, int type)
{
	h264_mbinfo_t *m = s->cur;
	h264_slice_t *sh = s->sh;
	int nact[2] = {sh->num_ref_idx_active[0], sh->num_ref_idx_active[1]};
	m->type = (int8_t)type;
	if (type == MBT_SKIP) {
		/* B_Direct_16x16 */
		m->direct = 0xf;
		for (int b8 = 0; b8 < 4; ++b8) direct_8x8(s, b8);
		if (decode_residual_inter(s, 1) < 0) return -1;
	} else if (type == MBT_P8x8 || type == MBT_P8x8REF0 || type == MBT_B8x8) {
		int sub[4];
		int is_b = (type == MBT_B8x8);
		int allow_t8;
		for (int i = 0; i < 4; ++i) {
			sub[i] = read_sub_mb_type(s);
			if (sub[i] < 0) return -1;
		}
		if (is_b) {
			for (int i = 0; i < 4; ++i)
				if (sub[i] == 0) {
					m->direct |= (uint8_t)(1 << i);
					direct_8x8(s, i);
				}
		}
		for (int lx = 0; lx < 2; ++lx) {
			for (int i = 0; i < 4; ++i) {
				int pf = is_b ? b_sub_pred[sub[i]] : 1;
				if (pf < 0 || !((pf >> lx) & 1)) continue;
				m->ref[lx][i] = (int8_t)((type == MBT_P8x8REF0) ? 0 : read_ref_idx(s, lx, i, nact[lx]));
			}
		}
		for (int lx = 0; lx < 2; ++lx) {
			for (int i = 0; i < 4; ++i) {
				int pf = is_b ? b_sub_pred[sub[i]] : 1;
				int shape = is_b ? b_sub_shape[sub[i]] : sub[i];
				int x0 = (i & 1) * 2, y0 = (i >> 1) * 2;
				int w = (shape == 0 || shape == 1) ? 2 : 1;
				int h = (shape == 0 || shape == 2) ? 2 : 1;
				if (pf < 0 || !((pf >> lx) & 1)) continue;
				for (int y = y0; y < y0 + 2; y += h)
					for (int x = x0; x < x0 + 2; x += w) {
						int16_t p[2];
						int dv[2];
						mvp(s, lx, x, y, w, m->ref[lx][i], 0, p);
						read_mvd(s, lx, x, y, dv);
						fill_mv(m, lx, x, y, w, h, p[0] + dv[0], p[1] + dv[1]);
						fill_mvd(m, lx, x, y, w, h, dv[0], dv[1]);
					}
			}
		}
		if (is_b) {
			/* need_transform_size_8x8 (h264.cpp:1296-1303, 9531-9541) */
			if (s->sps->direct_8x8_inference_flag) {
				allow_t8 = 1;
			} else {
				allow_t8 = 1;
				for (int i = 0; i < 4; ++i)
					if (!(sub[i] >= 1 && sub[i] <= 3)) allow_t8 = 0;
			}
		} else {
			allow_t8 = (sub[0] == 0 && sub[1] == 0 && sub[2] == 0 && sub[3] == 0);
		}
		if (decode_residual_inter(s, allow_t8) < 0) return -1;
	} else {
		/* 16x16, 16x8, 8x16 */
		int shape, pm;
		if (type >= MBT_B_FIRST) {
			int bt = type - MBT_B_FIRST; /* 0.. */
			pm = b_predmap[bt];
			shape = (bt < 3) ? 0 : ((bt & 1) ? 1 : 2); /* bt 3 = B_L0_L0_16x8, bt 4 = B_L0_L0_8x16 */
			if (bt < 3) pm = (pm & 1) | ((pm & 2) << 1); /* per partition bits: L0 part0, L1 part0 */
		} else {
			shape = type - MBT_P16x16; /* 0 16x16, 1 16x8, 2 8x16 */
			pm = (shape == 0) ? 1 : 3;
		}
		{
			int nparts = (shape == 0) ? 1 : 2;
			/* ref_idx for all partitions (L0 then L1), then mvd likewise */
			for (int lx = 0; lx < 2; ++lx)
				for (int p = 0; p < nparts; ++p) {
					int b8 = (shape == 1) ? p * 2 : p; /* first 8x8 of the partition */
					int ref;
					if (!((pm >> (lx * 2 + p)) & 1)) continue;
					ref = read_ref_idx(s, lx, b8, nact[lx]);
					if (shape == 0) { for (int k = 0; k < 4; ++k) m->ref[lx][k] = (int8_t)ref; }
					else if (shape == 1) { m->ref[lx][p * 2] = m->ref[lx][p * 2 + 1] = (int8_t)ref; }
					else { m->ref[lx][p] = m->ref[lx][p + 2] = (int8_t)ref; }
				}
			for (int lx = 0; lx < 2; ++lx)
				for (int p = 0; p < nparts; ++p) {
					int x = (shape == 2) ? p * 2 : 0, y = (shape == 1) ? p * 2 : 0;
					int w = (shape == 2) ? 2 : 4, h = (shape == 1) ? 2 : 4;
					int b8 = (shape == 1) ? p * 2 : p;
					int sh_ = (shape == 0) ? 0 : (shape == 1 ? 1 + p : 3 + p);
					int16_t pv[2];
					int dv[2];
					if (!((pm >> (lx * 2 + p)) & 1)) continue;
					mvp(s, lx, x, y, w, m->ref[lx][b8], sh_, pv);
					read_mvd(s, lx, x, y, dv);
					fill_mv(m, lx, x, y, w, h, pv[0] + dv[0], pv[1] + dv[1]);
					fill_mvd(m, lx, x, y, w, h, dv[0], dv[1]);
				}
		}
		if (decode_residual_inter(s, 1) < 0) return -1;
	}
	finish_mb_common(s);
	return 0;
}

/* ================================================================== slice data loop (h264.cpp:10210-10251) */
static int decode_mb(slice_ctx_t *s)
{
	int type = read_mb_type(s);
	if (type < 0) return -1;
	if (type == MBT_IPCM) return decode_pcm(s);
	if (type <= MBT_IPCM) return decode_intra(s, type);
	return decode_inter(s, type);
}

static void next_mb(slice_ctx_t *s)
{
	s->addr++;
	if (0 <= s->firstline) s->firstline--;
}

int h264_slice_data(h264_dec_t *d)
{
	slice_ctx_t s;
	h264_slice_t *sh = &d->sh;
	int ret = 0;
	int first_in_slice;
	memset(&s, 0, sizeof(s));
	s.d = d;
	s.sh = sh;
	s.pps = &d->pps[sh->pps_id];
	s.sps = &d->sps[s.pps->sps_id];
	s.cabac = s.pps->entropy_coding_mode_flag;
	s.slice_type = sh->slice_type;
	s.t8x8_mode = s.pps->transform_8x8_mode_flag;
	s.addr = sh->first_mb;
	s.firstline = d->mb_w;
	s.coef = d->pic->coef + d->pic->n_coef;
	set_qp(&s, sh->qp);
	vlc_init();
	if (s.addr >= d->n_mbs) return -1;
	first_in_slice = s.addr;

	/* per-slice deblock parameters and weighted-prediction record */
	if (d->slice_num >= 1024) return -1;
	d->slice_idc[d->slice_num] = (int8_t)sh->disable_deblocking_filter_idc;
	d->slice_alpha[d->slice_num] = (int8_t)sh->alpha_off;
	d->slice_beta[d->slice_num] = (int8_t)sh->beta_off;
	{
		m2r_picture_t *pic = d->pic;
		m2r_slice_t *sr;
		if (pic->n_slices >= pic->cap_slices) return -1;
		d->slice_rec = pic->n_slices++;
		sr = &pic->slice[d->slice_rec];
		memset(sr, 0, sizeof(*sr));
		sr->wp_mode = (uint8_t)sh->wp_mode;
		sr->log2wd[0] = (uint8_t)sh->log2wd[0];
		sr->log2wd[1] = (uint8_t)sh->log2wd[1];
		if (sh->wp_mode == M2R_WP_EXPLICIT) {
			memcpy(sr->w, sh->w, sizeof(sr->w));
			memcpy(sr->o, sh->o, sizeof(sr->o));
		} else if (sh->wp_mode == M2R_WP_IMPLICIT) {
			/* pred_weight_type2, h264.cpp:7001-7025 */
			for (int i = 0; i < sh->num_ref_idx_active[0] && i < 32; ++i)
				for (int j = 0; j < sh->num_ref_idx_active[1] && j < 32; ++j) {
					const h264_ref_t *r0 = &d->refs[0][i & 15], *r1 = &d->refs[1][j & 15];
					int w0 = 32, w1 = 32;
					if (!(r0->poc == r1->poc || r0->in_use != REF_SHORT || r1->in_use != REF_SHORT)) {
						int dsf;
						int td = r1->poc - r0->poc, tb = sh->poc - r0->poc, tx;
						td = td < -128 ? -128 : (td > 127 ? 127 : td);
						tb = tb < -128 ? -128 : (tb > 127 ? 127 : tb);
						tx = (16384 + iabs(td / 2)) / td;
						dsf = (tb * tx + 32) >> 6;
						w1 = dsf >> 2;
						if (w1 < -64 || 128 < w1) w0 = w1 = 32;
						else w0 = 64 - w1;
					}
					sr->iw[i][j][0] = (int8_t)w0;
					sr->iw[i][j][1] = (int8_t)w1;
				}
		}
	}

	if (s.cabac) {
		int idc = (sh->slice_type == 2) ? 0 : sh->cabac_init_idc + 1;
		size_t pos = (hb_pos(&d->bs, d->slice_rbsp) + 7) >> 3; /* cabac_alignment_one_bit */
		cabac_init_ctx(&d->cabac, s.qp, idc);
		d->cabac_start = d->slice_rbsp + pos;
		cabac_start(&d->cabac, d->cabac_start, d->slice_rbsp_end);
	}

	/* every MB record / coefficient / motion slot of the picture arena is sized for n_mbs MBs: slices that
	 * overlap (a damaged stream) would decode more than that and run past it; the picture is an error */
#define MB_ROOM() do { if (d->mbs_decoded + d->par_first_mb >= d->n_mbs) return -1; } while (0)
	for (;;) {
		MB_ROOM();
		if (s.slice_type != 2) {
			if (s.cabac) {
				init_mb(&s);
				if (read_mb_skip(&s)) {
					decode_skip(&s);
					d->mbs_decoded++;
					if (s.addr + 1 >= d->n_mbs) { ret = 1; break; }
					if (cabac_terminate(&d->cabac)) { next_mb(&s); break; }
					next_mb(&s);
					continue;
				}
			} else {
				uint32_t run = hb_ue(&d->bs);
				int more;
				if (run > (uint32_t)(d->n_mbs - s.addr)) run = (uint32_t)(d->n_mbs - s.addr);
				while (run--) {
					MB_ROOM();
					init_mb(&s);
					decode_skip(&s);
					d->mbs_decoded++;
					if (s.addr + 1 >= d->n_mbs) { ret = 1; goto out; }
					next_mb(&s);
				}
				more = hb_pos(&d->bs, d->slice_rbsp) < d->slice_rbsp_bits;
				if (!more) break;
				MB_ROOM();
				init_mb(&s);
			}
		} else {
			init_mb(&s);
		}
		s.cur->skip = 0;
		if (decode_mb(&s) < 0) return -1;
		d->mbs_decoded++;
		if (s.addr + 1 >= d->n_mbs) { ret = 1; break; }
		if (s.cabac) {
			if (cabac_terminate(&d->cabac)) { next_mb(&s); break; }
		} else if (hb_pos(&d->bs, d->slice_rbsp) >= d->slice_rbsp_bits) {
			next_mb(&s);
			break;
		}
		next_mb(&s);
	}
#undef MB_ROOM
out:
	d->pic->n_coef = (int32_t)(s.coef - d->pic->coef);
	/* a damaged stream's slices can reach the picture's last MB with MBs of it never coded (a slice header
	 * jumping ahead, overlapping slices): their records would be another picture's, whose coefficient /
	 * motion offsets this picture's pools do not hold.  Such a picture is an error, not a frame.  (A
	 * slice-parallel slice, par_first_mb > 0, counts only its own range; job_run_par checks the tiling.) */
	if (ret == 1 && d->par_first_mb == 0 && d->mbs_coded != d->n_mbs) ret = -1;
	/* picture-final firstline: value during the last MB of the picture (increment_mb_pos) */
	if (ret == 1) {
		int k = s.addr - first_in_slice; /* index of the last MB inside its slice */
		d->last_firstline = imax(d->mb_w - k, -1);
	}
	d->slice_num++;
	return ret;
}
