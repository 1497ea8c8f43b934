/*
 * h265gen — deterministic synthetic H.265 (Main, 8-bit 4:2:0) stream generator for the tests and the
 * bench (the repository's own encoder of random syntax: no pixels are coded, every syntax decision is
 * drawn from a seeded PRNG and written with a CABAC encoder).
 *
 * Pictures are intra (I slices: IDR_W_RADL first, then TRAIL_R), one slice each, in the tool set the
 * reference decoder accepts (h265.cpp: no PCM, transquant bypass, cu_qp_delta, scaling lists, tiles,
 * WPP): coding quadtrees with boundary splits, 2Nx2N and NxN intra CUs, all 35 luma modes through the
 * MPM / remaining-mode syntax, the 5 chroma modes, transform trees down to 4x4, residuals with
 * transform skip, sign data hiding, greater1 / greater2 / remaining levels, SAO (band and edge, merges)
 * and deblocking with slice offsets.  Levels are kept small so that no reconstruction leaves the
 * reference's CLIP255C domain (the oracle counts it; tools/make_h265_goldens.py keeps only clean streams).
 *
 *   h265gen --preset NAME --seed S --frames N -o out.265 [--dump syntax.txt]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../h264gen/bitwriter.h"
#include "h264_spec_tables.h"
#include "h265_dec.h"

/* ------------------------------------------------------------------ PRNG */
static uint64_t rs;
static uint32_t rnd(void)
{
	rs ^= rs << 13;
	rs ^= rs >> 7;
	rs ^= rs << 17;
	return (uint32_t)(rs >> 11);
}
static int rn(int n) { return (int)(rnd() % (uint32_t)n); }
static int chance(int pct) { return rn(100) < pct; }

/* ------------------------------------------------------------------ configuration */
typedef struct {
	const char *name;
	int w, h, ctb_log2, max_tb_log2, depth_intra;
	int qp, cb_off, cr_off, slice_cb, slice_cr;
	int sign_hiding, tskip, strong, sao, deblock, beta, tc;
	int split_pct, nxn_pct, cbf_pct, big_pct; /* split / NxN / coded-block / large-level probabilities */
	int frames;
	/* P / B pictures (0: an intra stream) */
	int gop;                  /* picture structure: 1 I P P P..., 2 hierarchical B, 3 low-delay B */
	int amp, depth_inter, cabac_init, merge_level, max_merge;
	int skip_pct, intra_pct, merge_pct, bi_pct, rqt_pct, mvd_max;
} cfg_t;

static const cfg_t presets[] = {
	/* name        w     h   ctb tb dep qp  cbo cro sco scr sdh ts st sao dbk  b   t  spl nxn cbf big frames */
	{"cov_h265_a", 208, 120, 4, 4, 1, 30, 0, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 55, 30, 60, 5, 3},
	{"cov_h265_b", 320, 200, 5, 5, 2, 26, 2, -3, 1, 2, 0, 0, 1, 1, 1, 2, -2, 45, 40, 55, 10, 3},
	{"cov_h265_c", 256, 136, 6, 5, 3, 34, -2, 4, 0, 0, 1, 1, 0, 1, 1, -4, 3, 40, 25, 50, 5, 3},
	{"cov_h265_nodbk", 192, 128, 5, 4, 1, 28, 0, 0, 0, 0, 1, 1, 1, 1, 0, 0, 0, 50, 30, 60, 5, 2},
	{"cov_h265_nosao", 192, 128, 6, 5, 2, 24, 0, 0, 0, 0, 1, 0, 1, 0, 1, 6, 6, 50, 30, 60, 5, 2},
	{"cov_h265_hiqp", 160, 96, 4, 4, 1, 45, 3, 3, 0, 0, 1, 1, 1, 1, 1, 6, 6, 50, 30, 40, 0, 2},
	{"c_h265_1080p", 1920, 1080, 6, 5, 1, 30, 0, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 35, 20, 50, 3, 8},
	/* P / B:        w    h   ctb tb dep qp  cbo cro sco scr sdh ts st sao dbk  b   t  spl nxn cbf big fr  gop amp dpi cin mrg mx skp int mrp bi rqt mvd */
	{"cov_h265_p", 200, 120, 5, 4, 1, 30, 0, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 45, 20, 50, 3, 6, 1, 1, 1, 0, 2, 5, 20, 10, 40, 0, 60, 24},
	{"cov_h265_hb", 232, 136, 4, 4, 1, 28, 1, -1, 0, 0, 1, 0, 1, 1, 1, 2, 2, 45, 20, 50, 3, 8, 2, 0, 0, 1, 3, 3, 25, 10, 40, 50, 55, 16},
	{"cov_h265_ldb", 296, 168, 6, 5, 2, 32, 0, 0, 1, -1, 0, 1, 1, 1, 1, -2, 0, 40, 20, 45, 3, 8, 3, 1, 2, 1, 4, 4, 20, 8, 45, 40, 60, 40},
	{"cov_h265_pnodbk", 168, 104, 4, 3, 1, 26, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 45, 20, 55, 3, 5, 1, 0, 1, 1, 2, 1, 15, 15, 50, 0, 65, 12},
	{"c_h265_1080p_pb", 1920, 1080, 6, 5, 1, 30, 0, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 35, 20, 50, 3, 8, 2, 1, 1, 1, 2, 5, 25, 5, 45, 40, 50, 32},
	{NULL, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
};

static cfg_t C;
static FILE *dumpf;

/* ------------------------------------------------------------------ CABAC encoder on the H.265 contexts */
static cenc_t E;

static void ctx_init(int qp, int init_type)
{
	const int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
	for (int i = 0; i < H265_NUM_CTX; ++i) {
		int pre = ((h265_cabac_init_mn[init_type][i][0] * q) >> 4) + h265_cabac_init_mn[init_type][i][1];
		pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
		E.st[i] = (pre <= 63) ? (uint8_t)((63 - pre) << 1) : (uint8_t)(((pre - 64) << 1) | 1);
	}
}

static void dec(int ctx, int bin) { cenc_decision(&E, ctx, bin); }
static void byp(int bin) { cenc_bypass(&E, bin); }
static void bypn(uint32_t v, int n)
{
	for (int i = n - 1; i >= 0; --i) byp((int)((v >> i) & 1));
}

/* ------------------------------------------------------------------ picture state */
static int W, H, CTB, cols, rows, W4, FW, FH;
static uint8_t *cb_log2, *ipm;

static int order_map(int mode)
{
	if (mode >= 6 && mode <= 14) return 2;
	if (mode >= 22 && mode <= 30) return 1;
	return 0;
}

/* scan position k -> x | y << 4 (6.5.3 - 6.5.5) */
static uint8_t scan_pos[3][4][64];
static void build_scans(void)
{
	for (int l = 1; l <= 3; ++l) {
		const int n = 1 << l;
		int k = 0;
		for (int s = 0; s <= 2 * (n - 1); ++s)
			for (int y = s; y >= 0; --y) {
				const int x = s - y;
				if (y < n && x < n) scan_pos[0][l][k++] = (uint8_t)(x | (y << 4));
			}
		k = 0;
		for (int y = 0; y < n; ++y)
			for (int x = 0; x < n; ++x) scan_pos[1][l][k++] = (uint8_t)(x | (y << 4));
		k = 0;
		for (int x = 0; x < n; ++x)
			for (int y = 0; y < n; ++y) scan_pos[2][l][k++] = (uint8_t)(x | (y << 4));
	}
}

/* one residual block: random sparse levels, written per 7.3.8.11 */
static void residual(int log2, int cidx, int scan)
{
	const int n = 1 << log2, chroma = cidx > 0;
	int lev[32 * 32];
	memset(lev, 0, sizeof(lev));
	/* the last significant coefficient, biased to low frequencies, and a few others before it in scan order */
	const int lsb = log2 - 2;
	const uint8_t *sbscan = scan_pos[scan][lsb ? lsb : 1];
	const uint8_t *inscan = scan_pos[scan][2];
	const int nsb = 1 << (2 * lsb);
	int last_sb = 0, last_k = 0;
	{
		const int r = rn(100);
		const int span = r < 50 ? (nsb < 2 ? 1 : (nsb + 3) / 4) : (r < 85 ? (nsb + 1) / 2 : nsb);
		last_sb = rn(span < 1 ? 1 : span);
		last_k = rn(r < 30 ? 4 : 16);
		if (nsb == 1 && rn(4) == 0) last_k = 0;
	}
	const int tskip = (log2 == 2 && C.tskip && chance(20));
	for (int i = 0; i <= last_sb; ++i) {
		const int xs = lsb ? (sbscan[i] & 15) : 0, ys = lsb ? (sbscan[i] >> 4) : 0;
		const int coded = (i == last_sb || i == 0) ? 1 : chance(60);
		if (!coded) continue;
		for (int k = 0; k < 16; ++k) {
			if (i == last_sb && k > last_k) break;
			const int x = (xs << 2) + (inscan[k] & 15), y = (ys << 2) + (inscan[k] >> 4);
			int v = 0;
			if (i == last_sb && k == last_k) v = 1;
			else if (chance(i == 0 ? 45 : 25)) v = 1;
			if (v) {
				if (chance(30)) v = 2;
				if (chance(12)) v = 3 + rn(3);
				if (log2 <= 3 && chance(C.big_pct)) v = 6 + rn(6);
				/* keep the residual of large blocks and low QPs modest */
				if (log2 >= 4 && v > 3 && C.qp < 30) v = 3;
				if (log2 >= 4 && v > 2 && C.qp >= 30) v = 2;
				if (C.qp >= 40) v = 1;
				if (chance(50)) v = -v;
			}
			lev[y * n + x] = v;
		}
	}
	if (tskip) dec(H265_CTX_TSKIP + chroma, 1);
	else if (log2 == 2 && C.tskip) dec(H265_CTX_TSKIP + chroma, 0);
	/* last position (in scan-swapped coordinates for the vertical scan) */
	int lx = (sbscan[last_sb] & 15) * 4 + (inscan[last_k] & 15), ly = (sbscan[last_sb] >> 4) * 4 + (inscan[last_k] >> 4);
	if (!lsb) {
		lx = inscan[last_k] & 15;
		ly = inscan[last_k] >> 4;
	}
	{
		int cx = lx, cy = ly;
		if (scan == 2) {
			cx = ly;
			cy = lx;
		}
		const int off = chroma ? 15 : 3 * (log2 - 2) + ((log2 - 1) >> 2);
		const int shift = chroma ? log2 - 2 : (log2 + 1) >> 2;
		const int max = 2 * log2 - 1;
		int pre[2], suf[2], sl[2];
		const int v[2] = {cx, cy};
		for (int a = 0; a < 2; ++a) {
			int p = 0;
			if (v[a] < 4) {
				p = v[a];
				sl[a] = 0;
				suf[a] = 0;
			} else {
				/* the prefix whose group holds v: (1 << ((p >> 1) - 1)) * (2 + (p & 1)) <= v */
				for (p = 4; p <= max; ++p) {
					const int base = (1 << ((p >> 1) - 1)) * (2 + (p & 1));
					const int len = (p >> 1) - 1;
					if (v[a] >= base && v[a] < base + (1 << len)) break;
				}
				sl[a] = (p >> 1) - 1;
				suf[a] = v[a] - (1 << ((p >> 1) - 1)) * (2 + (p & 1));
			}
			pre[a] = p;
		}
		for (int a = 0; a < 2; ++a) {
			const int base = a ? H265_CTX_LAST_Y : H265_CTX_LAST_X;
			for (int i = 0; i < pre[a]; ++i) dec(base + off + (i >> shift), 1);
			if (pre[a] < max) dec(base + off + (pre[a] >> shift), 0);
		}
		for (int a = 0; a < 2; ++a)
			if (pre[a] > 3) bypn((uint32_t)suf[a], sl[a]);
	}
	/* subblocks from the last one down */
	{
		uint8_t csbf[8][8];
		int greater1ctx = 1;
		memset(csbf, 0, sizeof(csbf));
		for (int i = last_sb; i >= 0; --i) {
			const int xs = lsb ? (sbscan[i] & 15) : 0, ys = lsb ? (sbscan[i] >> 4) : 0;
			int prev = 0, any = 0, infer_dc = 0;
			if (xs + 1 < (1 << lsb)) prev |= csbf[ys][xs + 1];
			if (ys + 1 < (1 << lsb)) prev |= csbf[ys + 1][xs] << 1;
			for (int k = 0; k < 16; ++k) {
				const int x = (xs << 2) + (inscan[k] & 15), y = (ys << 2) + (inscan[k] >> 4);
				if (lev[y * n + x]) any = 1;
			}
			if (i < last_sb && i > 0) {
				dec(H265_CTX_CSBF + ((prev & 1) | (prev >> 1)) + (chroma ? 2 : 0), any);
				infer_dc = 1;
			}
			csbf[ys][xs] = (uint8_t)((i < last_sb && i > 0) ? any : 1);
			if (!csbf[ys][xs]) continue;
			int sig_k[16], sig_v[16], nsig = 0;
			const int top = (i == last_sb) ? last_k : 15;
			for (int k = top; k >= 0; --k) {
				const int x = (xs << 2) + (inscan[k] & 15), y = (ys << 2) + (inscan[k] >> 4);
				const int sig = lev[y * n + x] != 0;
				if (i == last_sb && k == last_k) {
					/* implied */
				} else if (k == 0 && infer_dc && nsig == 0) {
					/* inferred 1: the DC of this subblock must be nonzero */
					if (!sig) lev[y * n + x] = 1;
				} else {
					int sctx;
					const int xp = inscan[k] & 15, yp = inscan[k] >> 4;
					if (log2 == 2) {
						static const uint8_t m4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
						sctx = m4[(y << 2) + x];
					} else if (x + y == 0) {
						sctx = 0;
					} else {
						if (prev == 0) sctx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
						else if (prev == 1) sctx = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
						else if (prev == 2) sctx = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
						else sctx = 2;
						if (!chroma) {
							if (xs + ys > 0) sctx += 3;
							sctx += (log2 == 3) ? (scan == 0 ? 9 : 15) : 21;
						} else {
							sctx += (log2 == 3) ? 9 : 12;
						}
					}
					dec(H265_CTX_SIG + (chroma ? 27 : 0) + sctx, sig);
				}
				if (lev[y * n + x]) {
					sig_k[nsig] = k;
					sig_v[nsig++] = lev[y * n + x];
				}
			}
			if (!nsig) continue;
			/* greater1 / greater2 */
			int need_rem = 0, first_g1 = -1, base[16];
			const int ctxset = ((!chroma && i != 0) ? 2 : 0) + (greater1ctx == 0);
			const int g1off = ctxset * 4 + (chroma ? 16 : 0);
			greater1ctx = 1;
			for (int j = 0; j < nsig; ++j) {
				const int a = abs(sig_v[j]);
				base[j] = 1;
				if (j < 8) {
					dec(H265_CTX_GT1 + g1off + greater1ctx, a > 1);
					if (a > 1) {
						greater1ctx = 0;
						base[j] = 2;
						if (first_g1 >= 0) need_rem |= 1 << j;
						else first_g1 = j;
					} else if (greater1ctx > 0 && greater1ctx < 3) {
						greater1ctx++;
					}
				} else {
					need_rem |= 1 << j;
				}
			}
			if (first_g1 >= 0) {
				const int a = abs(sig_v[first_g1]);
				dec(H265_CTX_GT2 + ctxset + (chroma ? 4 : 0), a > 2);
				if (a > 2) {
					base[first_g1] = 3;
					need_rem |= 1 << first_g1;
				}
			}
			/* sign data hiding: the first coefficient's sign follows the parity of the level sum */
			const int hide = C.sign_hiding && (sig_k[0] - sig_k[nsig - 1] > 3);
			if (hide) {
				int sum = 0;
				for (int j = 0; j < nsig; ++j) sum += abs(sig_v[j]);
				const int a = abs(sig_v[nsig - 1]);
				sig_v[nsig - 1] = (sum & 1) ? -a : a;
				const int x = (xs << 2) + (inscan[sig_k[nsig - 1]] & 15), y = (ys << 2) + (inscan[sig_k[nsig - 1]] >> 4);
				lev[y * n + x] = sig_v[nsig - 1];
			}
			for (int j = 0; j < nsig - hide; ++j) byp(sig_v[j] < 0);
			int rice = 0;
			for (int j = 0; j < nsig; ++j) {
				const int a = abs(sig_v[j]);
				if (need_rem & (1 << j)) {
					const int r = a - base[j];
					/* coeff_abs_level_remaining: prefix < 4: (p << rice) + suffix(rice); else EGk-style */
					if ((r >> rice) < 4) {
						const int p = r >> rice;
						for (int t = 0; t < p; ++t) byp(1);
						byp(0);
						bypn((uint32_t)(r & ((1 << rice) - 1)), rice);
					} else {
						int p = 4;
						while (r >= (1 << (p - 3 + rice + 1)) + (2 << rice)) p++;
						/* value = (1 << sl) + (2 << rice) + suffix(sl), sl = p - 3 + rice (h265.cpp:1345-1346) */
						const int sl = p - 3 + rice;
						const int suf = r - ((1 << sl) + (2 << rice));
						for (int t = 0; t < p; ++t) byp(1);
						byp(0);
						bypn((uint32_t)suf, sl);
					}
					if (a > (3 << rice) && rice < 4) rice++;
				}
			}
		}
	}
	if (dumpf) {
		fprintf(dumpf, "res c%d l%d s%d t%d:", cidx, log2, scan, tskip);
		for (int i = 0; i < n * n; ++i)
			if (lev[i]) fprintf(dumpf, " %d@%d", lev[i], i);
		fprintf(dumpf, "\n");
	}
}

static int order_luma[4], order_chroma, intra_split;

static void transform_tree(int x0, int y0, int log2, int depth, int cbf_cbcr, int blk, int pred_idx)
{
	int split = 0, cbf = 0;
	if (C.max_tb_log2 < log2) {
		split = 1;
	} else if (depth == 0 && intra_split) {
		split = 2;
	} else if (2 < log2 && depth < C.depth_intra) {
		split = chance(C.split_pct);
		dec(H265_CTX_SPLIT_TRANSFORM + 5 - log2, split);
	}
	if (log2 > 2) {
		if (cbf_cbcr & 2) {
			const int b = chance(C.cbf_pct);
			dec(H265_CTX_CBF_CHROMA + depth, b);
			cbf |= b << 1;
		}
		if (cbf_cbcr & 1) {
			const int b = chance(C.cbf_pct);
			dec(H265_CTX_CBF_CHROMA + depth, b);
			cbf |= b;
		}
	} else {
		cbf = cbf_cbcr;
	}
	if (split) {
		const int h = 1 << (log2 - 1);
		int pi = split == 2 ? 0 : pred_idx;
		const int pinc = split == 2;
		transform_tree(x0, y0, log2 - 1, depth + 1, cbf, 0, pi);
		pi += pinc;
		transform_tree(x0 + h, y0, log2 - 1, depth + 1, cbf, 1, pi);
		pi += pinc;
		transform_tree(x0, y0 + h, log2 - 1, depth + 1, cbf, 2, pi);
		pi += pinc;
		transform_tree(x0 + h, y0 + h, log2 - 1, depth + 1, cbf, 3, pi);
		return;
	}
	const int cl = chance(C.cbf_pct);
	dec(H265_CTX_CBF_LUMA + (depth == 0), cl);
	if (cl) residual(log2, 0, log2 <= 3 ? order_map(order_luma[pred_idx]) : 0);
	if (cbf) {
		if (log2 > 2 || blk == 3) {
			const int c = log2 > 2 ? log2 - 1 : 2;
			const int scan = c == 2 ? order_map(order_chroma) : 0;
			if (cbf & 2) residual(c, 1, scan);
			if (cbf & 1) residual(c, 2, scan);
		}
	}
}

static void mpm_cands(int a, int b, int cand[3])
{
	if (a == b) {
		if (a < 2) {
			cand[0] = 0;
			cand[1] = 1;
			cand[2] = 26;
		} else {
			cand[0] = a;
			cand[1] = 2 + ((a + 29) % 32);
			cand[2] = 2 + ((a - 2 + 1) % 32);
		}
	} else {
		cand[0] = a;
		cand[1] = b;
		cand[2] = (a != 0 && b != 0) ? 0 : ((a != 1 && b != 1) ? 1 : 26);
	}
}

static void coding_unit(int x0, int y0, int log2)
{
	int part = 1;
	for (int j = 0; j < (1 << (log2 - 2)); ++j) memset(cb_log2 + (size_t)((y0 >> 2) + j) * W4 + (x0 >> 2), log2, (size_t)1 << (log2 - 2));
	intra_split = 0;
	if (log2 == 3) {
		intra_split = chance(C.nxn_pct);
		dec(H265_CTX_PART_MODE, !intra_split);
		if (intra_split) part = 4;
	}
	const int pl = part == 4 ? log2 - 1 : log2;
	int modes[4], mpm[4], idx[4];
	for (int i = 0; i < part; ++i) {
		const int px = x0 + ((i & 1) << pl), py = y0 + ((i >> 1) << pl);
		int cand[3];
		const int a = px > 0 ? ipm[(size_t)(py >> 2) * W4 + (px >> 2) - 1] : 1;
		const int b = (py > 0 && ((py - 1) / CTB) == (py / CTB)) ? ipm[(size_t)((py >> 2) - 1) * W4 + (px >> 2)] : 1;
		mpm_cands(a, b, cand);
		/* half of the time a candidate, else any mode */
		if (chance(50)) {
			idx[i] = rn(3);
			modes[i] = cand[idx[i]];
			mpm[i] = 1;
		} else {
			modes[i] = rn(35);
			mpm[i] = 0;
			for (int k = 0; k < 3; ++k)
				if (cand[k] == modes[i]) {
					mpm[i] = 1;
					idx[i] = k;
				}
			if (!mpm[i]) {
				/* rem = mode minus the candidates below it */
				int s[3] = {cand[0], cand[1], cand[2]}, t;
				if (s[0] > s[1]) { t = s[0]; s[0] = s[1]; s[1] = t; }
				if (s[0] > s[2]) { t = s[0]; s[0] = s[2]; s[2] = t; }
				if (s[1] > s[2]) { t = s[1]; s[1] = s[2]; s[2] = t; }
				int r = modes[i];
				for (int k = 2; k >= 0; --k)
					if (modes[i] > s[k]) r--;
				idx[i] = r;
			}
		}
		order_luma[i] = modes[i];
		for (int j = 0; j < (1 << (pl - 2)); ++j) memset(ipm + (size_t)((py >> 2) + j) * W4 + (px >> 2), modes[i], (size_t)1 << (pl - 2));
	}
	for (int i = 0; i < part; ++i) dec(H265_CTX_PREV_INTRA_LUMA, mpm[i]);
	for (int i = 0; i < part; ++i) {
		if (mpm[i]) {
			byp(idx[i] > 0);
			if (idx[i] > 0) byp(idx[i] > 1);
		} else {
			bypn((uint32_t)idx[i], 5);
		}
	}
	if (part != 4) order_luma[1] = order_luma[2] = order_luma[3] = order_luma[0];
	{
		const int ci = rn(5);
		static const int base[4] = {0, 26, 10, 1};
		dec(H265_CTX_INTRA_CHROMA, ci != 4);
		if (ci != 4) bypn((uint32_t)ci, 2);
		order_chroma = ci == 4 ? order_luma[0] : (base[ci] == order_luma[0] ? 34 : base[ci]);
	}
	if (dumpf) fprintf(dumpf, "cu %d %d l%d p%d m %d %d %d %d c%d\n", x0, y0, log2, part, order_luma[0], order_luma[1], order_luma[2],
	                   order_luma[3], order_chroma);
	transform_tree(x0, y0, log2, 0, 3, 0, 0);
}

/* ------------------------------------------------------------------ P / B pictures */
/* The generator derives every block's motion itself (merge, AMVP, TMVP as the reference does them:
 * h265.cpp:3572-3931) to write AMVP differences against the predictor and to dump the motion for
 * tests/gen_check.py-style comparison with the parser.  Where the reference's result would depend on
 * memory it never wrote, the generator avoids the syntax (h265gen's own rules):
 *   - an L0-only AMVP block leaves its L1 vector unset (prediction_unit's mvxy[1]); a merge list whose
 *     pruning (memcmp of the whole motion) would compare such bytes with different ones is not chosen;
 *   - a P slice's temporal merge candidate leaves its L1 reference unset: never selected;
 *   - B slices code no L1-only AMVP block (the deblocking strength would read an unset vector);
 *   - prediction blocks at the top-right corner of a last-column CTU whose right edge is the picture's
 *     read past the neighbour array when the picture width is a multiple of the CTB: intra there. */
typedef struct {
	int16_t mv[2][2];
	int8_t ref[2];
} gpred_t;

typedef struct {
	gpred_t p;
	int undef;  /* mv[1] is the reference's unset stack memory (AMVP L0-only); 2: ref[1] unset (P temporal) */
	int origin; /* the block that made the motion (undef ones compare equal only with the same origin) */
} gmot_t;

typedef struct {
	uint8_t pu_intra, skip;
	gmot_t m;
} gnb_t;

typedef struct {
	uint8_t intra;
	gpred_t p;
} gcol_t;

static gnb_t *gnb;                       /* per 4x4 unit of the picture */
static gcol_t *gcol[8];                  /* per frame, 16x16 units */
static int gcol_stride, origin_seq;
static int8_t reg_frame[8][2][16];       /* per frame: its lists' frames (registered by every slice) */
static int frame_poc[8];
static int ref_poc[2][16];               /* the lists (persistent across slices, as in the reference) */
static int8_t ref_frm[2][16];
static int num_ref[2] = {1, 1}, col_l0 = 1, col_idx, cabac_init_flag, mvd_l1_zero, max_merge = 5;
static int cur_slot, cur_poc, bslice, inter_pic, lowdelay;
static int16_t colmv[8][8], tmvs[8][8];
static const gcol_t *col_ref;
static const int8_t (*col_lists)[16];
static const gnb_t nb_out = {1, 0, {{{{0, 0}, {0, 0}}, {-1, -1}}, 0, 0}};

static const gnb_t *gnb_at(int x, int y)
{
	if (x < 0 || y < 0 || x >= W || y >= H) return &nb_out;
	return &gnb[(size_t)(y >> 2) * W4 + (x >> 2)];
}

static void gnb_rect(int px, int py, int w, int h, int what, const gmot_t *m)
{
	for (int y = py; y < py + h && y < H; y += 4)
		for (int x = px; x < px + w && x < W; x += 4) {
			gnb_t *u = &gnb[(size_t)(y >> 2) * W4 + (x >> 2)];
			if (what == 0) { /* intra */
				u->pu_intra = 1;
				u->skip = 0;
			} else if (what == 1) { /* motion of a merged block */
				u->pu_intra = 0;
				u->skip = 1;
				u->m = *m;
			} else if (what == 2) { /* motion of an AMVP block */
				u->pu_intra = 0;
				u->skip = 0;
				u->m = *m;
			} else { /* the CU's skip flag */
				u->skip = (uint8_t)(what == 4);
			}
		}
}

static void gcol_fill(int px, int py, int w, int h, int intra, const gpred_t *p)
{
	for (int y = (py + 15) & ~15; y < py + h; y += 16)
		for (int x = (px + 15) & ~15; x < px + w; x += 16) {
			gcol_t *c = &gcol[cur_slot][(size_t)(y >> 4) * gcol_stride + (x >> 4)];
			c->intra = (uint8_t)intra;
			if (!intra) c->p = *p;
		}
}

static int16_t gscale(int poc0, int refpoc0, int poc1, int refpoc1)
{
	const int d1 = poc1 - refpoc1, d0 = poc0 - refpoc0;
	if (!d1) return 4096;
	const int td = d1 < -128 ? -128 : (d1 > 127 ? 127 : d1), tb = d0 < -128 ? -128 : (d0 > 127 ? 127 : d0);
	const int tx = (16384 + (abs(td) >> 1)) / td, v = (tb * tx + 32) >> 6;
	return (int16_t)(v < -4096 ? -4096 : (v > 4095 ? 4095 : v));
}

static int16_t gscale_mv(int mv, int sc)
{
	long v = (long)mv * sc;
	if (v >= 0) {
		v = (v + 127) >> 8;
		return (int16_t)(v > 32767 ? 32767 : v);
	}
	v = -((127 - v) >> 8);
	return (int16_t)(v < -32768 ? -32768 : v);
}

static const gcol_t *gcol_get(int px, int py, int w, int h)
{
	int bx = px + w, by = py + h;
	if ((py % CTB) + h < CTB && bx < W && by < H) {
		const gcol_t *r = &col_ref[(size_t)(by >> 4) * gcol_stride + (bx >> 4)];
		if (!r->intra) return r;
	}
	bx = px + w / 2;
	by = py + h / 2;
	return &col_ref[(size_t)(by >> 4) * gcol_stride + (bx >> 4)];
}

static void gadd_col(gpred_t *p, const gcol_t *col, int lx, int ref_idx)
{
	int cl = lowdelay ? lx : col_l0;
	int cr = col->p.ref[cl];
	if (cr < 0) {
		cl ^= 1;
		cr = col->p.ref[cl];
	}
	p->ref[lx] = (int8_t)ref_idx;
	const int sc = colmv[ref_frm[lx][ref_idx] & 7][col_lists[cl][cr] & 7];
	p->mv[lx][0] = gscale_mv(col->p.mv[cl][0], sc);
	p->mv[lx][1] = gscale_mv(col->p.mv[cl][1], sc);
}

/* the motion comparison of the merge list's pruning: 1 equal, 0 different, -1 depends on unset memory */
static int gmot_cmp(const gmot_t *a, const gmot_t *b)
{
	if (a->undef || b->undef) {
		if (a->undef && b->undef && a->origin == b->origin) return 1;
		if (a->p.ref[0] == b->p.ref[0] && a->p.ref[1] == b->p.ref[1] && !memcmp(a->p.mv[0], b->p.mv[0], 4)) return -1;
		return 0;
	}
	return !memcmp(&a->p, &b->p, sizeof(gpred_t));
}

/* the merge candidate idx selects; -1 if the reference's choice would read unset memory */
static int gmerge(int ua, int px, int py, int w, int h, int idx, gmot_t *out)
{
	gmot_t list[5];
	int num = 0, amb = 0;
	const int s = C.merge_level;
	memset(list, 0, sizeof(list));
#define ADD(nx, ny)                                                                                 \
	do {                                                                                            \
		const gnb_t *n_ = gnb_at(nx, ny);                                                           \
		if (!n_->pu_intra && (((px) >> s) != ((nx) >> s) || ((py) >> s) != ((ny) >> s))) {         \
			int dup_ = 0;                                                                       \
			for (int i_ = 0; i_ < num; ++i_) {                                                  \
				const int c_ = gmot_cmp(&n_->m, &list[i_]);                                     \
				if (c_ < 0) amb = 1;                                                            \
				if (c_ > 0) dup_ = 1;                                                           \
			}                                                                                   \
			if (!dup_) list[num++] = n_->m;                                                     \
		}                                                                                       \
	} while (0)
	if (!(ua & 1)) ADD(px - 1, py + h - 1);
	if (num <= idx) {
		if (!(ua & 2)) ADD(px + w - 1, py - 1);
		if (!(ua & 8)) ADD(px + w, py - 1);
		if (!(ua & 4)) ADD(px - 1, py + h);
		if (num <= idx && num < 4) ADD(px - 1, py - 1);
	}
#undef ADD
	if (num <= idx) {
		const gcol_t *col = gcol_get(px, py, w, h);
		if (!col->intra) {
			memset(&list[num], 0, sizeof(list[num]));
			gadd_col(&list[num].p, col, 0, 0);
			if (bslice) gadd_col(&list[num].p, col, 1, 0);
			else {
				list[num].p.ref[1] = -1;
				list[num].undef = 2;
			}
			num++;
		}
	}
	if (num > 1 && num <= idx && bslice) {
		static const int8_t l0c[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
		const int cut = num * (num - 1);
		for (int c = 0; c < cut; ++c) {
			const int i0 = l0c[c], i1 = l0c[c ^ 1];
			if (idx <= i0 || idx <= i1) break;
			const gpred_t a = list[i0].p, b = list[i1].p;
			if (a.ref[0] >= 0 && b.ref[1] >= 0 && (memcmp(a.mv[0], b.mv[1], 4) || ref_poc[0][a.ref[0]] != ref_poc[1][b.ref[1]])) {
				memset(&list[num], 0, sizeof(list[num]));
				memcpy(list[num].p.mv[0], a.mv[0], 4);
				memcpy(list[num].p.mv[1], b.mv[1], 4);
				list[num].p.ref[0] = a.ref[0];
				list[num].p.ref[1] = b.ref[1];
				if (idx < ++num) break;
			}
		}
	}
	while (num <= idx) {
		const int nref = bslice ? (num_ref[0] < num_ref[1] ? num_ref[0] : num_ref[1]) : num_ref[0];
		const int m = idx - num, r = m < nref ? m : 0;
		memset(&list[num], 0, sizeof(list[num]));
		list[num].p.ref[0] = (int8_t)r;
		list[num].p.ref[1] = (int8_t)(bslice ? r : -1);
		num++;
	}
	if (amb || list[idx].undef == 2) return -1;
	*out = list[idx];
	return 0;
}

/* AMVP (calc_mv and its helpers, h265.cpp:3742-3839) */
static void gmvp2nd(int lx, int ri, const gpred_t *n, int16_t d[2])
{
	int l = lx;
	for (int k = 0; k < 2; ++k) {
		if (n->ref[l] >= 0) {
			const int sc = tmvs[ref_frm[lx][ri] & 7][ref_frm[l][n->ref[l]] & 7];
			d[0] = gscale_mv(n->mv[l][0], sc);
			d[1] = gscale_mv(n->mv[l][1], sc);
			return;
		}
		l ^= 1;
	}
}

static const int16_t *gspatial(const gnb_t *n, int lx, int refpoc, int ri, int16_t m2[2], int *skip2, int *match2)
{
	if (n->pu_intra) return NULL;
	int l = lx;
	for (int k = 0; k < 2; ++k) {
		if (n->m.p.ref[l] >= 0) {
			if (ref_poc[l][n->m.p.ref[l]] == refpoc) {
				*skip2 = 1;
				return n->m.p.mv[l];
			}
			if (!*skip2 && !*match2) {
				gmvp2nd(lx, ri, &n->m.p, m2);
				*match2 = 1;
			}
		}
		l ^= 1;
	}
	*skip2 = 1;
	return NULL;
}

static const int16_t *gmvp_side(int ua, int side, int px, int py, int w, int h, int lx, int ri, int16_t m2[2], int *skip2)
{
	const int dir = side ? ua >> 1 : ua, refpoc = ref_poc[lx][ri];
	int match2 = 0;
	const int16_t *mv;
	if (!(dir & 4) && (mv = gspatial(side ? gnb_at(px + w, py - 1) : gnb_at(px - 1, py + h), lx, refpoc, ri, m2, skip2, &match2))) return mv;
	if (!(dir & 1) && (mv = gspatial(side ? gnb_at(px + w - 1, py - 1) : gnb_at(px - 1, py + h - 1), lx, refpoc, ri, m2, skip2, &match2)))
		return mv;
	if (side && !(ua & 3) && (mv = gspatial(gnb_at(px - 1, py - 1), lx, refpoc, ri, m2, skip2, &match2))) return mv;
	return match2 ? m2 : NULL;
}

static int gadd_mvp(const int16_t mv[2], int16_t l[2][2], int idx, int *n)
{
	const int16_t a = mv[0], b = mv[1];
	for (int i = 0; i < *n; ++i)
		if (l[i][0] == a && l[i][1] == b) return 0;
	l[*n][0] = a;
	l[*n][1] = b;
	return idx < ++*n;
}

static void gpredictor(int ua, int px, int py, int w, int h, int lx, int ri, int mvp_idx, const gcol_t *col, int16_t out[2])
{
	int16_t l[2][2], m2[2] = {0, 0};
	int n = 0, skip2 = 0;
	const int16_t *mvp = gmvp_side(ua, 0, px, py, w, h, lx, ri, m2, &skip2);
	if (!mvp || !gadd_mvp(mvp, l, mvp_idx, &n)) {
		mvp = gmvp_side(ua, 1, px, py, w, h, lx, ri, m2, &skip2);
		if (!mvp || !gadd_mvp(mvp, l, mvp_idx, &n)) {
			gpred_t t;
			int ok = 0;
			if (col) {
				gadd_col(&t, col, lx, ri);
				ok = gadd_mvp(t.mv[lx], l, mvp_idx, &n);
			}
			if (!ok) memset(l[n], 0, sizeof(l[0]) * (size_t)(2 - n));
		}
	}
	out[0] = l[mvp_idx][0];
	out[1] = l[mvp_idx][1];
}

/* mvd_coding (7.3.8.9) */
static void write_mvd(int dx, int dy)
{
	const int v[2] = {dx, dy};
	for (int k = 0; k < 2; ++k) dec(H265_CTX_ABS_MVD_GT, v[k] != 0);
	for (int k = 0; k < 2; ++k)
		if (v[k]) dec(H265_CTX_ABS_MVD_GT + 1, abs(v[k]) > 1);
	for (int k = 0; k < 2; ++k) {
		if (!v[k]) continue;
		if (abs(v[k]) > 1) { /* abs_mvd_minus2: EG1 */
			const int r = abs(v[k]) - 2;
			int bits = 0;
			while (r >= (2 << bits) - 2 + (2 << bits)) bits++;
			for (int t = 0; t < bits; ++t) byp(1);
			byp(0);
			bypn((uint32_t)(r - ((2 << bits) - 2)), bits + 1);
		}
		byp(v[k] < 0);
	}
}

static void write_merge_idx(int idx)
{
	if (max_merge > 1) {
		dec(H265_CTX_MERGE_IDX, idx > 0);
		for (int i = 1; i < max_merge - 1 && i <= idx; ++i) byp(idx > i);
	}
}

/* a merged block: its motion to the neighbour map and the motion field, and the dump */
static void gmerge_apply(int px, int py, int w, int h, int idx, const gmot_t *m)
{
	gmot_t q = *m;
	const int no_bidir = m->p.ref[0] >= 0 && m->p.ref[1] >= 0 && w + h == 12;
	if (no_bidir) q.p.ref[1] = -1;
	gnb_rect(px, py, w, h, 1, &q);
	gcol_fill(px, py, w, h, 0, &m->p);
	if (dumpf)
		fprintf(dumpf, "pu %d %d %d %d m%d r %d %d mv %d %d %d %d\n", px, py, w, h, idx, m->p.ref[0], no_bidir ? -1 : m->p.ref[1],
		        m->p.mv[0][0], m->p.mv[0][1], m->p.mv[1][0], m->p.mv[1][1]);
}

/* a merge index whose candidate the reference derives from written memory only (-1: none) */
static int gpick_merge(int ua, int px, int py, int w, int h, gmot_t *m)
{
	const int start = rn(max_merge);
	for (int k = 0; k < max_merge; ++k) {
		const int idx = (start + k) % max_merge;
		if (gmerge(ua, px, py, w, h, idx, m) == 0) return idx;
	}
	return -1;
}

/* prediction_unit: merge when allowed and drawn, else AMVP; returns 1 if merged */
static int gpu(int log2, int ua, int pred_ua, int px, int py, int w, int h)
{
	gmot_t m;
	int idx = -1;
	if (chance(C.merge_pct)) idx = gpick_merge(ua | pred_ua, px, py, w, h, &m);
	dec(H265_CTX_MERGE_FLAG, idx >= 0);
	if (idx >= 0) {
		write_merge_idx(idx);
		gmerge_apply(px, py, w, h, idx, &m);
		return 1;
	}
	int idc = 0;
	if (bslice) {
		idc = (w + h != 12 && chance(C.bi_pct)) ? 2 : 0; /* (no L1-only blocks) */
		if (w + h != 12) dec(H265_CTX_INTER_PRED_IDC + (C.ctb_log2 - log2), idc == 2);
		if (idc != 2) dec(H265_CTX_INTER_PRED_IDC + 4, 0);
	}
	const gcol_t *col = gcol_get(px, py, w, h);
	if (col->intra) col = NULL;
	memset(&m, 0, sizeof(m));
	m.p.ref[0] = m.p.ref[1] = -1;
	for (int lx = 0; lx < 2; ++lx) {
		if (lx == 1 && idc != 2) continue;
		const int ri = rn(num_ref[lx]);
		if (num_ref[lx] > 1) {
			const int nb = num_ref[lx] - 1, m2 = nb < 2 ? nb : 2;
			for (int i = 0; i < m2 && i <= ri; ++i) dec(H265_CTX_REF_IDX + i, ri > i);
			for (int i = 2; i < nb && i <= ri; ++i) byp(ri > i);
		}
		int dx = 0, dy = 0;
		if (lx == 0 || !mvd_l1_zero) {
			const int r = chance(15) ? 4 * C.mvd_max : C.mvd_max;
			dx = rn(2 * r + 1) - r;
			dy = rn(2 * r + 1) - r;
			write_mvd(dx, dy);
		}
		const int mvp_idx = rn(2);
		dec(H265_CTX_MVP_FLAG, mvp_idx);
		int16_t mvp[2];
		gpredictor(ua, px, py, w, h, lx, ri, mvp_idx, col, mvp);
		m.p.ref[lx] = (int8_t)ri;
		m.p.mv[lx][0] = (int16_t)(mvp[0] + dx);
		m.p.mv[lx][1] = (int16_t)(mvp[1] + dy);
	}
	if (idc == 0) {
		m.undef = 1;
		m.origin = ++origin_seq;
	}
	gnb_rect(px, py, w, h, 2, &m);
	gcol_fill(px, py, w, h, 0, &m.p);
	if (dumpf)
		fprintf(dumpf, "pu %d %d %d %d a%d r %d %d mv %d %d %d %d\n", px, py, w, h, idc, m.p.ref[0], m.p.ref[1], m.p.mv[0][0], m.p.mv[0][1],
		        m.p.mv[1][0], m.p.mv[1][1]);
	return 0;
}

/* transform_tree of an inter CU */
static void transform_tree_inter(int x0, int y0, int log2, int depth, int cbf_cbcr, int blk)
{
	int split = 0, cbf = 0;
	if (C.max_tb_log2 < log2) {
		split = 1;
	} else if (2 < log2 && depth < C.depth_inter) {
		split = chance(C.split_pct);
		dec(H265_CTX_SPLIT_TRANSFORM + 5 - log2, split);
	} else {
		split = depth == 0 && intra_split;
	}
	if (log2 > 2) {
		if (cbf_cbcr & 2) {
			const int b = chance(C.cbf_pct);
			dec(H265_CTX_CBF_CHROMA + depth, b);
			cbf |= b << 1;
		}
		if (cbf_cbcr & 1) {
			const int b = chance(C.cbf_pct);
			dec(H265_CTX_CBF_CHROMA + depth, b);
			cbf |= b;
		}
	} else {
		cbf = cbf_cbcr;
	}
	if (split) {
		const int h = 1 << (log2 - 1);
		transform_tree_inter(x0, y0, log2 - 1, depth + 1, cbf, 0);
		transform_tree_inter(x0 + h, y0, log2 - 1, depth + 1, cbf, 1);
		transform_tree_inter(x0, y0 + h, log2 - 1, depth + 1, cbf, 2);
		transform_tree_inter(x0 + h, y0 + h, log2 - 1, depth + 1, cbf, 3);
		return;
	}
	int cl = 1;
	if (depth || cbf) {
		cl = chance(C.cbf_pct);
		dec(H265_CTX_CBF_LUMA + (depth == 0), cl);
	}
	if (cl) residual(log2, 0, 0);
	if (cbf && (log2 > 2 || blk == 3)) {
		const int c = log2 > 2 ? log2 - 1 : 2;
		if (cbf & 2) residual(c, 1, 0);
		if (cbf & 1) residual(c, 2, 0);
	}
}

static const int8_t gav4[3][16] = {{0, 5, 10, 15, 0, 5, 10, 15, 0, 5, 10, 15, 0, 5, 10, 15},
                                   {4, 4, 6, 6, 4, 4, 6, 6, 12, 12, 14, 14, 12, 12, 14, 14},
                                   {0, 1, 0, 1, 4, 5, 4, 5, 0, 1, 0, 1, 4, 5, 4, 5}};
static const int8_t gav21[2][16] = {{0, 1, 2, 3, 0, 5, 2, 7, 8, 9, 10, 11, 8, 13, 10, 15}, {8, 9, 8, 9, 12, 13, 12, 13, 8, 9, 8, 9, 12, 13, 12, 13}};
static const int8_t gav12[2][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 4, 5, 14, 15}, {4, 4, 6, 6, 4, 4, 6, 6, 12, 12, 14, 14, 12, 12, 14, 14}};

static void coding_unit(int x0, int y0, int log2);

static void coding_unit_inter(int x0, int y0, int log2, int ua)
{
	const int len = 1 << log2;
	for (int j = 0; j < (1 << (log2 - 2)); ++j) memset(cb_log2 + (size_t)((y0 >> 2) + j) * W4 + (x0 >> 2), log2, (size_t)1 << (log2 - 2));
	/* the top-right corner of a last-column CTU at the picture's right edge (W a multiple of the CTB) */
	const int corner = (W % CTB) == 0 && x0 + len == W && (y0 % CTB) == 0 && y0 > 0;
	{
		const int ctx = (!(ua & 1) && gnb_at(x0 - 1, y0)->skip) + (!(ua & 2) && gnb_at(x0, y0 - 1)->skip);
		gmot_t m;
		int idx = -1;
		if (!corner && chance(C.skip_pct)) idx = gpick_merge(ua, x0, y0, len, len, &m);
		dec(H265_CTX_CU_SKIP + ctx, idx >= 0);
		if (idx >= 0) {
			if (dumpf) fprintf(dumpf, "icu %d %d l%d skip\n", x0, y0, log2);
			write_merge_idx(idx);
			gmerge_apply(x0, y0, len, len, idx, &m);
			gnb_rect(x0, y0, len, len, 4, NULL);
			return;
		}
	}
	if (corner || chance(C.intra_pct)) {
		dec(H265_CTX_PRED_MODE, 1);
		coding_unit(x0, y0, log2);
		gnb_rect(x0, y0, len, len, 0, NULL);
		gcol_fill(x0, y0, len, len, 1, NULL);
		return;
	}
	dec(H265_CTX_PRED_MODE, 0);
	/* part_mode: 2Nx2N, 2NxN, Nx2N, and the AMP modes when enabled above the minimum CU (no inter NxN) */
	int part = 0;
	{
		const int r = rn(100);
		if (r < 45) part = 0;
		else if (r < 65) part = 1;
		else if (r < 85) part = 2;
		else part = (C.amp && log2 > 3) ? 4 + rn(4) : 1 + rn(2);
		dec(H265_CTX_PART_MODE, part == 0);
		if (part) {
			const int horiz = part == 1 || part == 4 || part == 5;
			dec(H265_CTX_PART_MODE + 1, horiz);
			if (log2 > 3) {
				if (C.amp) {
					dec(H265_CTX_PART_MODE + 3, part < 4);
					if (part >= 4) byp(part & 1);
				}
			}
		}
	}
	if (dumpf) fprintf(dumpf, "icu %d %d l%d p%d\n", x0, y0, log2, part);
	int merged = 0;
	{
		const int hl = len >> 1, ql = len >> 2;
		switch (part) {
		case 0: merged = gpu(log2, ua, 0, x0, y0, len, len); break;
		case 1:
			gpu(log2, gav21[0][ua], 0, x0, y0, len, hl);
			gpu(log2, gav21[1][ua], 2, x0, y0 + hl, len, hl);
			break;
		case 2:
			gpu(log2, gav12[0][ua], 0, x0, y0, hl, len);
			gpu(log2, gav12[1][ua], 1, x0 + hl, y0, hl, len);
			break;
		case 4:
			gpu(log2, gav21[0][ua], 0, x0, y0, len, ql);
			gpu(log2, gav21[1][ua], 2, x0, y0 + ql, len, len - ql);
			break;
		case 5:
			gpu(log2, gav21[0][ua], 0, x0, y0, len, len - ql);
			gpu(log2, gav21[1][ua], 2, x0, y0 + len - ql, len, ql);
			break;
		case 6:
			gpu(log2, gav12[0][ua], 0, x0, y0, ql, len);
			gpu(log2, gav12[1][ua], 1, x0 + ql, y0, len - ql, len);
			break;
		default:
			gpu(log2, gav12[0][ua], 0, x0, y0, len - ql, len);
			gpu(log2, gav12[1][ua], 1, x0 + len - ql, y0, ql, len);
			break;
		}
	}
	int rqt = 1;
	if (!(part == 0 && merged)) {
		rqt = chance(C.rqt_pct);
		dec(H265_CTX_RQT_ROOT_CBF, rqt);
	}
	if (rqt) {
		intra_split = part != 0 && C.depth_inter == 0;
		transform_tree_inter(x0, y0, log2, 0, 3, 0);
	}
	gnb_rect(x0, y0, len, len, 3, NULL);
}

/* the slice's temporal state (colpics_t::init) */
static void inter_slice_setup(void)
{
	const int cl = col_l0 ^ 1;
	const int cf = ref_frm[cl][col_idx] & 7, cp = ref_poc[cl][col_idx];
	col_ref = gcol[cf];
	col_lists = (const int8_t(*)[16])reg_frame[cf];
	for (int i = 0; i < 8; ++i)
		for (int j = 0; j < 8; ++j) {
			colmv[i][j] = gscale(cur_poc, frame_poc[i], cp, frame_poc[j]);
			tmvs[i][j] = gscale(cur_poc, frame_poc[i], cur_poc, frame_poc[j]);
		}
	lowdelay = 1;
	for (int i = 0; i < 8; ++i)
		if (cur_poc < frame_poc[i]) lowdelay = 0;
	for (size_t i = 0; i < (size_t)W4 * (FH / 4); ++i) gnb[i] = nb_out;
}

static void quad_tree(int x0, int y0, int log2, int vx, int vy, int ua)
{
	if (vx <= 0 || vy <= 0) return;
	if (3 < log2) {
		int split = vx < (1 << log2) || vy < (1 << log2);
		if (!split) {
			const int l = x0 > 0 ? cb_log2[(size_t)(y0 >> 2) * W4 + (x0 >> 2) - 1] : 0;
			const int t = y0 > 0 ? cb_log2[(size_t)((y0 >> 2) - 1) * W4 + (x0 >> 2)] : 0;
			split = chance(C.split_pct + (log2 == 6 ? 30 : 0));
			dec(H265_CTX_SPLIT_CU + (l && l < log2) + (t && t < log2), split);
		}
		if (split) {
			const int h = 1 << (log2 - 1);
			quad_tree(x0, y0, log2 - 1, vx, vy, gav4[0][ua]);
			quad_tree(x0 + h, y0, log2 - 1, vx - h, vy < h ? vy : h, gav4[1][ua]);
			quad_tree(x0, y0 + h, log2 - 1, vx < 2 * h ? vx : 2 * h, vy - h, gav4[2][ua]);
			quad_tree(x0 + h, y0 + h, log2 - 1, (vx - h) < h ? vx - h : h, (vy - h) < h ? vy - h : h, 12);
			return;
		}
	}
	if (inter_pic) coding_unit_inter(x0, y0, log2, ua);
	else coding_unit(x0, y0, log2);
}

typedef struct {
	int type[3], band[3], eo[3], off[3][4];
} sao_t;

static void sao_ctu(sao_t *map, int cx, int cy)
{
	sao_t *s = &map[cy * cols + cx];
	memset(s, 0, sizeof(*s));
	if (!C.sao) return;
	if (cx > 0) {
		const int m = chance(25);
		dec(H265_CTX_SAO_MERGE, m);
		if (m) {
			*s = s[-1];
			return;
		}
	}
	if (cy > 0) {
		const int m = chance(25);
		dec(H265_CTX_SAO_MERGE, m);
		if (m) {
			*s = s[-cols];
			return;
		}
	}
	for (int ci = 0; ci < 3; ++ci) {
		int type = ci == 2 ? s->type[1] : rn(3);
		if (ci < 2) {
			dec(H265_CTX_SAO_TYPE, type != 0);
			if (type) byp(type == 2);
		}
		s->type[ci] = type;
		if (!type) continue;
		for (int j = 0; j < 4; ++j) {
			const int v = rn(8);
			s->off[ci][j] = v;
			for (int t = 0; t < v; ++t) byp(1);
			if (v < 7) byp(0);
		}
		if (type == 1) {
			for (int j = 0; j < 4; ++j)
				if (s->off[ci][j]) byp(chance(50));
			s->band[ci] = rn(32);
			bypn((uint32_t)s->band[ci], 5);
		} else if (ci < 2) {
			s->eo[ci] = rn(4);
			bypn((uint32_t)s->eo[ci], 2);
		}
	}
}

/* ------------------------------------------------------------------ headers */
static void nal(bw_t *out, int type, bw_t *rbsp)
{
	int zeros = 0;
	bw_byte(out, 0);
	bw_byte(out, 0);
	bw_byte(out, 0);
	bw_byte(out, 1);
	bw_byte(out, (uint8_t)(type << 1));
	bw_byte(out, 1); /* nuh_layer_id 0, nuh_temporal_id_plus1 1 */
	for (size_t i = 0; i < rbsp->n; ++i) {
		const uint8_t v = rbsp->b[i];
		if (zeros >= 2 && v <= 3) {
			bw_byte(out, 3);
			zeros = 0;
		}
		bw_byte(out, v);
		zeros = (v == 0) ? zeros + 1 : 0;
	}
}

static void ptl(bw_t *w)
{
	bw_bits(w, 1, 8);          /* general_profile_space 0, tier 0, profile_idc 1 (Main) */
	bw_bits(w, 0x60000000, 32); /* compatibility flags 1, 2 */
	bw_bits(w, 0x900000, 24);   /* progressive, frame-only ... + reserved */
	bw_bits(w, 0, 24);
	bw_bits(w, 120, 8);        /* level 4 */
}

static void write_vps(bw_t *out)
{
	bw_t w;
	bw_init(&w);
	bw_bits(&w, 0, 4);
	bw_bits(&w, 3, 2);
	bw_bits(&w, 0, 6);
	bw_bits(&w, 0, 3);
	bw_bit(&w, 1);
	bw_bits(&w, 0xffff, 16);
	ptl(&w);
	bw_bit(&w, 0); /* sub_layer_ordering_info_present */
	bw_ue(&w, 4);
	bw_ue(&w, 0);
	bw_ue(&w, 0);
	bw_bits(&w, 0, 6);
	bw_ue(&w, 0);
	bw_bit(&w, 0); /* timing */
	bw_bit(&w, 0); /* extension */
	bw_trailing(&w);
	nal(out, H265_VPS, &w);
	free(w.b);
}

/* --rps N (intra presets only): N short-term RPS sets in the SPS instead of 8, so the reference's motion-field
 * buffer count min(num_long_term_ref_pics_sps + num_short_term_ref_pic_sets, 8) is N */
static int g_rps_sets = 8;

static void write_sps(bw_t *out)
{
	bw_t w;
	bw_init(&w);
	bw_bits(&w, 0, 4);
	bw_bits(&w, 0, 3);
	bw_bit(&w, 1);
	ptl(&w);
	bw_ue(&w, 0); /* sps id */
	bw_ue(&w, 1); /* 4:2:0 */
	bw_ue(&w, (uint32_t)W);
	bw_ue(&w, (uint32_t)H);
	{
		const int cw = (FW - W) / 2, ch = (FH - H) / 2;
		(void)cw;
		(void)ch;
		bw_bit(&w, 0); /* conformance window: none (W, H are multiples of 8) */
	}
	bw_ue(&w, 0);
	bw_ue(&w, 0);
	bw_ue(&w, 4); /* log2_max_poc_lsb 8 */
	bw_bit(&w, 1);
	bw_ue(&w, 4);
	bw_ue(&w, 0);
	bw_ue(&w, 0);
	bw_ue(&w, 0);                             /* min cb 8 */
	bw_ue(&w, (uint32_t)(C.ctb_log2 - 3));    /* ctb */
	bw_ue(&w, 0);                             /* min tb 4 */
	bw_ue(&w, (uint32_t)(C.max_tb_log2 - 2)); /* max tb */
	bw_ue(&w, (uint32_t)(C.gop ? C.depth_inter : 1)); /* depth inter */
	bw_ue(&w, (uint32_t)C.depth_intra);
	bw_bit(&w, 0); /* scaling lists */
	bw_bit(&w, (uint32_t)C.amp);
	bw_bit(&w, (uint32_t)C.sao);
	bw_bit(&w, 0); /* pcm */
	/* 8 short-term RPS sets (I slices name set 0): the reference sizes its motion-field buffers by their
	 * count, min(num_long_term_ref_pics_sps + num_short_term_ref_pic_sets, 8) frames (h265.cpp:121-128) */
	bw_ue(&w, (uint32_t)g_rps_sets);
	for (int i = 0; i < g_rps_sets; ++i) {
		if (i) bw_bit(&w, 0); /* inter_ref_pic_set_prediction_flag */
		bw_ue(&w, (uint32_t)(1 + (i & 3)));
		bw_ue(&w, (uint32_t)(i >> 2));
		for (int k = 0; k < 1 + (i & 3); ++k) {
			bw_ue(&w, 0);
			bw_bit(&w, 1);
		}
		for (int k = 0; k < (i >> 2); ++k) {
			bw_ue(&w, 0);
			bw_bit(&w, 1);
		}
	}
	bw_bit(&w, 0); /* long-term */
	bw_bit(&w, (uint32_t)(C.gop != 0)); /* temporal mvp */
	bw_bit(&w, (uint32_t)C.strong);
	bw_bit(&w, 0); /* vui */
	bw_bit(&w, 0); /* extension */
	bw_trailing(&w);
	nal(out, H265_SPS, &w);
	free(w.b);
}

static void write_pps(bw_t *out)
{
	bw_t w;
	bw_init(&w);
	bw_ue(&w, 0);
	bw_ue(&w, 0);
	bw_bit(&w, 0);
	bw_bit(&w, 0);
	bw_bits(&w, 0, 3);
	bw_bit(&w, (uint32_t)C.sign_hiding);
	bw_bit(&w, (uint32_t)C.cabac_init); /* cabac_init_present */
	bw_ue(&w, 0);
	bw_ue(&w, 0);
	bw_se(&w, 0); /* init_qp 26 */
	bw_bit(&w, 0);
	bw_bit(&w, (uint32_t)C.tskip);
	bw_bit(&w, 0); /* cu_qp_delta */
	bw_se(&w, C.cb_off);
	bw_se(&w, C.cr_off);
	bw_bit(&w, 1); /* slice chroma qp offsets present */
	bw_bit(&w, 0);
	bw_bit(&w, 0);
	bw_bit(&w, 0);
	bw_bit(&w, 0); /* tiles */
	bw_bit(&w, 0); /* wpp */
	bw_bit(&w, 1); /* loop filter across slices */
	bw_bit(&w, 1); /* deblocking control */
	bw_bit(&w, 1); /* override enabled */
	bw_bit(&w, 0); /* pps disabled */
	bw_se(&w, 0);
	bw_se(&w, 0);
	bw_bit(&w, 0); /* scaling list data */
	bw_bit(&w, 0);
	bw_ue(&w, (uint32_t)(C.gop ? C.merge_level - 2 : 0));
	bw_bit(&w, 0);
	bw_bit(&w, 0);
	bw_trailing(&w);
	nal(out, H265_PPS, &w);
	free(w.b);
}

/* the picture structures (decode order: POC and slice type, 2 = I, 1 = P, 0 = B) */
static const int gop_poc[4][8] = {{0}, {0, 1, 2, 3, 4, 5, 6, 7}, {0, 4, 2, 1, 3, 8, 6, 5}, {0, 1, 2, 3, 4, 5, 6, 7}};
static const int gop_type[4][8] = {{2}, {2, 1, 1, 1, 1, 1, 1, 1}, {2, 1, 0, 0, 0, 1, 0, 0}, {2, 0, 0, 1, 2, 0, 0, 0}};

static void write_slice(bw_t *out, int idx)
{
	bw_t w;
	const int idr = idx == 0;
	const int type = C.gop ? gop_type[C.gop][idx] : 2, poc = C.gop ? gop_poc[C.gop][idx] : idx;
	bw_init(&w);
	bw_bit(&w, 1); /* first slice */
	if (idr) bw_bit(&w, 0); /* no_output_of_prior_pics */
	bw_ue(&w, 0);
	bw_ue(&w, (uint32_t)type);
	cur_slot = idx & 7; /* (P / B streams: at most 8 pictures, never output before the end: picture k in frame k) */
	cur_poc = poc;
	inter_pic = type < 2;
	bslice = type == 0;
	if (!idr) {
		bw_bits(&w, (uint32_t)(poc & 255), 8);
		if (!inter_pic) {
			/* the SPS RPS, index in log2ceil(n) bits (1 + floor(log2 n): 4 bits for the 8 sets, the reference's count,
			 * h265.cpp:757-759), none for a single set */
			bw_bit(&w, 1);
			if (g_rps_sets > 1) {
				int nb = 0;
				for (int n = g_rps_sets; n; n >>= 1) nb++;
				bw_bits(&w, 0, nb);
			}
		} else {
			/* every picture decoded so far, nearest first on each side, all used */
			int neg[8], pos[8], nn = 0, np = 0;
			for (int d = poc - 1; d >= 0; --d)
				for (int k = 0; k < idx; ++k)
					if (gop_poc[C.gop][k] == d && nn < 4) neg[nn++] = d;
			for (int d = poc + 1; d < 64; ++d)
				for (int k = 0; k < idx; ++k)
					if (gop_poc[C.gop][k] == d && np < 4) pos[np++] = d;
			bw_bit(&w, 0); /* short_term_ref_pic_set_sps_flag */
			bw_bit(&w, 0); /* inter_ref_pic_set_prediction_flag */
			bw_ue(&w, (uint32_t)nn);
			bw_ue(&w, (uint32_t)np);
			for (int k = 0, prev = poc; k < nn; prev = neg[k], ++k) {
				bw_ue(&w, (uint32_t)(prev - neg[k] - 1));
				bw_bit(&w, 1);
			}
			for (int k = 0, prev = poc; k < np; prev = pos[k], ++k) {
				bw_ue(&w, (uint32_t)(pos[k] - prev - 1));
				bw_bit(&w, 1);
			}
			/* init_ref_pic_list with every entry used: L0 = negatives then positives, L1 the other way */
			const int tot = nn + np;
			for (int lx = 0; lx < 2; ++lx)
				for (int k = 0; k < tot; ++k) {
					const int pc = lx == 0 ? (k < nn ? neg[k] : pos[k - nn]) : (k < np ? pos[k] : neg[k - np]);
					ref_poc[lx][k] = pc;
					for (int f = 0; f < idx; ++f)
						if (gop_poc[C.gop][f] == pc) ref_frm[lx][k] = (int8_t)f;
				}
			num_ref[0] = 1 + rn(tot < 15 ? tot : 15);
			if (bslice) num_ref[1] = 1 + rn(tot < 15 ? tot : 15);
		}
		if (C.gop) bw_bit(&w, 1); /* slice_temporal_mvp_enabled_flag */
	}
	frame_poc[cur_slot] = poc;
	if (C.sao) {
		bw_bit(&w, 1);
		bw_bit(&w, 1);
	}
	if (inter_pic) {
		bw_bit(&w, 1); /* num_ref_idx_active_override_flag */
		bw_ue(&w, (uint32_t)(num_ref[0] - 1));
		if (bslice) bw_ue(&w, (uint32_t)(num_ref[1] - 1));
		if (bslice) {
			mvd_l1_zero = rn(2);
			bw_bit(&w, (uint32_t)mvd_l1_zero);
		}
		if (C.cabac_init) {
			cabac_init_flag = rn(2);
			bw_bit(&w, (uint32_t)cabac_init_flag);
		}
		col_l0 = bslice ? rn(2) : 1;
		if (bslice) bw_bit(&w, (uint32_t)col_l0);
		if (num_ref[col_l0 ^ 1] > 1) { /* else collocated_ref_idx keeps the previous slice's value */
			col_idx = rn(num_ref[col_l0 ^ 1]);
			bw_ue(&w, (uint32_t)col_idx);
		}
		max_merge = C.max_merge - rn(2);
		if (max_merge < 1) max_merge = 1;
		bw_ue(&w, (uint32_t)(5 - max_merge));
	}
	/* every slice registers its (possibly stale) lists for the frame (colpics_t::init) */
	memcpy(reg_frame[cur_slot][0], ref_frm[0], 16);
	memcpy(reg_frame[cur_slot][1], ref_frm[1], 16);
	bw_se(&w, C.qp - 26);
	bw_se(&w, C.slice_cb);
	bw_se(&w, C.slice_cr);
	bw_bit(&w, 1); /* deblocking override */
	bw_bit(&w, (uint32_t)!C.deblock);
	if (C.deblock) {
		bw_se(&w, C.beta / 2);
		bw_se(&w, C.tc / 2);
	}
	if (C.sao || C.deblock) bw_bit(&w, 1); /* slice_loop_filter_across_slices */
	/* byte_alignment */
	bw_bit(&w, 1);
	while (!bw_aligned(&w)) bw_bit(&w, 0);
	/* slice data */
	cenc_start(&E, &w);
	ctx_init(C.qp, inter_pic ? 2 - (type ^ cabac_init_flag) : 0);
	memset(cb_log2, 0, (size_t)W4 * (FH / 4));
	memset(ipm, 1, (size_t)W4 * (FH / 4));
	if (inter_pic) inter_slice_setup();
	else if (gcol[cur_slot])
		for (size_t i = 0; i < (size_t)gcol_stride * (size_t)((H + 15) >> 4); ++i) gcol[cur_slot][i].intra = 1;
	{
		sao_t *map = (sao_t *)calloc((size_t)(cols * rows), sizeof(sao_t));
		for (int cy = 0; cy < rows; ++cy)
			for (int cx = 0; cx < cols; ++cx) {
				const int x0 = cx * CTB, y0 = cy * CTB;
				sao_ctu(map, cx, cy);
				quad_tree(x0, y0, C.ctb_log2, W - x0, (H - y0) < CTB ? H - y0 : CTB, (cy == 0 ? 10 : 0) | (cx == 0 ? 5 : 0) | 4);
				if (cx != cols - 1 || cy != rows - 1) cenc_terminate(&E, 0);
			}
		free(map);
	}
	cenc_terminate(&E, 1); /* end_of_slice_segment_flag (flush; its last bit is rbsp_stop_one_bit) */
	while (!bw_aligned(&w)) bw_bit(&w, 0);
	nal(out, idr ? H265_IDR_W_RADL : H265_TRAIL_R, &w);
	if (C.gop && idx + 1 > 8) fprintf(stderr, "h265gen: more than 8 pictures\n");
	free(w.b);
}

int main(int argc, char **argv)
{
	const char *preset = "cov_h265_a", *outp = NULL;
	int seed = 1, frames = -1;
	for (int i = 1; i < argc; ++i) {
		if (!strcmp(argv[i], "--preset") && i + 1 < argc) preset = argv[++i];
		else if (!strcmp(argv[i], "--seed") && i + 1 < argc) seed = atoi(argv[++i]);
		else if (!strcmp(argv[i], "--frames") && i + 1 < argc) frames = atoi(argv[++i]);
		else if (!strcmp(argv[i], "-o") && i + 1 < argc) outp = argv[++i];
		else if (!strcmp(argv[i], "--dump") && i + 1 < argc) dumpf = fopen(argv[++i], "w");
		else if (!strcmp(argv[i], "--rps") && i + 1 < argc) g_rps_sets = atoi(argv[++i]);
	}
	{
		int found = 0;
		for (int i = 0; presets[i].name; ++i)
			if (!strcmp(presets[i].name, preset)) {
				C = presets[i];
				found = 1;
			}
		if (!found || !outp) {
			fprintf(stderr, "usage: h265gen --preset NAME --seed S [--frames N] -o out.265\n");
			return 2;
		}
	}
	if (frames > 0) C.frames = frames;
	if (g_rps_sets < 1 || g_rps_sets > 8 || (C.gop && g_rps_sets != 8)) {
		fprintf(stderr, "h265gen: --rps 1..8, and only for intra presets\n");
		return 2;
	}
	rs = 0x9E3779B97F4A7C15ull ^ ((uint64_t)seed * 0x100000001B3ull);
	build_scans();
	W = C.w;
	H = C.h;
	CTB = 1 << C.ctb_log2;
	cols = (W + CTB - 1) / CTB;
	rows = (H + CTB - 1) / CTB;
	FW = cols * CTB;
	FH = rows * CTB;
	W4 = FW / 4;
	cb_log2 = (uint8_t *)malloc((size_t)W4 * (FH / 4));
	ipm = (uint8_t *)malloc((size_t)W4 * (FH / 4));
	gnb = (gnb_t *)malloc(sizeof(gnb_t) * (size_t)W4 * (FH / 4));
	gcol_stride = (W + 15) >> 4;
	for (int i = 0; i < 8; ++i) gcol[i] = (gcol_t *)calloc((size_t)gcol_stride * (size_t)((H + 15) >> 4), sizeof(gcol_t));
	if (C.gop && C.frames > 8) C.frames = 8;
	bw_t out;
	bw_init(&out);
	write_vps(&out);
	write_sps(&out);
	write_pps(&out);
	for (int f = 0; f < C.frames; ++f) {
		if (dumpf) fprintf(dumpf, "pic %d\n", f);
		write_slice(&out, f);
	}
	FILE *fo = fopen(outp, "wb");
	if (!fo) return 1;
	fwrite(out.b, 1, out.n, fo);
	fclose(fo);
	if (dumpf) fclose(dumpf);
	return 0;
}
