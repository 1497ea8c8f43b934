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
	{NULL, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
};

static cfg_t C;
static FILE *dumpf;

/* ------------------------------------------------------------------ CABAC encoder on the H.265 contexts */
static cenc_t E;

static void ctx_init(int qp)
{
	const int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
	for (int i = 0; i < H265_NUM_CTX; ++i) {
		int pre = ((h265_cabac_init_mn[0][i][0] * q) >> 4) + h265_cabac_init_mn[0][i][1];
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

static void quad_tree(int x0, int y0, int log2, int vx, int vy)
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
			quad_tree(x0, y0, log2 - 1, vx, vy);
			quad_tree(x0 + h, y0, log2 - 1, vx - h, vy < h ? vy : h);
			quad_tree(x0, y0 + h, log2 - 1, vx < 2 * h ? vx : 2 * h, vy - h);
			quad_tree(x0 + h, y0 + h, log2 - 1, (vx - h) < h ? vx - h : h, (vy - h) < h ? vy - h : h);
			return;
		}
	}
	coding_unit(x0, y0, log2);
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
	bw_ue(&w, 1);                             /* depth inter */
	bw_ue(&w, (uint32_t)C.depth_intra);
	bw_bit(&w, 0); /* scaling lists */
	bw_bit(&w, 0); /* amp */
	bw_bit(&w, (uint32_t)C.sao);
	bw_bit(&w, 0); /* pcm */
	bw_ue(&w, 1);  /* one short-term RPS: {-1} */
	bw_ue(&w, 1);
	bw_ue(&w, 0);
	bw_ue(&w, 0);
	bw_bit(&w, 1);
	bw_bit(&w, 0); /* long-term */
	bw_bit(&w, 0); /* temporal mvp */
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
	bw_bit(&w, 0);
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
	bw_ue(&w, 0);
	bw_bit(&w, 0);
	bw_bit(&w, 0);
	bw_trailing(&w);
	nal(out, H265_PPS, &w);
	free(w.b);
}

static void write_slice(bw_t *out, int idx)
{
	bw_t w;
	const int idr = idx == 0;
	bw_init(&w);
	bw_bit(&w, 1); /* first slice */
	if (idr) bw_bit(&w, 0); /* no_output_of_prior_pics */
	bw_ue(&w, 0);
	bw_ue(&w, 2); /* I */
	if (!idr) {
		bw_bits(&w, (uint32_t)(idx & 255), 8);
		bw_bit(&w, 1); /* the SPS RPS */
	}
	if (C.sao) {
		bw_bit(&w, 1);
		bw_bit(&w, 1);
	}
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
	ctx_init(C.qp);
	memset(cb_log2, 0, (size_t)W4 * (FH / 4));
	memset(ipm, 1, (size_t)W4 * (FH / 4));
	{
		sao_t *map = (sao_t *)calloc((size_t)(cols * rows), sizeof(sao_t));
		for (int cy = 0; cy < rows; ++cy)
			for (int cx = 0; cx < cols; ++cx) {
				const int x0 = cx * CTB, y0 = cy * CTB;
				sao_ctu(map, cx, cy);
				quad_tree(x0, y0, C.ctb_log2, W - x0, (H - y0) < CTB ? H - y0 : CTB);
				if (cx != cols - 1 || cy != rows - 1) cenc_terminate(&E, 0);
			}
		free(map);
	}
	cenc_terminate(&E, 1); /* end_of_slice_segment_flag (flush; its last bit is rbsp_stop_one_bit) */
	while (!bw_aligned(&w)) bw_bit(&w, 0);
	nal(out, idr ? H265_IDR_W_RADL : H265_TRAIL_R, &w);
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
