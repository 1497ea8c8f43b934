/*
 * m2vgen — deterministic synthetic MPEG-1/2 video elementary streams of intra pictures for the C1
 * config (MPEG-2 MP@ML 720x480, 4:2:0, I-only, 30 frames, fixed quantiser scale,
 * intra_dc_precision 0, procedural textures) and for coverage streams of the intra tools the
 * reference decodes (mpeg2.cpp): both DCT tables, alternate scan, linear / non-linear quantiser
 * scale, intra_dc_precision 0-3, frame / field DCT, per-MB quantiser changes, loaded quantiser
 * matrices (sequence header and quant matrix extension), escape codes, slices starting mid-row,
 * missing slices, MPEG-1 syntax (8/16-bit escapes, oddification).
 *
 * P / B coverage (presets *_pb): coded order I P B B P B B ..., every macroblock type of Tables B.3 /
 * B.4 (with / without MC, coded / not coded, quantiser changes, intra), skipped macroblocks (P: copies,
 * B: the last vectors repeated), frame / field / dual-prime motion types, field DCT, f_codes 1-4, motion
 * vectors against the decoder's predictors (kept inside the reference frames: the reference does not
 * bound its reads), non-intra quantiser matrices, lost slices.
 *
 *   m2vgen --preset c1|c1_pb|cov_m2v|cov_m2v_slices|cov_mpeg1|cov_m2v_pb|cov_m2v_pb_field|cov_mpeg1_pb
 *          [--seed N] [--frames N] [--size WxH] -o out.m2v
 *
 * Encoding: floating-point forward DCT of procedural 8x8 blocks, quantised to the levels the
 * decoder's dequantiser expects; codes from the VLC lists of m2dec_amd/csrc/host/mpeg2_tables.c.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../h264gen/bitwriter.h"
#include "mpeg2_dec.h"

typedef struct {
	int w, h, frames, mpeg2;
	int qscale_code;          /* fixed quantiser_scale_code (c1) */
	int vary;                 /* coverage: random tools per picture / MB */
	int slices_midrow;        /* slices that start inside a MB row */
	int drop_slice;           /* leave out one slice row now and then (lost-slice copy) */
	int intra_vlc_format, dc_precision;
	uint64_t seed;
	int pb;                   /* I P B B P B B ... (coded order) */
	int field_mc;             /* P / B pictures with frame_pred_frame_dct 0 (field / dual-prime MC, field DCT) */
} params_t;

static uint64_t rng_s;
static uint32_t rnd(void)
{
	rng_s ^= rng_s << 13;
	rng_s ^= rng_s >> 7;
	rng_s ^= rng_s << 17;
	return (uint32_t)(rng_s >> 11);
}
static int rnd_n(int n) { return (int)(rnd() % (uint32_t)n); }

static void put_code(bw_t *w, const char *c)
{
	for (; *c; ++c) bw_bit(w, *c == '1');
}

static const char *find_code(const m2v_code_t *t, int v)
{
	for (; t->code; ++t)
		if (t->value == v) return t->code;
	return NULL;
}

/* codes of table zero / one by (run, level); NULL: escape */
static const char *dct_code(int table, int run, int level)
{
	if (table) {
		for (const m2v_dct_code_t *t = m2v_dct1; t->code; ++t)
			if (t->run == run && t->level == level) return t->code;
		for (const m2v_dct_code_t *t = m2v_dct0; t->code; ++t)
			if (strlen(t->code) >= 14 && t->run == run && t->level == level) return t->code;
		return NULL;
	}
	for (const m2v_dct_code_t *t = m2v_dct0; t->code; ++t)
		if (t->run == run && t->level == level) return t->code;
	return NULL;
}

static void start_code(bw_t *w, int code)
{
	while (w->na) bw_bit(w, 0);
	bw_byte(w, 0);
	bw_byte(w, 0);
	bw_byte(w, 1);
	bw_byte(w, (uint8_t)code);
}

/* ---------------------------------------------------------------- picture content */
static double sample(int comp, int x, int y, int t, int seed)
{
	/* moving gradients, rings, checker patches and noise: low and high frequencies everywhere */
	const double fx = x / 37.0 + 0.13 * t + 0.7 * comp + seed * 0.011, fy = y / 23.0 - 0.07 * t;
	double v = 128 + 60 * sin(fx) * cos(fy) + 30 * sin((x * x + y * y) / (900.0 + 40 * comp) + 0.2 * t);
	if (((x >> 5) + (y >> 5) + t) % 7 == 0) v += ((x >> 2) ^ (y >> 2)) & 1 ? 40 : -40;
	v += (int)(rnd() % 9) - 4;
	return v < 0 ? 0 : v > 255 ? 255 : v;
}

static void fdct8(const double in[64], double out[64])
{
	for (int u = 0; u < 8; ++u)
		for (int v = 0; v < 8; ++v) {
			double s = 0;
			for (int x = 0; x < 8; ++x)
				for (int y = 0; y < 8; ++y)
					s += in[y * 8 + x] * cos((2 * x + 1) * u * M_PI / 16) * cos((2 * y + 1) * v * M_PI / 16);
			const double cu = u ? 1 : M_SQRT1_2, cv = v ? 1 : M_SQRT1_2;
			out[v * 8 + u] = 0.25 * cu * cv * s;
		}
}

typedef struct {
	int intra_vlc_format, alternate_scan, q_scale_type, dc_precision, frame_pred_frame_dct;
	const uint8_t *qmat;       /* intra matrix (raster) */
	int qcode;
	int16_t dc_pred[3];
	int mpeg2;
} enc_t;

static void put_dc(bw_t *w, int cc, int diff)
{
	int size = 0, a = abs(diff);
	while (a >> size) size++;
	put_code(w, find_code(cc ? m2v_dc_chroma : m2v_dc_luma, size));
	if (size) bw_bits(w, (uint32_t)(diff > 0 ? diff : diff + (1 << size) - 1), size);
}

static void put_block(bw_t *w, enc_t *e, const double pix[64], int cc, int force_escape)
{
	double F[64];
	const int qs = m2v_q_scale[e->q_scale_type][e->qcode];
	const uint8_t *scan = m2v_scan[e->alternate_scan];
	const int maxl = e->mpeg2 ? 2047 : 255;
	int dc, run = 0;
	fdct8(pix, F);
	/* DC: F[0] = 8 * mean; dc_level in units of 2^(3 - precision) */
	dc = (int)lrint(F[0] / (1 << (3 - e->dc_precision)));
	{
		const int mx = (1 << (8 + e->dc_precision)) - 1;
		dc = dc < 0 ? 0 : dc > mx ? mx : dc;
	}
	put_dc(w, cc, dc - e->dc_pred[cc]);
	e->dc_pred[cc] = (int16_t)dc;
	for (int i = 1; i < 64; ++i) {
		const int z = scan[i];
		const double q = e->qmat[z] * qs / 16.0;
		int l = (int)lrint(F[z] / q);
		if (l > maxl) l = maxl;
		if (l < -maxl) l = -maxl;
		if (!l) {
			run++;
			continue;
		}
		{
			const char *c = force_escape ? NULL : dct_code(e->intra_vlc_format, run, abs(l));
			if (c) {
				put_code(w, c);
				bw_bit(w, l < 0);
			} else {
				put_code(w, "000001");
				bw_bits(w, (uint32_t)run, 6);
				if (e->mpeg2) {
					bw_bits(w, (uint32_t)l & 0xfff, 12);
				} else if (abs(l) < 128) {
					bw_bits(w, (uint32_t)l & 0xff, 8);
				} else if (l > 0) {
					bw_bits(w, 0x00, 8);
					bw_bits(w, (uint32_t)l, 8);
				} else {
					bw_bits(w, 0x80, 8);
					bw_bits(w, (uint32_t)(l + 256), 8);
				}
			}
		}
		run = 0;
	}
	put_code(w, e->intra_vlc_format ? "0110" : "10");
}

static void put_mb(bw_t *w, enc_t *e, int mbx, int mby, int t, int seed, int quant, int dct_type, int force_escape)
{
	double blk[64];
	put_code(w, quant ? "01" : "1");
	if (!e->frame_pred_frame_dct && e->mpeg2) bw_bit(w, dct_type);
	if (quant) bw_bits(w, (uint32_t)e->qcode, 5);
	for (int b = 0; b < 4; ++b) {
		for (int y = 0; y < 8; ++y)
			for (int x = 0; x < 8; ++x) {
				const int px = mbx * 16 + (b & 1) * 8 + x;
				const int py = dct_type ? mby * 16 + (b >> 1) + 2 * y : mby * 16 + (b >> 1) * 8 + y;
				blk[y * 8 + x] = sample(0, px, py, t, seed);
			}
		put_block(w, e, blk, 0, force_escape);
	}
	for (int c = 0; c < 2; ++c) {
		for (int y = 0; y < 8; ++y)
			for (int x = 0; x < 8; ++x) blk[y * 8 + x] = sample(1 + c, mbx * 8 + x, mby * 8 + y, t, seed);
		put_block(w, e, blk, 1 + c, force_escape);
	}
}

static void put_qmat(bw_t *w, const uint8_t *q, const uint8_t *scan)
{
	for (int i = 0; i < 64; ++i) bw_bits(w, q[scan[i]], 8);
}

/* ---------------------------------------------------------------- P / B pictures */
/* the decoder state the syntax depends on (mpeg2.cpp m2d_mb_current: mv predictors, type of the last
 * coded MB, intra DC predictors), mirrored so that every vector lands where the generator wants it */
typedef struct {
	int16_t pmv[2][2][2];
	int prev_type;            /* M2V_MBF_* of the last coded MB (persists over slices and pictures) */
	int ctype;                /* 2 P, 3 B */
	int r_size[2][2];
	int frame_mode;           /* 3: frame_pred_frame_dct, 1: frame picture with field MC / DCT choices */
	int w, h;                 /* frame (multiple of 16) */
	int vary;
} pbstate_t;

static pbstate_t g_pb;

static void pb_reset_mv(void) { memset(g_pb.pmv, 0, sizeof(g_pb.pmv)); }

static void enc_reset_dc(enc_t *e)
{
	e->dc_pred[0] = e->dc_pred[1] = e->dc_pred[2] = (int16_t)(1 << (7 + e->dc_precision));
}

/* is a 16 x 16 prediction with vector (mvx, mvy) (half samples) of the MB at (mbx, mby) inside the
 * frame?  field: one field's 16 x 8 lines (vertical vector in field lines) */
static int mv_inside(int mbx, int mby, int mvx, int mvy, int field)
{
	const int W = g_pb.w, H = field ? g_pb.h / 2 : g_pb.h, lh = field ? 8 : 16, ch = field ? 4 : 8;
	const int x = mbx * 16 + (mvx >> 1), y = mby * lh + (mvy >> 1);
	const int cx = mvx / 2, cy = mvy / 2;
	const int xc = mbx * 16 + 2 * (cx >> 1), yc = mby * ch + (cy >> 1);
	if (x < 0 || y < 0 || x + 16 + (mvx & 1) > W || y + lh + (mvy & 1) > H) return 0;
	if (xc < 0 || yc < 0 || xc + 16 + 2 * (cx & 1) > W || yc + ch + (cy & 1) > H / 2) return 0;
	return 1;
}

/* one vector component: `mv` against the predictor *pmv (stored << is_field), as m2d_one_mv decodes */
static void put_one_mv(bw_t *w, int16_t *pmv, int mv, int r_size, int is_field)
{
	const int limit = 16 << r_size;
	int delta = mv - (*pmv >> is_field);
	if (delta < -limit) delta += 2 * limit;
	if (delta >= limit) delta -= 2 * limit;
	if (!delta) {
		bw_bit(w, 1);
	} else {
		const int a = abs(delta) - 1;
		put_code(w, find_code(m2v_motion_code, (a >> r_size) + 1));
		bw_bit(w, delta < 0);
		if (r_size) bw_bits(w, (uint32_t)(a & ((1 << r_size) - 1)), r_size);
	}
	*pmv = (int16_t)(mv << is_field);
}

/* a random vector component in [-limit, limit) biased to small values */
static int rnd_mv(int r_size)
{
	const int limit = 16 << r_size;
	const int k = rnd_n(4);
	int v = k == 0 ? 0 : k == 1 ? rnd_n(9) - 4 : rnd_n(2 * limit) - limit;
	return v;
}

/* motion vectors of direction s for motion type mt (2 frame, 1 field, 3 dual prime) of the MB at
 * (mbx, mby), chosen inside the frame */
static void put_mvs(bw_t *w, int s, int mt, int mbx, int mby)
{
	const int *rs = g_pb.r_size[s];
	if (mt == 1) {
		for (int i = 0; i < 2; ++i) {
			int vx = 0, vy = 0;
			for (int tries = 0; tries < 16; ++tries) {
				vx = rnd_mv(rs[0]);
				vy = rnd_mv(rs[1]);
				if (mv_inside(mbx, mby, vx, vy, 1)) break;
				vx = vy = 0;
			}
			bw_bit(w, rnd_n(2)); /* motion_vertical_field_select */
			put_one_mv(w, &g_pb.pmv[s][i][0], vx, rs[0], 0);
			put_one_mv(w, &g_pb.pmv[s][i][1], vy, rs[1], 1);
		}
		return;
	}
	{
		int vx = 0, vy = 0;
		for (int tries = 0; tries < 16; ++tries) {
			vx = rnd_mv(rs[0]);
			vy = rnd_mv(rs[1]);
			if (mv_inside(mbx, mby, vx, vy, 0)) break;
			vx = vy = 0;
		}
		put_one_mv(w, &g_pb.pmv[s][0][0], vx, rs[0], 0);
		if (mt == 3) { /* dmvector: 0, or 1 s */
			const int d = rnd_n(3);
			bw_bit(w, d != 0);
			if (d) bw_bit(w, d == 2);
		}
		/* dual prime: the vertical component is parsed as a field vector (the reference then predicts
		 * a frame with it) */
		put_one_mv(w, &g_pb.pmv[s][0][1], vy, rs[1], mt == 3);
		if (mt == 3) {
			const int d = rnd_n(3);
			bw_bit(w, d != 0);
			if (d) bw_bit(w, d == 2);
		}
		g_pb.pmv[s][1][0] = g_pb.pmv[s][0][0];
		g_pb.pmv[s][1][1] = g_pb.pmv[s][0][1];
	}
}

/* a non-intra block: a few small coefficients (table B.14; a first coefficient of run 0 / level 1 as
 * "1s"), sometimes escaped, then end of block */
static void put_inter_block(bw_t *w, enc_t *e, int force_escape)
{
	const int n = 1 + rnd_n(3);
	int idx = -1;
	for (int k = 0; k < n; ++k) {
		const int run = rnd_n(k ? 8 : 4);
		const int level = 1 + (rnd_n(4) == 0);
		const int neg = rnd_n(2);
		if (idx + 1 + run >= 64) break;
		idx += 1 + run;
		if (k == 0 && run == 0 && level == 1) {
			bw_bit(w, 1);
			bw_bit(w, neg);
			continue;
		}
		{
			const char *c = (force_escape && rnd_n(2)) ? NULL : dct_code(0, run, level);
			const int l = neg ? -level : level;
			if (c) {
				put_code(w, c);
				bw_bit(w, neg);
			} else {
				put_code(w, "000001");
				bw_bits(w, (uint32_t)run, 6);
				if (e->mpeg2) bw_bits(w, (uint32_t)l & 0xfff, 12);
				else bw_bits(w, (uint32_t)l & 0xff, 8);
			}
		}
	}
	put_code(w, "10");
}

/* the B-skip prediction of the MB at (mbx, mby) (m2d_skip_mb_B: the last MB's directions, frame MC with
 * the first predictor of each) stays inside the frame */
static int b_skip_ok(int mbx, int mby)
{
	const int dir = g_pb.prev_type & (M2V_MBF_FWD | M2V_MBF_BWD);
	const int bi = dir == (M2V_MBF_FWD | M2V_MBF_BWD);
	const int one = bi ? 0 : (dir >> 1);
	for (int s = 0; s < 2; ++s) {
		if (!bi && s != one) continue;
		if (!mv_inside(mbx, mby, g_pb.pmv[s][0][0], g_pb.pmv[s][0][1], 0)) return 0;
	}
	return 1;
}

/* one coded macroblock of a P / B picture (6.2.5 order: type, motion type, dct_type, quantiser,
 * vectors, coded_block_pattern, blocks) */
static void put_pb_mb(bw_t *w, enc_t *e, int mbx, int mby, int t, int seed, int mpeg2)
{
	int type;
	if (g_pb.ctype == 2) {
		static const int tp[] = {9, 9, 9, 8, 1, 1, 4, 25, 24, 20};
		type = tp[rnd_n(10)];
	} else {
		static const int tb[] = {3, 11, 11, 2, 10, 10, 1, 9, 9, 4, 27, 25, 26, 20};
		type = tb[rnd_n(14)];
	}
	put_code(w, find_code(g_pb.ctype == 2 ? m2v_mb_type_p : m2v_mb_type_b, type));
	{
		const int prev_intra = (g_pb.prev_type & M2V_MBF_INTRA) != 0;
		const int mc = type & (M2V_MBF_FWD | M2V_MBF_BWD);
		int mt = 2;
		g_pb.prev_type = type;
		if (mc && g_pb.frame_mode == 1) {
			const int k = rnd_n(g_pb.ctype == 2 ? 7 : 5);
			mt = k < 3 ? 2 : k < 5 ? 1 : 3; /* (dual prime in P pictures only) */
			bw_bits(w, (uint32_t)mt, 2);
		}
		if (g_pb.frame_mode == 1 && (type & (M2V_MBF_INTRA | M2V_MBF_PATTERN))) bw_bit(w, rnd_n(2)); /* dct_type */
		if (type & M2V_MBF_QUANT) {
			e->qcode = 1 + rnd_n(20);
			bw_bits(w, (uint32_t)e->qcode, 5);
		}
		if (type & M2V_MBF_INTRA) {
			double blk[64];
			if (!prev_intra) enc_reset_dc(e);
			for (int b = 0; b < 4; ++b) {
				for (int y = 0; y < 8; ++y)
					for (int x = 0; x < 8; ++x) blk[y * 8 + x] = sample(0, mbx * 16 + (b & 1) * 8 + x, mby * 16 + (b >> 1) * 8 + y, t, seed);
				put_block(w, e, blk, 0, rnd_n(16) == 0);
			}
			for (int c = 0; c < 2; ++c) {
				for (int y = 0; y < 8; ++y)
					for (int x = 0; x < 8; ++x) blk[y * 8 + x] = sample(1 + c, mbx * 8 + x, mby * 8 + y, t, seed);
				put_block(w, e, blk, 1 + c, rnd_n(16) == 0);
			}
			return;
		}
		if (prev_intra) pb_reset_mv();
		if (mc) {
			if (type & M2V_MBF_FWD) put_mvs(w, 0, mt, mbx, mby);
			if (type & M2V_MBF_BWD) put_mvs(w, 1, mt, mbx, mby);
		} else { /* P "no MC": the co-located MB, predictors reset */
			pb_reset_mv();
			enc_reset_dc(e);
		}
		if (type & M2V_MBF_PATTERN) {
			const int cbp = 1 + rnd_n(63);
			put_code(w, find_code(m2v_cbp, cbp));
			for (int i = 0; i < 6; ++i)
				if (cbp & (1 << (5 - i))) put_inter_block(w, e, rnd_n(12) == 0);
		}
		(void)mpeg2;
	}
}

/* the slices of a P / B picture: one per MB row (a row left out now and then); macroblocks inside a
 * slice skipped at random where the syntax and the in-frame rule allow */
static void put_pb_slices(bw_t *w, enc_t *e, int mbw, int mbh, int t, int seed, int drop_row)
{
	for (int y = 0; y < mbh; ++y) {
		int skip = 0;
		if (y == drop_row) continue;
		start_code(w, y + 1);
		bw_bits(w, (uint32_t)e->qcode, 5);
		bw_bit(w, 0);
		enc_reset_dc(e);
		pb_reset_mv();
		for (int x = 0; x < mbw; ++x) {
			if (x > 0 && x < mbw - 1 && rnd_n(5) == 0 && (g_pb.ctype == 2 || b_skip_ok(x, y))) {
				skip++;
				continue;
			}
			if (skip && g_pb.ctype == 2) { /* m2d_skip_mb_P: predictors reset after the copies */
				pb_reset_mv();
				enc_reset_dc(e);
			}
			{
				int inc = skip + 1;
				while (inc > 33) {
					put_code(w, "00000001000");
					inc -= 33;
				}
				put_code(w, find_code(m2v_mb_inc, inc));
			}
			skip = 0;
			put_pb_mb(w, e, x, y, t, seed, e->mpeg2);
		}
	}
}

int main(int argc, char **argv)
{
	params_t p = {720, 480, 30, 1, 8, 0, 0, 0, 1, 0, 1, 0, 0};
	const char *out = NULL, *preset = "c1";
	for (int i = 1; i < argc; ++i) {
		if (!strcmp(argv[i], "--preset") && i + 1 < argc) preset = argv[++i];
		else if (!strcmp(argv[i], "--seed") && i + 1 < argc) p.seed = strtoull(argv[++i], NULL, 0);
		else if (!strcmp(argv[i], "--frames") && i + 1 < argc) p.frames = -atoi(argv[++i]); /* applied after the preset */
		else if (!strcmp(argv[i], "--size") && i + 1 < argc) {
			if (sscanf(argv[++i], "%dx%d", &p.w, &p.h) != 2) return 2;
			p.w = -p.w;
		} else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
		else {
			fprintf(stderr, "usage: m2vgen --preset c1|c1_pb|cov_m2v|cov_m2v_slices|cov_mpeg1|cov_m2v_pb|cov_m2v_pb_field|cov_mpeg1_pb [--seed N] [--frames N] [--size WxH] -o out.m2v\n");
			return 2;
		}
	}
	{
		const int fr = p.frames < 0 ? -p.frames : 0, sw = p.w < 0 ? -p.w : 0, sh = p.h;
		if (!strcmp(preset, "c1")) {
			p.w = 720, p.h = 480, p.frames = 30, p.mpeg2 = 1, p.qscale_code = 8, p.vary = 0;
			p.intra_vlc_format = 1, p.dc_precision = 0;
		} else if (!strcmp(preset, "cov_m2v") || !strcmp(preset, "cov_m2v_slices")) {
			p.w = 176, p.h = 144, p.frames = 8, p.mpeg2 = 1, p.vary = 1;
			p.slices_midrow = p.drop_slice = !strcmp(preset, "cov_m2v_slices");
		} else if (!strcmp(preset, "cov_mpeg1")) {
			p.w = 176, p.h = 144, p.frames = 6, p.mpeg2 = 0, p.vary = 1;
		} else if (!strcmp(preset, "c1_pb")) { /* C1's geometry with P / B pictures (GPU reconstruction bench) */
			p.w = 720, p.h = 480, p.frames = 30, p.mpeg2 = 1, p.qscale_code = 8, p.vary = 0, p.pb = 1;
			p.intra_vlc_format = 1, p.dc_precision = 0;
		} else if (!strcmp(preset, "cov_m2v_pb") || !strcmp(preset, "cov_m2v_pb_field")) {
			p.w = 176, p.h = 144, p.frames = 10, p.mpeg2 = 1, p.vary = 1, p.pb = 1, p.drop_slice = 1;
			p.field_mc = !strcmp(preset, "cov_m2v_pb_field");
		} else if (!strcmp(preset, "cov_mpeg1_pb")) {
			p.w = 176, p.h = 144, p.frames = 10, p.mpeg2 = 0, p.vary = 1, p.pb = 1;
		} else {
			fprintf(stderr, "m2vgen: unknown preset %s\n", preset);
			return 2;
		}
		if (fr) p.frames = fr;
		if (sw) p.w = sw, p.h = sh;
	}
	if (!out || (p.w & 15) || (p.h & 15)) return 2;
	rng_s = 0x9e3779b97f4a7c15ull ^ (p.seed * 0x2545f4914f6cdd1dull + 1);
	bw_t w;
	bw_init(&w);
	const int mbw = p.w / 16, mbh = p.h / 16;
	uint8_t seq_intra[64];
	int seq_loaded = p.vary && rnd_n(2);
	for (int i = 0; i < 64; ++i) seq_intra[i] = (uint8_t)(i ? 8 + rnd_n(40) : 8);
	/* the decoder's intra matrix: set by a sequence header, replaced by a quant matrix extension until
	 * the next sequence header (mpeg2.cpp:258-266, 381-403) */
	static uint8_t ext_intra[64];
	const uint8_t *cur_qmat = m2v_default_intra_qmat;
	g_pb.w = p.w;
	g_pb.h = p.h;
	g_pb.vary = p.vary;
	for (int t = 0; t < p.frames; ++t) {
		enc_t e;
		/* coded order I P B B P B B ... (an I picture every 9 in the coverage streams) */
		const int ctype = !p.pb || t == 0 || (p.vary && t % 9 == 0) ? 1 : (t % 3 == 1 ? 2 : 3);
		memset(&e, 0, sizeof(e));
		e.mpeg2 = p.mpeg2;
		if (t == 0 || (p.vary && t % 3 == 0)) {
			/* sequence header (+ extension): 6.2.2.1, 6.2.2.3 */
			start_code(&w, 0xb3);
			bw_bits(&w, (uint32_t)p.w, 12);
			bw_bits(&w, (uint32_t)p.h, 12);
			bw_bits(&w, 2, 4);      /* aspect 4:3 */
			bw_bits(&w, 4, 4);      /* 29.97 Hz */
			bw_bits(&w, 20000, 18); /* bit rate / 400 */
			bw_bit(&w, 1);
			bw_bits(&w, 112, 10);   /* vbv_buffer_size */
			bw_bit(&w, 0);
			bw_bit(&w, seq_loaded);
			if (seq_loaded) put_qmat(&w, seq_intra, m2v_scan[0]);
			cur_qmat = seq_loaded ? seq_intra : m2v_default_intra_qmat;
			if (p.pb && p.vary && rnd_n(2)) { /* a non-intra matrix */
				uint8_t ni[64];
				for (int i = 0; i < 64; ++i) ni[i] = (uint8_t)(8 + rnd_n(33));
				bw_bit(&w, 1);
				put_qmat(&w, ni, m2v_scan[0]);
			} else {
				bw_bit(&w, 0);          /* default non-intra matrix */
			}
			if (p.mpeg2) {
				start_code(&w, 0xb5);
				bw_bits(&w, 1, 4);      /* sequence extension */
				bw_bits(&w, 0x48, 8);   /* main profile, main level */
				bw_bit(&w, 1);          /* progressive_sequence */
				bw_bits(&w, 1, 2);      /* 4:2:0 */
				bw_bits(&w, 0, 2);
				bw_bits(&w, 0, 2);
				bw_bits(&w, 0, 12);
				bw_bit(&w, 1);
				bw_bits(&w, 0, 8);
				bw_bit(&w, 0);          /* low_delay */
				bw_bits(&w, 0, 2);
				bw_bits(&w, 0, 5);
				if (p.vary && rnd_n(2)) { /* sequence display extension */
					start_code(&w, 0xb5);
					bw_bits(&w, 2, 4);
					bw_bits(&w, 5, 3);
					bw_bit(&w, 1);
					bw_bits(&w, 0x010101, 24);
					bw_bits(&w, (uint32_t)p.w, 14);
					bw_bit(&w, 1);
					bw_bits(&w, (uint32_t)p.h, 14);
				}
			}
			start_code(&w, 0xb8); /* GOP */
			bw_bits(&w, 0, 25);
			bw_bit(&w, 1);
			bw_bit(&w, 0);
		}
		/* picture header, 6.2.3 */
		start_code(&w, 0x00);
		{
			/* temporal_reference: display order of I0 P3 B1 B2 P6 B4 B5 ... */
			const int tr = ctype == 2 ? t + 2 : ctype == 3 ? t - 1 : t;
			bw_bits(&w, (uint32_t)tr & 1023, 10);
		}
		bw_bits(&w, (uint32_t)ctype, 3);
		bw_bits(&w, 0xffff, 16);
		g_pb.ctype = ctype;
		if (ctype != 1) {
			/* f_codes 1-4 (r_size 0-3); MPEG-2 sends them in the picture coding extension and 0111 here */
			for (int s2 = 0; s2 < 2; ++s2)
				for (int c = 0; c < 2; ++c) g_pb.r_size[s2][c] = p.vary ? rnd_n(4) : 1;
			if (!p.mpeg2) { /* one f_code per direction */
				g_pb.r_size[0][1] = g_pb.r_size[0][0];
				g_pb.r_size[1][1] = g_pb.r_size[1][0];
			}
			bw_bits(&w, p.mpeg2 ? 7 : (uint32_t)(g_pb.r_size[0][0] + 1), 4); /* full_pel 0 + f_code */
			if (ctype == 3) bw_bits(&w, p.mpeg2 ? 7 : (uint32_t)(g_pb.r_size[1][0] + 1), 4);
		}
		bw_bit(&w, 0);
		e.qmat = cur_qmat;
		e.qcode = p.vary ? 1 + rnd_n(ctype == 1 ? 31 : 20) : p.qscale_code;
		if (p.mpeg2) {
			e.intra_vlc_format = p.vary ? rnd_n(2) : p.intra_vlc_format;
			e.alternate_scan = p.vary ? rnd_n(2) : 0;
			e.q_scale_type = p.vary ? rnd_n(2) : 0;
			e.dc_precision = p.vary ? rnd_n(4) : p.dc_precision;
			e.frame_pred_frame_dct = p.vary ? rnd_n(2) : 1;
			if (ctype != 1 && p.field_mc) e.frame_pred_frame_dct = 0;
			start_code(&w, 0xb5); /* picture coding extension, 6.2.3.1 */
			bw_bits(&w, 8, 4);
			if (ctype == 1) {
				bw_bits(&w, 0xffff, 16); /* f_codes (I picture) */
			} else {
				bw_bits(&w, (uint32_t)(g_pb.r_size[0][0] + 1), 4);
				bw_bits(&w, (uint32_t)(g_pb.r_size[0][1] + 1), 4);
				bw_bits(&w, ctype == 3 ? (uint32_t)(g_pb.r_size[1][0] + 1) : 15, 4);
				bw_bits(&w, ctype == 3 ? (uint32_t)(g_pb.r_size[1][1] + 1) : 15, 4);
			}
			bw_bits(&w, (uint32_t)e.dc_precision, 2);
			bw_bits(&w, 3, 2);       /* frame picture */
			bw_bit(&w, 0);           /* top_field_first */
			bw_bit(&w, e.frame_pred_frame_dct);
			bw_bit(&w, 0);           /* concealment_motion_vectors */
			bw_bit(&w, e.q_scale_type);
			bw_bit(&w, e.intra_vlc_format);
			bw_bit(&w, e.alternate_scan);
			bw_bit(&w, 0);           /* repeat_first_field */
			bw_bit(&w, 1);           /* chroma_420_type */
			bw_bit(&w, 1);           /* progressive_frame */
			bw_bit(&w, 0);           /* composite_display_flag */
			if (p.vary && rnd_n(3) == 0) { /* quant matrix extension (intra matrix, in the current scan) */
				start_code(&w, 0xb5);
				bw_bits(&w, 3, 4);
				bw_bit(&w, 1);
				for (int i = 0; i < 64; ++i) ext_intra[i] = (uint8_t)(i ? 6 + rnd_n(50) : 8);
				put_qmat(&w, ext_intra, m2v_scan[e.alternate_scan]);
				bw_bit(&w, 0);
				bw_bit(&w, 0);
				bw_bit(&w, 0);
				e.qmat = cur_qmat = ext_intra;
			}
		} else {
			e.dc_precision = 0;
			e.frame_pred_frame_dct = 1;
		}
		g_pb.frame_mode = (p.mpeg2 && !e.frame_pred_frame_dct) ? 1 : 3;
		if (ctype != 1) {
			const int drop_row = (p.drop_slice && rnd_n(3) == 0) ? 1 + rnd_n(mbh - 2) : -1;
			put_pb_slices(&w, &e, mbw, mbh, t, (int)p.seed, drop_row);
			continue;
		}
		/* slices: one per MB row; coverage: some rows split inside the row, a row left out */
		const int drop_row = (p.drop_slice && t > 0 && t % 2 == 0) ? 1 + rnd_n(mbh - 2) : -1;
		for (int y = 0; y < mbh; ++y) {
			if (y == drop_row) continue;
			/* (never in row 0: every slice of row 0 starts a new picture's frame in the reference,
			 * m2d_read_slice -> m2d_update_frames, mpeg2.cpp:641-643) */
			const int split = (p.slices_midrow && y > 0 && rnd_n(2)) ? 1 + rnd_n(mbw - 1) : mbw;
			for (int x0 = 0; x0 < mbw; x0 = split > x0 ? split : mbw) {
				const int x1 = split > x0 ? split : mbw;
				start_code(&w, y + 1);
				bw_bits(&w, (uint32_t)e.qcode, 5);
				if (p.vary && rnd_n(4) == 0) { /* extra_bit_slice with intra_slice info + one extra byte */
					bw_bit(&w, 1);
					bw_bits(&w, 0x80, 8);
					bw_bit(&w, 1);
					bw_bits(&w, 0x5a, 8);
				}
				bw_bit(&w, 0);
				e.dc_pred[0] = e.dc_pred[1] = e.dc_pred[2] = (int16_t)(1 << (7 + e.dc_precision));
				for (int x = x0; x < x1; ++x) {
					/* macroblock_address_increment: 1, or x0 + 1 for the first MB of a mid-row slice */
					int inc = (x == x0) ? x0 + 1 : 1;
					while (inc > 33) {
						put_code(&w, "00000001000");
						inc -= 33;
					}
					put_code(&w, find_code(m2v_mb_inc, inc));
					if (x == x0 && x0 > 0) /* the reference resets the DC predictors after the copy */
						e.dc_pred[0] = e.dc_pred[1] = e.dc_pred[2] = (int16_t)(1 << (7 + e.dc_precision));
					const int quant = p.vary && rnd_n(5) == 0;
					if (quant) e.qcode = 1 + rnd_n(31);
					const int dct_type = (!e.frame_pred_frame_dct && p.mpeg2) ? rnd_n(2) : 0;
					put_mb(&w, &e, x, y, t, (int)p.seed, quant, dct_type, p.vary && rnd_n(16) == 0);
				}
			}
		}
		g_pb.prev_type = M2V_MBF_INTRA;
	}
	start_code(&w, 0xb7); /* sequence end */
	{
		FILE *f = fopen(out, "wb");
		if (!f) return 1;
		fwrite(w.b, 1, w.n, f);
		fclose(f);
	}
	return 0;
}
