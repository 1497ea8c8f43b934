/* h264gen command line: deterministic synthetic H.264 streams for tests and bench.py.
 *
 *   h264gen --preset c2|c3|c5|cov_cabac|cov_cavlc|cov_wp|cov_wp_quirks|cov_slices|cov_tools|cov_tools_cavlc
 *           [--seed N] [--frames N]
 *           [--size WxH] [--set key=value ...] -o out.264
 *
 * Presets follow SURVEY.md §8(d): c2 = Baseline 720p CAVLC IPPP, c3 = 1080p CABAC IBBP 8x8,
 * c5 = 4K multi-slice; cov_* are small streams that stress one tool each.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gen.h"

static void preset(params_t *p, const char *name)
{
	memset(p, 0, sizeof(*p));
	p->width = 1920; p->height = 1088; p->crop_bottom = 8;
	p->frames = 60; p->cabac = 1; p->bframes = 2; p->t8x8 = 1; p->gop = 30; p->idr_period = 0;
	p->slices = 1; p->profile = 100; p->level = 40; p->wp_p = 0; p->wp_b = 2; p->direct = 2;
	p->qp_min = 22; p->qp_max = 36; p->deblock = 1; p->pcm_permille = 0; p->mv_px = 48;
	p->num_ref_frames = 3; p->l0_active = 2; p->l1_active = 1;
	p->p_skip_pct = 25; p->p_intra_pct = 5; p->i4_pct = 40; p->i8_pct = 40; p->sub8x8_pct = 10;
	p->coef_pct = 45; p->planar = 0; p->seed = 1;
	if (!strcmp(name, "c3")) return;
	if (!strcmp(name, "c2")) {
		p->width = 1280; p->height = 720; p->crop_bottom = 0; p->cabac = 0; p->bframes = 0; p->t8x8 = 0;
		p->profile = 66; p->level = 31; p->wp_b = 0; p->qp_min = 22; p->qp_max = 38; p->mv_px = 64;
		p->num_ref_frames = 2; p->l0_active = 2; p->l1_active = 1; p->i8_pct = 0; p->i4_pct = 60;
		return;
	}
	if (!strcmp(name, "c5")) {
		p->width = 3840; p->height = 2160; p->crop_bottom = 0; p->slices = 8; p->level = 51; p->frames = 30;
		return;
	}
	if (!strcmp(name, "cov_cabac")) {
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->pcm_permille = 10;
		p->sub8x8_pct = 30; p->t8x8 = 1; p->gop = 8; p->mv_px = 80; p->qp_min = 10; p->qp_max = 40;
		return;
	}
	if (!strcmp(name, "cov_cabac4x4")) {
		/* B_8x8 with every sub-partition size (transform 8x8 off) */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->pcm_permille = 10;
		p->sub8x8_pct = 40; p->t8x8 = 0; p->gop = 8; p->mv_px = 80; p->i8_pct = 0; p->i4_pct = 60;
		return;
	}
	if (!strcmp(name, "cov_cavlc")) {
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->cabac = 0; p->t8x8 = 0;
		p->profile = 77; p->level = 30; p->pcm_permille = 10; p->sub8x8_pct = 30; p->gop = 8; p->mv_px = 80;
		p->i8_pct = 0; p->i4_pct = 60; p->qp_min = 10; p->qp_max = 40;
		return;
	}
	if (!strcmp(name, "cov_wp")) {
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->wp_p = 1; p->wp_b = 1;
		p->gop = 0;
		return;
	}
	if (!strcmp(name, "cov_wp_quirks")) {
		/* explicit weighting at the edges the reference's SSE2 path handles its own way (int16
		 * saturation, int8 weight 128) and DC-only blocks at large adjustments: oracle_quirk_hits > 0 */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->wp_p = 1; p->wp_b = 1;
		p->gop = 8; p->t8x8 = 1; p->quirks = 1; p->qp_min = 24; p->qp_max = 36;
		return;
	}
	if (!strcmp(name, "cov_tools")) {
		/* the reference paths no other preset reaches: plane prediction (luma 16x16 and chroma),
		 * constrained intra prediction, deblocking idc 2 across 3 slices, SPS scaling lists */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->slices = 3; p->gop = 8;
		p->planar = 1; p->cip = 1; p->idc2 = 1; p->scaling = 1; p->p_intra_pct = 25; p->i4_pct = 30;
		p->i8_pct = 30; p->pcm_permille = 5;
		return;
	}
	if (!strcmp(name, "cov_tools_cavlc")) {
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 16; p->slices = 3; p->gop = 8;
		p->cabac = 0; p->t8x8 = 0; p->profile = 77; p->level = 30; p->i8_pct = 0; p->i4_pct = 50;
		p->planar = 1; p->cip = 1; p->idc2 = 1; p->p_intra_pct = 25; p->pcm_permille = 5;
		return;
	}
	if (!strcmp(name, "cov_slices")) {
		p->width = 384; p->height = 256; p->crop_bottom = 0; p->frames = 12; p->slices = 5; p->gop = 6;
		return;
	}
	if (!strcmp(name, "cov_reflists")) {
		/* list modification, adaptive marking (MMCO 1 / 2 / 3 / 4 / 6), long-term references in P and B
		 * lists and in temporal direct, frame_num wrapping every 16 pictures */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 40; p->gop = 20; p->num_ref_frames = 4;
		p->l0_active = 3; p->l1_active = 2; p->direct = 0; p->log2_fn = 4; p->reorder_pct = 60; p->mmco_pct = 60;
		p->long_term = 1; p->mv_px = 40;
		return;
	}
	if (!strcmp(name, "cov_reflists_cavlc")) {
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 30; p->cabac = 0; p->t8x8 = 0; p->profile = 77;
		p->level = 30; p->i8_pct = 0; p->i4_pct = 60; p->gop = 15; p->num_ref_frames = 4; p->l0_active = 4;
		p->l1_active = 2; p->direct = 2; p->log2_fn = 4; p->reorder_pct = 70; p->mmco_pct = 50; p->long_term = 1;
		p->mv_px = 40;
		return;
	}
	if (!strcmp(name, "cov_mmco5")) {
		/* MMCO 5 every 9th anchor: references dropped, frame_num and POC restart at the picture */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 30; p->gop = 0; p->mmco5 = 9;
		p->num_ref_frames = 3; p->reorder_pct = 30; p->mv_px = 40;
		return;
	}
	if (!strcmp(name, "cov_poc1")) {
		/* POC type 1 (offset_for_ref_frame 1 per frame, delta_pic_order_cnt[0] per picture) with B pictures */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 24; p->gop = 12; p->poc_type = 1;
		p->log2_fn = 4; p->mv_px = 40;
		return;
	}
	if (!strcmp(name, "cov_poc2")) {
		/* POC type 2 (output order = decoding order), IPPP with non-reference P pictures */
		p->width = 320; p->height = 192; p->crop_bottom = 0; p->frames = 24; p->gop = 12; p->poc_type = 2;
		p->bframes = 0; p->log2_fn = 4; p->nonref_pct = 35; p->mmco_pct = 30; p->mv_px = 40;
		return;
	}
	fprintf(stderr, "h264gen: unknown preset %s\n", name);
	exit(2);
}

static void set_kv(params_t *p, const char *kv)
{
	char key[64];
	const char *eq = strchr(kv, '=');
	long v;
	if (!eq || eq - kv >= (long)sizeof(key)) { fprintf(stderr, "bad --set %s\n", kv); exit(2); }
	memcpy(key, kv, (size_t)(eq - kv));
	key[eq - kv] = 0;
	v = strtol(eq + 1, NULL, 0);
#define F(name) if (!strcmp(key, #name)) { p->name = (int)v; return; }
	F(width) F(height) F(crop_bottom) F(frames) F(cabac) F(bframes) F(t8x8) F(gop) F(idr_period) F(slices)
	F(profile) F(level) F(wp_p) F(wp_b) F(direct) F(qp_min) F(qp_max) F(deblock) F(pcm_permille) F(mv_px)
	F(num_ref_frames) F(l0_active) F(l1_active) F(p_skip_pct) F(p_intra_pct) F(i4_pct) F(i8_pct)
	F(sub8x8_pct) F(coef_pct) F(planar) F(cip) F(idc2) F(scaling) F(quirks)
	F(poc_type) F(log2_fn) F(reorder_pct) F(mmco_pct) F(long_term) F(mmco5) F(nonref_pct)
#undef F
	fprintf(stderr, "h264gen: unknown key %s\n", key);
	exit(2);
}

int main(int argc, char **argv)
{
	params_t p;
	const char *out = NULL, *dump = NULL, *refdump = NULL;
	FILE *df = NULL, *rf = NULL;
	bw_t o;
	FILE *f;
	int n;
	preset(&p, "c3");
	for (int i = 1; i < argc; ++i) {
		if (!strcmp(argv[i], "--preset") && i + 1 < argc) preset(&p, argv[++i]);
		else if (!strcmp(argv[i], "--seed") && i + 1 < argc) p.seed = strtoull(argv[++i], NULL, 0);
		else if (!strcmp(argv[i], "--frames") && i + 1 < argc) p.frames = atoi(argv[++i]);
		else if (!strcmp(argv[i], "--size") && i + 1 < argc) {
			if (sscanf(argv[++i], "%dx%d", &p.width, &p.height) != 2) return 2;
		} else if (!strcmp(argv[i], "--set") && i + 1 < argc) set_kv(&p, argv[++i]);
		else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
		else if (!strcmp(argv[i], "--dump") && i + 1 < argc) dump = argv[++i];
		else if (!strcmp(argv[i], "--dump-refs") && i + 1 < argc) refdump = argv[++i];
		else {
			fprintf(stderr, "usage: h264gen --preset NAME [--seed N] [--frames N] [--size WxH] [--set k=v] -o out.264\n");
			return 2;
		}
	}
	if (!out || p.width % 16 || p.height % 16 || p.frames < 1) {
		fprintf(stderr, "h264gen: need -o and 16-aligned size\n");
		return 2;
	}
	if (!p.cabac) p.t8x8 = 0;
	bw_init(&o);
	if (dump && !(df = fopen(dump, "wb"))) return 1;
	if (refdump && !(rf = fopen(refdump, "wb"))) return 1;
	n = gen_stream(&p, &o, df, rf);
	if (df) fclose(df);
	if (rf) fclose(rf);
	f = fopen(out, "wb");
	if (!f) return 1;
	fwrite(o.b, 1, o.n, f);
	fclose(f);
	fprintf(stderr, "h264gen: %d pictures, %zu bytes -> %s\n", n, o.n, out);
	free(o.b);
	return 0;
}
