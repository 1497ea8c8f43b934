/*
 * H.265 / HEVC host parser and the reference-shaped h265d_func table (h265.h:37, h265.cpp:5010-5025).
 *
 * The parse follows the reference decoder's semantics (h265.cpp; functions cited inline) and emits the
 * per-picture reconstruction records of include/m2d_recon.h (h265r_*) instead of reconstructing:
 * every sample operation happens in the back end (gfx950: m2dec_amd/csrc/hip/h265_hip.hip).  Reference
 * behaviours kept on purpose, since they decide the output:
 *   - decode_picture handles one slice NAL per call and returns -2 on end of data or any error
 *     (h265.cpp:4898-4920, setjmp / error_report);
 *   - only TRAIL_N, TRAIL_R and IDR_W_RADL slices are decoded (h265.cpp:4872-4877);
 *   - the frame LRU over at most 8 frames and the 16-entry POC-sorted DPB that outputs only when full,
 *     pops data[0] on every get (h265.cpp:180-205, 4931-5008);
 *   - deblocking offsets are taken from the slice header only when it overrides them, and otherwise
 *     kept from the previous slice (h265.cpp:894-901);
 *   - the slice's POC from the previous slice's lsb / msb (h265.cpp:736-750);
 *   - the sign-hidden coefficient is negated after dequantisation (h265.cpp:1645-1647).
 */
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "h264_dec.h" /* bit reader (hb_*) and the CABAC range tables, shared with the H.264 parser */
#include "h265_dec.h"

int m2d_stream_next_byte(dec_bits *st); /* bitio.c */
extern int m2dec_host_cpu_ok;           /* cpucheck.c */

#define H265_ERR(d) longjmp(*(d)->jb, 1)

/* M2DEC_AMD_H265_DUMP=path: the parsed syntax in tools/h265gen --dump's format (tests/test_h265_cpu.py
 * compares the two), and a check that each slice's CABAC data ends with end_of_slice_segment_flag = 1 */
static FILE *g_dump;
static int g_dump_init;

typedef struct {
	h265_dec_t *d;
	jmp_buf *jb;
} perr_t;

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------ NAL units */
/* the next NAL unit (after a start code) into d->unit, emulation-prevention bytes removed; its two
 * header bytes stay in front.  -1 at the end of the data */
static int next_unit(h265_dec_t *d)
{
	dec_bits *st = &d->stream_i;
	int zeros = 0, c;
	if (!d->pending) {
		for (;;) {
			c = m2d_stream_next_byte(st);
			if (c < 0) return -1;
			if (c == 0) {
				zeros++;
			} else {
				if (c == 1 && zeros >= 2) break;
				zeros = 0;
			}
		}
	}
	d->pending = 0;
	d->unit_len = 0;
	zeros = 0;
	for (;;) {
		c = m2d_stream_next_byte(st);
		if (c < 0) break;
		if (zeros >= 2 && c == 1) {
			d->unit_len -= (size_t)zeros;
			d->pending = 1;
			break;
		}
		if (zeros >= 2 && c == 3) { /* emulation_prevention_three_byte (7.4.2) */
			zeros = 0;
			continue;
		}
		if (d->unit_len + 16 >= d->unit_cap) {
			size_t cap = d->unit_cap ? 2 * d->unit_cap : (1u << 16);
			uint8_t *n = (uint8_t *)realloc(d->unit, cap);
			if (!n) return -1;
			d->unit = n;
			d->unit_cap = cap;
		}
		d->unit[d->unit_len++] = (uint8_t)c;
		zeros = (c == 0) ? zeros + 1 : 0;
	}
	if (!d->unit) {
		d->unit = (uint8_t *)calloc(1, 64);
		if (!d->unit) return -1;
		d->unit_cap = 64;
	}
	memset(d->unit + d->unit_len, 0, 16);
	return 0;
}

/* ------------------------------------------------------------------ parameter sets (h265.cpp:231-691) */
static void profile_tier_level(h264_bits_t *b, int max_sub_layers_m1)
{
	hb_get(b, 8);
	hb_get(b, 32);
	hb_get(b, 24);
	hb_get(b, 24);
	hb_get(b, 8); /* general_level_idc */
	if (max_sub_layers_m1) {
		uint32_t present = hb_get(b, 16);
		for (int i = 0; i < max_sub_layers_m1; ++i) {
			if (present & (1u << 15)) {
				hb_get(b, 8);
				hb_get(b, 32);
				hb_get(b, 24);
				hb_get(b, 24);
			}
			if (present & (1u << 14)) hb_get(b, 8);
			present <<= 2;
		}
	}
}

static int ue_max(perr_t *e, h264_bits_t *b, uint32_t max)
{
	uint32_t v = hb_ue(b);
	if (v > max) H265_ERR(e);
	return (int)v;
}

static int se_range(perr_t *e, h264_bits_t *b, int lo, int hi)
{
	int v = hb_se(b);
	if (v < lo || v > hi) H265_ERR(e);
	return v;
}

/* short_term_ref_pic_set, h265.cpp:392-485 (the reference's inter-RPS prediction included) */
static void st_rps_nopred(perr_t *e, h264_bits_t *b, h265_st_rps_t *r)
{
	const int neg = ue_max(e, b, 16), pos = ue_max(e, b, (uint32_t)(16 - neg));
	int cnt = 0;
	r->num_pics[0] = (uint8_t)neg;
	r->num_pics[1] = (uint8_t)pos;
	for (int s = 0; s < 2; ++s) {
		int val = 0;
		r->used[s] = 0;
		for (int i = 0; i < r->num_pics[s]; ++i) {
			const int delta = ue_max(e, b, 32767) + 1;
			val += s ? delta : -delta;
			r->delta_poc[s][i] = (int16_t)val;
			const int used = (int)hb_get1(b);
			r->used[s] |= (uint16_t)(used << i);
			cnt += used;
		}
	}
	r->total_curr = (uint8_t)cnt;
}

static int rps_pred_core(int16_t *dst, const int16_t *refd, int delta_rps, uint32_t used_flag, uint32_t use_delta, uint16_t *used,
                         int idx, int neg, int j)
{
	const int dpoc = refd[j] + delta_rps;
	if (((neg ? -dpoc : dpoc) < 0) && (use_delta & (1u << j))) {
		dst[idx] = (int16_t)dpoc;
		if (used_flag & (1u << j)) *used |= (uint16_t)(1u << idx);
		idx++;
	}
	return idx;
}

static void st_rps_pred_part(h265_st_rps_t *dst, const h265_st_rps_t *ref, int delta_rps, uint32_t used_flag, uint32_t use_delta, int s0)
{
	uint16_t used0 = 0;
	const int sh_neg = s0 ? 0 : ref->num_pics[0], sh_pos = s0 ? ref->num_pics[0] : 0;
	int i = 0;
	const h265_st_rps_t *r = ref;
	/* h265.cpp:434-439 over ref.ref[s0 ^ 1] backwards */
	for (int j = r->num_pics[s0 ^ 1] - 1; j >= 0; --j)
		i = rps_pred_core(dst->delta_poc[s0], r->delta_poc[s0 ^ 1], delta_rps, used_flag >> sh_neg, use_delta >> sh_neg, &used0, i,
		                  s0 != 0, j);
	{
		const uint32_t mask = 1u << (ref->num_pics[0] + ref->num_pics[1]);
		if ((((s0 != 0) ? -delta_rps : delta_rps) < 0) && (use_delta & mask)) {
			dst->delta_poc[s0][i] = (int16_t)delta_rps;
			if (used_flag & mask) used0 |= (uint16_t)(1u << i);
			i++;
		}
	}
	for (int j = 0; j < r->num_pics[s0]; ++j)
		i = rps_pred_core(dst->delta_poc[s0], r->delta_poc[s0], delta_rps, used_flag >> sh_pos, use_delta >> sh_pos, &used0, i, s0 != 0, j);
	dst->num_pics[s0] = (uint8_t)i;
	dst->used[s0] = used0;
}

static void st_rps_pred(perr_t *e, h264_bits_t *b, h265_st_rps_t *dst, const h265_st_rps_t *ref)
{
	const int sign = (int)hb_get1(b);
	const int abs_delta = ue_max(e, b, 32767) + 1;
	const int delta_rps = sign ? -abs_delta : abs_delta;
	const int num = ref->num_pics[0] + ref->num_pics[1];
	uint32_t used_flag = 0, use_delta = 0;
	int cnt = 0;
	/* a predicted set holds at most num + 1 entries; delta_poc[s] has 16 per side, so a reference set of
	 * 16 (the most st_rps_nopred lets through; a conformant one has <= 15) cannot be predicted from */
	if (num >= 16) H265_ERR(e);
	for (int j = 0; j <= num; ++j) {
		const uint32_t used_by = hb_get1(b);
		cnt += (int)used_by;
		if (used_by) {
			used_flag |= 1u << j;
			use_delta |= 1u << j;
		} else if (hb_get1(b)) {
			use_delta |= 1u << j;
		}
	}
	st_rps_pred_part(dst, ref, delta_rps, used_flag, use_delta, 0);
	st_rps_pred_part(dst, ref, delta_rps, used_flag, use_delta, 1);
	dst->total_curr = (uint8_t)cnt;
}

static int log2ceil(uint32_t n)
{
	/* h265.cpp:523-534: 1 + floor(log2(n)) for n > 0 */
	int r = 0;
	while (n) {
		r++;
		n >>= 1;
	}
	return r;
}

static void parse_sps(perr_t *e, h264_bits_t *b)
{
	h265_dec_t *d = e->d;
	h265_sps_t s;
	int max_sub_m1, id;
	memset(&s, 0, sizeof(s));
	hb_get(b, 4); /* vps id */
	max_sub_m1 = (int)hb_get(b, 3);
	hb_get1(b);
	profile_tier_level(b, max_sub_m1);
	id = ue_max(e, b, 15);
	s.chroma_format_idc = ue_max(e, b, 3);
	if (s.chroma_format_idc == 3) s.separate_colour_plane = (int)hb_get1(b);
	s.pic_w = (int)hb_ue(b);
	s.pic_h = (int)hb_ue(b);
	if (hb_get1(b))
		for (int i = 0; i < 4; ++i) s.crop[i] = (int)hb_ue(b);
	s.bit_depth_luma_m8 = ue_max(e, b, 6);
	s.bit_depth_chroma_m8 = ue_max(e, b, 6);
	s.log2_max_poc_lsb = ue_max(e, b, 12) + 4;
	{
		const int present = (int)hb_get1(b);
		for (int i = present ? 0 : max_sub_m1; i <= max_sub_m1; ++i) {
			hb_ue(b);
			hb_ue(b);
			hb_ue(b);
		}
	}
	s.log2_min_cb = ue_max(e, b, 2) + 3;
	s.log2_ctb = s.log2_min_cb + ue_max(e, b, 3);
	s.log2_min_tb = ue_max(e, b, 2) + 2;
	s.log2_max_tb = s.log2_min_tb + ue_max(e, b, 3);
	s.max_th_depth_inter = ue_max(e, b, 5);
	s.max_th_depth_intra = ue_max(e, b, 5);
	s.scaling_list_enabled = (int)hb_get1(b);
	if (s.scaling_list_enabled) H265_ERR(e); /* the reference has no scaling lists (h265.cpp:333, 4760-4763) */
	s.amp = (int)hb_get1(b);
	s.sao = (int)hb_get1(b);
	s.pcm = (int)hb_get1(b);
	if (s.pcm) {
		hb_get(b, 4);
		hb_get(b, 4);
		s.log2_min_pcm = ue_max(e, b, 2) + 3;
		s.log2_max_pcm = s.log2_min_pcm + ue_max(e, b, 3);
		hb_get1(b);
	} else {
		s.log2_min_pcm = 8; /* h265.cpp:540 */
		s.log2_max_pcm = 8;
	}
	s.num_st_rps = ue_max(e, b, 64);
	for (int i = 0; i < s.num_st_rps; ++i) {
		if (i && hb_get1(b)) st_rps_pred(e, b, &s.st_rps[i], &s.st_rps[i - 1]);
		else st_rps_nopred(e, b, &s.st_rps[i]);
	}
	s.long_term_present = (int)hb_get1(b);
	if (s.long_term_present) {
		s.num_lt_sps = ue_max(e, b, 32);
		for (int i = 0; i < s.num_lt_sps; ++i) {
			hb_get(b, s.log2_max_poc_lsb);
			hb_get1(b);
		}
	}
	s.temporal_mvp = (int)hb_get1(b);
	s.strong_intra_smoothing = (int)hb_get1(b);
	/* (vui and extensions: nothing the decode uses, as in the reference) */
	if (s.chroma_format_idc != 1 || s.bit_depth_luma_m8 || s.bit_depth_chroma_m8 || s.log2_ctb > 6 || s.log2_max_tb > 5 ||
	    s.pic_w <= 0 || s.pic_h <= 0 || s.pic_w > 8192 || s.pic_h > 8192)
		H265_ERR(e);
	s.ctb_cols = (s.pic_w + (1 << s.log2_ctb) - 1) >> s.log2_ctb;
	s.ctb_rows = (s.pic_h + (1 << s.log2_ctb) - 1) >> s.log2_ctb;
	s.stride = s.ctb_cols << s.log2_ctb;
	s.num_ctb_log2 = log2ceil((uint32_t)(s.ctb_cols * s.ctb_rows));
	s.frame_num = imin(s.num_lt_sps + s.num_st_rps, H265R_MAX_FRAMES);
	s.valid = 1;
	d->sps[id] = s;
}

static void parse_pps(perr_t *e, h264_bits_t *b)
{
	h265_dec_t *d = e->d;
	h265_pps_t p;
	int id;
	memset(&p, 0, sizeof(p));
	id = ue_max(e, b, 63);
	p.sps_id = ue_max(e, b, 15);
	p.dependent_slices = (int)hb_get1(b);
	p.output_flag_present = (int)hb_get1(b);
	p.num_extra_bits = (int)hb_get(b, 3);
	p.sign_hiding = (int)hb_get1(b);
	p.cabac_init_present = (int)hb_get1(b);
	p.num_ref_idx_default[0] = ue_max(e, b, 14) + 1;
	p.num_ref_idx_default[1] = ue_max(e, b, 14) + 1;
	p.init_qp = 26 + se_range(e, b, -26, 25);
	p.constrained_intra = (int)hb_get1(b);
	p.transform_skip = (int)hb_get1(b);
	p.cu_qp_delta = (int)hb_get1(b);
	if (p.cu_qp_delta) p.diff_cu_qp_delta_depth = ue_max(e, b, 52);
	p.cb_qp_offset = se_range(e, b, -12, 12);
	p.cr_qp_offset = se_range(e, b, -12, 12);
	p.slice_chroma_qp_offsets_present = (int)hb_get1(b);
	p.weighted_pred = (int)hb_get1(b);
	p.weighted_bipred = (int)hb_get1(b);
	p.transquant_bypass = (int)hb_get1(b);
	p.tiles = (int)hb_get1(b);
	p.entropy_sync = (int)hb_get1(b);
	if (p.tiles) H265_ERR(e); /* (tiles: not built) */
	p.loop_filter_across_slices = (int)hb_get1(b);
	p.deblocking_control = (int)hb_get1(b);
	if (p.deblocking_control) {
		p.deblocking_override_enabled = (int)hb_get1(b);
		p.pps_deblocking_disabled = (int)hb_get1(b);
		if (!p.pps_deblocking_disabled) {
			p.pps_beta_offset_div2 = se_range(e, b, -12, 12);
			p.pps_tc_offset_div2 = se_range(e, b, -12, 12);
		}
	}
	p.scaling_list_data = (int)hb_get1(b);
	if (p.scaling_list_data) H265_ERR(e);
	p.lists_modification = (int)hb_get1(b);
	p.log2_parallel_merge_level = (int)hb_ue(b) + 2;
	p.slice_header_extension = (int)hb_get1(b);
	/* the reference's unsupported tools are errors here rather than assert(0) (h265.cpp:3008, 4092) */
	if (p.cu_qp_delta || p.transquant_bypass || p.entropy_sync) H265_ERR(e);
	p.valid = 1;
	d->pps[id] = p;
}

/* ------------------------------------------------------------------ slice header (h265.cpp:752-934) */
static void update_poc(h265_slice_t *sh, unsigned lsb, const h265_sps_t *s)
{
	const unsigned prev_lsb = (unsigned)sh->poc_lsb;
	const unsigned half = 8u << (s->log2_max_poc_lsb - 4);
	sh->poc_lsb = (int)lsb;
	if (sh->nal_type >= H265_BLA_W_LP && sh->nal_type <= H265_BLA_N_LP) sh->poc_msb = 0;
	else if (lsb < prev_lsb && prev_lsb - lsb >= half) sh->poc_msb++;
	else if (prev_lsb < lsb && lsb - prev_lsb > half) sh->poc_msb--;
	sh->poc = ((16 * sh->poc_msb) << (s->log2_max_poc_lsb - 4)) + (int)lsb;
}

static void parse_slice_header(perr_t *e, h264_bits_t *b, const h265_sps_t *s, const h265_pps_t *p)
{
	h265_slice_t *sh = &e->d->sh;
	sh->dependent = 0;
	if (!sh->first_slice) {
		if (p->dependent_slices) sh->dependent = (int)hb_get1(b);
		sh->address = (int)hb_get(b, s->num_ctb_log2);
		if (sh->address > s->ctb_cols * s->ctb_rows - 1) H265_ERR(e);
	} else {
		sh->address = 0;
	}
	if (sh->dependent) H265_ERR(e);
	if (p->num_extra_bits) hb_get(b, p->num_extra_bits);
	sh->slice_type = ue_max(e, b, 2);
	sh->pic_output = p->output_flag_present ? (int)hb_get1(b) : 1;
	if (sh->nal_type != H265_IDR_W_RADL && sh->nal_type != H265_IDR_N_LP) {
		const unsigned lsb = hb_get(b, s->log2_max_poc_lsb);
		update_poc(sh, lsb, s);
		if (hb_get1(b)) {
			int idx = 0;
			if (s->num_st_rps > 1) idx = (int)hb_get(b, log2ceil((uint32_t)s->num_st_rps));
			/* the reference reads log2ceil(n) bits, one more than the spec for a power of two (kept), and
			 * never checks the index against the SPS's sets */
			if (idx >= s->num_st_rps) H265_ERR(e);
			sh->rps = s->st_rps[idx];
		} else {
			if (s->num_st_rps && hb_get1(b)) {
				const int dm1 = ue_max(e, b, (uint32_t)s->num_st_rps - 1);
				st_rps_pred(e, b, &sh->rps, &s->st_rps[s->num_st_rps - dm1 - 1]);
			} else {
				st_rps_nopred(e, b, &sh->rps);
			}
		}
		if (s->long_term_present) H265_ERR(e); /* h265.cpp:768 */
		sh->temporal_mvp = s->temporal_mvp ? (int)hb_get1(b) : 0;
	} else {
		sh->poc_lsb = sh->poc_msb = sh->poc = 0; /* init_pic_order_cnt */
		memset(&sh->rps, 0, sizeof(sh->rps));
	}
	if (s->sao) {
		sh->sao_luma = (int)hb_get1(b);
		sh->sao_chroma = (int)hb_get1(b);
	} else {
		sh->sao_luma = sh->sao_chroma = 0;
	}
	if (sh->slice_type != 2) H265_ERR(e); /* P / B slices: the inter path is not built yet */
	sh->slice_qp = p->init_qp + hb_se(b);
	if (sh->slice_qp < 0 || sh->slice_qp > 51) H265_ERR(e);
	{
		int cb = 0, cr = 0;
		if (p->slice_chroma_qp_offsets_present) {
			cb = se_range(e, b, -12, 12);
			cr = se_range(e, b, -12, 12);
		}
		cb += p->cb_qp_offset;
		cr += p->cr_qp_offset;
		if (cb < -12 || cb > 12 || cr < -12 || cr > 12) H265_ERR(e);
		sh->qpc_delta[0] = cb;
		sh->qpc_delta[1] = cr;
	}
	sh->deblocking_disabled = p->pps_deblocking_disabled;
	sh->deblocking_override = p->deblocking_override_enabled ? (int)hb_get1(b) : 0;
	if (sh->deblocking_override) {
		sh->deblocking_disabled = (int)hb_get1(b);
		if (!sh->deblocking_disabled) {
			sh->beta_offset_div2 = se_range(e, b, -6, 6);
			sh->tc_offset_div2 = se_range(e, b, -6, 6);
		}
	}
	if (p->loop_filter_across_slices && (sh->sao_luma || sh->sao_chroma || !sh->deblocking_disabled))
		sh->loop_filter_across_slices = (int)hb_get1(b);
	else
		sh->loop_filter_across_slices = p->loop_filter_across_slices;
	if (p->slice_header_extension) {
		uint32_t n = hb_ue(b);
		while (n--) hb_get(b, 8);
	}
	/* byte_alignment(): the reference skips to the next byte boundary, a whole byte if aligned */
	{
		const int mis = b->bits & 7;
		hb_get(b, mis ? mis : 8);
	}
}

/* ------------------------------------------------------------------ CABAC (9.3.4.3) */
/* The engine keeps the spec's 9-bit ivlOffset as the top bits of a 64-bit window: value == win >> cnt,
 * with cnt look-ahead bits below it, refilled a byte at a time (bytes past the end read as 0, as the
 * reference's bit reader does).  Renormalisation is one count-leading-zeros instead of a bit loop. */
typedef struct {
	const uint8_t *p, *end;
	uint64_t win;
	uint32_t range;
	int cnt;
	uint8_t ctx[H265_NUM_CTX];
	uint64_t bins;
} cab_t;

static inline void cab_refill(cab_t *c)
{
	while (c->cnt <= 46) { /* value (9 bits) + look-ahead stays within 63 bits */
		c->win = (c->win << 8) | (c->p < c->end ? *c->p++ : 0u);
		c->cnt += 8;
	}
}

/* context state transitions (9.3.4.3.2.2) for a context byte (pStateIdx << 1 | valMps) after an MPS (0) or
 * an LPS (1), so that the decision below needs no data-dependent branch */
static uint8_t cab_next[128][2];
static pthread_once_t cab_once = PTHREAD_ONCE_INIT;

static void cab_build_next(void)
{
	for (int v = 0; v < 128; ++v) {
		const int s = v >> 1, mps = v & 1;
		cab_next[v][0] = (uint8_t)(((s + (s < 62)) << 1) | mps);
		cab_next[v][1] = (uint8_t)((h264_trans_idx_lps[s] << 1) | (s == 0 ? !mps : mps));
	}
}

static void cab_init_ctx(cab_t *c, int init_type, int qp)
{
	const int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
	for (int i = 0; i < H265_NUM_CTX; ++i) {
		int pre = ((h265_cabac_init_mn[init_type][i][0] * q) >> 4) + h265_cabac_init_mn[init_type][i][1];
		pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
		c->ctx[i] = (pre <= 63) ? (uint8_t)((63 - pre) << 1) : (uint8_t)(((pre - 64) << 1) | 1);
	}
}

static void cab_start(cab_t *c, const uint8_t *p, const uint8_t *end)
{
	pthread_once(&cab_once, cab_build_next);
	c->p = p;
	c->end = end;
	c->range = 510;
	c->win = 0;
	c->cnt = -9; /* the first 9 bits are ivlOffset itself */
	cab_refill(c);
}

static inline int cab_decision(cab_t *c, int ci)
{
	const int v = c->ctx[ci];
	const uint32_t lps = h264_range_lps[v >> 1][(c->range >> 6) & 3];
	const uint32_t rm = c->range - lps;
	const uint64_t scaled = (uint64_t)rm << c->cnt;
	const int is_lps = c->win >= scaled;
	const uint64_t m = -(uint64_t)is_lps;
	int n;
	c->bins++;
	c->win -= scaled & m;
	c->range = rm ^ ((rm ^ lps) & (uint32_t)m);
	c->ctx[ci] = cab_next[v][is_lps];
	n = __builtin_clz(c->range) - 23; /* shifts until range >= 256 */
	c->range <<= n;
	c->cnt -= n;
	if (c->cnt < 16) cab_refill(c);
	return (v & 1) ^ is_lps;
}

static inline int cab_bypass(cab_t *c)
{
	uint64_t r;
	c->bins++;
	if (--c->cnt < 16) cab_refill(c);
	r = (uint64_t)c->range << c->cnt;
	if (c->win >= r) {
		c->win -= r;
		return 1;
	}
	return 0;
}

/* k <= 16 bypass bins at once, MSB first: k compare-subtract steps are one long division of the
 * window by range << (cnt - k) (win < range << cnt bounds the quotient by 2^k) */
static inline uint32_t cab_bypass_k(cab_t *c, int k)
{
	uint64_t scaled, q;
	c->bins += (uint64_t)k;
	c->cnt -= k;
	scaled = (uint64_t)c->range << c->cnt;
	q = c->win / scaled;
	c->win -= q * scaled;
	if (c->cnt < 16) cab_refill(c);
	return (uint32_t)q;
}

static inline uint32_t cab_bypass_n(cab_t *c, int n)
{
	uint32_t v = 0;
	while (n > 16) {
		v = (v << 16) | cab_bypass_k(c, 16);
		n -= 16;
	}
	return n > 0 ? (v << n) | cab_bypass_k(c, n) : v;
}

/* a unary run of bypass 1s ended by a 0, looking at most 16 bins ahead: the number of 1s with the 0
 * consumed, or -1 (nothing consumed) if the next 16 bins are all 1 */
static inline int cab_bypass_ones(cab_t *c)
{
	const uint64_t scaled = (uint64_t)c->range << (c->cnt - 16);
	const uint32_t q = (uint32_t)(c->win / scaled); /* the next 16 bins, not consumed */
	const int ones = __builtin_clz(~(q << 16) | 1u);
	if (ones >= 16) return -1;
	c->bins += (uint64_t)ones + 1;
	c->cnt -= ones + 1;
	c->win -= (uint64_t)(q >> (15 - ones)) * ((uint64_t)c->range << c->cnt);
	if (c->cnt < 16) cab_refill(c);
	return ones;
}

/* end_of_slice_segment_flag (h265.cpp:1350-1365) */
static inline int cab_terminate(cab_t *c)
{
	c->range -= 2;
	if (c->win >= ((uint64_t)c->range << c->cnt)) return 1;
	if (c->range < 256) {
		c->range <<= 1;
		if (--c->cnt < 16) cab_refill(c);
	}
	return 0;
}

/* ------------------------------------------------------------------ slice data (intra) */
typedef struct {
	perr_t *e;
	h265_dec_t *d;
	const h265_sps_t *s;
	const h265_pps_t *p;
	const h265_slice_t *sh;
	cab_t c;
	int qp_y, scale[3];
	int order_luma[4], order_chroma, intra_split;
	int W4;                    /* luma 4x4 units per row (frame width / 4) */
	int16_t blk[32 * 32];
	int lev[32 * 32];          /* raw levels (the syntax dump only) */
} sctx_t;

static const uint8_t level_scale[6] = {40, 45, 51, 57, 64, 72};

static int qp_chroma(int qpi)
{
	/* qpi_to_qpc (h265.cpp:2965-2973) for 0 <= qpi < 52 */
	static const int8_t t[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
	                             18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33,
	                             34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45};
	return t[((qpi % 52) + 52) % 52];
}

static void set_qp(sctx_t *x, int qp)
{
	x->qp_y = qp;
	for (int c = 0; c < 3; ++c) {
		const int q = c ? qp_chroma(qp + x->sh->qpc_delta[c - 1]) : qp;
		x->scale[c] = level_scale[q % 6] << (q / 6);
	}
}

/* the record arrays of the picture */
static h265r_tu_t *new_tu(sctx_t *x)
{
	h265_dec_t *d = x->d;
	if ((size_t)d->pic.n_tu >= d->cap_tu) {
		size_t cap = d->cap_tu ? 2 * d->cap_tu : 4096;
		h265r_tu_t *n = (h265r_tu_t *)realloc(d->pic.tu, cap * sizeof(h265r_tu_t));
		if (!n) H265_ERR(x->e);
		d->pic.tu = n;
		d->cap_tu = cap;
	}
	h265r_tu_t *t = &d->pic.tu[d->pic.n_tu++];
	memset(t, 0, sizeof(*t));
	return t;
}

static uint32_t new_coef(sctx_t *x, int n)
{
	h265_dec_t *d = x->d;
	if ((size_t)(d->pic.n_coef + n) > d->cap_coef) {
		size_t cap = d->cap_coef ? 2 * d->cap_coef : (1u << 20);
		while (cap < (size_t)(d->pic.n_coef + n)) cap *= 2;
		int16_t *nc = (int16_t *)realloc(d->pic.coef, cap * sizeof(int16_t));
		if (!nc) H265_ERR(x->e);
		d->pic.coef = nc;
		d->cap_coef = cap;
	}
	const uint32_t off = (uint32_t)d->pic.n_coef;
	d->pic.n_coef += n;
	return off;
}

/* map the 4x4 units of a block (plane 0 luma, 1 chroma) to record t */
static void map_block(sctx_t *x, int plane, int px, int py, int log2, int t)
{
	h265_dec_t *d = x->d;
	const int W4 = plane ? d->frame_w / 8 : d->frame_w / 4;
	int32_t *m = d->pic.map + (plane ? (size_t)(d->frame_w / 4) * (size_t)(d->frame_h / 4) : 0);
	const int n = 1 << (log2 - 2);
	for (int j = 0; j < n; ++j)
		for (int i = 0; i < n; ++i) m[(size_t)((py >> 2) + j) * (size_t)W4 + (size_t)((px >> 2) + i)] = t;
}

/* scan orders (6.5.3 - 6.5.5): position k -> (x, y) packed x | y << 4, for 2x2 / 4x4 / 8x8 blocks */
static uint8_t scan_pos[3][4][64]; /* [scanIdx][log2 1..3 -> 0..2 used][k] */
static pthread_once_t scan_once = PTHREAD_ONCE_INIT;

/* sig_coeff_flag context offsets (9.3.4.2.5) by [size class: 4x4 / 8x8 diagonal (and chroma 8x8) / 8x8
 * horizontal-vertical / 16+][chroma][prev csbf pattern 0..3][a sub-block other than the first][scan]
 * [scan position k 0..15], H265_CTX_SIG-relative (chroma's +27 included): one table read per
 * coefficient instead of the derivation's branches */
static uint8_t sig_ctx_tab[4][2][4][2][3][16];

static void build_sig_ctx(void)
{
	for (int cls = 0; cls < 4; ++cls)
		for (int ch = 0; ch < 2; ++ch)
			for (int prev = 0; prev < 4; ++prev)
				for (int nf = 0; nf < 2; ++nf)
					for (int scan = 0; scan < 3; ++scan)
						for (int k = 0; k < 16; ++k) {
							const int xp = scan_pos[scan][2][k] & 15, yp = scan_pos[scan][2][k] >> 4;
							int sctx;
							if (cls == 0) {
								static const uint8_t m4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
								sctx = m4[(yp << 2) + xp];
							} else if (!nf && xp + yp == 0) {
								sctx = 0;
							} else {
								if (prev == 0) sctx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
								else if (prev == 1) sctx = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
								else if (prev == 2) sctx = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
								else sctx = 2;
								if (!ch) {
									if (nf) sctx += 3;
									sctx += (cls == 1) ? 9 : (cls == 2 ? 15 : 21);
								} else {
									sctx += (cls == 3) ? 12 : 9;
								}
							}
							sig_ctx_tab[cls][ch][prev][nf][scan][k] = (uint8_t)(sctx + (ch ? 27 : 0));
						}
}

static void build_scans(void)
{
	for (int l = 1; l <= 3; ++l) {
		const int n = 1 << l;
		int k = 0;
		/* up-right diagonal */
		for (int s = 0; s <= 2 * (n - 1); ++s)
			for (int y = s; y >= 0; --y) {
				const int xx = s - y;
				if (y < n && xx < n) scan_pos[0][l][k++] = (uint8_t)(xx | (y << 4));
			}
		k = 0;
		for (int y = 0; y < n; ++y)
			for (int xx = 0; xx < n; ++xx) scan_pos[1][l][k++] = (uint8_t)(xx | (y << 4)); /* horizontal */
		k = 0;
		for (int xx = 0; xx < n; ++xx)
			for (int y = 0; y < n; ++y) scan_pos[2][l][k++] = (uint8_t)(xx | (y << 4)); /* vertical */
	}
	build_sig_ctx();
}

/* scanIdx from the intra mode (order_map, h265.cpp:2235-2244) */
static int order_map(int mode)
{
	if (mode >= 6 && mode <= 14) return 2;
	if (mode >= 22 && mode <= 30) return 1;
	return 0;
}

static inline int16_t sat16(int v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }

/* residual_coding (h265.cpp:2186-2233, spec 7.3.8.11): the dequantised coefficients of one block into
 * x->blk (raster, zeroed), and the residual kind the reference's transform dispatch picks for them */
static int residual_coding(sctx_t *x, int log2, int cidx, int scan, int is_intra)
{
	cab_t *c = &x->c;
	const int n = 1 << log2, chroma = cidx > 0;
	int tskip = 0;
	int last_x, last_y;
	uint32_t xy_or = 0;
	memset(x->blk, 0, sizeof(int16_t) * (size_t)(n * n));
	if (g_dump) memset(x->lev, 0, sizeof(int) * (size_t)(n * n));
	if (log2 == 2 && x->p->transform_skip) tskip = cab_decision(c, H265_CTX_TSKIP + chroma);
	{
		/* last_sig_coeff_x/y_prefix, then the suffixes */
		const int off = chroma ? 15 : 3 * (log2 - 2) + ((log2 - 1) >> 2);
		const int shift = chroma ? log2 - 2 : (log2 + 1) >> 2;
		const int max = 2 * log2 - 1;
		int px = 0, py = 0;
		while (px < max && cab_decision(c, H265_CTX_LAST_X + off + (px >> shift))) px++;
		while (py < max && cab_decision(c, H265_CTX_LAST_Y + off + (py >> shift))) py++;
		last_x = px;
		last_y = py;
		if (px > 3) last_x = (1 << ((px >> 1) - 1)) * (2 + (px & 1)) + (int)cab_bypass_n(c, (px >> 1) - 1);
		if (py > 3) last_y = (1 << ((py >> 1) - 1)) * (2 + (py & 1)) + (int)cab_bypass_n(c, (py >> 1) - 1);
		if (scan == 2) {
			const int t = last_x;
			last_x = last_y;
			last_y = t;
		}
	}
	{
		const int lsb = log2 - 2;                 /* subblocks per side: 1 << lsb */
		const uint8_t *sbscan = scan_pos[scan][lsb ? lsb : 1];
		const uint8_t *inscan = scan_pos[scan][2];
		uint8_t csbf[8][8];
		int last_sb = 0, last_pos = 0, greater1ctx = 1;
		const int scale = x->scale[cidx];
		/* size class of the sig_coeff_flag contexts (sig_ctx_tab); chroma 8x8 counts as diagonal */
		const int cls = log2 == 2 ? 0 : (log2 == 3 ? ((scan == 0 || chroma) ? 1 : 2) : 3);
		const int rnd = 1 << (log2 - 2), sh = log2 - 1;
		memset(csbf, 0, sizeof(csbf));
		/* the subblock and in-subblock scan positions of the last coefficient */
		{
			const int sbn = 1 << (2 * lsb);
			for (int k = 0; k < sbn; ++k) {
				const int sx = lsb ? (sbscan[k] & 15) : 0, sy = lsb ? (sbscan[k] >> 4) : 0;
				if (sx == (last_x >> 2) && sy == (last_y >> 2)) last_sb = k;
			}
			for (int k = 0; k < 16; ++k)
				if ((inscan[k] & 15) == (last_x & 3) && (inscan[k] >> 4) == (last_y & 3)) last_pos = k;
		}
		for (int i = last_sb; i >= 0; --i) {
			const int xs = lsb ? (sbscan[i] & 15) : 0, ys = lsb ? (sbscan[i] >> 4) : 0;
			int prev = 0, coded, infer_dc = 0;
			if (xs + 1 < (1 << lsb)) prev |= csbf[ys][xs + 1];
			if (ys + 1 < (1 << lsb)) prev |= csbf[ys + 1][xs] << 1;
			if (i < last_sb && i > 0) {
				coded = cab_decision(c, H265_CTX_CSBF + ((prev & 1) | (prev >> 1)) + (chroma ? 2 : 0));
				infer_dc = 1;
			} else {
				coded = 1;
			}
			csbf[ys][xs] = (uint8_t)coded;
			if (!coded) continue;
			/* sig_coeff_flag (9.3.4.2.5) for scan positions in the subblock, highest first */
			int sig_pos[16], nsig = 0;
			const uint8_t *const sctab = sig_ctx_tab[cls][chroma][prev][xs + ys > 0][scan];
			for (int k = (i == last_sb) ? last_pos : 15; k >= 0; --k) {
				int sig;
				if (i == last_sb && k == last_pos) {
					sig = 1;
				} else if (k == 0 && infer_dc && nsig == 0) {
					sig = 1;
				} else {
					sig = cab_decision(c, H265_CTX_SIG + sctab[k]);
				}
				if (sig) sig_pos[nsig++] = k;
			}
			if (nsig == 0) continue;
			/* greater1 / greater2 (h265.cpp:1593-1623) */
			int lvl[16], need_rem = 0, first_g1 = -1;
			{
				const int ctxset = ((!chroma && i != 0) ? 2 : 0) + (greater1ctx == 0);
				const int g1off = ctxset * 4 + (chroma ? 16 : 0);
				greater1ctx = 1;
				for (int j = 0; j < nsig; ++j) {
					lvl[j] = 1;
					if (j < 8) {
						if (cab_decision(c, H265_CTX_GT1 + g1off + greater1ctx)) {
							greater1ctx = 0;
							lvl[j] = 2;
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
					if (cab_decision(c, H265_CTX_GT2 + ctxset + (chroma ? 4 : 0))) {
						lvl[first_g1] = 3;
						need_rem |= 1 << first_g1;
					}
				}
			}
			const int hide = x->p->sign_hiding && (sig_pos[0] - sig_pos[nsig - 1] > 3);
			const uint32_t signs = cab_bypass_n(c, nsig - hide);
			uint32_t smask = 1u << (nsig - 1 - hide);
			int rice = 0, sum = 0, last_raster = 0;
			for (int j = 0; j < nsig; ++j) {
				int a = lvl[j];
				if (need_rem & (1 << j)) {
					/* coeff_abs_level_remaining (h265.cpp:1335-1348) */
					int pfx = cab_bypass_ones(c);
					if (pfx < 0) { /* 16 or more 1s: bin by bin up to the cap */
						pfx = 0;
						while (pfx < 20 && cab_bypass(c)) pfx++;
					}
					if (pfx < 4) a += (pfx << rice) + (int)cab_bypass_n(c, rice);
					else a += (1 << (pfx - 4 + rice + 1)) + (2 << rice) + (int)cab_bypass_n(c, pfx - 4 + rice + 1);
					if (a > (3 << rice) && rice < 4) rice++;
				}
				sum += a;
				const int k = sig_pos[j];
				const int xc = (xs << 2) + (inscan[k] & 15), yc = (ys << 2) + (inscan[k] >> 4);
				const int raster = yc * n + xc;
				const int neg = (signs & smask) != 0;
				smask >>= 1;
				if (g_dump) x->lev[raster] = neg ? -a : a;
				/* scaling_default_base (h265.cpp:1681-1684): level * scale, rounded, >> (log2 - 1), int16 */
				{
					const int v = neg ? -a : a;
					x->blk[raster] = sat16((v * scale + rnd) >> sh);
				}
				xy_or |= (uint32_t)raster;
				last_raster = raster;
			}
			if (hide && (sum & 1)) {
				x->blk[last_raster] = (int16_t)-x->blk[last_raster];
				if (g_dump) x->lev[last_raster] = -x->lev[last_raster];
			}
		}
	}
	if (g_dump) {
		fprintf(g_dump, "res c%d l%d s%d t%d:", cidx, log2, scan, tskip);
		for (int i = 0; i < n * n; ++i)
			if (x->lev[i]) fprintf(g_dump, " %d@%d", x->lev[i], i);
		fprintf(g_dump, "\n");
	}
	if (tskip) return H265R_RES_SKIP;
	if (is_intra && cidx == 0 && log2 == 2) return H265R_RES_DST;
	return xy_or == 0 ? H265R_RES_DC : H265R_RES_FULL;
}

static void put_residual(sctx_t *x, h265r_tu_t *t, int k, int log2, int kind)
{
	const int n = 1 << (2 * log2);
	t->res[k] = (uint8_t)kind;
	t->coef[k] = new_coef(x, n);
	memcpy(x->d->pic.coef + t->coef[k], x->blk, sizeof(int16_t) * (size_t)n);
}

/* deblocking edges of a transform block (record_tu_intra, h265modules.h:491-503, 618-625) */
static void record_tu_edges(sctx_t *x, int x0, int y0, int log2)
{
	h265_dec_t *d = x->d;
	const int n = 1 << (log2 - 2);
	const uint8_t v = (uint8_t)((x->qp_y << 2) | 2); /* (qpP + qpQ + 1) >> 1 with one QP per slice */
	if (x->sh->deblocking_disabled) return;
	if (!(x0 & 7) && x0 > 0)
		for (int j = 0; j < n; ++j) d->pic.bs_v[(size_t)((y0 >> 2) + j) * (size_t)(d->frame_w / 8) + (size_t)(x0 >> 3)] = v;
	if (!(y0 & 7) && y0 > 0)
		for (int i = 0; i < n; ++i) d->pic.bs_h[(size_t)(y0 >> 3) * (size_t)(d->frame_w / 4) + (size_t)((x0 >> 2) + i)] = v;
}

/* transform_tree (h265.cpp:2919-2956, 3026-3075): intra */
static void transform_tree(sctx_t *x, int x0, int y0, int log2, int depth, int cbf_cbcr, int vx, int vy, int ua, int blk,
                           int pred_idx, int *cparent)
{
	const h265_sps_t *s = x->s;
	cab_t *c = &x->c;
	int split, cbf = 0;
	if (s->log2_max_tb < log2) split = 1;
	else if (depth == 0 && x->intra_split) split = 2;
	else split = (s->log2_min_tb < log2 && depth < s->max_th_depth_intra) ? cab_decision(c, H265_CTX_SPLIT_TRANSFORM + 5 - log2) : 0;
	if (log2 > 2) {
		if (cbf_cbcr & 2) cbf |= cab_decision(c, H265_CTX_CBF_CHROMA + depth) << 1;
		if (cbf_cbcr & 1) cbf |= cab_decision(c, H265_CTX_CBF_CHROMA + depth);
	} else {
		cbf = cbf_cbcr;
	}
	if (split) {
		const int h = 1 << (log2 - 1);
		int pi = split == 2 ? 0 : pred_idx;
		const int pinc = split == 2 ? 1 : 0;
		int cidx = -1;
		if (log2 - 1 == 2) {
			/* 4x4 luma children: the 4x4 chroma block is predicted here, its residual comes with child 3 */
			h265r_tu_t *t = new_tu(x);
			cidx = (int)(t - x->d->pic.tu);
			t->x = (uint16_t)(x0 >> 1);
			t->y = (uint16_t)(y0 >> 1);
			t->log2 = 2;
			t->plane = 1;
			t->mode = (uint8_t)x->order_chroma;
			t->flags = H265R_TU_PRED;
			t->avail_top = (int16_t)((ua & 2) ? -1 : (vx >> 1));
			t->avail_left = (int16_t)((ua & 1) ? -1 : (vy >> 1));
			map_block(x, 1, x0 >> 1, y0 >> 1, 2, cidx);
		}
		transform_tree(x, x0, y0, log2 - 1, depth + 1, cbf, vx, vy, ua, 0, pi, &cidx);
		pi += pinc;
		transform_tree(x, x0 + h, y0, log2 - 1, depth + 1, cbf, vx - h, imin(vy, h), ua & ~1, 1, pi, &cidx);
		pi += pinc;
		transform_tree(x, x0, y0 + h, log2 - 1, depth + 1, cbf, imin(vx, 2 * h), vy - h, ua & ~2, 2, pi, &cidx);
		pi += pinc;
		transform_tree(x, x0 + h, y0 + h, log2 - 1, depth + 1, cbf, imin(vx - h, h), imin(vy - h, h), 0, 3, pi, &cidx);
		return;
	}
	/* a leaf: intra prediction records (intra_prediction, h265.cpp:2906-2913), then the residual */
	int ly, lc = -1;
	{
		h265r_tu_t *t = new_tu(x);
		ly = (int)(t - x->d->pic.tu);
		t->x = (uint16_t)x0;
		t->y = (uint16_t)y0;
		t->log2 = (uint8_t)log2;
		t->plane = 0;
		t->mode = (uint8_t)x->order_luma[pred_idx];
		t->flags = H265R_TU_PRED;
		t->strong = (uint8_t)s->strong_intra_smoothing;
		t->avail_top = (int16_t)((ua & 2) ? -1 : vx);
		t->avail_left = (int16_t)((ua & 1) ? -1 : vy);
		map_block(x, 0, x0, y0, log2, ly);
	}
	if (log2 > 2) {
		h265r_tu_t *t = new_tu(x);
		lc = (int)(t - x->d->pic.tu);
		t->x = (uint16_t)(x0 >> 1);
		t->y = (uint16_t)(y0 >> 1);
		t->log2 = (uint8_t)(log2 - 1);
		t->plane = 1;
		t->mode = (uint8_t)x->order_chroma;
		t->flags = H265R_TU_PRED;
		t->avail_top = (int16_t)((ua & 2) ? -1 : (vx >> 1));
		t->avail_left = (int16_t)((ua & 1) ? -1 : (vy >> 1));
		map_block(x, 1, x0 >> 1, y0 >> 1, log2 - 1, lc);
	}
	cbf = cbf * 2 | cab_decision(c, H265_CTX_CBF_LUMA + (depth == 0));
	/* transform_unit (h265.cpp:2246-2270) */
	if (cbf & 1) {
		const int scan = log2 <= 3 ? order_map(x->order_luma[pred_idx]) : 0;
		const int kind = residual_coding(x, log2, 0, scan, 1);
		put_residual(x, &x->d->pic.tu[ly], 0, log2, kind);
	}
	if (cbf & 6) {
		int cl = log2 - 1, target = lc;
		if (log2 == 2) {
			cl = 2;
			target = (blk == 3) ? *cparent : -1;
		}
		if (target >= 0) {
			const int scan = cl == 2 ? order_map(x->order_chroma) : 0;
			if (cbf & 4) put_residual(x, &x->d->pic.tu[target], 0, cl, residual_coding(x, cl, 1, scan, 0));
			if (cbf & 2) put_residual(x, &x->d->pic.tu[target], 1, cl, residual_coding(x, cl, 2, scan, 0));
		}
	}
	record_tu_edges(x, x0, y0, log2);
}

/* MPM candidates (intra_pred_candidate, h265.cpp:1385-1409) */
static void mpm_cands(int a, int b, int cand[3])
{
	if (a == b) {
		if (a < 2) {
			cand[0] = 0;
			cand[1] = 1;
			cand[2] = 26;
		} else {
			cand[0] = a;
			cand[1] = ((a - 3) & 31) + 2;
			cand[2] = ((a - 1) & 31) + 2;
		}
	} else {
		cand[0] = a;
		cand[1] = b;
		cand[2] = (a != 0 && b != 0) ? 0 : ((a != 1 && b != 1) ? 1 : 26);
	}
}

/* cu_header_intra + pred_intra (h265.cpp:4016-4059) */
static void coding_unit(sctx_t *x, int x0, int y0, int log2, int vx, int vy, int ua)
{
	h265_dec_t *d = x->d;
	cab_t *c = &x->c;
	const int W4 = x->W4;
	int part = 1, flags = 0;
	for (int j = 0; j < (1 << (log2 - 2)); ++j)
		memset(d->cb_log2 + (size_t)((y0 >> 2) + j) * (size_t)W4 + (size_t)(x0 >> 2), log2, (size_t)1 << (log2 - 2));
	x->intra_split = 0;
	if (log2 == x->s->log2_min_cb && cab_decision(c, H265_CTX_PART_MODE) == 0) {
		x->intra_split = 1;
		part = 4;
	}
	if (x->s->pcm && log2 >= x->s->log2_min_pcm && log2 <= x->s->log2_max_pcm) H265_ERR(x->e); /* pcm_flag: h265.cpp:4023-4025 */
	for (int i = 0; i < part; ++i) flags |= cab_decision(c, H265_CTX_PREV_INTRA_LUMA) << i;
	{
		const int pl = part == 4 ? log2 - 1 : log2; /* PU size */
		for (int i = 0; i < part; ++i) {
			const int px = x0 + ((i & 1) << pl), py = y0 + ((i >> 1) << pl);
			int cand[3], mode;
			const int a = px > 0 ? d->ipm[(size_t)(py >> 2) * (size_t)W4 + (size_t)((px >> 2) - 1)] : 1;
			const int b = (py > 0 && ((py - 1) >> x->s->log2_ctb) == (py >> x->s->log2_ctb))
			                  ? d->ipm[(size_t)((py >> 2) - 1) * (size_t)W4 + (size_t)(px >> 2)]
			                  : 1;
			mpm_cands(a, b, cand);
			if (flags & (1 << i)) {
				const int idx = cab_bypass(c) ? 1 + cab_bypass(c) : 0;
				mode = cand[idx];
			} else {
				int t;
				mode = (int)cab_bypass_n(c, 5);
				/* ascending candidates */
				if (cand[0] > cand[1]) { t = cand[0]; cand[0] = cand[1]; cand[1] = t; }
				if (cand[0] > cand[2]) { t = cand[0]; cand[0] = cand[2]; cand[2] = t; }
				if (cand[1] > cand[2]) { t = cand[1]; cand[1] = cand[2]; cand[2] = t; }
				for (int k = 0; k < 3; ++k) mode += (cand[k] <= mode);
			}
			x->order_luma[i] = mode;
			for (int j = 0; j < (1 << (pl - 2)); ++j)
				memset(d->ipm + (size_t)((py >> 2) + j) * (size_t)W4 + (size_t)(px >> 2), mode, (size_t)1 << (pl - 2));
		}
		if (part != 4) x->order_luma[1] = x->order_luma[2] = x->order_luma[3] = x->order_luma[0];
	}
	{
		/* intra_chroma_pred_mode (h265.cpp:1282-1288) and its direction (intra_chroma_pred_dir, :1367-1383) */
		const int idx = cab_decision(c, H265_CTX_INTRA_CHROMA) ? (int)cab_bypass_n(c, 2) : 4;
		const int lm = x->order_luma[0];
		static const int base[4] = {0, 26, 10, 1};
		x->order_chroma = idx == 4 ? lm : (base[idx] == lm ? 34 : base[idx]);
	}
	if (g_dump)
		fprintf(g_dump, "cu %d %d l%d p%d m %d %d %d %d c%d\n", x0, y0, log2, part, x->order_luma[0], x->order_luma[1],
		        x->order_luma[2], x->order_luma[3], x->order_chroma);
	transform_tree(x, x0, y0, log2, 0, 3, vx, vy, ua, 0, 0, NULL);
}

/* coding_quadtree (quad_tree, h265.cpp:4100-4123) */
static void quad_tree(sctx_t *x, int x0, int y0, int log2, int vx, int vy, int ua)
{
	h265_dec_t *d = x->d;
	if (vx <= 0 || vy <= 0) return;
	if (x->s->log2_min_cb < log2) {
		int split = vx < (1 << log2) || vy < (1 << log2);
		if (!split) {
			const int W4 = x->W4;
			const int l = x0 > 0 ? d->cb_log2[(size_t)(y0 >> 2) * (size_t)W4 + (size_t)((x0 >> 2) - 1)] : 0;
			const int t = y0 > 0 ? d->cb_log2[(size_t)((y0 >> 2) - 1) * (size_t)W4 + (size_t)(x0 >> 2)] : 0;
			const int inc = (l && l < log2) + (t && t < log2);
			split = cab_decision(&x->c, H265_CTX_SPLIT_CU + inc);
		}
		if (split) {
			const int h = 1 << (log2 - 1);
			quad_tree(x, x0, y0, log2 - 1, vx, vy, ua);
			quad_tree(x, x0 + h, y0, log2 - 1, vx - h, imin(vy, h), ua & ~1);
			quad_tree(x, x0, y0 + h, log2 - 1, imin(vx, 2 * h), vy - h, ua & ~2);
			quad_tree(x, x0 + h, y0 + h, log2 - 1, imin(vx - h, h), imin(vy - h, h), 0);
			return;
		}
	}
	coding_unit(x, x0, y0, log2, vx, vy, ua);
}

/* sao (h265.cpp:1017-1130) into the picture's per-CTU record, merges resolved */
static void sao_syntax(sctx_t *x, int cx, int cy)
{
	cab_t *c = &x->c;
	const int cols = x->s->ctb_cols;
	h265r_sao_t *sa = &x->d->pic.sao[(size_t)cy * (size_t)cols + (size_t)cx];
	memset(sa, 0, sizeof(*sa));
	if (!x->sh->sao_luma && !x->sh->sao_chroma) return;
	if (cx > 0 && cab_decision(c, H265_CTX_SAO_MERGE)) {
		*sa = sa[-1];
		return;
	}
	if (cy > 0 && cab_decision(c, H265_CTX_SAO_MERGE)) {
		*sa = sa[-cols];
		return;
	}
	for (int ci = 0; ci < 3; ++ci) {
		if (ci == 0 ? !x->sh->sao_luma : !x->sh->sao_chroma) continue;
		int type;
		if (ci == 2) {
			type = sa->type[1];
		} else {
			type = cab_decision(c, H265_CTX_SAO_TYPE) ? 1 + cab_bypass(c) : 0;
		}
		sa->type[ci] = (uint8_t)type;
		if (!type) continue;
		for (int j = 0; j < 4; ++j) {
			int v = 0;
			while (v < 7 && cab_bypass(c)) v++;
			sa->off[ci][j] = (int8_t)v;
		}
		if (type == 1) {
			for (int j = 0; j < 4; ++j)
				if (sa->off[ci][j] && cab_bypass(c)) sa->off[ci][j] = (int8_t)-sa->off[ci][j];
			sa->band[ci] = (uint8_t)cab_bypass_n(c, 5);
		} else {
			if (ci == 0) sa->eo[0] = (uint8_t)cab_bypass_n(c, 2);
			if (ci == 1) sa->eo[1] = (uint8_t)cab_bypass_n(c, 2);
			if (ci == 2) sa->eo[2] = sa->eo[1];
			sa->off[ci][2] = (int8_t)-sa->off[ci][2];
			sa->off[ci][3] = (int8_t)-sa->off[ci][3];
		}
	}
}

/* grow the per-picture arrays to the frame geometry */
static void pic_arrays(perr_t *e, int fw, int fh, int cols, int rows)
{
	h265_dec_t *d = e->d;
	const size_t units = (size_t)(fw / 4) * (size_t)(fh / 4);
	const size_t nmap = units + (size_t)(fw / 8) * (size_t)(fh / 8);
	const size_t nbs = (size_t)(fh / 4) * (size_t)(fw / 8);
	if (nmap > d->cap_map) {
		free(d->pic.map);
		d->pic.map = (int32_t *)malloc(nmap * sizeof(int32_t));
		d->cap_map = d->pic.map ? nmap : 0;
	}
	if (nbs > d->cap_bs) {
		free(d->pic.bs_v);
		free(d->pic.bs_h);
		d->pic.bs_v = (uint8_t *)malloc(nbs);
		d->pic.bs_h = (uint8_t *)malloc(nbs);
		d->cap_bs = (d->pic.bs_v && d->pic.bs_h) ? nbs : 0;
	}
	if ((size_t)(cols * rows) > d->cap_sao) {
		free(d->pic.sao);
		d->pic.sao = (h265r_sao_t *)malloc(sizeof(h265r_sao_t) * (size_t)(cols * rows));
		d->cap_sao = d->pic.sao ? (size_t)(cols * rows) : 0;
	}
	if (units > d->cap_units) {
		free(d->cb_log2);
		free(d->ipm);
		d->cb_log2 = (uint8_t *)malloc(units);
		d->ipm = (uint8_t *)malloc(units);
		d->cap_units = (d->cb_log2 && d->ipm) ? units : 0;
	}
	if (!d->cap_map || !d->cap_bs || !d->cap_sao || !d->cap_units) H265_ERR(e);
	memset(d->pic.map, 0xff, nmap * sizeof(int32_t));
	memset(d->pic.bs_v, 0, nbs);
	memset(d->pic.bs_h, 0, nbs);
	memset(d->cb_log2, 0, units);
	memset(d->ipm, 1, units);
}

/* slice_data (h265.cpp:4735-4845) of an I slice */
static void slice_data(perr_t *e, const h265_sps_t *s, const h265_pps_t *p, const uint8_t *data, const uint8_t *end)
{
	h265_dec_t *d = e->d;
	sctx_t *x = (sctx_t *)malloc(sizeof(sctx_t));
	if (!x) H265_ERR(e);
	memset(x, 0, offsetof(sctx_t, blk));
	x->e = e;
	x->d = d;
	x->s = s;
	x->p = p;
	x->sh = &d->sh;
	x->W4 = d->frame_w / 4;
	set_qp(x, d->sh.slice_qp);
	cab_init_ctx(&x->c, 0, d->sh.slice_qp);
	cab_start(&x->c, data, end);
	{
		const int ctb = 1 << s->log2_ctb;
		int addr = d->sh.address;
		for (;;) {
			const int cx = addr % s->ctb_cols, cy = addr / s->ctb_cols;
			const int x0 = cx << s->log2_ctb, y0 = cy << s->log2_ctb;
			/* availability at the CTU (coding_tree_unit, h265.cpp:4738): left / top inside the slice */
			const int idx = addr - d->sh.address;
			const int ua = ((cy == 0 || idx < s->ctb_cols) ? 2 : 0) | ((cx == 0 || idx == 0) ? 1 : 0);
			sao_syntax(x, cx, cy);
			quad_tree(x, x0, y0, s->log2_ctb, s->pic_w - x0, imin(s->pic_h - y0, ctb), ua);
			addr++;
			if (addr >= s->ctb_cols * s->ctb_rows) break;
			if (cab_terminate(&x->c)) break;
		}
		if (addr < s->ctb_cols * s->ctb_rows) { /* the slice ended early: only whole pictures are handled */
			free(x);
			H265_ERR(e);
		}
		if (g_dump && !cab_terminate(&x->c)) fprintf(g_dump, "error: end_of_slice_segment_flag 0\n");
	}
	d->cabac_bins += x->c.bins;
	free(x);
}

/* ------------------------------------------------------------------ frames and output (h265.cpp:152-220, 4931-5008) */
static int dpb_has(const h265_dec_t *d, int idx)
{
	for (int i = 0; i < d->dpb_size; ++i)
		if (d->dpb[i].frame_idx == idx) return 1;
	return 0;
}

static void find_empty_frame(h265_dec_t *d)
{
	int max_idx = 0, max_val = -1;
	for (int i = 0; i < d->num_frames; ++i) d->lru[i] = dpb_has(d, i) ? 0 : (int8_t)(d->lru[i] + 1);
	for (int i = 0; i < d->num_frames; ++i)
		if (max_val < d->lru[i]) {
			max_val = d->lru[i];
			max_idx = i;
		}
	d->lru[max_idx] = 0;
	d->index = max_idx;
}

static void insert_dpb(h265_dec_t *d, int frame_idx, int poc, int is_idr)
{
	int size = d->dpb_size, pos;
	if (d->dpb_max <= size) {
		size -= 1;
		d->dpb_output = d->dpb[0].frame_idx;
	} else {
		d->dpb_output = -1;
	}
	pos = 0;
	if (size > 0) {
		while (pos < size && !(poc < d->dpb[pos].poc)) pos++;
		memmove(&d->dpb[pos + 1], &d->dpb[pos], sizeof(d->dpb[0]) * (size_t)(size - pos));
	}
	d->dpb[pos].frame_idx = (int8_t)frame_idx;
	d->dpb[pos].poc = poc;
	d->dpb[pos].is_idr = (uint8_t)is_idr;
	d->dpb_size = size + 1;
}

/* slice_layer (h265.cpp:4849-4866) */
static void slice_layer(perr_t *e, int nal_type)
{
	h265_dec_t *d = e->d;
	h264_bits_t b;
	h265_slice_t *sh = &d->sh;
	hb_init(&b, d->unit + 2, d->unit_len - 2);
	sh->nal_type = nal_type;
	sh->first_slice = (int)hb_get1(&b);
	if (!sh->first_slice) H265_ERR(e); /* one slice per picture (see the header comment) */
	if (!d->num_frames) H265_ERR(e);
	find_empty_frame(d);
	if (nal_type >= H265_BLA_W_LP && nal_type <= H265_RSV_IRAP_23) sh->no_output_of_prior_pics = (int)hb_get1(&b);
	sh->pps_id = ue_max(e, &b, 63);
	{
		const h265_pps_t *p = &d->pps[sh->pps_id];
		const h265_sps_t *s = &d->sps[p->sps_id];
		if (!p->valid || !s->valid) H265_ERR(e);
		if (s->stride != d->frame_w || (s->ctb_rows << s->log2_ctb) != d->frame_h) H265_ERR(e);
		parse_slice_header(e, &b, s, p);
		/* the frame's geometry as the reference sets it in ctu_init (h265.cpp:4776-4783) */
		{
			m2d_frame_t *f = &d->frames[d->index];
			f->width = (int16_t)s->stride;
			f->height = (int16_t)(s->ctb_rows << s->log2_ctb);
			f->crop[0] = (int16_t)s->crop[0];
			f->crop[1] = (int16_t)(s->crop[1] + f->width - s->pic_w);
			f->crop[2] = (int16_t)s->crop[2];
			f->crop[3] = (int16_t)(s->crop[3] + f->height - s->pic_h);
		}
		pic_arrays(e, d->frame_w, d->frame_h, s->ctb_cols, s->ctb_rows);
		if (g_dump) fprintf(g_dump, "pic %d\n", d->pictures);
		d->pic.n_tu = 0;
		d->pic.n_coef = 0;
		{
			const size_t pos = (size_t)(b.p - (d->unit + 2)) - (size_t)(b.bits >> 3);
			slice_data(e, s, p, d->unit + 2 + pos, d->unit + d->unit_len);
		}
		{
			h265r_picture_t *pic = &d->pic;
			pic->width = d->frame_w;
			pic->height = d->frame_h;
			pic->pic_w = s->pic_w;
			pic->pic_h = s->pic_h;
			pic->ctb_log2 = s->log2_ctb;
			pic->slot = d->index;
			pic->flags = (sh->deblocking_disabled ? 0 : H265R_PIC_DEBLOCK) | (sh->sao_luma ? H265R_PIC_SAO_LUMA : 0) |
			             (sh->sao_chroma ? H265R_PIC_SAO_CHROMA : 0);
			pic->beta_offset = sh->beta_offset_div2 * 2;
			pic->tc_offset = sh->tc_offset_div2 * 2;
			pic->cb_qp_offset = p->cb_qp_offset;
			pic->cr_qp_offset = p->cr_qp_offset;
			if (!d->have_be || d->be.submit(d->be.self, pic) < 0) H265_ERR(e);
		}
	}
	d->pictures++;
	insert_dpb(d, d->index, sh->poc, nal_type == H265_IDR_W_RADL || nal_type == H265_IDR_N_LP);
}

/* ------------------------------------------------------------------ m2d_func_table_t */
static h265_dec_t *CTX(void *p) { return (h265_dec_t *)p; }

static int hdr_dummy(void *a, void *b)
{
	(void)a;
	(void)b;
	return 0;
}

static int api_init(void *ctx, int dpb_max, int (*cb)(void *, void *), void *arg)
{
	h265_dec_t *d = CTX(ctx);
	(void)dpb_max; /* (the reference ignores it too: h265.cpp:57-68) */
	if (!d || !m2dec_host_cpu_ok) return -1;
	memset(d, 0, sizeof(*d));
	pthread_once(&scan_once, build_scans);
	if (!g_dump_init) {
		const char *p = getenv("M2DEC_AMD_H265_DUMP");
		g_dump_init = 1;
		if (p) g_dump = fopen(p, "w");
	}
	d->header_callback = cb ? cb : hdr_dummy;
	d->header_callback_arg = arg;
	d->dpb_max = 16;
	d->dpb_output = -1;
	d->device = 0;
	dec_bits_open(&d->stream_i, NULL);
	return 0;
}

static dec_bits *api_stream_pos(void *ctx) { return &CTX(ctx)->stream_i; }

/* h265d_get_info (h265.cpp:132-151): the SPS of pps[slice_header.pps_id] */
static int api_get_info(void *ctx, m2d_info_t *info)
{
	h265_dec_t *d = CTX(ctx);
	if (!d || !info) return -1;
	const h265_sps_t *s = &d->sps[d->pps[d->sh.pps_id].sps_id];
	const int w = s->ctb_cols << s->log2_ctb, h = s->ctb_rows << s->log2_ctb;
	info->src_width = (int16_t)w;
	info->src_height = (int16_t)h;
	info->disp_width = (int16_t)w;
	info->disp_height = (int16_t)h;
	info->frame_num = (int16_t)s->frame_num;
	info->crop[0] = (int16_t)s->crop[0];
	info->crop[1] = (int16_t)(w - s->pic_w + s->crop[1]);
	info->crop[2] = (int16_t)s->crop[2];
	info->crop[3] = (int16_t)(h - s->pic_h + s->crop[3]);
	info->additional_size = 16; /* (the reference's second frame holds its line buffers: none needed here) */
	return 0;
}

static int api_set_frames(void *ctx, int n, m2d_frame_t *frames, uint8_t *work, int work_len)
{
	h265_dec_t *d = CTX(ctx);
	(void)work_len;
	if (!d || n < 1 || !frames || !work) return -1;
	const h265_sps_t *s = &d->sps[d->pps[d->sh.pps_id].sps_id];
	d->num_frames = imin(n, H265R_MAX_FRAMES);
	memcpy(d->frames, frames, sizeof(m2d_frame_t) * (size_t)d->num_frames);
	memset(d->lru, 0, sizeof(d->lru));
	d->dpb_max = 16;
	d->dpb_size = 0;
	d->dpb_output = -1;
	d->frame_w = s->ctb_cols << s->log2_ctb;
	d->frame_h = s->ctb_rows << s->log2_ctb;
	if (!d->have_be) {
		if (h265_hip_backend_create(&d->be, d->device) < 0) {
			fprintf(stderr, "m2dec_amd: no gfx950 device for the H.265 reconstruction\n");
			return -1;
		}
		d->have_be = 1;
	}
	return d->be.set_frames(d->be.self, d->num_frames, d->frames, d->frame_w, d->frame_h);
}

/* h265d_decode_picture (h265.cpp:4898-4920) */
static int api_decode_picture(void *ctx)
{
	h265_dec_t *d = CTX(ctx);
	jmp_buf jb;
	perr_t e;
	if (!d) return -1;
	e.d = d;
	e.jb = &jb;
	if (setjmp(jb)) return -2;
	for (;;) {
		if (next_unit(d) < 0 || d->unit_len < 2) H265_ERR(&e);
		const int type = (d->unit[0] >> 1) & 63;
		h264_bits_t b;
		hb_init(&b, d->unit + 2, d->unit_len - 2);
		switch (type) {
		case H265_TRAIL_N:
		case H265_TRAIL_R:
		case H265_IDR_W_RADL:
			slice_layer(&e, type);
			return 1;
		case H265_SPS:
			parse_sps(&e, &b);
			d->header_callback(d->header_callback_arg, d->stream_i.id);
			break;
		case H265_PPS:
			parse_pps(&e, &b);
			break;
		default: /* VPS, AUD, SEI, other slice types: nothing the decode uses (h265.cpp:4878-4894) */
			break;
		}
	}
}

static int peek_idx(h265_dec_t *d, int bypass)
{
	if (d->dpb_size <= 0) return -1;
	return bypass ? d->dpb[0].frame_idx : d->dpb_output;
}

static int api_peek(void *ctx, m2d_frame_t *frame, int bypass)
{
	h265_dec_t *d = CTX(ctx);
	if (!d || !frame) return -1;
	const int idx = peek_idx(d, bypass);
	if (idx < 0) return 0;
	if (d->have_be && d->be.sync_frame(d->be.self, idx) < 0) return -1;
	*frame = d->frames[idx];
	return 1;
}

static int api_get(void *ctx, m2d_frame_t *frame, int bypass)
{
	h265_dec_t *d = CTX(ctx);
	const int r = api_peek(ctx, frame, bypass);
	if (r < 0) return -1;
	if (d->dpb_size > 0) { /* force_pop_dpb, whether a frame was returned or not (h265.cpp:4969-4976, 5000-5008) */
		memmove(&d->dpb[0], &d->dpb[1], sizeof(d->dpb[0]) * (size_t)d->dpb_size);
		d->dpb_size--;
		d->dpb_output = -1;
	}
	return r;
}

static const m2d_func_table_t h265d_func_ = {
	sizeof(h265_dec_t), api_init, api_stream_pos, api_get_info, api_set_frames, api_decode_picture, api_peek, api_get,
};

const m2d_func_table_t *const h265d_func = &h265d_func_;

/* ------------------------------------------------------------------ extra C ABI */
int m2dec_amd_h265_set_backend(void *ctx, const h265r_backend_t *be)
{
	h265_dec_t *d = CTX(ctx);
	if (!d) return -1;
	if (!be) {
		d->have_be = 0;
		return 0;
	}
	if (d->have_be && d->be.destroy) d->be.destroy(d->be.self);
	d->be = *be;
	d->have_be = 1;
	return 0;
}

int m2dec_amd_h265_set_device(void *ctx, int device)
{
	h265_dec_t *d = CTX(ctx);
	if (!d || device < 0) return -1;
	d->device = device;
	return 0;
}

void m2dec_amd_h265_release(void *ctx)
{
	h265_dec_t *d = CTX(ctx);
	if (!d) return;
	if (g_dump) fflush(g_dump);
	if (d->have_be && d->be.destroy) d->be.destroy(d->be.self);
	d->have_be = 0;
	free(d->unit);
	free(d->pic.tu);
	free(d->pic.coef);
	free(d->pic.map);
	free(d->pic.bs_v);
	free(d->pic.bs_h);
	free(d->pic.sao);
	free(d->cb_log2);
	free(d->ipm);
	d->unit = NULL;
	d->unit_cap = 0;
	memset(&d->pic, 0, sizeof(d->pic));
	d->cap_tu = d->cap_coef = d->cap_map = d->cap_bs = d->cap_sao = d->cap_units = 0;
	d->cb_log2 = d->ipm = NULL;
}

/* test hook: write the parsed syntax of every later H.265 context to `path` (NULL: stop) */
int m2dec_amd_h265_set_dump(const char *path)
{
	if (g_dump) fclose(g_dump);
	g_dump = path ? fopen(path, "w") : NULL;
	g_dump_init = 1;
	return path && !g_dump ? -1 : 0;
}

uint64_t m2dec_amd_h265_cabac_bins(const void *ctx) { return ctx ? ((const h265_dec_t *)ctx)->cabac_bins : 0; }
