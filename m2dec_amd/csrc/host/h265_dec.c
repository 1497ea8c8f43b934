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
#define _GNU_SOURCE /* pthread_setname_np */
#include <limits.h>
#include <pthread.h>
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "h264_dec.h" /* bit reader (hb_*) and the CABAC range tables, shared with the H.264 parser */
#include "h265_dec.h"

int m2d_stream_next_byte(dec_bits *st); /* bitio.c */
extern int m2dec_host_cpu_ok;           /* cpucheck.c */

#define H265_ERR(d) longjmp(*(d)->jb, 1)

/* M2DEC_AMD_H265_DUMP=path: the parsed syntax in tools/h265gen --dump's format (tests/test_h265_cpu.py
 * compares the two), and a check that each slice's CABAC data ends with end_of_slice_segment_flag = 1 */
static FILE *g_dump;
static int g_dump_init;

/* coverage counters of the inter derivation (tests/test_h265_cpu.py: which paths the goldens exercise) */
enum { H265_HIT_MERGE_SPATIAL, H265_HIT_MERGE_TEMPORAL, H265_HIT_MERGE_COMBINED, H265_HIT_MERGE_ZERO, H265_HIT_NO_BIDIR,
       H265_HIT_MVP_A, H265_HIT_MVP_B, H265_HIT_MVP_SCALED, H265_HIT_MVP_TEMPORAL, H265_HIT_MVP_ZERO, H265_HIT_BI,
       H265_HIT_LOWDELAY, H265_HIT_NOT_LOWDELAY, H265_HIT_COL_STALE, H265_HIT_BS_MOTION, H265_HIT_INTRA_CU, H265_HIT_N };
static long g_hits[H265_HIT_N];
#define HIT(k) __atomic_fetch_add(&g_hits[k], 1, __ATOMIC_RELAXED)

int m2dec_amd_h265_parser_hits(long *out, int n, int reset)
{
	for (int i = 0; i < n && i < H265_HIT_N; ++i) out[i] = __atomic_load_n(&g_hits[i], __ATOMIC_RELAXED);
	if (reset)
		for (int i = 0; i < H265_HIT_N; ++i) __atomic_store_n(&g_hits[i], 0, __ATOMIC_RELAXED);
	return H265_HIT_N;
}

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

/* find_frame_idx_from_dpb (h265.cpp:785-793): by POC in the output DPB, data[0]'s frame (or 0) otherwise */
static int find_frame_idx(const h265_dec_t *d, int poc)
{
	for (int i = 0; i < d->dpb_size; ++i)
		if (d->dpb[i].poc == poc) return d->dpb[i].frame_idx;
	return d->dpb_size ? d->dpb[0].frame_idx : 0;
}

/* init_ref_pic_list_short_lx (h265.cpp:795-809): entries of one RPS side from list position `at`; unused
 * entries are skipped but counted, and keep what the list held (the lists persist across slices) */
static int ref_list_side(h265_dec_t *d, int lx, int at, int side, int rest)
{
	h265_slice_t *sh = &d->sh;
	unsigned used = sh->rps.used[side];
	int i;
	for (i = 0; i < sh->rps.num_pics[side] && i < rest; ++i) {
		if (used & 1) {
			const int poc = sh->poc + sh->rps.delta_poc[side][i];
			sh->ref_poc[lx][at + i] = poc;
			sh->ref_frame[lx][at + i] = (int8_t)find_frame_idx(d, poc);
		}
		used >>= 1;
	}
	return i;
}

/* init_ref_pic_list (h265.cpp:811-820), as written: every round restarts the list's own side at entry 0 */
static void init_ref_lists(perr_t *e)
{
	h265_slice_t *sh = &e->d->sh;
	if (sh->rps.num_pics[0] + sh->rps.num_pics[1] == 0) H265_ERR(e); /* (the reference loops forever) */
	for (int lx = 0; lx < 2; ++lx) {
		const int num = imax(sh->num_ref_idx[lx], sh->rps.total_curr);
		int idx = 0;
		while (idx < num) {
			idx += ref_list_side(e->d, lx, 0, lx, num - idx);
			idx += ref_list_side(e->d, lx, idx, lx ^ 1, num - idx);
		}
	}
}

/* slice_header_nonintra (h265.cpp:822-856).  Fields a slice does not code keep the previous slice's value,
 * as in the reference (collocated_ref_idx, cabac_init_flag, mvd_l1_zero_flag, num_ref_idx of L1 in P) */
static void slice_header_inter(perr_t *e, h264_bits_t *b, const h265_sps_t *s, const h265_pps_t *p)
{
	h265_slice_t *sh = &e->d->sh;
	const int bslice = sh->slice_type == 0;
	if (hb_get1(b)) {
		sh->num_ref_idx[0] = ue_max(e, b, 14) + 1;
		if (bslice) sh->num_ref_idx[1] = ue_max(e, b, 14) + 1;
	} else {
		sh->num_ref_idx[0] = p->num_ref_idx_default[0];
		sh->num_ref_idx[1] = p->num_ref_idx_default[1];
	}
	if (p->lists_modification && sh->rps.total_curr > 1) H265_ERR(e); /* assert(0) in the reference */
	init_ref_lists(e);
	if (bslice) sh->mvd_l1_zero = (int)hb_get1(b);
	if (p->cabac_init_present) sh->cabac_init_flag = (int)hb_get1(b);
	if (sh->temporal_mvp) {
		const int l0 = bslice ? (int)hb_get1(b) : 1;
		sh->col_from_l0 = l0;
		if (l0 && sh->num_ref_idx[0] > 1) sh->col_ref_idx = ue_max(e, b, (uint32_t)sh->num_ref_idx[0] - 1);
		else if (!l0 && sh->num_ref_idx[1] > 1) sh->col_ref_idx = ue_max(e, b, (uint32_t)sh->num_ref_idx[1] - 1);
		else if (sh->col_ref_idx) HIT(H265_HIT_COL_STALE);
	}
	if ((bslice && p->weighted_bipred) || (sh->slice_type == 1 && p->weighted_pred)) H265_ERR(e); /* assert(0) */
	sh->max_merge_cand = 5 - ue_max(e, b, 4);
	/* the merge-level test compares CTU-relative positions (h265.cpp:3597-3599); a conformant level is at
	 * most the CTB size, where absolute positions give the same answer */
	if (p->log2_parallel_merge_level > s->log2_ctb) H265_ERR(e);
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
	if (sh->slice_type != 2) slice_header_inter(e, b, s, p);
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
	/* P / B slices */
	int inter, bslice;
	int lowdelay;              /* no frame's POC above the current one (colpics_t::update_lowdelay) */
	int16_t colmv[8][8], tmv[8][8]; /* temporal_mvscale_t over the 8 frames' POCs (h265modules.h:684-708) */
	const h265_col_t *col_ref; /* the collocated picture's motion field */
	const int8_t (*col_lists)[16]; /* ... and the frames of its reference lists (frameidx_record_t) */
	h265_col_t *col_cur;       /* the current picture's motion field */
	int col_stride;
	struct h265_job *job;      /* parse-ahead: the job this parse runs for (CTU-row hooks), NULL sequentially */
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

/* ------------------------------------------------------------------ P / B coding units (h265.cpp:3012-4123) */
/* The reference keeps what later blocks read of a block in left / top neighbour arrays per CTU; every read
 * it makes of them (for positions its availability bits allow) is the block at that picture position, so
 * here they are one map of 4x4 units (d->nb) addressed by position.  Positions outside the picture read
 * the arrays' initial state (neighbour_init, h265.cpp:4743-4750: intra, not skipped). */
static const h265_nb_t nb_outside = {1, 0, 0, 0, 0, 0, {{{0, 0}, {0, 0}}, {-1, -1}}};

static inline h265_nb_t *nb_at(sctx_t *x, int px, int py)
{
	if (px < 0 || py < 0 || px >= x->s->pic_w || py >= x->s->pic_h) return (h265_nb_t *)&nb_outside;
	return &x->d->nb[(size_t)(py >> 2) * (size_t)x->W4 + (size_t)(px >> 2)];
}

/* the 4x4 units of a rectangle inside the picture */
#define NB_RECT(x, px, py, w, h, u, body)                                                                      \
	for (int yy_ = (py); yy_ < (py) + (h) && yy_ < (x)->s->pic_h; yy_ += 4)                                  \
		for (int xx_ = (px); xx_ < (px) + (w) && xx_ < (x)->s->pic_w; xx_ += 4) {                            \
			h265_nb_t *u = &(x)->d->nb[(size_t)(yy_ >> 2) * (size_t)(x)->W4 + (size_t)(xx_ >> 2)];       \
			body;                                                                                     \
		}

/* colpics_t::fill (h265modules.h:835-850): the 16x16 units whose top-left sample the block covers */
static void col_fill(sctx_t *x, int px, int py, int w, int h, int intra, const h265_pred_t *pred)
{
	for (int y = (py + 15) & ~15; y < py + h; y += 16)
		for (int xx = (px + 15) & ~15; xx < px + w; xx += 16) {
			h265_col_t *c = &x->col_cur[(size_t)(y >> 4) * (size_t)x->col_stride + (size_t)(xx >> 4)];
			c->intra = (uint8_t)intra;
			if (!intra) c->pred = *pred;
		}
}

/* temporal_mvscale_t::scale (h265modules.h:685-696) */
static int16_t tmv_scale_of(int poc0, int refpoc0, int poc1, int refpoc1)
{
	const int diff1 = poc1 - refpoc1, diff0 = poc0 - refpoc0;
	if (diff1 == 0) return 4096;
	const int td = diff1 < -128 ? -128 : (diff1 > 127 ? 127 : diff1), tb = diff0 < -128 ? -128 : (diff0 > 127 ? 127 : diff0);
	const int tx = (16384 + (abs(td) >> 1)) / td;
	const int v = (tb * tx + 32) >> 6;
	return (int16_t)(v < -4096 ? -4096 : (v > 4095 ? 4095 : v));
}

/* scale_mv (h265.cpp:3622-3631) */
static int16_t scale_mv(int mv, int scale)
{
	int v = mv * scale;
	if (v >= 0) {
		v = (v + 127) >> 8;
		return (int16_t)(v <= 32767 ? v : 32767);
	}
	v = -((127 - v) >> 8);
	return (int16_t)(v >= -32768 ? v : -32768);
}

/* frameidx_record_t::frameidx (h265modules.h:667-669) of the current slice's lists */
static inline int cur_frame(const sctx_t *x, int lx, int ref) { return x->sh->ref_frame[lx][ref] & 7; }

/* colpics_t::get_ref (h265modules.h:793-807): the bottom-right 16x16 unit if it is inside the CTU row and the
 * picture and not intra, else the centre unit */
static const h265_col_t *col_get(const sctx_t *x, int px, int py, int w, int h)
{
	const int ctb = x->s->log2_ctb;
	int bx = px + w, by = py + h;
	if (!((((py & ((1 << ctb) - 1)) + h) >> ctb)) && bx < x->s->pic_w && by < x->s->pic_h) {
		const h265_col_t *r = &x->col_ref[(size_t)(by >> 4) * (size_t)x->col_stride + (size_t)(bx >> 4)];
		if (!r->intra) return r;
	}
	bx = px + (w >> 1);
	by = py + (h >> 1);
	return &x->col_ref[(size_t)(by >> 4) * (size_t)x->col_stride + (size_t)(bx >> 4)];
}

/* add_colpic_candidate (h265.cpp:3633-3645) */
static void add_col(const sctx_t *x, h265_pred_t *pred, const h265_col_t *col, int lx, int ref_idx)
{
	int col_lx = x->lowdelay ? lx : x->sh->col_from_l0;
	int col_ref = col->pred.ref[col_lx];
	if (col_ref < 0) {
		col_lx ^= 1;
		col_ref = col->pred.ref[col_lx];
	}
	pred->ref[lx] = (int8_t)ref_idx;
	const int sc = x->colmv[cur_frame(x, lx, ref_idx)][x->col_lists[col_lx][col_ref] & 7];
	pred->mv[lx][0] = scale_mv(col->pred.mv[col_lx][0], sc);
	pred->mv[lx][1] = scale_mv(col->pred.mv[col_lx][1], sc);
}

/* add_merge_candidate (h265.cpp:3597-3610) */
static void add_merge(sctx_t *x, h265_pred_t *list, int *num, int px, int py, int nx, int ny)
{
	const h265_nb_t *n = nb_at(x, nx, ny);
	const int s = x->p->log2_parallel_merge_level;
	if (n->pu_intra || ((px >> s) == (nx >> s) && (py >> s) == (ny >> s))) return;
	for (int i = 0; i < *num; ++i)
		if (!memcmp(&n->pred, &list[i], sizeof(h265_pred_t))) return;
	list[(*num)++] = n->pred;
}

/* the merge candidate merge_idx selects (prediction_unit_merge, h265.cpp:3685-3721) */
static void merge_cand(sctx_t *x, int ua, int px, int py, int w, int h, int idx, h265_pred_t *out)
{
	h265_pred_t list[5];
	int num = 0, spatial;
	memset(list, 0, sizeof(list));
	if (!(ua & 1)) add_merge(x, list, &num, px, py, px - 1, py + h - 1);
	if (num <= idx) {
		if (!(ua & 2)) add_merge(x, list, &num, px, py, px + w - 1, py - 1);
		if (!(ua & 8)) add_merge(x, list, &num, px, py, px + w, py - 1);
		if (!(ua & 4)) add_merge(x, list, &num, px, py, px - 1, py + h);
		if (num <= idx && num < 4) add_merge(x, list, &num, px, py, px - 1, py - 1); /* (no availability test) */
	}
	spatial = num;
	if (num <= idx && x->sh->temporal_mvp) { /* add_colpic_candidate_merge (:3647-3656) */
		const h265_col_t *col = col_get(x, px, py, w, h);
		if (!col->intra) {
			add_col(x, &list[num], col, 0, 0);
			if (x->bslice) add_col(x, &list[num], col, 1, 0);
			else list[num].ref[1] = -1; /* (left uninitialised in a P slice by the reference: the spec's value) */
			num++;
		}
	}
	const int temporal_end = num;
	if (num > 1 && num <= idx && x->bslice) { /* add_merge_combind_candidate (:3658-3683) */
		static const int8_t l0_cand[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
		const int cutoff = num * (num - 1);
		for (int c = 0; c < cutoff; ++c) {
			const int i0 = l0_cand[c], i1 = l0_cand[c ^ 1];
			if (idx <= i0 || idx <= i1) break;
			const h265_pred_t a = list[i0], bb = list[i1];
			if (a.ref[0] >= 0 && bb.ref[1] >= 0) {
				if (memcmp(a.mv[0], bb.mv[1], sizeof(a.mv[0])) || x->sh->ref_poc[0][a.ref[0]] != x->sh->ref_poc[1][bb.ref[1]]) {
					memcpy(list[num].mv[0], a.mv[0], sizeof(a.mv[0]));
					memcpy(list[num].mv[1], bb.mv[1], sizeof(a.mv[0]));
					list[num].ref[0] = a.ref[0];
					list[num].ref[1] = bb.ref[1];
					if (idx < ++num) break;
				}
			}
		}
	}
	const int combined_end = num;
	HIT(idx < spatial ? H265_HIT_MERGE_SPATIAL
	                  : (idx < temporal_end ? H265_HIT_MERGE_TEMPORAL : (idx < combined_end ? H265_HIT_MERGE_COMBINED : H265_HIT_MERGE_ZERO)));
	while (num <= idx) { /* merge_zero_mv (:3612-3620): the selected one always takes reference 0 */
		const int nref = x->bslice ? imin(x->sh->num_ref_idx[0], x->sh->num_ref_idx[1]) : x->sh->num_ref_idx[0];
		const int m = idx - num, r = m < nref ? m : 0;
		list[num].ref[0] = (int8_t)r;
		list[num].ref[1] = (int8_t)(x->bslice ? r : -1);
		memset(list[num].mv, 0, sizeof(list[num].mv));
		num++;
	}
	*out = list[idx];
}

/* mvp2nd (h265.cpp:3755-3767) */
static void mvp2nd(const sctx_t *x, int lx, int ref_idx, const h265_pred_t *n, int16_t dst[2])
{
	int lxi = lx;
	for (int l = 0; l < 2; ++l) {
		const int nr = n->ref[lxi];
		if (nr >= 0) {
			const int sc = x->tmv[cur_frame(x, lx, ref_idx)][cur_frame(x, lxi, nr)];
			dst[0] = scale_mv(n->mv[lxi][0], sc);
			dst[1] = scale_mv(n->mv[lxi][1], sc);
			break;
		}
		lxi ^= 1;
	}
}

/* find_spatial_mvp (h265.cpp:3769-3790) */
static const int16_t *find_spatial_mvp(const sctx_t *x, const h265_nb_t *n, int lx, int refpoc, int ref_idx, int16_t m2[2],
                                       int *skip2nd, int *match2nd)
{
	if (n->pu_intra) return NULL;
	int lxi = lx;
	for (int li = 0; li < 2; ++li) {
		if (n->pred.ref[lxi] >= 0) {
			if (x->sh->ref_poc[lxi][n->pred.ref[lxi]] == refpoc) {
				*skip2nd = 1;
				return n->pred.mv[lxi];
			} else if (!*skip2nd && !*match2nd) {
				mvp2nd(x, lx, ref_idx, &n->pred, m2);
				*match2nd = 1;
			}
		}
		lxi ^= 1;
	}
	*skip2nd = 1;
	return NULL;
}

/* mvp_one_dir (h265.cpp:3792-3819): side 0 = A0, A1; side 1 = B0, B1 and (left and top available) B2 */
static const int16_t *mvp_one_dir(sctx_t *x, int ua, int side, int px, int py, int w, int h, int lx, int ref_idx, int16_t m2[2],
                                  int *skip2nd)
{
	const int dir = side ? ua >> 1 : ua;
	const int refpoc = x->sh->ref_poc[lx][ref_idx];
	int match2nd = 0;
	const int16_t *mv;
	if (!(dir & 4)) {
		mv = find_spatial_mvp(x, side ? nb_at(x, px + w, py - 1) : nb_at(x, px - 1, py + h), lx, refpoc, ref_idx, m2, skip2nd, &match2nd);
		if (mv) return mv;
	}
	if (!(dir & 1)) {
		mv = find_spatial_mvp(x, side ? nb_at(x, px + w - 1, py - 1) : nb_at(x, px - 1, py + h - 1), lx, refpoc, ref_idx, m2, skip2nd,
		                      &match2nd);
		if (mv) return mv;
	}
	if (side && !(ua & 3)) {
		mv = find_spatial_mvp(x, nb_at(x, px - 1, py - 1), lx, refpoc, ref_idx, m2, skip2nd, &match2nd);
		if (mv) return mv;
	}
	return match2nd ? m2 : NULL;
}

/* add_mvp (h265.cpp:3742-3753) */
static int add_mvp(const int16_t mv[2], int16_t list[2][2], int mvp_idx, int *n)
{
	const int16_t a = mv[0], b = mv[1];
	for (int i = 0; i < *n; ++i)
		if (list[i][0] == a && list[i][1] == b) return 0;
	list[*n][0] = a;
	list[*n][1] = b;
	return mvp_idx < ++*n;
}

/* calc_mv (h265.cpp:3821-3839) */
static void calc_mv(sctx_t *x, int ua, int px, int py, int w, int h, int lx, int ref_idx, int mvp_idx, const int mvd[2],
                    const h265_col_t *col, int16_t out[2])
{
	int16_t list[2][2], m2[2] = {0, 0};
	int n = 0, skip2nd = 0;
	const int16_t *mvp = mvp_one_dir(x, ua, 0, px, py, w, h, lx, ref_idx, m2, &skip2nd);
	int hit = H265_HIT_MVP_A;
	if (!mvp || !add_mvp(mvp, list, mvp_idx, &n)) {
		mvp = mvp_one_dir(x, ua, 1, px, py, w, h, lx, ref_idx, m2, &skip2nd);
		hit = H265_HIT_MVP_B;
		if (!mvp || !add_mvp(mvp, list, mvp_idx, &n)) {
			h265_pred_t t;
			int ok = 0;
			hit = H265_HIT_MVP_TEMPORAL;
			if (col) {
				add_col(x, &t, col, lx, ref_idx);
				ok = add_mvp(t.mv[lx], list, mvp_idx, &n);
			}
			if (!ok) {
				memset(list[n], 0, sizeof(list[0]) * (size_t)(2 - n));
				hit = H265_HIT_MVP_ZERO;
			}
		}
	}
	HIT(hit);
	if (mvp == m2) HIT(H265_HIT_MVP_SCALED);
	out[0] = (int16_t)(mvd[0] + list[mvp_idx][0]);
	out[1] = (int16_t)(mvd[1] + list[mvp_idx][1]);
}

/* deblocking strengths of a prediction block's left / top edges (h265d_deblocking_t::record_pu,
 * h265modules.h:504-582, 636-642): written over whatever the edge held */
static inline int mv_big(const int16_t a[2], const int16_t b[2])
{
	const int dx = a[0] - b[0], dy = a[1] - b[1];
	return dx * dx >= 16 || dy * dy >= 16;
}

static int pu_strength_motion(const sctx_t *x, const h265_nb_t *n, const int16_t cmv[2][2], int cf0, int cf1, int c_sw);

static int pu_strength(const sctx_t *x, const h265_nb_t *n, const int16_t cmv[2][2], int cf0, int cf1, int c_sw)
{
	if (n->pu_intra) return 2;
	if (n->pu_nz) return 1;
	int r = pu_strength_motion(x, n, cmv, cf0, cf1, c_sw);
	if (r) HIT(H265_HIT_BS_MOTION);
	return r;
}

static int pu_strength_motion(const sctx_t *x, const h265_nb_t *n, const int16_t cmv[2][2], int cf0, int cf1, int c_sw)
{
	int nf0 = n->pred.ref[0] >= 0 ? x->sh->ref_frame[0][n->pred.ref[0]] : -1;
	int nf1 = n->pred.ref[1] >= 0 ? x->sh->ref_frame[1][n->pred.ref[1]] : -1;
	int n_sw = 0;
	if (nf0 < nf1) {
		const int t = nf0;
		nf0 = nf1;
		nf1 = t;
		n_sw = 1;
	}
	/* inter_strength (:532-542), called with the two swap flags exchanged (h265modules.h:559) */
	const int a_sw = c_sw, b_sw = n_sw;
	if (nf0 != cf0 || nf1 != cf1) return 1;
	if (nf0 == nf1)
		return (mv_big(n->pred.mv[0], cmv[0]) || mv_big(n->pred.mv[1], cmv[1])) && (mv_big(n->pred.mv[0], cmv[1]) || mv_big(n->pred.mv[1], cmv[0]));
	return (nf0 >= 0 && mv_big(n->pred.mv[a_sw], cmv[b_sw])) || (nf1 >= 0 && mv_big(n->pred.mv[a_sw ^ 1], cmv[b_sw ^ 1]));
}

static void record_pu(sctx_t *x, int px, int py, int w, int h, int r0, int r1, const int16_t mv[2][2])
{
	h265_dec_t *d = x->d;
	if (x->sh->deblocking_disabled) return;
	int f0 = r0 >= 0 ? x->sh->ref_frame[0][r0] : -1, f1 = r1 >= 0 ? x->sh->ref_frame[1][r1] : -1, c_sw = 0;
	if (f0 < f1) {
		const int t = f0;
		f0 = f1;
		f1 = t;
		c_sw = 1;
	}
	const int q = x->qp_y << 2;
	if (!(px & 7) && px > 0)
		for (int j = 0; j < h >> 2; ++j)
			d->pic.bs_v[(size_t)((py >> 2) + j) * (size_t)(d->frame_w / 8) + (size_t)(px >> 3)] =
			    (uint8_t)(q | pu_strength(x, nb_at(x, px - 1, py + 4 * j), mv, f0, f1, c_sw));
	if (!(py & 7) && py > 0)
		for (int i = 0; i < w >> 2; ++i)
			d->pic.bs_h[(size_t)(py >> 3) * (size_t)(d->frame_w / 4) + (size_t)((px >> 2) + i)] =
			    (uint8_t)(q | pu_strength(x, nb_at(x, px + 4 * i, py - 1), mv, f0, f1, c_sw));
}

/* transform-block edges of an inter CU (record_tu, h265modules.h:507-524, 627-634): the larger of what the
 * edge holds, the block's coded luma and the neighbour's transform block */
static void record_tu_inter(sctx_t *x, int x0, int y0, int log2, int nz)
{
	h265_dec_t *d = x->d;
	const int n = 1 << (log2 - 2), q = x->qp_y << 2;
	if (x->sh->deblocking_disabled) return;
	if (!(x0 & 7) && x0 > 0)
		for (int j = 0; j < n; ++j) {
			uint8_t *e = &d->pic.bs_v[(size_t)((y0 >> 2) + j) * (size_t)(d->frame_w / 8) + (size_t)(x0 >> 3)];
			const h265_nb_t *nb = nb_at(x, x0 - 1, y0 + 4 * j);
			const int s = imax(imax(nz, nb->tu_intra ? 2 : nb->tu_nz), *e & 3);
			*e = (uint8_t)(q | s);
		}
	if (!(y0 & 7) && y0 > 0)
		for (int i = 0; i < n; ++i) {
			uint8_t *e = &d->pic.bs_h[(size_t)(y0 >> 3) * (size_t)(d->frame_w / 4) + (size_t)((x0 >> 2) + i)];
			const h265_nb_t *nb = nb_at(x, x0 + 4 * i, y0 - 1);
			const int s = imax(imax(nz, nb->tu_intra ? 2 : nb->tu_nz), *e & 3);
			*e = (uint8_t)(q | s);
		}
}

/* one prediction block out: the motion compensation record, deblocking, the neighbour map and the motion field */
static void emit_pu(sctx_t *x, int px, int py, int w, int h, int r0, int r1, const int16_t mv[2][2])
{
	h265_dec_t *d = x->d;
	if ((size_t)d->pic.n_pu >= d->cap_pu) {
		const size_t cap = d->cap_pu ? 2 * d->cap_pu : 4096;
		h265r_pu_t *n = (h265r_pu_t *)realloc(d->pic.pu, cap * sizeof(h265r_pu_t));
		if (!n) H265_ERR(x->e);
		d->pic.pu = n;
		d->cap_pu = cap;
	}
	h265r_pu_t *u = &d->pic.pu[d->pic.n_pu++];
	u->x = (uint16_t)px;
	u->y = (uint16_t)py;
	u->w = (uint8_t)w;
	u->h = (uint8_t)h;
	u->ref[0] = (int8_t)(r0 >= 0 ? x->sh->ref_frame[0][r0] : -1);
	u->ref[1] = (int8_t)(r1 >= 0 ? x->sh->ref_frame[1][r1] : -1);
	memcpy(u->mv, mv, sizeof(u->mv));
	if (r0 < 0) memset(u->mv[0], 0, sizeof(u->mv[0]));
	if (r1 < 0) memset(u->mv[1], 0, sizeof(u->mv[1]));
}

/* prediction_unit_merge (h265.cpp:3685-3721) with merge_pred (:3572-3595) */
static void merge_pu(sctx_t *x, int ua, int px, int py, int w, int h)
{
	cab_t *c = &x->c;
	h265_pred_t p;
	{
		const int max = x->sh->max_merge_cand;
		int idx = 0;
		if (max > 1 && cab_decision(c, H265_CTX_MERGE_IDX)) { /* merge_idx (:1143-1155) */
			for (idx = 1; idx < max - 1; ++idx)
				if (!cab_bypass(c)) break;
		}
		merge_cand(x, ua, px, py, w, h, idx, &p);
		const int no_bidir = p.ref[0] >= 0 && p.ref[1] >= 0 && w + h == 12;
		if (no_bidir) HIT(H265_HIT_NO_BIDIR);
		else if (p.ref[0] >= 0 && p.ref[1] >= 0) HIT(H265_HIT_BI);
		const int r0 = p.ref[0], r1 = (no_bidir || (p.ref[0] < 0 && p.ref[1] < 0)) ? -1 : p.ref[1];
		emit_pu(x, px, py, w, h, r0, r1, (const int16_t(*)[2])p.mv);
		record_pu(x, px, py, w, h, r0, no_bidir ? -1 : p.ref[1], (const int16_t(*)[2])p.mv);
		{ /* copy_predinfo (:3119-3130) */
			h265_pred_t q = p;
			if (no_bidir) q.ref[1] = -1;
			NB_RECT(x, px, py, w, h, u, {
				u->pu_nz = 0;
				u->pu_intra = 0;
				u->skip = 1;
				u->pred = q;
			})
		}
		col_fill(x, px, py, w, h, 0, &p);
		if (g_dump)
			fprintf(g_dump, "pu %d %d %d %d m%d r %d %d mv %d %d %d %d\n", px, py, w, h, idx, p.ref[0], no_bidir ? -1 : p.ref[1], p.mv[0][0],
			        p.mv[0][1], p.mv[1][0], p.mv[1][1]);
	}
}

/* prediction_unit (h265.cpp:3905-3931): 1 if merged */
static int prediction_unit(sctx_t *x, int log2, int ua, int px, int py, int w, int h, int pred_ua)
{
	cab_t *c = &x->c;
	h265_pred_t p;
	if (cab_decision(c, H265_CTX_MERGE_FLAG)) {
		merge_pu(x, ua | pred_ua, px, py, w, h);
		return 1;
	}
	int pred_idc = 0;
	if (x->bslice) { /* inter_pred_idc (:1210-1216) */
		const int depth = x->s->log2_ctb - log2;
		if (w + h != 12 && cab_decision(c, H265_CTX_INTER_PRED_IDC + depth)) pred_idc = 2;
		else pred_idc = cab_decision(c, H265_CTX_INTER_PRED_IDC + 4);
	}
	/* the collocated block (a null one dereferenced by the reference when TMVP is off: none here) */
	const h265_col_t *col = x->sh->temporal_mvp ? col_get(x, px, py, w, h) : NULL;
	if (col && col->intra) col = NULL;
	int16_t mv[2][2] = {{0, 0}, {0, 0}};
	int ref[2] = {-1, -1};
	for (int lx = 0; lx < 2; ++lx) {
		if (pred_idc == (lx ^ 1)) continue; /* L0 only: no L1; L1 only: no L0 */
		int r = 0;
		const int num = x->sh->num_ref_idx[lx] - 1;
		if (num > 0) { /* ref_idx_lx (:1218-1237) */
			const int m2 = imin(num, 2);
			for (r = 0; r < m2; ++r)
				if (!cab_decision(c, H265_CTX_REF_IDX + r)) break;
			if (r == m2)
				for (; r < num; ++r)
					if (!cab_bypass(c)) break;
		}
		int mvd[2] = {0, 0};
		if (lx == 0 || pred_idc == 1 || !x->sh->mvd_l1_zero) { /* mvd_coding (:3723-3740) */
			int a0 = cab_decision(c, H265_CTX_ABS_MVD_GT), a1 = cab_decision(c, H265_CTX_ABS_MVD_GT);
			if (a0) a0 += cab_decision(c, H265_CTX_ABS_MVD_GT + 1);
			if (a1) a1 += cab_decision(c, H265_CTX_ABS_MVD_GT + 1);
			int v[2] = {a0, a1};
			for (int k = 0; k < 2; ++k) {
				if (!v[k]) continue;
				if (v[k] > 1) { /* abs_mvd_minus2: EG1 (:1243-1247) */
					int bits = 0;
					while (cab_bypass(c)) bits++;
					v[k] += (2 << bits) - 2 + (int)cab_bypass_n(c, bits + 1);
				}
				if (cab_bypass(c)) v[k] = -v[k];
			}
			mvd[0] = v[0];
			mvd[1] = v[1];
		}
		const int mvp_idx = cab_decision(c, H265_CTX_MVP_FLAG);
		ref[lx] = r;
		calc_mv(x, ua, px, py, w, h, lx, r, mvp_idx, mvd, col, mv[lx]);
	}
	if (pred_idc == 2) HIT(H265_HIT_BI);
	emit_pu(x, px, py, w, h, ref[0], ref[1], (const int16_t(*)[2])mv);
	record_pu(x, px, py, w, h, ref[0], ref[1], (const int16_t(*)[2])mv);
	p.ref[0] = (int8_t)ref[0];
	p.ref[1] = (int8_t)ref[1];
	memcpy(p.mv, mv, sizeof(mv));
	NB_RECT(x, px, py, w, h, u, { /* fill_pred (:3851-3866) */
		u->pu_intra = 0;
		u->pu_nz = 0;
		u->skip = 0;
		u->pred = p;
	})
	col_fill(x, px, py, w, h, 0, &p);
	if (g_dump)
		fprintf(g_dump, "pu %d %d %d %d a%d r %d %d mv %d %d %d %d\n", px, py, w, h, pred_idc, ref[0], ref[1], mv[0][0], mv[0][1], mv[1][0],
		        mv[1][1]);
	return 0;
}

/* transform_tree of an inter CU (h265.cpp:3026-3075 with is_intra false): residual-only records */
static void transform_tree_inter(sctx_t *x, int x0, int y0, int log2, int depth, int cbf_cbcr, int blk)
{
	const h265_sps_t *s = x->s;
	cab_t *c = &x->c;
	int split, cbf = 0;
	if (s->log2_max_tb < log2) split = 1;
	else if (s->log2_min_tb < log2 && depth < s->max_th_depth_inter) split = cab_decision(c, H265_CTX_SPLIT_TRANSFORM + 5 - log2);
	else split = depth == 0 && x->intra_split;
	if (log2 > 2) {
		if (cbf_cbcr & 2) cbf |= cab_decision(c, H265_CTX_CBF_CHROMA + depth) << 1;
		if (cbf_cbcr & 1) cbf |= cab_decision(c, H265_CTX_CBF_CHROMA + depth);
	} else {
		cbf = cbf_cbcr;
	}
	if (split) {
		const int h = 1 << (log2 - 1);
		transform_tree_inter(x, x0, y0, log2 - 1, depth + 1, cbf, 0);
		transform_tree_inter(x, x0 + h, y0, log2 - 1, depth + 1, cbf, 1);
		transform_tree_inter(x, x0, y0 + h, log2 - 1, depth + 1, cbf, 2);
		transform_tree_inter(x, x0 + h, y0 + h, log2 - 1, depth + 1, cbf, 3);
		return;
	}
	cbf = cbf * 2 | ((depth || cbf) ? cab_decision(c, H265_CTX_CBF_LUMA + (depth == 0)) : 1);
	if (cbf & 1) { /* transform_unit (:2246-2270), scans all 0 (zero_scan_order) */
		h265r_tu_t *t = new_tu(x);
		const int k = (int)(t - x->d->pic.tu);
		t->x = (uint16_t)x0;
		t->y = (uint16_t)y0;
		t->log2 = (uint8_t)log2;
		map_block(x, 0, x0, y0, log2, k);
		put_residual(x, &x->d->pic.tu[k], 0, log2, residual_coding(x, log2, 0, 0, 0));
	}
	if ((cbf & 6) && (log2 > 2 || blk == 3)) {
		const int cl = log2 > 2 ? log2 - 1 : 2, cx = log2 > 2 ? x0 >> 1 : (x0 - 4) >> 1, cy = log2 > 2 ? y0 >> 1 : (y0 - 4) >> 1;
		h265r_tu_t *t = new_tu(x);
		const int k = (int)(t - x->d->pic.tu);
		t->x = (uint16_t)cx;
		t->y = (uint16_t)cy;
		t->log2 = (uint8_t)cl;
		t->plane = 1;
		map_block(x, 1, cx, cy, cl, k);
		if (cbf & 4) put_residual(x, &x->d->pic.tu[k], 0, cl, residual_coding(x, cl, 1, 0, 0));
		if (cbf & 2) put_residual(x, &x->d->pic.tu[k], 1, cl, residual_coding(x, cl, 2, 0, 0));
	}
	record_tu_inter(x, x0, y0, log2, cbf & 1);
	NB_RECT(x, x0, y0, 1 << log2, 1 << log2, u, { /* cu_inter_tu_fill (:3012-3024) */
		u->pu_nz = (uint8_t)(cbf & 1);
		u->tu_intra = 0;
		u->tu_nz = (uint8_t)(cbf & 1);
		u->pu_intra = 0;
	})
}

/* availability of the blocks of a split (h265.cpp:3933-3947): bit 1 left, 2 top, 4 bottom-left, 8 top-right */
static const int8_t av4x4[3][16] = {{0, 5, 10, 15, 0, 5, 10, 15, 0, 5, 10, 15, 0, 5, 10, 15},
                                    {4, 4, 6, 6, 4, 4, 6, 6, 12, 12, 14, 14, 12, 12, 14, 14},
                                    {0, 1, 0, 1, 4, 5, 4, 5, 0, 1, 0, 1, 4, 5, 4, 5}};
static const int8_t av2x1[2][16] = {{0, 1, 2, 3, 0, 5, 2, 7, 8, 9, 10, 11, 8, 13, 10, 15},
                                    {8, 9, 8, 9, 12, 13, 12, 13, 8, 9, 8, 9, 12, 13, 12, 13}};
static const int8_t av1x2[2][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 4, 5, 14, 15},
                                    {4, 4, 6, 6, 4, 4, 6, 6, 12, 12, 14, 14, 12, 12, 14, 14}};

/* pred_inter (h265.cpp:4061-4084) with prediction_unit_cases (:3949-4009) */
static void coding_unit_inter(sctx_t *x, int x0, int y0, int log2, int vx, int vy, int ua)
{
	h265_dec_t *d = x->d;
	cab_t *c = &x->c;
	const int len = 1 << log2;
	for (int j = 0; j < (1 << (log2 - 2)); ++j)
		memset(d->cb_log2 + (size_t)((y0 >> 2) + j) * (size_t)x->W4 + (size_t)(x0 >> 2), log2, (size_t)1 << (log2 - 2));
	{
		const int ctx = (!(ua & 1) && nb_at(x, x0 - 1, y0)->skip) + (!(ua & 2) && nb_at(x, x0, y0 - 1)->skip);
		if (cab_decision(c, H265_CTX_CU_SKIP + ctx)) { /* cu_skip_flag (:1138-1141) */
			if (g_dump) fprintf(g_dump, "icu %d %d l%d skip\n", x0, y0, log2);
			merge_pu(x, ua, x0, y0, len, len);
			NB_RECT(x, x0, y0, len, len, u, {
				u->tu_intra = 0;
				u->skip = 1;
				u->pu_nz = 0;
				u->tu_nz = 0;
			})
			return;
		}
	}
	if (cab_decision(c, H265_CTX_PRED_MODE)) { /* pred_mode_flag: intra */
		HIT(H265_HIT_INTRA_CU);
		coding_unit(x, x0, y0, log2, vx, vy, ua & 3);
		NB_RECT(x, x0, y0, len, len, u, { /* cu_intra_pred_mode_fill (:3077-3088) */
			u->tu_intra = 1;
			u->pu_intra = 1;
			u->skip = 0;
		})
		col_fill(x, x0, y0, len, len, 1, NULL);
		return;
	}
	/* part_mode (:1165-1208) */
	int part;
	{
		const int min = x->s->log2_min_cb;
		if (cab_decision(c, H265_CTX_PART_MODE)) {
			part = 0;
		} else {
			part = 2 - cab_decision(c, H265_CTX_PART_MODE + 1);
			if (min < log2) {
				if (x->s->amp && !cab_decision(c, H265_CTX_PART_MODE + 3)) part = (part + 1) * 2 + cab_bypass(c);
			} else if (log2 > 3 && part == 2) {
				part += cab_decision(c, H265_CTX_PART_MODE + 2) ^ 1;
			}
		}
	}
	if (g_dump) fprintf(g_dump, "icu %d %d l%d p%d\n", x0, y0, log2, part);
	int merged = 0;
	{
		const int hl = len >> 1, ql = len >> 2;
		switch (part) {
		case 0: merged = prediction_unit(x, log2, ua, x0, y0, len, len, 0); break;
		case 1:
			prediction_unit(x, log2, av2x1[0][ua], x0, y0, len, hl, 0);
			prediction_unit(x, log2, av2x1[1][ua], x0, y0 + hl, len, hl, 2);
			break;
		case 2:
			prediction_unit(x, log2, av1x2[0][ua], x0, y0, hl, len, 0);
			prediction_unit(x, log2, av1x2[1][ua], x0 + hl, y0, hl, len, 1);
			break;
		case 3: /* NxN (the reference's fourth block reads an unset top-left neighbour: its position here) */
			prediction_unit(x, log2, av4x4[0][ua], x0, y0, hl, hl, 0);
			prediction_unit(x, log2, av4x4[1][ua], x0 + hl, y0, hl, hl, 0);
			prediction_unit(x, log2, av4x4[2][ua], x0, y0 + hl, hl, hl, 0);
			prediction_unit(x, log2, 12, x0 + hl, y0 + hl, hl, hl, 0);
			break;
		case 4:
			prediction_unit(x, log2, av2x1[0][ua], x0, y0, len, ql, 0);
			prediction_unit(x, log2, av2x1[1][ua], x0, y0 + ql, len, len - ql, 2);
			break;
		case 5:
			prediction_unit(x, log2, av2x1[0][ua], x0, y0, len, len - ql, 0);
			prediction_unit(x, log2, av2x1[1][ua], x0, y0 + len - ql, len, ql, 2);
			break;
		case 6:
			prediction_unit(x, log2, av1x2[0][ua], x0, y0, ql, len, 0);
			prediction_unit(x, log2, av1x2[1][ua], x0 + ql, y0, len - ql, len, 1);
			break;
		default:
			prediction_unit(x, log2, av1x2[0][ua], x0, y0, len - ql, len, 0);
			prediction_unit(x, log2, av1x2[1][ua], x0 + len - ql, y0, ql, len, 1);
			break;
		}
	}
	if ((part == 0 && merged) || cab_decision(c, H265_CTX_RQT_ROOT_CBF)) {
		x->intra_split = part != 0 && x->s->max_th_depth_inter == 0;
		transform_tree_inter(x, x0, y0, log2, 0, 3, 0);
	} else {
		NB_RECT(x, x0, y0, len, len, u, { /* cu_inter_zerocoef_fill (:3101-3108) */
			u->pu_nz = 0;
			u->tu_nz = 0;
		})
	}
	NB_RECT(x, x0, y0, len, len, u, { /* cu_inter_skip_mode_fill (:3090-3099) */
		u->tu_intra = 0;
		u->skip = 0;
	})
}

/* coding_quadtree (quad_tree, h265.cpp:4100-4123); ua: the 4 availability bits of the block */
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
			quad_tree(x, x0, y0, log2 - 1, vx, vy, av4x4[0][ua]);
			quad_tree(x, x0 + h, y0, log2 - 1, vx - h, imin(vy, h), av4x4[1][ua]);
			quad_tree(x, x0, y0 + h, log2 - 1, imin(vx, 2 * h), vy - h, av4x4[2][ua]);
			quad_tree(x, x0 + h, y0 + h, log2 - 1, imin(vx - h, h), imin(vy - h, h), 12);
			return;
		}
	}
	if (x->inter) coding_unit_inter(x, x0, y0, log2, vx, vy, ua);
	else coding_unit(x, x0, y0, log2, vx, vy, ua & 3);
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
	if (units > d->cap_nb) {
		free(d->nb);
		d->nb = (h265_nb_t *)malloc(units * sizeof(h265_nb_t));
		d->cap_nb = d->nb ? units : 0;
	}
	{
		const size_t ncol = (size_t)(fw / 16) * (size_t)(fh / 16);
		if (ncol > d->cap_col) {
			int ok = 1;
			for (int i = 0; i < H265R_MAX_FRAMES; ++i) {
				free(d->col[i]);
				d->col[i] = (h265_col_t *)calloc(ncol, sizeof(h265_col_t));
				ok &= d->col[i] != NULL;
			}
			d->cap_col = ok ? ncol : 0;
		}
	}
	if (!d->cap_map || !d->cap_bs || !d->cap_sao || !d->cap_units || !d->cap_nb || !d->cap_col) H265_ERR(e);
	memset(d->pic.map, 0xff, nmap * sizeof(int32_t));
	memset(d->pic.bs_v, 0, nbs);
	memset(d->pic.bs_h, 0, nbs);
	memset(d->cb_log2, 0, units);
	memset(d->ipm, 1, units);
}

/* the temporal motion state of a P / B slice (colpics_t::init, h265modules.h:758-774) */
static void inter_setup(sctx_t *x)
{
	h265_dec_t *d = x->d;
	const h265_slice_t *sh = x->sh;
	const int cl = sh->col_from_l0 ^ 1;
	const int col_frm = sh->ref_frame[cl][sh->col_ref_idx] & 7, col_poc = sh->ref_poc[cl][sh->col_ref_idx];
	x->col_ref = d->col[col_frm];
	x->col_lists = (const int8_t(*)[16])d->col_frame[col_frm];
	for (int i = 0; i < 8; ++i)
		for (int j = 0; j < 8; ++j) {
			x->colmv[i][j] = tmv_scale_of(sh->poc, d->frame_poc[i], col_poc, d->frame_poc[j]);
			x->tmv[i][j] = tmv_scale_of(sh->poc, d->frame_poc[i], sh->poc, d->frame_poc[j]);
		}
	x->lowdelay = 1;
	for (int i = 0; i < 8; ++i)
		if (sh->poc < d->frame_poc[i]) x->lowdelay = 0;
	HIT(x->lowdelay ? H265_HIT_LOWDELAY : H265_HIT_NOT_LOWDELAY);
	/* the neighbour map starts as neighbour_init's state everywhere (only decoded positions are read) */
	for (size_t i = 0, n = (size_t)x->W4 * (size_t)(d->frame_h / 4); i < n; ++i) d->nb[i] = nb_outside;
}

static void job_row_wait(struct h265_job *j, int row);
static void job_row_done(struct h265_job *j, int rows);

/* slice_data (h265.cpp:4735-4845); job: the parse-ahead job it runs for (NULL: the caller's thread) */
static void slice_data(perr_t *e, const h265_sps_t *s, const h265_pps_t *p, const uint8_t *data, const uint8_t *end,
                       struct h265_job *job)
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
	x->inter = d->sh.slice_type < 2;
	x->bslice = d->sh.slice_type == 0;
	x->col_cur = d->col[d->index];
	x->col_stride = (s->pic_w + 15) >> 4;
	x->job = job;
	set_qp(x, d->sh.slice_qp);
	/* initType (ctu_init, h265.cpp:4756) */
	cab_init_ctx(&x->c, x->inter ? 2 - (d->sh.slice_type ^ d->sh.cabac_init_flag) : 0, d->sh.slice_qp);
	if (x->inter) {
		inter_setup(x);
	} else { /* every block of an I picture is intra in its motion field (pred_intra's colpics fill) */
		for (size_t i = 0, n = (size_t)x->col_stride * (size_t)((s->pic_h + 15) >> 4); i < n; ++i) x->col_cur[i].intra = 1;
	}
	cab_start(&x->c, data, end);
	{
		const int ctb = 1 << s->log2_ctb;
		int addr = d->sh.address;
		for (;;) {
			const int cx = addr % s->ctb_cols, cy = addr / s->ctb_cols;
			const int x0 = cx << s->log2_ctb, y0 = cy << s->log2_ctb;
			/* availability at the CTU (coding_tree_unit, h265.cpp:4738): left / top inside the slice */
			const int idx = addr - d->sh.address;
			const int ua = ((cy == 0 || idx < s->ctb_cols) ? 10 : 0) | ((cx == 0 || idx == 0) ? 5 : 0) | 4;
			/* parse ahead: the collocated picture's motion field is read up to this CTU row (TMVP) */
			if (job && (cx == 0 || idx == 0)) job_row_wait(job, cy);
			sao_syntax(x, cx, cy);
			quad_tree(x, x0, y0, s->log2_ctb, s->pic_w - x0, imin(s->pic_h - y0, ctb), ua);
			if (job && cx == s->ctb_cols - 1) job_row_done(job, cy + 1);
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
	d->fresh[max_idx] = 1;
}

static long pipe_last_seq(const h265_dec_t *d);

static void pipe_note_insert(h265_dec_t *d);

static void insert_dpb(h265_dec_t *d, int frame_idx, int poc, int is_idr)
{
	pipe_note_insert(d);
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
	d->dpb[pos].seq = pipe_last_seq(d); /* (slice_layer dispatched the picture just before) */
	d->dpb_size = size + 1;
}

/* the slice data of the picture in frame d->index into d->pic (records) and the frame's motion field: on the
 * caller's thread (job NULL) or on a parse-ahead worker over the job's private view d */
static void picture_parse(perr_t *e, const h265_sps_t *s, const h265_pps_t *p, const uint8_t *data, const uint8_t *end,
                          struct h265_job *job)
{
	h265_dec_t *d = e->d;
	const h265_slice_t *sh = &d->sh;
	pic_arrays(e, d->frame_w, d->frame_h, s->ctb_cols, s->ctb_rows);
	if (g_dump) fprintf(g_dump, "pic %d\n", d->pictures);
	d->pic.n_tu = 0;
	d->pic.n_coef = 0;
	d->pic.n_pu = 0;
	slice_data(e, s, p, data, end, job);
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
}

/* ------------------------------------------------------------------ parse ahead
 *
 * The reference decodes a picture per decode_picture call on the caller's thread (h265.cpp:4898-5008).  Here
 * the caller's thread keeps everything header-level — NAL units, parameter sets, the slice header, the frame
 * LRU, POC, reference lists, DPB and output — in the reference's order, and hands each picture's slice data
 * (the CABAC parse into records: ~10-20 ms for a 1080p picture) to a worker of the context's pool; parsed
 * pictures go to the back end in decode order, by whichever worker finishes the next one.
 *
 * A picture's parse reads one other picture's state, the collocated picture's motion field (TMVP,
 * h265modules.h:731-874), and of it only the CTU rows up to the current one (the bottom-right candidate is
 * taken inside the CTU row, else the centre): a P / B picture starts once its collocated picture's parse has
 * started and follows it row by row.  It writes its own frame's motion field, after every earlier reader and
 * writer of that field finished.  Workers never touch the caller's context memory (which the caller may
 * free): a job carries a private decoder view (slice header, frame geometry, the frames' POC / list
 * snapshots, its records and maps), copies of its SPS / PPS and its slice NAL; the motion fields and the
 * back end's copy live in the pipeline's heap state.  peek / get wait until the picture of the frame they
 * hand out was submitted.  M2DEC_AMD_H265_THREADS (default 8; 0 = the sequential path, as with the syntax
 * dump). */
#define H265_RING 16

enum { JOB_FREE, JOB_QUEUED, JOB_RUNNING, JOB_PARSED };

typedef struct h265_job {
	long seq;
	int state, err;
	h265_dec_t *w;                 /* private view: sh, index, geometry, frame_poc / col_frame, records, maps */
	h265_sps_t sps;
	h265_pps_t pps;
	uint8_t *nal;
	size_t nal_len, nal_cap, data_off;
	long after;                    /* every job up to this seq is parsed before this one starts (-1: none) */
	struct h265_job *col;          /* the job writing the collocated motion field, while in flight */
	long col_seq;
	int rows_done;                 /* CTU rows parsed; INT_MAX once the job ended */
	struct h265_pipe *P;
} h265_job_t;

typedef struct h265_pipe {
	pthread_mutex_t mu;
	pthread_cond_t cv_work, cv_done;
	pthread_t th[16];
	int nth, started, quit, submitting;
	h265_job_t jobs[H265_RING];    /* the job of seq s: jobs[s % H265_RING] */
	long head;                     /* jobs dispatched */
	long sub;                      /* jobs submitted to the back end (decode order) */
	long parsed_below;             /* every job below this seq is parsed */
	long col_writer[H265R_MAX_FRAMES], col_reader[H265R_MAX_FRAMES]; /* motion fields: last writer, latest reader */
	long frame_seq[H265R_MAX_FRAMES]; /* the last picture decoded into each frame (-1: none) */
	h265_col_t *col[H265R_MAX_FRAMES];
	size_t cap_col;
	h265r_backend_t be;
	int have_be;
	int err_seen;                  /* a picture failed: decode_picture returns -2 from now on */
	long fail_seq;                 /* the first picture that failed (LONG_MAX: none): it and every later one
	                                  are never output, as the sequential path never decodes past it */
	/* the caller's DPB as it was before each dispatched picture's insert_dpb, and the entries get popped since
	 * (caller's thread only): on a failure the DPB goes back to its state before the failed picture, less what
	 * was output meanwhile — exactly the sequential path's DPB when its decode_picture returned -2 there */
	struct {
		h265_dpb_elem_t dpb[16];
		int size;
		long npop, seq;
	} hist[H265_RING];
	long popped[4 * H265_RING];
	long npop;
	int rolled_back;
	uint64_t bins;
} h265_pipe_t;

/* the sequence number of the picture dispatched last (-1: sequential path) */
static long pipe_last_seq(const h265_dec_t *d) { return d->pipe ? d->pipe->head - 1 : -1; }

/* parse ahead: the DPB before the dispatched picture's insert (pipe_purge_failed) */
static void pipe_note_insert(h265_dec_t *d)
{
	h265_pipe_t *P = d->pipe;
	if (!P || P->head <= 0) return;
	const int h = (int)((P->head - 1) % H265_RING);
	memcpy(P->hist[h].dpb, d->dpb, sizeof(d->dpb));
	P->hist[h].size = d->dpb_size;
	P->hist[h].npop = P->npop;
	P->hist[h].seq = P->head - 1;
}

static double h265_now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

static int pipe_threads(const h265_dec_t *d)
{
	if (d->threads >= 0) return d->threads > 16 ? 16 : d->threads;
	const char *e = getenv("M2DEC_AMD_H265_THREADS");
	const int n = e && *e ? atoi(e) : (m2d_cpu_share() < 8 ? m2d_cpu_share() : 8); /* (cpushare.c) */
	return n < 0 ? 0 : (n > 16 ? 16 : n);
}

/* the parse-ahead path is in use (the syntax dump is written in decode order: sequential) */
static int pipe_on(h265_dec_t *d)
{
	if (d->pipe) return 1;
	if (g_dump || !d->have_be || pipe_threads(d) == 0) return 0;
	h265_pipe_t *P = (h265_pipe_t *)calloc(1, sizeof(h265_pipe_t));
	if (!P) return 0;
	pthread_mutex_init(&P->mu, NULL);
	pthread_cond_init(&P->cv_work, NULL);
	pthread_cond_init(&P->cv_done, NULL);
	P->nth = pipe_threads(d);
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) P->col_writer[i] = P->col_reader[i] = P->frame_seq[i] = -1;
	P->fail_seq = LONG_MAX;
	for (int i = 0; i < H265_RING; ++i) P->jobs[i].P = P;
	P->be = d->be;
	P->have_be = d->have_be;
	d->pipe = P;
	return 1;
}

static void job_row_wait(h265_job_t *j, int row)
{
	h265_job_t *c = j->col;
	if (!c) return;
	h265_pipe_t *P = j->P;
	pthread_mutex_lock(&P->mu);
	while (c->seq == j->col_seq && c->rows_done <= row) pthread_cond_wait(&P->cv_done, &P->mu);
	pthread_mutex_unlock(&P->mu);
}

static void job_row_done(h265_job_t *j, int rows)
{
	h265_pipe_t *P = j->P;
	pthread_mutex_lock(&P->mu);
	j->rows_done = rows;
	pthread_cond_broadcast(&P->cv_done);
	pthread_mutex_unlock(&P->mu);
}

/* submit the parsed jobs that are next in decode order (mutex held; one submitter at a time, the back end's
 * calls made outside the mutex) */
static void pipe_submit_locked(h265_pipe_t *P)
{
	while (!P->submitting && P->sub < P->head && P->jobs[P->sub % H265_RING].state == JOB_PARSED) {
		h265_job_t *j = &P->jobs[P->sub % H265_RING];
		P->submitting = 1;
		pthread_mutex_unlock(&P->mu);
		int r = -1;
		const int tr = getenv("M2DEC_AMD_H265_TRACE") != NULL;
		if (tr) fprintf(stderr, "h265 job %ld submit %.3f\n", j->seq, h265_now());
		/* (nothing after a failed picture reaches the back end: the sequential path never decodes it, so the frames
		 * it would overwrite keep their content for the output that follows) */
		if (!j->err && P->have_be && j->seq < P->fail_seq) r = P->be.submit(P->be.self, &j->w->pic);
		else if (P->have_be && P->be.stage) P->be.stage(P->be.self, &j->w->pic, 1); /* (its staged arena back) */
		if (tr) fprintf(stderr, "h265 job %ld submitted %.3f\n", j->seq, h265_now());
		pthread_mutex_lock(&P->mu);
		if (r < 0) { /* a slice-data error on a worker (j->err) or a refused submission */
			P->err_seen = 1;
			if (j->seq < P->fail_seq) P->fail_seq = j->seq;
		}
		P->bins += j->w->cabac_bins;
		j->state = JOB_FREE;
		P->sub++;
		P->submitting = 0;
		pthread_cond_broadcast(&P->cv_done);
	}
}

static void job_run(h265_pipe_t *P, h265_job_t *j)
{
	h265_dec_t *w = j->w;
	jmp_buf jb;
	perr_t e;
	e.d = w;
	e.jb = &jb;
	w->cabac_bins = 0;
	if (setjmp(jb)) {
		j->err = 1;
		return;
	}
	picture_parse(&e, &j->sps, &j->pps, j->nal + j->data_off, j->nal + j->nal_len, j);
	(void)P;
}

static void *pipe_worker(void *arg)
{
	h265_pipe_t *P = (h265_pipe_t *)arg;
	pthread_setname_np(pthread_self(), "m2d-h265");
	pthread_mutex_lock(&P->mu);
	for (;;) {
		h265_job_t *j = NULL;
		/* the oldest job whose writes may start and whose collocated picture's parse has started (a worker then
		 * waits only on a running job: the chain of such waits ends at one that does not wait) */
		for (long sq = P->parsed_below; sq < P->head && !j; ++sq) {
			h265_job_t *c = &P->jobs[sq % H265_RING];
			if (c->state != JOB_QUEUED || c->after >= P->parsed_below) continue;
			if (c->col && c->col->seq == c->col_seq && c->col->state == JOB_QUEUED) continue;
			j = c;
		}
		if (!j) {
			if (P->quit) break;
			pthread_cond_wait(&P->cv_work, &P->mu);
			continue;
		}
		j->state = JOB_RUNNING;
		pthread_mutex_unlock(&P->mu);
		m2d_place_self(); /* (numa.c) */
		if (getenv("M2DEC_AMD_H265_TRACE")) fprintf(stderr, "h265 job %ld start %.3f\n", j->seq, h265_now());
		job_run(P, j);
		/* the records into the back end's page-locked arena here, in parallel, rather than on the serial
		 * submission (h265r_backend_t.stage) */
		if (!j->err && P->have_be && P->be.stage) P->be.stage(P->be.self, &j->w->pic, 0);
		if (getenv("M2DEC_AMD_H265_TRACE")) fprintf(stderr, "h265 job %ld end %.3f\n", j->seq, h265_now());
		pthread_mutex_lock(&P->mu);
		j->state = JOB_PARSED;
		j->rows_done = INT_MAX;
		while (P->parsed_below < P->head && P->jobs[P->parsed_below % H265_RING].state == JOB_PARSED) P->parsed_below++;
		pthread_cond_broadcast(&P->cv_done);
		pthread_cond_broadcast(&P->cv_work);
		pipe_submit_locked(P);
	}
	pthread_mutex_unlock(&P->mu);
	return NULL;
}

/* wait until every dispatched picture went to the back end (before the motion fields or the back end change) */
static void pipe_drain(h265_dec_t *d)
{
	h265_pipe_t *P = d->pipe;
	if (!P) return;
	pthread_mutex_lock(&P->mu);
	while (P->sub < P->head) pthread_cond_wait(&P->cv_done, &P->mu);
	pthread_mutex_unlock(&P->mu);
}

/* the motion fields of the frames, sized for the CTB-aligned frame as pic_arrays sizes them (on the caller's
 * thread, no job in flight) */
static size_t col_units(int fw, int fh) { return (size_t)(fw / 16) * (size_t)(fh / 16); }

static int pipe_cols(h265_pipe_t *P, int fw, int fh)
{
	const size_t ncol = col_units(fw, fh);
	if (ncol <= P->cap_col) return 0;
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) {
		free(P->col[i]);
		P->col[i] = (h265_col_t *)calloc(ncol, sizeof(h265_col_t));
		if (!P->col[i]) {
			P->cap_col = 0;
			return -1;
		}
	}
	P->cap_col = ncol;
	return 0;
}

static int pipe_dispatch(perr_t *e, const h265_sps_t *s, const h265_pps_t *p, size_t data_off)
{
	h265_dec_t *d = e->d;
	h265_pipe_t *P = d->pipe;
	const h265_slice_t *sh = &d->sh;
	if (col_units(d->frame_w, d->frame_h) > P->cap_col) {
		pipe_drain(d);
		if (pipe_cols(P, d->frame_w, d->frame_h) < 0) return -1;
	}
	pthread_mutex_lock(&P->mu);
	while (P->head - P->sub >= H265_RING && !P->err_seen) pthread_cond_wait(&P->cv_done, &P->mu);
	const int failed = P->err_seen;
	h265_job_t *j = &P->jobs[P->head % H265_RING];
	pthread_mutex_unlock(&P->mu);
	if (failed) return -1;
	/* (the job is FREE: no worker reads it until it is queued below) */
	if (!j->w && !(j->w = (h265_dec_t *)calloc(1, sizeof(h265_dec_t)))) return -1;
	h265_dec_t *w = j->w;
	if (d->unit_len + 16 > j->nal_cap) {
		free(j->nal);
		j->nal_cap = d->unit_len + 16 + (d->unit_len >> 2);
		if (!(j->nal = (uint8_t *)malloc(j->nal_cap))) {
			j->nal_cap = 0;
			return -1;
		}
	}
	memcpy(j->nal, d->unit, d->unit_len + 16); /* (next_unit zero-pads 16 bytes) */
	j->nal_len = d->unit_len;
	j->data_off = data_off;
	j->sps = *s;
	j->pps = *p;
	j->err = 0;
	w->sh = *sh;
	w->index = d->index;
	w->frame_w = d->frame_w;
	w->frame_h = d->frame_h;
	w->pictures = d->pictures;
	memcpy(w->frame_poc, d->frame_poc, sizeof(w->frame_poc));
	memcpy(w->col_frame, d->col_frame, sizeof(w->col_frame));
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) w->col[i] = P->col[i];
	w->cap_col = P->cap_col;
	pthread_mutex_lock(&P->mu);
	const long sq = P->head;
	const int idx = d->index;
	j->seq = sq;
	j->after = P->col_writer[idx] > P->col_reader[idx] ? P->col_writer[idx] : P->col_reader[idx];
	j->col = NULL;
	j->col_seq = -1;
	if (sh->slice_type < 2) {
		const int cf = sh->ref_frame[sh->col_from_l0 ^ 1][sh->col_ref_idx] & 7;
		const long k = P->col_writer[cf];
		if (k >= P->sub) { /* (in flight: not submitted yet) */
			j->col = &P->jobs[k % H265_RING];
			j->col_seq = k;
		}
		if (P->col_reader[cf] < sq) P->col_reader[cf] = sq;
	}
	P->col_writer[idx] = sq;
	P->col_reader[idx] = -1;
	P->frame_seq[idx] = sq;
	j->rows_done = 0;
	j->state = JOB_QUEUED;
	P->head++;
	while (P->started < P->nth) {
		if (pthread_create(&P->th[P->started], NULL, pipe_worker, P) != 0) break;
		P->started++;
	}
	if (!P->started) { /* no worker could be started: the picture fails here (decode_picture returns -2, as for a
	                     * slice-data error) and is retired at once, so no drain waits for a job nobody runs */
		j->err = 1;
		j->state = JOB_PARSED;
		j->rows_done = INT_MAX;
		while (P->parsed_below < P->head && P->jobs[P->parsed_below % H265_RING].state == JOB_PARSED) P->parsed_below++;
		pipe_submit_locked(P);
		pthread_mutex_unlock(&P->mu);
		return -1;
	}
	pthread_cond_broadcast(&P->cv_work);
	pthread_mutex_unlock(&P->mu);
	return 0;
}

static void pipe_stop(h265_dec_t *d)
{
	h265_pipe_t *P = d->pipe;
	if (!P) return;
	pipe_drain(d);
	pthread_mutex_lock(&P->mu);
	P->quit = 1;
	pthread_cond_broadcast(&P->cv_work);
	pthread_mutex_unlock(&P->mu);
	for (int i = 0; i < P->started; ++i) pthread_join(P->th[i], NULL);
	d->cabac_bins += P->bins;
	for (int i = 0; i < H265_RING; ++i) {
		h265_job_t *j = &P->jobs[i];
		if (j->w) {
			h265_dec_t *w = j->w;
			free(w->pic.tu);
			free(w->pic.coef);
			free(w->pic.map);
			free(w->pic.bs_v);
			free(w->pic.bs_h);
			free(w->pic.sao);
			free(w->pic.pu);
			free(w->cb_log2);
			free(w->ipm);
			free(w->nb);
			free(w);
		}
		free(j->nal);
	}
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) free(P->col[i]);
	pthread_cond_destroy(&P->cv_work);
	pthread_cond_destroy(&P->cv_done);
	pthread_mutex_destroy(&P->mu);
	free(P);
	d->pipe = NULL;
}

/* peek / get: the last picture dispatched into frame idx was retired (submitted, its reconstruction the back
 * end's to wait for, or failed).  Returns 1 when some picture failed on a worker: the sequential path (and the
 * reference, h265.cpp:4904) stops at the failing picture, so it and every picture dispatched after it are never
 * output (pipe_purge_failed). */
static int pipe_wait_frame(h265_dec_t *d, int idx)
{
	h265_pipe_t *P = d->pipe;
	if (!P || idx < 0 || idx >= H265R_MAX_FRAMES) return 0;
	pthread_mutex_lock(&P->mu);
	while (P->frame_seq[idx] >= P->sub) pthread_cond_wait(&P->cv_done, &P->mu);
	const int failed = P->fail_seq != LONG_MAX;
	pthread_mutex_unlock(&P->mu);
	return failed;
}

/* after a failure: the DPB back to its state before the failed picture's insert, less the entries get popped
 * since (caller's thread, once); 1 if it changed */
static int pipe_purge_failed(h265_dec_t *d)
{
	h265_pipe_t *P = d->pipe;
	if (P->rolled_back) return 0;
	pthread_mutex_lock(&P->mu);
	const long f = P->fail_seq;
	pthread_mutex_unlock(&P->mu);
	if (f == LONG_MAX || f >= P->head) return 0;
	P->rolled_back = 1;
	const int h = (int)(f % H265_RING);
	if (P->hist[h].seq != f) return 0; /* (failed in its dispatch: never inserted, nothing after it either) */
	int k = 0;
	for (int i = 0; i < P->hist[h].size; ++i) {
		const h265_dpb_elem_t *el = &P->hist[h].dpb[i];
		int gone = 0;
		for (long q = P->hist[h].npop; q < P->npop && !gone; ++q) gone = P->popped[q % (4 * H265_RING)] == el->seq;
		if (!gone) d->dpb[k++] = *el;
	}
	d->dpb_size = k;
	d->dpb_output = -1;
	return 1;
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
		/* the reference has motion-field buffers for min(num_long_term_ref_pics_sps + num_short_term_ref_pic_sets, 8)
		 * frames (set_second_frame, h265.cpp:121-128) and writes the current frame's for every picture: a frame
		 * index at or above that count is reference UB (parity unpinned).  Here every one of the
		 * H265R_MAX_FRAMES frames has its motion field, so only an index beyond those is an error (an
		 * all-intra stream with few RPS sets decodes) */
		if (d->index >= H265R_MAX_FRAMES) H265_ERR(e);
		parse_slice_header(e, &b, s, p);
		/* ctu_init (h265.cpp:4777) and colpics_t::init's register_reflist (h265modules.h:769): every slice */
		d->frame_poc[d->index] = sh->poc;
		memcpy(d->col_frame[d->index], sh->ref_frame, sizeof(sh->ref_frame));
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
		const size_t pos = (size_t)(b.p - (d->unit + 2)) - (size_t)(b.bits >> 3);
		if (pipe_on(d)) {
			if (pipe_dispatch(e, s, p, 2 + pos) < 0) H265_ERR(e);
		} else {
			picture_parse(e, s, p, d->unit + 2 + pos, d->unit + d->unit_len, NULL);
			if (!d->have_be || d->be.submit(d->be.self, &d->pic) < 0) H265_ERR(e);
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
	d->threads = -1;
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
	pipe_drain(d); /* (the back end is reconfigured below: nothing of the old geometry may still go to it) */
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
		if (d->pipe) {
			d->pipe->be = d->be;
			d->pipe->have_be = 1;
		}
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
	if (d->pipe && __atomic_load_n(&d->pipe->err_seen, __ATOMIC_ACQUIRE)) return -2; /* (as the reference at that picture) */
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
	int idx = peek_idx(d, bypass);
	if (idx < 0) return 0;
	if (pipe_wait_frame(d, idx) && pipe_purge_failed(d)) {
		idx = peek_idx(d, bypass);
		if (idx < 0) return 0;
		(void)pipe_wait_frame(d, idx);
	}
	if (d->hold && idx < 16 && d->fresh[idx]) { /* the frame's previous content is still read by the caller (driver_mt.c: its MD5) */
		pthread_mutex_lock(&d->hold->mu);
		while (m2dec_hold_busy(d->hold, d->frames[idx].luma)) {
			d->hold->waits++;
			pthread_cond_wait(&d->hold->cv, &d->hold->mu);
		}
		pthread_mutex_unlock(&d->hold->mu);
	}
	m2d_tl('Y', idx, 0);
	if (d->have_be && d->be.sync_frame(d->be.self, idx) < 0) return -1;
	if (idx < 16) d->fresh[idx] = 0;
	m2d_tl('y', idx, 0);
	*frame = d->frames[idx];
	return 1;
}

static int api_get(void *ctx, m2d_frame_t *frame, int bypass)
{
	h265_dec_t *d = CTX(ctx);
	const int r = api_peek(ctx, frame, bypass);
	if (r < 0) return -1;
	if (d->dpb_size > 0) { /* force_pop_dpb, whether a frame was returned or not (h265.cpp:4969-4976, 5000-5008) */
		if (d->pipe) d->pipe->popped[d->pipe->npop++ % (4 * H265_RING)] = d->dpb[0].seq;
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
void h265_set_hold(void *ctx, struct m2dec_hold *hold)
{
	h265_dec_t *d = CTX(ctx);
	if (d) d->hold = hold;
}

int m2dec_amd_h265_set_backend(void *ctx, const h265r_backend_t *be)
{
	h265_dec_t *d = CTX(ctx);
	if (!d) return -1;
	pipe_drain(d); /* (no picture in flight goes to the old back end after this) */
	if (!be) {
		pipe_stop(d);
		d->have_be = 0;
		return 0;
	}
	if (d->have_be && d->be.destroy) d->be.destroy(d->be.self);
	d->be = *be;
	d->have_be = 1;
	if (d->pipe) d->pipe->be = d->be;
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
	pipe_stop(d);
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
	free(d->nb);
	for (int i = 0; i < H265R_MAX_FRAMES; ++i) {
		free(d->col[i]);
		d->col[i] = NULL;
	}
	free(d->pic.pu);
	d->nb = NULL;
	d->cap_nb = d->cap_col = d->cap_pu = 0;
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

uint64_t m2dec_amd_h265_cabac_bins(const void *ctx)
{
	const h265_dec_t *d = (const h265_dec_t *)ctx;
	if (!d) return 0;
	uint64_t n = d->cabac_bins;
	if (d->pipe) {
		pthread_mutex_lock(&d->pipe->mu);
		n += d->pipe->bins;
		pthread_mutex_unlock(&d->pipe->mu);
	}
	return n;
}

/* parse-ahead workers of this context (0: sequential, on the caller's thread); before the first picture */
int m2dec_amd_h265_set_threads(void *ctx, int threads)
{
	h265_dec_t *d = CTX(ctx);
	if (!d || d->pipe) return -1;
	d->threads = threads < 0 ? 0 : threads;
	return 0;
}
