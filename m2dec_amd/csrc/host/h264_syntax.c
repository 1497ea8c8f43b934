/*
 * H.264 high-level syntax for the m2dec_amd host parser: SPS/PPS, slice header, POC, reference
 * list construction / modification, reference marking and the output (DPB) model.
 *
 * Everything here follows the reference decoder's behaviour (not only the spec), because output
 * order and reference selection change the bytes a caller sees.  Anchors:
 *   SPS            h264.cpp:254-362     PPS          h264.cpp:406-442
 *   slice header   h264.cpp:1417-1567   POC          h264.cpp:1121-1216
 *   list init      h264.cpp:10935-10960 list modif.  h264.cpp:1608-1653
 *   weights        h264.cpp:1655-1683   marking      h264.cpp:1685-1723, 10665-10873
 *   DPB bumping    h264.cpp:695-867     frame LRU    h264.cpp:924-962
 *   picture end    h264.cpp:11022-11050 (post_process)
 */
#include <stdio.h>
#include <stdlib.h>
#include <limits.h>
#include <pthread.h>
#include "h264_dec.h"

#define UE_RANGE(dst, b, max) do { uint32_t t_ = hb_ue(b); if ((uint32_t)(max) < t_) return -1; (dst) = (int)t_; } while (0)
#define SE_RANGE(dst, b, min, max) do { int32_t t_ = hb_se(b); if (t_ < (min) || (max) < t_) return -1; (dst) = t_; } while (0)

/* ------------------------------------------------------------------ SPS (h264.cpp:254-362) */
static int is_high_profile(int p)
{
	return p == 44 || p == 83 || p == 86 || p == 100 || p == 110 || p == 118 || p == 128 || p == 122 || p == 244;
}

static int skip_scaling_list(h264_bits_t *b, int size)
{
	int last = 8, next = 8;
	for (int i = 0; i < size; ++i) {
		if (next != 0) {
			int delta;
			SE_RANGE(delta, b, -128, 127);
			next = (last + delta + 256) & 255;
		}
		last = (next == 0) ? last : next;
	}
	return 0;
}

static int max_dpb_mbs(int profile_idc, int level_idc, int constraint)
{
	(void)constraint;
	if (profile_idc == 100 && level_idc == 9) level_idc = 10;
	switch (level_idc) {
	case 10: return 396;
	case 11: return 900;
	case 12: case 13: case 20: return 2376;
	case 21: return 4752;
	case 22: case 30: return 8100;
	case 31: return 18000;
	case 32: return 20480;
	case 40: case 41: return 32768;
	case 42: return 34816;
	case 50: return 110400;
	case 51: return 184320;
	default: return -1;
	}
}

int h264_parse_sps(h264_dec_t *d, h264_bits_t *b)
{
	int profile = hb_get(b, 8);
	int cflags = hb_get(b, 8);
	int level = hb_get(b, 8);
	int id, tmp;
	h264_sps_t *s;

	UE_RANGE(id, b, 31);
	s = &d->sps[id];
	s->profile_idc = profile;
	s->constraint_flags = cflags;
	s->level_idc = level;
	if (is_high_profile(profile)) {
		int chroma_idc;
		UE_RANGE(chroma_idc, b, 3);
		if (chroma_idc == 3) hb_get1(b);
		UE_RANGE(tmp, b, 6);
		UE_RANGE(tmp, b, 6);
		hb_get1(b);
		if (hb_get1(b)) {
			/* h264.cpp:280-296 reads 6 4x4 flags and then 8 (or 12) 8x8 flags; replicate. */
			int max = (chroma_idc != 3) ? 8 : 12;
			for (int i = 0; i < 6; ++i)
				if (hb_get1(b) && skip_scaling_list(b, 16) < 0) return -1;
			for (int i = 0; i < max; ++i)
				if (hb_get1(b) && skip_scaling_list(b, 64) < 0) return -1;
		}
	}
	UE_RANGE(tmp, b, 27);
	s->log2_max_frame_num = tmp + 4;
	UE_RANGE(s->poc_type, b, 2);
	if (s->poc_type == 0) {
		UE_RANGE(tmp, b, 27);
		s->log2_max_poc_lsb = tmp + 4;
	} else if (s->poc_type == 1) {
		int32_t delta = 0;
		s->delta_pic_order_always_zero_flag = hb_get1(b);
		s->offset_for_non_ref_pic = hb_se(b);
		s->offset_for_top_to_bottom_field = hb_se(b);
		UE_RANGE(s->num_ref_frames_in_poc_cycle, b, 255);
		for (int i = 0; i < s->num_ref_frames_in_poc_cycle; ++i) {
			delta += hb_se(b);
			s->offset_for_ref_frame[i] = delta;
		}
	}
	UE_RANGE(s->num_ref_frames, b, 16);
	s->gaps_allowed = hb_get1(b);
	s->width = (int)(hb_ue(b) + 1) * 16;
	s->height = (int)(hb_ue(b) + 1) * 16;
	s->max_dpb_in_mbs = max_dpb_mbs(profile, level, cflags);
	if ((s->frame_mbs_only_flag = hb_get1(b)) == 0) hb_get1(b);
	s->direct_8x8_inference_flag = hb_get1(b);
	if (hb_get1(b)) {
		for (int i = 0; i < 4; ++i) s->crop[i] = (int)hb_ue(b) * 2;
	} else {
		memset(s->crop, 0, sizeof(s->crop));
	}
	/* VUI is not needed for decoding; the reference parses and ignores it. */
	s->valid = 1;
	return id;
}

/* ------------------------------------------------------------------ PPS (h264.cpp:406-442) */
static int more_rbsp_data(h264_bits_t *b, const uint8_t *start, size_t len)
{
	size_t last;
	size_t pos = hb_pos(b, start);
	/* position of the rbsp_stop_one_bit = last 1 bit in the RBSP */
	while (len > 0 && start[len - 1] == 0) len--;
	if (len == 0) return 0;
	last = (len - 1) * 8 + (7 - __builtin_ctz(start[len - 1]));
	return pos < last;
}

int h264_parse_pps(h264_dec_t *d, h264_bits_t *b, size_t rbsp_len)
{
	int id, tmp;
	h264_pps_t *p;

	UE_RANGE(id, b, 255);
	p = &d->pps[id];
	UE_RANGE(p->sps_id, b, 31);
	p->entropy_coding_mode_flag = hb_get1(b);
	p->pic_order_present_flag = hb_get1(b);
	if (hb_ue(b) != 0) return -1; /* FMO not implemented (h264.cpp:418-421) */
	UE_RANGE(tmp, b, 31); p->num_ref_idx_active[0] = tmp + 1;
	UE_RANGE(tmp, b, 31); p->num_ref_idx_active[1] = tmp + 1;
	p->weighted_pred_flag = hb_get1(b);
	p->weighted_bipred_idc = hb_get(b, 2);
	SE_RANGE(tmp, b, -26, 25); p->pic_init_qp = tmp + 26;
	SE_RANGE(tmp, b, -26, 25);
	SE_RANGE(p->chroma_qp_index[0], b, -12, 12);
	p->chroma_qp_index[1] = p->chroma_qp_index[0];
	p->deblocking_filter_control_present_flag = hb_get1(b);
	p->constrained_intra_pred_flag = hb_get1(b);
	p->redundant_pic_cnt_present_flag = hb_get1(b);
	if (more_rbsp_data(b, d->nal + 1, rbsp_len)) {
		p->transform_8x8_mode_flag = hb_get1(b);
		hb_get1(b); /* pic_scaling_matrix_present_flag: lists are not parsed (h264.cpp:437-438) */
		SE_RANGE(p->chroma_qp_index[1], b, -12, 12);
	}
	p->valid = 1;
	return 0;
}

/* ------------------------------------------------------------------ DPB (h264.cpp:695-867) */
void h264_dpb_init(h264_dpb_t *dpb, int maxsize)
{
	memset(dpb, 0, sizeof(*dpb));
	dpb->max = maxsize;
	dpb->output = -1;
}

static void dpb_insert_non_idr(h264_dpb_t *dpb, int poc, int frame_idx)
{
	int size = dpb->size;
	h264_dpb_elem_t *end = dpb->data + size;
	h264_dpb_elem_t *dd = end;

	if (0 < size) {
		do {
			--dd;
		} while (dd != dpb->data && !dd->is_terminal && (poc < dd->poc));
		if (size < dpb->max) {
			dpb->size = size + 1;
			dpb->output = -1;
			if (dd->is_terminal || (dd->poc < poc)) ++dd;
			memmove(dd + 1, dd, (size_t)(end - dd) * sizeof(*dd));
		} else {
			dpb->output = dpb->data[0].frame_idx;
			if (dpb->data[0].is_terminal) dpb->is_ready = 0;
			memmove(dpb->data, dpb->data + 1, (size_t)(dd - dpb->data) * sizeof(*dd));
		}
	} else {
		dpb->size = 1;
		dpb->output = -1;
	}
	dd->poc = poc;
	dd->frame_idx = (int16_t)frame_idx;
	dd->is_idr = 0;
	dd->is_terminal = 0;
}

static void dpb_insert_idr(h264_dpb_t *dpb, int poc, int frame_idx)
{
	int size = dpb->size;
	h264_dpb_elem_t *dd;
	(void)poc;
	if (size < dpb->max) {
		dpb->size = size + 1;
	} else {
		size--;
		dpb->output = dpb->data[0].frame_idx;
		if (dpb->data[0].is_terminal) dpb->is_ready = 0;
		memmove(dpb->data, dpb->data + 1, (size_t)size * sizeof(dpb->data[0]));
	}
	dd = &dpb->data[size];
	dd->poc = 0;
	dd->frame_idx = (int16_t)frame_idx;
	dd->is_idr = 1;
	dd->is_terminal = 0;
	if (0 < size) {
		dd[-1].is_terminal = 1;
		dpb->is_ready = 1;
	}
}

static int dpb_force_pop(h264_dpb_t *dpb)
{
	int size = dpb->size;
	int idx = dpb->output;
	if (0 <= idx) {
		dpb->output = -1;
		return idx;
	} else if (size == 0) {
		return -1;
	}
	size -= 1;
	dpb->size = size;
	dpb->output = -1;
	if (dpb->data[0].is_terminal) dpb->is_ready = 0;
	idx = dpb->data[0].frame_idx;
	memmove(dpb->data, dpb->data + 1, (size_t)size * sizeof(dpb->data[0]));
	return idx;
}

static int dpb_force_peek(h264_dpb_t *dpb)
{
	if (0 <= dpb->output) return dpb->output;
	if (dpb->size == 0) return -1;
	return dpb->data[0].frame_idx;
}

/* h264d_peek_decoded_frame, h264.cpp:817-840 */
int h264_dpb_peek(h264_dpb_t *dpb, int bypass)
{
	if (!bypass) return dpb->is_ready ? dpb_force_peek(dpb) : dpb->output;
	return dpb_force_peek(dpb);
}

/* h264d_get_decoded_frame, h264.cpp:842-867 */
int h264_dpb_pop(h264_dpb_t *dpb, int bypass)
{
	int idx;
	if (!bypass) {
		if (dpb->is_ready) {
			idx = dpb_force_pop(dpb);
		} else {
			idx = dpb->output;
			dpb->output = -1;
		}
	} else {
		idx = dpb_force_pop(dpb);
	}
	return idx;
}

static int dpb_exist(const h264_dpb_t *dpb, int frame_idx)
{
	for (int i = 0; i < dpb->size; ++i)
		if (dpb->data[i].frame_idx == frame_idx) return 1;
	return 0;
}

/* ------------------------------------------------------------------ frame LRU (h264.cpp:924-962) */
/* lookahead context: a virtual frame id per picture, unique among the live pictures (the reference
 * lists and the current one), reused as late as possible (round robin over 64 ids).  The parser
 * compares frame_idx values only for equality (bS motion tests, the co-located ref map, the record
 * ref slots), so the API-visible context can translate ids to its real LRU slots picture by
 * picture (h264_async.c). */
static void alloc_virtual_frame(h264_dec_t *d)
{
	uint64_t live = 0;
	for (int i = 0; i < 16; ++i) {
		if (d->refs[0][i].in_use) live |= 1ull << (d->refs[0][i].frame_idx & 63);
		if (d->refs[1][i].in_use) live |= 1ull << (d->refs[1][i].frame_idx & 63);
	}
	for (int k = 0; k < 64; ++k) {
		const int v = (d->vid_next + k) & 63;
		if (!(live >> v & 1)) {
			d->curr_idx = v;
			d->vid_next = (v + 1) & 63;
			return;
		}
	}
	d->curr_idx = 0; /* 64 live pictures: impossible (<= 32 reference entries) */
}

static void find_empty_frame(h264_dec_t *d)
{
	int max_idx = 0, max_val = -1;
	if (d->lookahead) {
		alloc_virtual_frame(d);
		return;
	}
	for (int i = 0; i < d->num_frames; ++i) {
		if (dpb_exist(&d->dpb, i)) d->lru[i] = 0;
		else d->lru[i] += 1;
	}
	for (int i = 0; i < 16; ++i) {
		if (d->refs[0][i].in_use) d->lru[d->refs[0][i].frame_idx] = 0;
		if (d->refs[1][i].in_use) d->lru[d->refs[1][i].frame_idx] = 0;
	}
	if (d->hold) {
		/* frames the caller still holds are skipped; when only frames in use (lru 0) are left, wait for
		 * a release rather than take one (with none held: the reference's choice below) */
		m2dec_hold_t *h = d->hold;
		pthread_mutex_lock(&h->mu);
		for (;;) {
			int held = 0;
			max_idx = 0;
			max_val = -1;
			for (int i = 0; i < d->num_frames; ++i) {
				if (m2dec_hold_busy(h, d->frames[i].luma)) {
					held = 1;
					continue;
				}
				if (max_val < d->lru[i]) {
					max_val = d->lru[i];
					max_idx = i;
				}
			}
			if (!held || max_val > 0) break;
			h->waits++;
			pthread_cond_wait(&h->cv, &h->mu);
		}
		pthread_mutex_unlock(&h->mu);
		d->lru[max_idx] = 0;
		d->curr_idx = max_idx;
		return;
	}
	for (int i = 0; i < d->num_frames; ++i) {
		if (max_val < d->lru[i]) {
			max_val = d->lru[i];
			max_idx = i;
		}
	}
	d->lru[max_idx] = 0;
	d->curr_idx = max_idx;
}

/* ------------------------------------------------------------------ POC (h264.cpp:1121-1216) */
static void calc_poc0(h264_slice_t *h, int log2_max_lsb, uint32_t lsb, int mmco5_prev)
{
	uint32_t prev_lsb, prev_msb;
	int max_lsb_2;
	int32_t msb;
	if (h->idr || mmco5_prev) {
		prev_msb = 0;
		prev_lsb = 0;
	} else {
		prev_lsb = h->poc0_lsb;
		prev_msb = h->poc0_msb;
	}
	h->poc0_lsb = lsb;
	max_lsb_2 = (1 << log2_max_lsb) >> 1;
	if (((int)lsb < (int)prev_lsb) && (max_lsb_2 <= (int)(prev_lsb - lsb))) {
		msb = (int32_t)prev_msb + max_lsb_2 * 2;
	} else if (((int)prev_lsb < (int)lsb) && (max_lsb_2 < (int)(lsb - prev_lsb))) {
		msb = (int32_t)prev_msb - max_lsb_2 * 2;
	} else {
		msb = (int32_t)prev_msb;
	}
	h->poc0_msb = (uint32_t)msb;
	h->poc = msb + (int32_t)lsb;
}

static void calc_poc1(h264_slice_t *h, const h264_sps_t *s, int nal_ref_idc, int mmco5_prev)
{
	uint32_t frame_num = h->frame_num;
	int poc;
	if (!h->idr && !mmco5_prev) {
		if (frame_num < h->prev_frame_num) h->poc1_num_offset += 1u << s->log2_max_frame_num;
	} else {
		h->poc1_num_offset = 0;
	}
	if (s->num_ref_frames_in_poc_cycle) {
		frame_num += h->poc1_num_offset;
		if (frame_num != 0) {
			int cycle_cnt = 0;
			int cycle_sum = s->offset_for_ref_frame[s->num_ref_frames_in_poc_cycle - 1];
			frame_num--;
			if (frame_num != 0 && !nal_ref_idc) frame_num--;
			while (cycle_sum <= (int)frame_num) {
				frame_num -= cycle_sum;
				cycle_cnt++;
			}
			poc = cycle_cnt * cycle_sum + s->offset_for_ref_frame[frame_num & 255];
		} else {
			poc = s->offset_for_ref_frame[0];
		}
		if (!nal_ref_idc) poc += s->offset_for_non_ref_pic;
	} else {
		poc = 0;
	}
	h->poc = poc + h->delta_poc[0];
}

static void calc_poc2(h264_slice_t *h, const h264_sps_t *s, int nal_ref_idc, int mmco5_prev)
{
	uint32_t frame_num = h->frame_num;
	if (h->idr || mmco5_prev) {
		h->poc2_prev_frameoffset = 0;
	} else if (frame_num < h->prev_frame_num) {
		h->poc2_prev_frameoffset += 1u << s->log2_max_frame_num;
	}
	h->poc = (int)((frame_num + h->poc2_prev_frameoffset) * 2) - (nal_ref_idc == 0);
}

/* ------------------------------------------------------------------ list init (h264.cpp:10876-10960) */
static int unwrap_num(int s, int frame_num, int max_frame_num)
{
	return (frame_num < s) ? s - max_frame_num : s;
}

/* strict weak ordering; returns 1 if l goes before r */
static int ref_before_p(const h264_ref_t *l, const h264_ref_t *r, int frame_num, int max_frame_num)
{
	if (l->in_use == REF_SHORT) {
		if (r->in_use == REF_SHORT)
			return unwrap_num((int)l->num, frame_num, max_frame_num) > unwrap_num((int)r->num, frame_num, max_frame_num);
		return 1;
	} else if (l->in_use == REF_LONG) {
		if (r->in_use == REF_SHORT) return 0;
		if (r->in_use == REF_LONG) return l->num < r->num;
		return 1;
	}
	return 0;
}

static int poc_before_l0(int l, int r, int cur)
{
	if (l < cur) return (cur < r) || (l > r);
	return (cur < r) && (l < r);
}

static int poc_before_l1(int l, int r, int cur)
{
	if (l > cur) return (cur > r) || (l < r);
	return (cur > r) && (l > r);
}

static int ref_before_b(const h264_ref_t *l, const h264_ref_t *r, int cur, int lx)
{
	if (l->in_use == REF_SHORT) {
		if (r->in_use == REF_SHORT)
			return lx ? poc_before_l1(l->poc, r->poc, cur) : poc_before_l0(l->poc, r->poc, cur);
		return 1;
	} else if (l->in_use == REF_LONG) {
		if (r->in_use == REF_SHORT) return 0;
		if (r->in_use == REF_LONG) return l->poc < r->poc;
		return 1;
	}
	return 0;
}

/* the comparators are strict orders on distinct keys, so any correct sort matches std::sort */
static void sort_refs_p(h264_ref_t *ref, int n, int frame_num, int max_frame_num)
{
	for (int i = 1; i < n; ++i) {
		h264_ref_t t = ref[i];
		int j = i - 1;
		while (j >= 0 && ref_before_p(&t, &ref[j], frame_num, max_frame_num)) {
			ref[j + 1] = ref[j];
			j--;
		}
		ref[j + 1] = t;
	}
}

static void sort_refs_b(h264_ref_t *ref, int n, int cur, int lx)
{
	for (int i = 1; i < n; ++i) {
		h264_ref_t t = ref[i];
		int j = i - 1;
		while (j >= 0 && ref_before_b(&t, &ref[j], cur, lx)) {
			ref[j + 1] = ref[j];
			j--;
		}
		ref[j + 1] = t;
	}
}

/* ------------------------------------------------------------------ diagnostics
 * Counters of the reference-picture paths a stream took (tests/test_reflists_cpu.py asserts that each
 * golden stream reaches the path it was made for), and M2DEC_AMD_H264_REFDUMP=path: the active lists of
 * every P / B slice in tools/h264gen's gen_refdump_t layout, compared with the generator's own by
 * tests/gen_check.py.  Both are written by the context that parses slice data (the lookahead context of a
 * parse-ahead pipeline, or the decoder itself), not by the pipeline's API context. */
static long g_hits[M2DEC_AMD_H264_HITS];
#define HIT(i) __atomic_fetch_add(&g_hits[i], 1, __ATOMIC_RELAXED)

int m2dec_amd_h264_parser_hits(long *out, int n, int reset)
{
	if (n > M2DEC_AMD_H264_HITS) n = M2DEC_AMD_H264_HITS;
	for (int i = 0; i < n; ++i) out[i] = reset ? __atomic_exchange_n(&g_hits[i], 0, __ATOMIC_RELAXED) : __atomic_load_n(&g_hits[i], __ATOMIC_RELAXED);
	return n;
}

void h264_hit(int i) { HIT(i); }

static int counting(const h264_dec_t *d) { return !(d->as && !d->lookahead); }

static pthread_mutex_t g_rd_mu = PTHREAD_MUTEX_INITIALIZER;
static FILE *g_rd;
static int g_rd_opened;

/* the list dump to `path` from now on (NULL: off); M2DEC_AMD_H264_REFDUMP sets the first one */
int m2dec_amd_h264_set_refdump(const char *path)
{
	pthread_mutex_lock(&g_rd_mu);
	if (g_rd) fclose(g_rd);
	g_rd = path && *path ? fopen(path, "wb") : NULL;
	g_rd_opened = 1;
	pthread_mutex_unlock(&g_rd_mu);
	return path && *path && !g_rd ? -1 : 0;
}

static void refdump(const h264_dec_t *d, int nal_ref_idc)
{
	const h264_slice_t *h = &d->sh;
	struct {
		int32_t pic, first_mb, slice_type, poc, n[2], poc_l[2][16];
		int8_t lt[2][16];
	} r;
	(void)nal_ref_idc;
	pthread_mutex_lock(&g_rd_mu);
	if (!g_rd_opened) {
		const char *p = getenv("M2DEC_AMD_H264_REFDUMP");
		g_rd_opened = 1;
		g_rd = p && *p ? fopen(p, "wb") : NULL;
	}
	FILE *f = g_rd;
	if (f) {
		memset(&r, 0, sizeof(r));
		r.pic = (int32_t)d->pictures;
		r.first_mb = h->first_mb;
		r.slice_type = h->slice_type;
		r.poc = h->poc;
		r.n[0] = h->slice_type != 2 ? h->num_ref_idx_active[0] : 0;
		r.n[1] = h->slice_type == 1 ? h->num_ref_idx_active[1] : 0;
		for (int lx = 0; lx < 2; ++lx)
			for (int i = 0; i < r.n[lx] && i < 16; ++i) {
				r.poc_l[lx][i] = d->refs[lx][i].in_use ? d->refs[lx][i].poc : -999999;
				r.lt[lx][i] = (int8_t)(d->refs[lx][i].in_use == REF_LONG);
			}
		fwrite(&r, sizeof(r), 1, f);
		fflush(f);
	}
	pthread_mutex_unlock(&g_rd_mu);
}

/* std::remove_if over [first, last): compacts survivors forward, tail keeps its old contents */
static void remove_if_target(h264_ref_t *first, h264_ref_t *last, uint32_t num, int mode)
{
	h264_ref_t *out = first;
	for (h264_ref_t *it = first; it != last; ++it) {
		if (!(it->num == num && it->in_use == mode)) {
			if (out != it) *out = *it;
			out++;
		}
	}
}

/* ref_pic_list_reordering, h264.cpp:1608-1653 */
static int list_modification(h264_bits_t *b, h264_ref_t *refs, uint32_t frame_num, int max_frame_num, int count)
{
	if (!hb_get1(b)) return 0;
	for (int idx = 0; idx < 16; ++idx) {
		int op;
		uint32_t num;
		int mode;
		UE_RANGE(op, b, 3);
		if (op == 3) break;
		if (count) HIT(H264_HIT_MOD0 + op);
		num = hb_ue(b);
		if (op < 2) {
			int v;
			if (op == 0) {
				v = (int)frame_num - (int)num - 1;
				while (v < 0) v += max_frame_num;
			} else {
				v = (int)frame_num + (int)num + 1;
				while (max_frame_num <= v) v -= max_frame_num;
			}
			num = (uint32_t)v;
			frame_num = num;
			mode = REF_SHORT;
		} else {
			mode = REF_LONG;
		}
		if (refs[idx].num == num && refs[idx].in_use == mode) {
			remove_if_target(&refs[idx + 1], refs + 16, num, mode);
		} else {
			int t;
			for (t = 0; t < 16; ++t)
				if (refs[t].num == num && refs[t].in_use == mode) break;
			if (t < 16) {
				h264_ref_t tmp = refs[t];
				remove_if_target(&refs[idx + 1], refs + 16, num, mode);
				memmove(&refs[idx + 1], &refs[idx], (size_t)(16 - (idx + 1)) * sizeof(refs[0]));
				refs[idx] = tmp;
			}
		}
	}
	return 0;
}

static int clip3i(int lo, int hi, int v)
{
	return v < lo ? lo : (v > hi ? hi : v);
}

/* dist_scale_factor, h264.cpp:1244-1254 */
static int dist_scale_factor(int poc0, int poc1, int cur)
{
	if (poc1 == poc0) return 256;
	{
		int td = clip3i(-128, 127, poc1 - poc0);
		int tb = clip3i(-128, 127, cur - poc0);
		int tx = (16384 + abs(td / 2)) / td;
		return (tb * tx + 32) >> 6;
	}
}

static int pred_weight_table(h264_bits_t *b, h264_slice_t *h, int lx)
{
	int dl = 1 << h->log2wd[0];
	int dc = 1 << h->log2wd[1];
	for (int i = 0; i < h->num_ref_idx_active[lx]; ++i) {
		if (hb_get1(b)) {
			int w, o;
			SE_RANGE(w, b, -128, 127);
			SE_RANGE(o, b, -128, 127);
			h->w[lx][i][0] = (int8_t)w;
			h->o[lx][i][0] = (int8_t)o;
		} else {
			h->w[lx][i][0] = (int8_t)dl; /* int8 store: 1 << 7 wraps (h264.h:219, Appendix A #16) */
			h->o[lx][i][0] = 0;
		}
		if (hb_get1(b)) {
			for (int j = 1; j < 3; ++j) {
				int w, o;
				SE_RANGE(w, b, -128, 127);
				SE_RANGE(o, b, -128, 127);
				h->w[lx][i][j] = (int8_t)w;
				h->o[lx][i][j] = (int8_t)o;
			}
		} else {
			for (int j = 1; j < 3; ++j) {
				h->w[lx][i][j] = (int8_t)dc;
				h->o[lx][i][j] = 0;
			}
		}
	}
	return 0;
}

static int dec_ref_pic_marking(h264_bits_t *b, h264_slice_t *h)
{
	uint32_t tmp = hb_get1(b);
	int op5 = 0;
	if (h->nal_unit_type == 5) {
		h->no_output_of_prior_pics = (int)tmp;
		h->long_term_reference_flag = hb_get1(b);
	} else {
		h->no_output_of_prior_pics = 0;
		h->adaptive_marking = (int)tmp;
		if (tmp) {
			for (int i = 0; i < 16; ++i) {
				h264_mmco_t *m = &h->mmco[i];
				UE_RANGE(m->op, b, 6);
				if (m->op == 0) break;
				if (m->op == 5) {
					op5 = 1;
				} else {
					uint32_t a = hb_ue(b);
					if (m->op == 3) m->arg2 = hb_ue(b);
					m->arg1 = a;
				}
			}
		}
	}
	h->mmco5 = op5;
	return 0;
}

/* ------------------------------------------------------------------ slice header (h264.cpp:1417-1567) */
int h264_slice_header(h264_dec_t *d, h264_bits_t *b, int nal_unit_type, int nal_ref_idc)
{
	h264_slice_t *h = &d->sh;
	h264_sps_t *s;
	h264_pps_t *p;
	int tmp;
	int mmco5_prev = h->mmco5;
	int max_frame_num;
	uint32_t first_mb = hb_ue(b);

	h->first_mb = (int)first_mb;
	UE_RANGE(tmp, b, 9);
	h->slice_type = (4 < tmp) ? tmp - 5 : tmp;
	if (3 <= h->slice_type) return -1;
	UE_RANGE(h->pps_id, b, 255);
	p = &d->pps[h->pps_id];
	if (!p->valid || !d->sps[p->sps_id].valid) return -1;
	d->active_sps = p->sps_id;
	s = &d->sps[p->sps_id];
	h->nal_unit_type = nal_unit_type;
	h->nal_ref_idc = nal_ref_idc;
	h->frame_num = hb_get(b, s->log2_max_frame_num);
	if (!s->frame_mbs_only_flag) {
		if (hb_get1(b)) hb_get1(b); /* field pictures are not supported (Appendix A #14) */
	}
	h->idr = (nal_unit_type == 5);
	if (h->idr) UE_RANGE(h->idr_pic_id, b, 65535);
	if (s->poc_type == 0) {
		uint32_t lsb = hb_get(b, s->log2_max_poc_lsb);
		h->delta_poc_bottom = p->pic_order_present_flag ? hb_se(b) : 0;
		if (h->first_mb == 0) calc_poc0(h, s->log2_max_poc_lsb, lsb, mmco5_prev);
	} else if (s->poc_type == 1) {
		if (!s->delta_pic_order_always_zero_flag) {
			h->delta_poc[0] = hb_se(b);
			if (p->pic_order_present_flag) h->delta_poc[1] = hb_se(b);
		} else {
			h->delta_poc[0] = 0;
			h->delta_poc[1] = 0;
		}
		if (h->first_mb == 0) calc_poc1(h, s, nal_ref_idc, mmco5_prev);
	} else {
		if (h->first_mb == 0) calc_poc2(h, s, nal_ref_idc, mmco5_prev);
	}
	if (p->redundant_pic_cnt_present_flag) hb_ue(b);
	max_frame_num = 1 << s->log2_max_frame_num;
	h->wp_mode = M2R_WP_DEFAULT;
	if (h->slice_type != 2) {
		if (h->slice_type == 1) h->direct_spatial = hb_get1(b);
		if (hb_get1(b)) {
			UE_RANGE(tmp, b, 31); h->num_ref_idx_active[0] = tmp + 1;
			if (h->slice_type == 1) { UE_RANGE(tmp, b, 31); h->num_ref_idx_active[1] = tmp + 1; }
		} else {
			h->num_ref_idx_active[0] = p->num_ref_idx_active[0];
			h->num_ref_idx_active[1] = p->num_ref_idx_active[1];
		}
		if (h->slice_type == 0) {
			sort_refs_p(d->refs[0], s->num_ref_frames, (int)h->frame_num, max_frame_num);
		} else {
			sort_refs_b(d->refs[0], s->num_ref_frames, h->poc, 0);
			sort_refs_b(d->refs[1], s->num_ref_frames, h->poc, 1);
			/* is_same_list (h264.cpp:10952) also compares the col pointers, which never match
			 * between the two arrays, so the spec's L1 swap never happens in the reference. */
			for (int i = s->num_ref_frames; i < 16; ++i) {
				d->refs[0][i].in_use = REF_UNUSED;
				d->refs[1][i].in_use = REF_UNUSED;
			}
		}
		if (list_modification(b, d->refs[0], h->frame_num, max_frame_num, counting(d)) < 0) return -1;
		if (h->slice_type == 1) {
			if (list_modification(b, d->refs[1], h->frame_num, max_frame_num, counting(d)) < 0) return -1;
			if (!h->direct_spatial) {
				/* create_map_col_to_list0, h264.cpp:1269-1277 */
				const h264_colpic_t *col = &d->colpic[d->refs[1][0].col];
				int poc1 = d->refs[1][0].poc;
				int len = s->num_ref_frames;
				for (int i = 0; i < len; ++i) {
					int fidx = col->map_col_frameidx[i];
					int k = -1;
					if (fidx >= 0) {
						for (k = 0; k < len; ++k)
							if (d->refs[0][k].frame_idx == fidx) break;
						if (k >= len) k = -1;
					}
					d->map_col_to_list0[i] = (int8_t)k;
					d->dist_scale[i] = (int16_t)clip3i(-1024, 1023, dist_scale_factor(d->refs[0][i].poc, poc1, h->poc));
				}
			}
			if (p->weighted_bipred_idc == 1) {
				UE_RANGE(h->log2wd[0], b, 7);
				UE_RANGE(h->log2wd[1], b, 7);
				pred_weight_table(b, h, 0);
				pred_weight_table(b, h, 1);
				h->wp_mode = M2R_WP_EXPLICIT;
			} else if (p->weighted_bipred_idc == 2) {
				h->wp_mode = M2R_WP_IMPLICIT;
			}
		} else if (p->weighted_pred_flag) {
			UE_RANGE(h->log2wd[0], b, 7);
			UE_RANGE(h->log2wd[1], b, 7);
			pred_weight_table(b, h, 0);
			h->wp_mode = M2R_WP_EXPLICIT;
		}
	}
	if (nal_ref_idc) {
		if (dec_ref_pic_marking(b, h) < 0) return -1;
	} else {
		h->mmco5 = 0;
	}
	if (counting(d)) {
		if (h->slice_type != 2) {
			int lt = 0;
			for (int lx = 0; lx < (h->slice_type == 1 ? 2 : 1); ++lx)
				for (int i = 0; i < h->num_ref_idx_active[lx] && i < 16; ++i) lt |= d->refs[lx][i].in_use == REF_LONG;
			if (lt) HIT(H264_HIT_LT_LIST);
			if (h->slice_type == 0) {
				for (int i = 0; i < h->num_ref_idx_active[0] && i < 16; ++i)
					if (d->refs[0][i].in_use == REF_SHORT && d->refs[0][i].num > h->frame_num) {
						HIT(H264_HIT_FN_WRAP);
						break;
					}
			}
		}
		if (s->poc_type == 1) HIT(H264_HIT_POC1);
		if (s->poc_type == 2) HIT(H264_HIT_POC2);
		if (nal_ref_idc && h->idr && h->long_term_reference_flag) HIT(H264_HIT_LT_IDR);
		if (nal_ref_idc && !h->idr && h->adaptive_marking)
			for (int i = 0; i < 16 && h->mmco[i].op; ++i) HIT(H264_HIT_MMCO1 + h->mmco[i].op - 1);
		refdump(d, nal_ref_idc);
	}
	h->cabac_init_idc = 0;
	if (p->entropy_coding_mode_flag && h->slice_type != 2) UE_RANGE(h->cabac_init_idc, b, 2);
	tmp = p->pic_init_qp + hb_se(b);
	if (tmp < 0) tmp += 52;
	else if (52 <= tmp) tmp -= 52;
	h->qp = tmp;
	if (p->deblocking_filter_control_present_flag) {
		UE_RANGE(h->disable_deblocking_filter_idc, b, 2);
		if (h->disable_deblocking_filter_idc != 1) {
			SE_RANGE(h->alpha_off, b, -6, 6);
			SE_RANGE(h->beta_off, b, -6, 6);
			h->alpha_off *= 2;
			h->beta_off *= 2;
		} else {
			h->alpha_off = h->beta_off = 0;
		}
	} else {
		h->disable_deblocking_filter_idc = 0;
		h->alpha_off = h->beta_off = 0;
	}
	if (d->dpb.max < 0) {
		int n = s->max_dpb_in_mbs / ((s->width * s->height) >> 8);
		d->dpb.max = 16 < n ? 16 : n;
	}
	return 0;
}

/* ------------------------------------------------------------------ marking (h264.cpp:10665-10873) */
static h264_ref_t *sliding_window(h264_ref_t *refs, int frame_idx, int frame_num, int max_frame_num, int num_ref_frames, int poc)
{
	int min_num = INT_MAX, min_idx = 0, empty = -1, n_long = 0, n_short = 0;
	for (int i = 0; i < 16; ++i) {
		int u = refs[i].in_use;
		if (u == REF_UNUSED) {
			if (empty < 0) empty = i;
		} else if (u == REF_SHORT) {
			int num = (int)refs[i].num;
			if (frame_num < num) num -= max_frame_num;
			if (num < min_num) {
				min_num = num;
				min_idx = i;
			}
			n_short++;
		} else {
			n_long++;
		}
	}
	if (n_short + n_long < num_ref_frames) refs += (0 <= empty) ? empty : num_ref_frames - 1;
	else refs += min_idx;
	refs->in_use = REF_SHORT;
	refs->frame_idx = (int16_t)frame_idx;
	refs->num = (uint32_t)frame_num;
	refs->poc = poc;
	return refs;
}

static void mmco_discard(h264_ref_t *refs, int in_use, uint32_t num)
{
	for (int i = 0; i < 16; ++i) {
		if (refs[i].num == num && refs[i].in_use == in_use) {
			refs[i].in_use = REF_UNUSED;
			break;
		}
	}
}

static int marking_mmco(const h264_slice_t *h, h264_ref_t *refs, int frame_idx, int frame_num, int max_frame_num, int num_ref_frames, int poc)
{
	int op5 = 0, op6 = 0;
	for (int i = 0; i < 16; ++i) {
		const h264_mmco_t *m = &h->mmco[i];
		if (m->op == 0) break;
		switch (m->op) {
		case 1: {
			int num = frame_num - (int)m->arg1 - 1;
			while (num < 0) num += max_frame_num;
			mmco_discard(refs, REF_SHORT, (uint32_t)num);
			break;
		}
		case 2:
			mmco_discard(refs, REF_LONG, m->arg1);
			break;
		case 3: {
			uint32_t target = (uint32_t)(frame_num - (int)m->arg1 - 1);
			while ((int)target < 0) target += (uint32_t)max_frame_num;
			for (int k = 0; k < 16; ++k) {
				if (refs[k].in_use == REF_LONG && refs[k].num == m->arg2) {
					refs[k].in_use = REF_UNUSED;
				} else if (refs[k].in_use == REF_SHORT && refs[k].num == target) {
					refs[k].in_use = REF_LONG;
					refs[k].num = m->arg2;
				}
			}
			break;
		}
		case 4:
			for (int k = 0; k < 16; ++k)
				if (refs[k].in_use == REF_LONG && m->arg1 <= refs[k].num) refs[k].in_use = REF_UNUSED;
			break;
		case 5:
			op5 = 1;
			for (int k = 0; k < 16; ++k) refs[k].in_use = REF_UNUSED;
			break;
		case 6: {
			h264_ref_t *r;
			op6 = 1;
			r = sliding_window(refs, frame_idx, frame_num, max_frame_num, num_ref_frames, poc);
			r->in_use = REF_LONG;
			r->num = m->arg1;
			break;
		}
		default:
			break;
		}
	}
	if (!op6) {
		if (op5) frame_num = poc = 0;
		sliding_window(refs, frame_idx, frame_num, max_frame_num, num_ref_frames, poc);
	}
	return op5;
}

static void post_ref_pic_marking(h264_dec_t *d, int lx, int max_frame_num, int num_ref_frames)
{
	h264_slice_t *h = &d->sh;
	h264_ref_t *refs = d->refs[lx];
	int frame_num = (int)h->frame_num;
	int poc = h->poc;
	if (h->nal_unit_type == 5) {
		refs[0].in_use = h->long_term_reference_flag ? REF_LONG : REF_SHORT;
		refs[0].frame_idx = (int16_t)d->curr_idx;
		refs[0].num = (uint32_t)frame_num;
		refs[0].poc = poc;
		for (int i = 1; i < 16; ++i) refs[i].in_use = REF_UNUSED;
	} else {
		if (!h->idr && !h->mmco5) {
			/* gap_mbs, h264.cpp:10806-10825 */
			int prev = (int)h->prev_frame_num;
			int gap = frame_num - prev;
			while (gap < 0) gap += max_frame_num;
			if (0 < --gap) {
				if (16 < gap) {
					gap = 16;
					prev = frame_num - 17;
				}
				do {
					if (max_frame_num <= ++prev) prev -= max_frame_num;
					sliding_window(refs, d->curr_idx, prev, max_frame_num, num_ref_frames, poc);
				} while (--gap);
			}
		}
		if (h->adaptive_marking) {
			if (marking_mmco(h, refs, d->curr_idx, frame_num, max_frame_num, num_ref_frames, poc)) h->frame_num = 0;
		} else {
			sliding_window(refs, d->curr_idx, frame_num, max_frame_num, num_ref_frames, poc);
		}
	}
}

/* ------------------------------------------------------------------ picture begin / end */
int h264_picture_begin(h264_dec_t *d)
{
	const h264_sps_t *s = &d->sps[d->active_sps];
	m2d_frame_t *f;
	find_empty_frame(d);
	f = &d->frames[d->curr_idx];
	f->width = (int16_t)s->width;
	f->height = (int16_t)s->height;
	for (int i = 0; i < 4; ++i) f->crop[i] = (int16_t)s->crop[i];
	f->cnt = d->sh.poc;
	d->mbs_decoded = 0;
	d->mbs_coded = 0;
	d->slice_num = 0;
	d->in_picture = 1;
	if (d->as) { /* parse-ahead: the job owns MB info and records (h264_async.c) */
		d->pic = NULL;
		return 0;
	}
	for (int i = 0; i < d->n_mbs; ++i) {
		d->mbi[i].type = -1;
		d->mbi[i].slice = -1;
	}
	d->pic = d->backend.acquire(d->backend.self, d->mb_w, d->mb_h);
	if (!d->pic) return -1;
	d->pic->slot = d->curr_idx;
	d->pic->n_inter = 0;
	d->pic->n_coef = 0;
	d->pic->n_slices = 0;
	d->pic->n_intra = 0;
	d->pic->deblock = 0;
	return 0;
}

/* post_process, h264.cpp:11022-11050, in three parts (deblocking happens inside the back end):
 * the deblock edge enables that deblock_pb derives from the picture-final firstline (needs the
 * picture's parsed MB info) ... */
void h264_picture_resolve_deblock(h264_dec_t *d)
{
	{
		m2r_deblock_t *dbk = d->pic->dbk;
		int any = 0;
		for (int y = 0; y < d->mb_h; ++y) {
			for (int x = 0; x < d->mb_w; ++x) {
				int a = y * d->mb_w + x;
				int sl = d->mbi[a].slice;
				int idc = (sl >= 0) ? d->slice_idc[sl] : 0;
				uint8_t fl = dbk[a].flags & (M2R_DBK_LEFT_BS4 | M2R_DBK_TOP_BS4);
				if (idc == 1) {
					fl |= M2R_DBK_OFF;
				} else {
					if (x != 0 && (!idc || d->last_firstline != d->mb_w)) fl |= M2R_DBK_LEFT;
					if (y != 0 && (!idc || d->last_firstline < 0)) fl |= M2R_DBK_TOP;
					any = 1;
				}
				dbk[a].flags = fl;
				dbk[a].alpha_off = (sl >= 0) ? d->slice_alpha[sl] : 0;
				dbk[a].beta_off = (sl >= 0) ? d->slice_beta[sl] : 0;
			}
		}
		d->pic->deblock = any;
	}
}

/* ... the reference marking, the co-located store swap and the DPB insertion (need only the slice
 * headers: the parse-ahead pipeline runs this before the picture's slice data is parsed) ... */
int h264_picture_mark(h264_dec_t *d)
{
	h264_slice_t *h = &d->sh;
	const h264_sps_t *s = &d->sps[d->active_sps];
	int max_frame_num = 1 << s->log2_max_frame_num;
	int num_ref_frames = s->num_ref_frames;
	if (h->nal_ref_idc) {
		h264_ref_t *r = NULL;
		int target;
		post_ref_pic_marking(d, 0, max_frame_num, num_ref_frames);
		post_ref_pic_marking(d, 1, max_frame_num, num_ref_frames);
		/* record_map_col_ref_frameidx, h264.cpp:10962-10968 (after marking, as the reference) */
		{
			int8_t *map = d->colpic[d->curr_col].map_col_frameidx;
			int i;
			for (i = 0; i < num_ref_frames; ++i) map[i] = (int8_t)d->refs[0][i].frame_idx;
			for (; i < 16; ++i) map[i] = (int8_t)d->refs[0][0].frame_idx;
		}
		/* find_l1_curr_pic + swap of the co-located store, h264.cpp:10970-10984 / 11040 */
		target = h->mmco5 ? 0 : h->poc;
		for (int i = 0; i < 16; ++i) {
			if (d->refs[1][i].in_use) {
				if (d->refs[1][i].poc == target) { r = &d->refs[1][i]; break; }
				if (!r) r = &d->refs[1][i];
			}
		}
		if (!r) r = &d->refs[1][0];
		{
			int t = r->col;
			r->col = (int16_t)d->curr_col;
			d->curr_col = t;
		}
		if (h->idr | h->mmco5) dpb_insert_idr(&d->dpb, h->poc, d->curr_idx);
		else dpb_insert_non_idr(&d->dpb, h->poc, d->curr_idx);
	} else {
		dpb_insert_non_idr(&d->dpb, h->poc, d->curr_idx);
	}
	h->prev_frame_num = h->frame_num;
	d->in_picture = 0;
	d->pictures++;
	return 1;
}

/* ... all three in order (synchronous parse) */
int h264_picture_finish(h264_dec_t *d)
{
	int err;
	h264_picture_resolve_deblock(d);
	err = d->backend.submit(d->backend.self, d->pic);
	if (!err && d->backend.flush) err = d->backend.flush(d->backend.self);
	d->pic = NULL;
	if (err < 0) return -1;
	return h264_picture_mark(d);
}
