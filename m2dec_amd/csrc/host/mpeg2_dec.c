/*
 * m2d_func — the reference's MPEG-1/2 video decoder table (mpeg2.cpp:1800-1811) for this library:
 * BASELINE.json configs[0] (C1), MPEG-2 MP@ML I-frame-only on the CPU.  Behaviour follows the
 * reference function by function:
 *
 *   init / stream_pos / get_info / set_frames      mpeg2.cpp:226-245, 1632-1651, 111-128
 *   decode_picture (m2d_decode_data)               mpeg2.cpp:1583-1604 (returns 1 per picture, -1 at
 *                                                  the end of the data)
 *   peek / get_decoded_frame, frame LRU, out_state mpeg2.cpp:1543-1573, 130-194
 *   headers: sequence / extensions / GOP / picture mpeg2.cpp:320-623
 *   slice + macroblock loop, skipped MBs, lost     mpeg2.cpp:625-660, 715-766, 1427-1524
 *   slices (copy from the forward reference)
 *   intra DC (prediction, clamp, precision)        mpeg2.cpp:920-939
 *   coefficient VLC (B.14 / B.15), escape, dequant mpeg2.cpp:945-1118 (MPEG-2 mismatch control /
 *   with +-2048 saturation                         MPEG-1 oddification, as the reference applies them)
 *   integer Chen-Wang IDCT (rows -> int16, columns idct.cpp:35-40, 69-236, 286-373
 *   with (x + 8192) >> 14), CLIP255C store
 *   luma placement per dct_type, NV12 chroma       mpeg2.cpp:1120-1153, idct.cpp:379-393
 *
 * Not implemented: P / B pictures (motion compensation, motioncomp.cpp) -> decode_picture returns
 * -1 at their picture header; MPEG-PS demux (.vob).  The VLC tables are this repo's transcription
 * of Annex B (mpeg2_tables.c), tested against the reference's own tables (tests/test_mpeg2_cpu.py).
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "h264_dec.h" /* h264_bits_t: the RBSP-style bit reader, used here on start-code units */
#include "mpeg2_dec.h"

int m2d_stream_next_byte(dec_bits *st); /* bitio.c */

/* ------------------------------------------------------------------ VLC look-up tables */
typedef struct {
	uint8_t len;   /* code length without the sign bit; 0: invalid */
	int8_t run;    /* -1: EOB (level 1) / escape (level 0) */
	uint8_t level;
} dct_lut_t;

typedef struct {
	uint8_t len;   /* 0: invalid */
	int8_t value;
} vlc_lut_t;

#define DCT_BITS 16
#define INC_BITS 11
#define DC_BITS 10
#define MC_BITS 10
#define MBT_BITS 6
#define CBP_BITS 9

static dct_lut_t lut_dct[2][1 << DCT_BITS];
static vlc_lut_t lut_inc[1 << INC_BITS], lut_dcl[1 << DC_BITS], lut_dcc[1 << DC_BITS], lut_mc[1 << MC_BITS];
static vlc_lut_t lut_mbp[1 << MBT_BITS], lut_mbb[1 << MBT_BITS], lut_cbp[1 << CBP_BITS];
static pthread_once_t lut_once = PTHREAD_ONCE_INIT;

static void fill_vlc(vlc_lut_t *lut, int bits, const m2v_code_t *t)
{
	for (; t->code; ++t) {
		const int n = (int)strlen(t->code);
		const int v = (int)strtol(t->code, NULL, 2);
		for (int k = 0; k < 1 << (bits - n); ++k) {
			lut[(v << (bits - n)) | k].len = (uint8_t)n;
			lut[(v << (bits - n)) | k].value = (int8_t)t->value;
		}
	}
}

static void fill_dct(dct_lut_t *lut, const m2v_dct_code_t *t)
{
	for (; t->code; ++t) {
		const int n = (int)strlen(t->code);
		const int v = (int)strtol(t->code, NULL, 2);
		for (int k = 0; k < 1 << (DCT_BITS - n); ++k) {
			dct_lut_t *e = &lut[(v << (DCT_BITS - n)) | k];
			e->len = (uint8_t)n;
			e->run = (int8_t)t->run;
			e->level = (uint8_t)t->level;
		}
	}
}

static void build_luts(void)
{
	fill_dct(lut_dct[0], m2v_dct0);
	for (const m2v_dct_code_t *t = m2v_dct0; t->code; ++t) /* the 14..16-bit codes of table zero ... */
		if (strlen(t->code) >= 14) {
			const m2v_dct_code_t one[2] = {*t, {0, 0, 0}};
			fill_dct(lut_dct[1], one);
		}
	fill_dct(lut_dct[1], m2v_dct1); /* ... and table one's own codes */
	fill_vlc(lut_inc, INC_BITS, m2v_mb_inc);
	fill_vlc(lut_dcl, DC_BITS, m2v_dc_luma);
	fill_vlc(lut_dcc, DC_BITS, m2v_dc_chroma);
	fill_vlc(lut_mc, MC_BITS, m2v_motion_code);
	fill_vlc(lut_mbp, MBT_BITS, m2v_mb_type_p);
	fill_vlc(lut_mbb, MBT_BITS, m2v_mb_type_b);
	fill_vlc(lut_cbp, CBP_BITS, m2v_cbp);
}

/* ------------------------------------------------------------------ C-ABI probes for the tests */
/* decode one DCT-coefficient codeword of `table` (0: B.14, 1: B.15) from the front of bits[]:
 * returns its length with the sign bit (0: invalid) and the run / sign-folded level, as parse_coef's
 * look-up does (run -1: EOB when level != 0, escape when level == 0). */
int m2dec_amd_m2v_dct_code(int table, uint32_t bits32, int *run, int *level)
{
	pthread_once(&lut_once, build_luts);
	const dct_lut_t *e = &lut_dct[table & 1][bits32 >> (32 - DCT_BITS)];
	if (!e->len) return 0;
	*run = e->run;
	if (e->run < 0) {
		*level = e->level ? 3 : 0; /* EOB / escape: no sign bit */
		return e->len;
	}
	*level = (e->level << 1) | (int)((bits32 >> (31 - e->len)) & 1);
	return e->len + 1;
}

/* decode one codeword of a plain VLC table (0: macroblock_address_increment after its first 0 bit,
 * 1: dct_dc_size_luminance, 2: dct_dc_size_chrominance, 3: motion_code after its first 0 bit, with
 * the sign folded in as the reference's table: -value) */
int m2dec_amd_m2v_vlc_code(int table, uint32_t bits32, int *value)
{
	pthread_once(&lut_once, build_luts);
	const vlc_lut_t *e;
	switch (table) {
	case 0: /* the leading '0' was consumed by the caller, as in m2d_macroblock_address_increment */
		e = &lut_inc[(bits32 >> (32 - INC_BITS + 1)) & ((1 << INC_BITS) - 1)];
		if (!e->len || e->len < 2) return 0;
		*value = e->value;
		return e->len - 1;
	case 1: e = &lut_dcl[bits32 >> (32 - DC_BITS)]; break;
	case 2: e = &lut_dcc[bits32 >> (32 - DC_BITS)]; break;
	case 3:
		e = &lut_mc[(bits32 >> (32 - MC_BITS + 1)) & ((1 << MC_BITS) - 1)];
		if (!e->len || e->len < 2) return 0;
		*value = ((bits32 >> (32 - e->len)) & 1) ? -e->value : e->value;
		return e->len; /* (len - 1 code bits after the 0) + the sign bit */
	default: return 0;
	}
	if (!e->len) return 0;
	*value = e->value;
	return e->len;
}

/* ------------------------------------------------------------------ start-code units */
/* the next start code's unit: returns its code byte (0..255) and leaves the payload up to the next
 * start code in m->unit, or -1 at the end of the data (m2d_find_mpeg_data, m2d.cpp:130-155) */
static int next_unit(mpeg2_dec_t *m)
{
	dec_bits *st = &m->stream_i;
	int zeros = 0, c, code;
	if (!m->pending) {
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
	m->pending = 0;
	code = m2d_stream_next_byte(st);
	if (code < 0) return -1;
	m->unit_len = 0;
	zeros = 0;
	for (;;) {
		c = m2d_stream_next_byte(st);
		if (c < 0) break;
		if (zeros >= 2 && c == 1) {
			m->unit_len -= (size_t)zeros;
			m->pending = 1;
			break;
		}
		if (m->unit_len + 16 >= m->unit_cap) {
			size_t cap = m->unit_cap ? 2 * m->unit_cap : (1u << 16);
			uint8_t *n = (uint8_t *)realloc(m->unit, cap);
			if (!n) return -1;
			m->unit = n;
			m->unit_cap = cap;
		}
		m->unit[m->unit_len++] = (uint8_t)c;
		zeros = (c == 0) ? zeros + 1 : 0;
	}
	if (!m->unit) {
		m->unit = (uint8_t *)calloc(1, 64);
		if (!m->unit) return -1;
		m->unit_cap = 64;
	}
	memset(m->unit + m->unit_len, 0, 16);
	return code;
}

/* ------------------------------------------------------------------ frames (mpeg2.cpp:130-220) */
static int find_valid_frame(int ref0, int ref1, int *lru, int num)
{
	int max_idx = -1, max_val = -1;
	for (int i = 0; i < num; ++i) {
		if (i != ref0 && i != ref1) {
			const int val = lru[i];
			lru[i] = val + 1;
			if (max_val < val) {
				max_val = val;
				max_idx = i;
			}
		}
	}
	if (max_idx < 0) max_idx = ref0; /* no available frame */
	lru[max_idx] = 0;
	return max_idx;
}

static void update_frames(mpeg2_dec_t *m, int next_coding_type, int temporal_reference)
{
	int curr;
	if (m->index < 0) { /* just after set_frames */
		m->out_state = (next_coding_type == M2V_I || next_coding_type == M2V_P) ? 2 : 0;
		m->index = 0;
		return;
	}
	curr = find_valid_frame(m->ref[0], m->ref[1], m->lru, m->num);
	if (next_coding_type == M2V_I || next_coding_type == M2V_P) {
		m->ref[0] = m->ref[1];
		m->ref[1] = curr;
		if (m->out_state < 4) m->out_state += 2;
	} else {
		m->out_state |= 1;
	}
	m->index = curr;
	m->frames[curr].cnt = temporal_reference;
	m->copy_src = m->ref[0]; /* set_ptrdiff(frames, 0, ref0_idx, curr_frame) */
}


/* ------------------------------------------------------------------ macroblock position */
static void set_frame_size(mpeg2_dec_t *m, int w, int h)
{
	const int mbx = (w + 15) >> 4, mby = (h + 15) >> 4;
	m->mbmax_x = mbx;
	m->mbmax_y = mby;
	m->fw = mbx * 16;
}

static void inc_mb_pos(mpeg2_dec_t *m)
{
	int x = m->mb_x + 1;
	const int w = m->mbmax_x;
	if (w <= x) {
		int inc_y = 0;
		do {
			x -= w;
			inc_y += 1;
		} while (w < x);
		m->mb_y += inc_y;
	}
	m->mb_x = x;
}

static int is_last(const mpeg2_dec_t *m)
{
	return (m->mb_y == m->mbmax_y - 1 && m->mbmax_x - 1 <= m->mb_x) || m->mbmax_y <= m->mb_y;
}

/* ------------------------------------------------------------------ records of the picture */
/* the picture's slots and an empty record per MB (flags 0: the MB keeps what the frame holds) */
static int picture_open(mpeg2_dec_t *m)
{
	m2v_picture_t *p = &m->pic;
	const int n = m->mbmax_x * m->mbmax_y;
	if (n <= 0) return -1;
	if (p->n_mbs != n || !p->mb) {
		free(p->mb);
		p->mb = (m2v_mb_t *)malloc(sizeof(m2v_mb_t) * (size_t)n);
		if (!p->mb) return -1;
	}
	if (m->coef_cap < (size_t)n * 6 * 64) {
		free(p->coef);
		m->coef_cap = (size_t)n * 6 * 64;
		p->coef = (int16_t *)malloc(sizeof(int16_t) * m->coef_cap);
		if (!p->coef) {
			m->coef_cap = 0;
			return -1;
		}
	}
	memset(p->mb, 0, sizeof(m2v_mb_t) * (size_t)n);
	for (int i = 0; i < n; ++i) {
		p->mb[i].mbx = (uint16_t)(i % m->mbmax_x);
		p->mb[i].mby = (uint16_t)(i / m->mbmax_x);
	}
	p->n_mbs = n;
	p->n_coef = 0;
	p->width = m->fw;
	p->height = m->mbmax_y * 16;
	p->cur = m->index < 0 ? 0 : m->index;
	p->fwd = m->ref[0];
	p->bwd = m->coding_type == M2V_B ? m->ref[1] : -1;
	p->copy = m->copy_src; /* -1: the very first picture, copies are in place (no-ops) */
	m->pic_open = 1;
	return 0;
}

/* the current MB position lies inside the picture (a damaged stream's address increments may run past it) */
static int mb_inside(const mpeg2_dec_t *m)
{
	return m->mb_x >= 0 && m->mb_x < m->mbmax_x && m->mb_y >= 0 && m->mb_y < m->mbmax_y;
}

static m2v_mb_t *rec_cur(mpeg2_dec_t *m)
{
	return &m->pic.mb[m->mb_y * m->mbmax_x + m->mb_x];
}

/* the records of the picture into its frame (CPU), or to the GPU */
static int picture_close(mpeg2_dec_t *m)
{
	if (!m->pic_open) return 0;
	m->pic_open = 0;
	if (m->gpu) return m2v_hip_submit(m->gpu, &m->pic);
	m2v_recon_picture_cpu(&m->pic, m->frames, &m->clip_out_of_domain, &m->mc_out_of_frame);
	return 0;
}

/* skipped / lost MB: a copy of the forward reference (m2d_skip_mb_P's copy, m2d_copy_slice) */
static int copy_in_place(const mpeg2_dec_t *m)
{
	return m->pic.copy < 0 || m->pic.copy == m->pic.cur;
}

/* (an in-place copy leaves the MB as it is — a slice starting mid-row re-"skips" MBs already decoded,
 * which the very first picture keeps) */
static void copy_mb(mpeg2_dec_t *m)
{
	m2v_mb_t *r = rec_cur(m);
	if (copy_in_place(m)) return;
	r->flags = M2V_REC_COPY;
	r->cbp = 0;
}

static void mb_reset(mpeg2_dec_t *m)
{
	const int dc = (m->dc_max + 1) >> 1;
	m->dc_pred[0] = m->dc_pred[1] = m->dc_pred[2] = (int16_t)dc;
	memset(m->pmv, 0, sizeof(m->pmv));
}

/* ------------------------------------------------------------------ headers */
static void load_qmat(uint8_t *q, const uint8_t *scan, h264_bits_t *b)
{
	for (int i = 0; i < 64; ++i) q[scan[i]] = (uint8_t)hb_get(b, 8);
}

static void set_default_state(mpeg2_dec_t *m)
{
	m->mpeg2 = 0;
	m->intra_vlc_format = 0;
	m->concealment_mv = 0;
	m->dc_scale = 3;
	m->dc_max = 255;
	m->frame_mode = 3;
	m->scan = m2v_scan[0];
	m->q_scale_type = 0;
}

static void sequence_header(mpeg2_dec_t *m, h264_bits_t *b)
{
	static const uint8_t flat16[64] = {
		16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
		16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
		16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16};
	m->hsize = (int)hb_get(b, 12);
	m->vsize = (int)hb_get(b, 12);
	hb_skip(b, 4 + 4);       /* aspect_ratio_information, frame_rate_code */
	hb_skip(b, 18 + 1 + 10 + 1); /* bit_rate_value, marker, vbv_buffer_size, constrained_parameters_flag */
	if (hb_get(b, 1)) {
		load_qmat(m->qmat_store[0], m2v_scan[0], b);
		m->qmat[0] = m->qmat_store[0];
	} else {
		m->qmat[0] = m2v_default_intra_qmat;
	}
	if (hb_get(b, 1)) {
		load_qmat(m->qmat_store[1], m2v_scan[0], b);
		m->qmat[1] = m->qmat_store[1];
	} else {
		m->qmat[1] = flat16;
	}
	set_frame_size(m, m->hsize, m->vsize);
	m->header_callback(m->header_callback_arg, m->stream_i.id);
}

static void extension(mpeg2_dec_t *m, h264_bits_t *b)
{
	const int id = (int)hb_get(b, 4);
	switch (id) {
	case 1: /* sequence_extension, mpeg2.cpp:358-379 */
		hb_skip(b, 8 + 1 + 2);   /* profile_and_level, progressive_sequence, chroma_format */
		m->hsize |= (int)hb_get(b, 2) << 12;
		m->vsize |= (int)hb_get(b, 2) << 12;
		set_frame_size(m, m->hsize, m->vsize);
		m->mpeg2 = 1;
		m->header_callback(m->header_callback_arg, m->stream_i.id);
		break;
	case 2: { /* sequence_display_extension, mpeg2.cpp:506-521 (video_format and colour_description in 4 bits) */
		const int format = (int)hb_get(b, 4);
		uint32_t wh;
		if (format & 1) hb_skip(b, 24);
		wh = hb_get(b, 29);
		m->disp_h = (int)(wh & 0x3fff);
		m->disp_w = (int)(wh >> 15);
		break;
	}
	case 3: /* quant_matrix_extension: loaded in the current scan order, as the reference (mpeg2.cpp:381-403) */
		for (int i = 0; i < 4; ++i) {
			if (hb_get(b, 1)) {
				load_qmat(m->qmat_store[i], m->scan, b);
				if (i < 2) m->qmat[i] = m->qmat_store[i];
			}
		}
		break;
	case 8: { /* picture_coding_extension, mpeg2.cpp:457-504 */
		const uint32_t f = hb_get(b, 16);
		uint32_t bits;
		m->r_size[0][0] = (int)(f >> 12) - 1;
		m->r_size[0][1] = (int)((f >> 8) & 15) - 1;
		m->r_size[1][0] = (int)((f >> 4) & 15) - 1;
		m->r_size[1][1] = (int)(f & 15) - 1;
		if (!m->coding_type) /* no picture header: guess from the f_codes */
			m->coding_type = ((f & 0xff) == 0xff) ? (((f & 0xff00) == 0xff00) ? M2V_I : M2V_P) : M2V_B;
		bits = hb_get(b, 14);
		m->intra_dc_precision = (int)(bits >> 12) & 3;
		m->picture_structure = (int)(bits >> 10) & 3;
		m->frame_pred_frame_dct = (int)(bits >> 8) & 1;
		m->concealment_mv = (int)(bits >> 7) & 1;
		m->q_scale_type = (int)(bits >> 6) & 1;
		m->intra_vlc_format = (int)(bits >> 5) & 1;
		m->alternate_scan = (int)(bits >> 4) & 1;
		m->dc_scale = 3 - m->intra_dc_precision;
		m->dc_max = (1 << (m->intra_dc_precision + 8)) - 1;
		m->scan = m2v_scan[m->alternate_scan];
		if (m->picture_structure == 1 || m->picture_structure == 2) m->frame_mode = 0;
		else if (m->picture_structure == 3) m->frame_mode = m->frame_pred_frame_dct ? 3 : 1;
		break;
	}
	default: /* display / copyright / scalable extensions: nothing the decoder uses */
		break;
	}
}

static int picture_header(mpeg2_dec_t *m, h264_bits_t *b)
{
	m->temporal_reference = (int)hb_get(b, 10);
	m->coding_type = (int)hb_get(b, 3);
	hb_skip(b, 16); /* vbv_delay */
	m->mb_x = -1;
	m->mb_y = 0;
	if (m->coding_type != M2V_I && m->coding_type != M2V_P && m->coding_type != M2V_B) return -1; /* D pictures */
	if (m->coding_type != M2V_I) {
		/* full_pel + f_code read as one 4-bit value minus 1, as the reference does (mpeg2.cpp:609-618);
		 * MPEG-2's picture coding extension replaces them */
		m->r_size[0][0] = m->r_size[0][1] = (int)hb_get(b, 4) - 1;
		if (m->coding_type == M2V_B) m->r_size[1][0] = m->r_size[1][1] = (int)hb_get(b, 4) - 1;
	}
	while (hb_get(b, 1)) hb_skip(b, 9); /* extra_information_picture as the reference reads it (mpeg2.cpp:617-619) */
	return 0;
}

/* ------------------------------------------------------------------ blocks */
/* parse_coef (mpeg2.cpp:1021-1113): coefficients from scan index `idx` into coef[] (raster; what is
 * below idx is kept), dequantised (intra ((|l| 2) W qs) >> 4, inter ((2|l| + 1) W qs) >> 5, sign,
 * +-2048 saturation), then MPEG-2 mismatch control over the block (coef[0] included when the
 * parse starts after it) or MPEG-1 oddification.  `level` values are sign-folded: (|l| << 1) | s. */
static int parse_coef(mpeg2_dec_t *m, h264_bits_t *b, int16_t *coef, int inter, int idx)
{
	const dct_lut_t *lut = lut_dct[inter ? 0 : m->intra_vlc_format];
	const uint8_t *qm = m->qmat[inter];
	const uint8_t *scan = m->scan;
	int mismatch = idx ? coef[0] : 0;
	memset(coef + idx, 0, sizeof(int16_t) * (size_t)(64 - idx));
	for (;; ++idx) {
		const dct_lut_t *e = &lut[hb_show(b, DCT_BITS)];
		int level, z;
		if (!e->len) return -1; /* undefined code: the reference abandons the slice (longjmp) */
		hb_skip(b, e->len);
		if (e->run >= 0) {
			idx += e->run;
			level = (e->level << 1) | (int)hb_get(b, 1);
		} else if (e->level) {
			break; /* end of block */
		} else { /* escape */
			idx += (int)hb_get(b, 6);
			if (m->mpeg2) {
				int v = (int)hb_get(b, 12);
				const int sign = v >> 11;
				level = ((((v ^ (-sign & 0xfff)) + sign) * 2) | sign);
			} else {
				int v = (int)hb_get(b, 8);
				if ((v & 0x7f) == 0) v = (int)hb_get(b, 8) - (v & 0x80) * 2;
				else v = (int8_t)v;
				level = v < 0 ? ((-v * 2) | 1) : v * 2;
			}
		}
		if (idx >= 64) break;
		z = scan[idx];
		{
			const int q = qm[z] * m->q_scale;
			const int t = inter ? (((level | 1) * q) >> 5) : (((level >> 1) * q) >> 4);
			int v = (level & 1) ? -t : t;
			v = v <= 2047 ? (v >= -2048 ? v : -2048) : 2047;
			mismatch += v;
			coef[z] = (int16_t)v;
		}
	}
	if (m->mpeg2) {
		if (!(mismatch & 1)) coef[63] ^= 1;
	} else {
		for (int i = 0; i < 64; ++i) {
			const int c = coef[i];
			if (c && !(c & 1)) coef[i] = (int16_t)(c > 0 ? c - 1 : c + 1);
		}
	}
	return 0;
}

/* the AC coefficients of an intra block (coef[0] holds the DC) */
static int intra_ac(mpeg2_dec_t *m, h264_bits_t *b)
{
	return parse_coef(m, b, m->coef, 0, 1);
}

/* mpeg2.cpp:920-939 */
static int intra_dc(mpeg2_dec_t *m, h264_bits_t *b, int cc, int *bad)
{
	const vlc_lut_t *e = cc ? &lut_dcc[hb_show(b, DC_BITS)] : &lut_dcl[hb_show(b, DC_BITS)];
	int size, diff = 0, dc;
	if (!e->len) {
		*bad = 1;
		return 0;
	}
	hb_skip(b, e->len);
	size = e->value;
	if (size) diff = (int)hb_get(b, size);
	dc = m->dc_pred[cc];
	if (size) {
		const int half = 1 << (size - 1);
		if (!(diff & half)) diff = diff + 1 - half * 2;
		dc += diff;
		m->dc_pred[cc] = (int16_t)dc;
		dc = dc < 0 ? 0 : dc > m->dc_max ? m->dc_max : dc;
	}
	return dc << m->dc_scale;
}

/* a non-intra block (m2d_parse_inter_block, mpeg2.cpp:1327-1341): a first coefficient coded "1s" is
 * level 1 at scan position 0, dequantised without saturation; then parse_coef from there */
static int inter_block(mpeg2_dec_t *m, h264_bits_t *b, int16_t *coef)
{
	const uint32_t bits = hb_show(b, 2);
	int idx = 0;
	if (bits & 2) {
		const int level = (int)bits; /* (1 << 1) | sign */
		const int t = ((level | 1) * (m->q_scale * m->qmat[1][0])) >> 5;
		hb_skip(b, 2);
		coef[0] = (int16_t)((level & 1) ? -t : t);
		idx = 1;
	}
	return parse_coef(m, b, coef, 1, idx);
}

/* ------------------------------------------------------------------ motion vectors */
/* m2d_one_mv (mpeg2.cpp:1189-1210): one component against its predictor *pmv (stored << is_field) */
static int one_mv(h264_bits_t *b, int16_t *pmv, int r_size, int is_field, int *bad)
{
	int mv;
	if (hb_get(b, 1) == 0) {
		const vlc_lut_t *e = &lut_mc[hb_show(b, MC_BITS - 1)]; /* index = the code with its leading 0 */
		int code, residual, limit;
		if (!e->len || e->len < 2) {
			*bad = 1;
			return 0;
		}
		/* e->len: the code's length with its leading 0; the sign bit follows the code */
		code = (hb_show(b, e->len) & 1) ? -e->value : e->value;
		hb_skip(b, e->len);
		if (r_size < 0) r_size = 0;
		residual = r_size > 0 ? 1 + (int)hb_get(b, r_size) : 1;
		mv = code >= 0 ? ((code - 1) << r_size) + residual : ((code + 1) << r_size) - residual;
		mv += *pmv >> is_field;
		limit = 16 << r_size;
		mv = (-limit <= mv) ? ((mv < limit) ? mv : mv - limit * 2) : mv + limit * 2;
	} else {
		mv = *pmv >> is_field;
	}
	*pmv = (int16_t)(mv << is_field);
	return mv;
}

/* m2d_motion_vectors (mpeg2.cpp:1245-1275) of direction s into the record */
static int motion_vectors(mpeg2_dec_t *m, h264_bits_t *b, int s, m2v_mb_t *r)
{
	int bad = 0;
	const int *rs = m->r_size[s];
	if (m->mv_count == 1) {
		if (m->mv_field && !m->mv_dmv) hb_skip(b, 1); /* motion_vertical_field_select (unused by the reference) */
		r->mv[s][0][0] = (int16_t)one_mv(b, &m->pmv[s][0][0], rs[0], 0, &bad);
		if (m->mv_dmv && hb_get(b, 1)) hb_skip(b, 1); /* dmvector (parsed, unused by the reference) */
		r->mv[s][0][1] = (int16_t)one_mv(b, &m->pmv[s][0][1], rs[1], m->mv_field, &bad);
		if (m->mv_dmv && hb_get(b, 1)) hb_skip(b, 1);
		m->pmv[s][1][0] = m->pmv[s][0][0];
		m->pmv[s][1][1] = m->pmv[s][0][1];
	} else {
		for (int i = 0; i < 2; ++i) {
			if (hb_get(b, 1)) r->field_sel |= (uint8_t)(1u << (2 * s + i));
			r->mv[s][i][0] = (int16_t)one_mv(b, &m->pmv[s][i][0], rs[0], 0, &bad);
			r->mv[s][i][1] = (int16_t)one_mv(b, &m->pmv[s][i][1], rs[1], 1, &bad);
		}
		r->flags |= M2V_REC_FIELD;
	}
	return bad ? -1 : 0;
}

/* ------------------------------------------------------------------ macroblocks */
static int vlc(h264_bits_t *b, const vlc_lut_t *lut, int bits, int *bad)
{
	const vlc_lut_t *e = &lut[hb_show(b, bits)];
	if (!e->len) {
		*bad = 1;
		return 0;
	}
	hb_skip(b, e->len);
	return e->value;
}

/* m2d_decode_macroblock_mode (mpeg2.cpp:834-872): macroblock_type, motion type, dct_type */
static int mb_modes(mpeg2_dec_t *m, h264_bits_t *b, int *bad)
{
	int type, idx;
	/* (motion types of frame / field pictures: count, field format, dual prime; m2d_motion_type) */
	static const int8_t mt[2][4][3] = {{{2, 1, 0}, {2, 1, 0}, {1, 0, 0}, {1, 1, 1}},
	                                   {{1, 1, 0}, {1, 1, 0}, {2, 1, 0}, {1, 1, 1}}};
	if (m->coding_type == M2V_P) type = vlc(b, lut_mbp, MBT_BITS, bad);
	else if (m->coding_type == M2V_B) type = vlc(b, lut_mbb, MBT_BITS, bad);
	else type = hb_get(b, 1) ? M2V_MBF_INTRA : (hb_get(b, 1) ? M2V_MBF_INTRA | M2V_MBF_QUANT : (*bad = 1, 0));
	if (*bad) return 0;
	if (type & (M2V_MBF_FWD | M2V_MBF_BWD)) {
		int f;
		if (m->frame_mode & 1) {
			idx = (m->frame_mode == 1) ? (int)hb_get(b, 2) : 2;
			f = 0;
		} else {
			idx = (int)hb_get(b, 2);
			f = 1;
		}
		m->mv_count = mt[f][idx][0];
		m->mv_field = mt[f][idx][1];
		m->mv_dmv = mt[f][idx][2];
	} else {
		idx = (m->frame_mode == 0);
		m->mv_count = mt[idx][2 - idx][0];
		m->mv_field = mt[idx][2 - idx][1];
		m->mv_dmv = mt[idx][2 - idx][2];
	}
	if (m->frame_mode == 1 && (type & (M2V_MBF_INTRA | M2V_MBF_PATTERN))) m->dct_type = (int)hb_get(b, 1);
	else m->dct_type = (m->frame_mode != 0) ? 0 : 1;
	return type;
}

/* one intra macroblock (mpeg2.cpp:1162-1187): quantiser, concealment vectors (parsed), 6 blocks */
static int intra_mb(mpeg2_dec_t *m, h264_bits_t *b, int type, m2v_mb_t *r)
{
	int bad = 0;
	if (type & M2V_MBF_QUANT) m->q_scale = m2v_q_scale[m->q_scale_type][hb_get(b, 5)];
	if (m->concealment_mv) { /* parsed (they update the predictors), not used for reconstruction */
		m2v_mb_t tmp;
		memset(&tmp, 0, sizeof(tmp));
		if (motion_vectors(m, b, 0, &tmp) < 0) return -1;
		hb_skip(b, 1); /* marker */
	}
	r->flags = M2V_REC_INTRA | (m->dct_type ? M2V_REC_DCT_FIELD : 0);
	r->cbp = 63;
	r->coef = (uint32_t)m->pic.n_coef;
	if ((size_t)m->pic.n_coef + 6 * 64 > m->coef_cap) return -1; /* (an MB parsed twice: damaged slices) */
	for (int i = 0; i < 6; ++i) {
		int16_t *c = m->pic.coef + m->pic.n_coef;
		m->coef[0] = (int16_t)intra_dc(m, b, i < 4 ? 0 : i - 3, &bad);
		if (bad || intra_ac(m, b) < 0) return -1;
		memcpy(c, m->coef, sizeof(m->coef));
		m->pic.n_coef += 64;
	}
	return 0;
}

/* one non-intra macroblock (m2d_parse_inter_macroblock, mpeg2.cpp:1355-1395) */
static int inter_mb(mpeg2_dec_t *m, h264_bits_t *b, int type, m2v_mb_t *r)
{
	if (type & M2V_MBF_QUANT) m->q_scale = m2v_q_scale[m->q_scale_type][hb_get(b, 5)];
	r->flags = m->dct_type ? M2V_REC_DCT_FIELD : 0;
	if (type & (M2V_MBF_FWD | M2V_MBF_BWD)) {
		if ((type & M2V_MBF_FWD) && motion_vectors(m, b, 0, r) < 0) return -1;
		if ((type & M2V_MBF_BWD) && motion_vectors(m, b, 1, r) < 0) return -1;
		r->flags |= ((type & M2V_MBF_FWD) ? M2V_REC_FWD : 0) | ((type & M2V_MBF_BWD) ? M2V_REC_BWD : 0);
		if (m->mv_count == 1) r->flags &= (uint8_t)~M2V_REC_FIELD;
	} else {
		/* P "no MC": m2d_skip_mb_P(mb, 0) — the co-located MB of the forward reference, predictors reset */
		r->flags |= M2V_REC_FWD;
		mb_reset(m);
	}
	r->cbp = 0;
	r->coef = (uint32_t)m->pic.n_coef;
	if (type & M2V_MBF_PATTERN) {
		int bad = 0;
		const int cbp = vlc(b, lut_cbp, CBP_BITS, &bad);
		if (bad) return -1;
		r->cbp = (uint8_t)cbp;
		if ((size_t)m->pic.n_coef + 6 * 64 > m->coef_cap) return -1; /* (an MB parsed twice: damaged slices) */
		for (int i = 0; i < 6; ++i)
			if (cbp & (1 << (5 - i))) {
				if (inter_block(m, b, m->pic.coef + m->pic.n_coef) < 0) return -1;
				m->pic.n_coef += 64;
			}
	}
	return 0;
}

/* m2d_parse_macroblock (mpeg2.cpp:1401-1420) */
static int parse_mb(mpeg2_dec_t *m, h264_bits_t *b)
{
	int bad = 0;
	const int prev_intra = (m->prev_type & M2V_MBF_INTRA) != 0;
	const int type = mb_modes(m, b, &bad);
	m2v_mb_t *r = rec_cur(m);
	if (bad) return -1;
	m->prev_type = type;
	memset(r->mv, 0, sizeof(r->mv));
	r->field_sel = 0;
	if (type & M2V_MBF_INTRA) {
		if (!prev_intra) {
			const int dc = (m->dc_max + 1) >> 1;
			m->dc_pred[0] = m->dc_pred[1] = m->dc_pred[2] = (int16_t)dc;
		}
		if (intra_mb(m, b, type, r) < 0) goto bad;
		return 0;
	}
	if (prev_intra) memset(m->pmv, 0, sizeof(m->pmv));
	if (inter_mb(m, b, type, r) < 0) goto bad;
	return 0;
bad:
	/* an undefined code inside the MB (damaged data): the record is dropped — its blocks may point past the
	 * coefficients written — and the slice is abandoned by the caller */
	r->flags = 0;
	r->cbp = 0;
	return -1;
}

/* skipped macroblocks before the current one (mb->skip_mb, mpeg2.cpp:740-766, 773-810): P (and I,
 * whose table entry is the P one) copy the forward reference, then reset the predictors; B repeat
 * the prediction of the last coded MB — its directions and the first vector of each (frame MC) */
static void skip_mbs(mpeg2_dec_t *m, int n)
{
	if (m->coding_type != M2V_B) {
		for (int k = 0; k < n; ++k) {
			inc_mb_pos(m);
			if (!mb_inside(m)) break;
			copy_mb(m);
		}
		mb_reset(m);
		return;
	}
	{
		const int dir = m->prev_type & (M2V_MBF_FWD | M2V_MBF_BWD);
		const int bi = dir == (M2V_MBF_FWD | M2V_MBF_BWD);
		const int one = bi ? 0 : (dir >> 1); /* (an intra last MB: forward) */
		for (int k = 0; k < n; ++k) {
			m2v_mb_t *r;
			inc_mb_pos(m);
			if (!mb_inside(m)) break;
			r = rec_cur(m);
			memset(r->mv, 0, sizeof(r->mv));
			r->field_sel = 0;
			r->cbp = 0;
			if (bi) {
				r->flags = M2V_REC_FWD | M2V_REC_BWD;
				memcpy(r->mv[0][0], m->pmv[0][0], sizeof(r->mv[0][0]));
				memcpy(r->mv[1][0], m->pmv[1][0], sizeof(r->mv[1][0]));
			} else {
				r->flags = one ? M2V_REC_BWD : M2V_REC_FWD;
				memcpy(r->mv[one][0], m->pmv[one][0], sizeof(r->mv[one][0]));
			}
		}
	}
}

/* macroblock_address_increment (mpeg2.cpp:1427-1453) */
static int mb_increment(h264_bits_t *b, int *bad)
{
	int val = 0;
	if (hb_get(b, 1)) return 1;
	for (;;) {
		const vlc_lut_t *e = &lut_inc[hb_show(b, INC_BITS - 1)];
		if (!e->len || e->len < 2) {
			*bad = 1;
			return 0;
		}
		hb_skip(b, e->len - 1);
		val += e->value;
		if (e->value != 0) break;
		val += 33;
		if (hb_get(b, 1)) {
			val += 1;
			break;
		}
	}
	return val;
}

/* slice (mpeg2.cpp:625-660) + m2d_decode_macroblocks (1502-1524); 1: the picture's last MB done */
static int slice(mpeg2_dec_t *m, h264_bits_t *b, int code)
{
	const int vpos = code - 1;
	int err = 0;
	m->q_scale = m2v_q_scale[m->q_scale_type][hb_get(b, 5)];
	if (vpos == 0) {
		picture_close(m); /* (an unfinished picture before this one) */
		update_frames(m, m->coding_type, m->temporal_reference);
		if (picture_open(m) < 0) return -1;
	}
	if (!m->pic_open || m->mbmax_y <= vpos) return 0;
	if (1 < vpos - m->mb_y && !copy_in_place(m)) { /* lost rows: copied from the forward reference (m2d_copy_slice) */
		for (int y = m->mb_y + 1; y < vpos; ++y)
			for (int x = 0; x < m->mbmax_x; ++x) {
				m2v_mb_t *r = &m->pic.mb[y * m->mbmax_x + x];
				r->flags = M2V_REC_COPY;
				r->cbp = 0;
			}
	}
	m->mb_x = -1;
	m->mb_y = vpos;
	if (hb_get(b, 1)) { /* extra_bit_slice: intra_slice_flag, intra_slice, reserved / MPEG-1 extra info */
		hb_skip(b, 8);
		while (hb_get(b, 1)) hb_skip(b, 8);
	}
	mb_reset(m);
	do {
		int bad = 0;
		const int inc = mb_increment(b, &bad);
		if (bad) return 0;
		if (1 < inc) skip_mbs(m, inc - 1);
		inc_mb_pos(m);
		if (!mb_inside(m)) return 0; /* an increment past the picture: slice abandoned */
		if (parse_mb(m, b) < 0) return 0; /* undefined code: slice abandoned */
		if (is_last(m)) {
			m->mb_x = -1;
			m->mb_y = 0;
			err = 1;
			break;
		}
	} while (hb_show(b, 23) != 0);
	return err;
}

/* ------------------------------------------------------------------ CPU reconstruction (C1) */
#define W1 2841
#define W2 2676
#define W3 2408
#define W5 1609
#define W6 1108
#define W7 565

/* idct.cpp:69-236: one row, results stored back as int16 */
static void idct_row(int16_t *s)
{
	const int32_t s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3], s4 = s[4], s5 = s[5], s6 = s[6], s7 = s[7];
	int32_t a0 = s0 * 2048 + 128, a1 = s4 * 2048, t;
	int32_t e0 = a0 - a1, e1 = a0 + a1;
	int32_t o4 = W7 * (s1 + s7) + (W1 - W7) * s1;
	int32_t o5 = W7 * (s1 + s7) - (W1 + W7) * s7;
	int32_t o6 = W3 * (s5 + s3) - (W3 - W5) * s5;
	int32_t o7 = W3 * (s5 + s3) - (W3 + W5) * s3;
	int32_t p4 = o4 - o6, p6 = o4 + o6, p5 = o5 - o7, p7 = o5 + o7;
	int32_t q5 = ((p4 + p5) * 181 + 128) >> 8;
	int32_t q4 = ((p4 - p5) * 181 + 128) >> 8;
	int32_t x2 = W6 * (s2 + s6) - (W2 + W6) * s6;
	int32_t x3 = W6 * (s2 + s6) + (W2 - W6) * s2;
	t = e0;
	e0 = e0 - x2;
	x2 = t + x2;
	t = e1;
	e1 = e1 - x3;
	x3 = t + x3;
	s[0] = (int16_t)((x3 + p6) >> 8);
	s[1] = (int16_t)((x2 + q5) >> 8);
	s[2] = (int16_t)((e0 + q4) >> 8);
	s[3] = (int16_t)((e1 + p7) >> 8);
	s[4] = (int16_t)((e1 - p7) >> 8);
	s[5] = (int16_t)((e0 - q4) >> 8);
	s[6] = (int16_t)((x2 - q5) >> 8);
	s[7] = (int16_t)((x3 - p6) >> 8);
}

static inline uint8_t clip255c(uint64_t *bad, int v)
{
	if (v < -256 || v > 767) (*bad)++; /* CLIP255C table domain (m2d.cpp:157-289) */
	return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

/* idct.cpp:286-422: columns with (x + 8192) >> 14, ClipStore (intra) or AddStore (inter); dst column
 * step `step` (1 luma, 2 NV12 chroma) */
static void idct_block(int16_t *c, uint8_t *dst, int stride, int step, int add, uint64_t *bad)
{
	for (int r = 0; r < 8; ++r) idct_row(c + 8 * r);
	for (int col = 0; col < 8; ++col, ++c, dst += step) {
		const int32_t s0 = c[0], s1 = c[8], s2 = c[16], s3 = c[24], s4 = c[32], s5 = c[40], s6 = c[48], s7 = c[56];
		int32_t x8 = W3 * (s5 + s3) + 4;
		const int32_t x6a = (x8 - (W3 - W5) * s5) >> 3, x7a = (x8 - (W3 + W5) * s3) >> 3;
		x8 = W7 * (s1 + s7) + 4;
		const int32_t x4a = (x8 + (W1 - W7) * s1) >> 3, x5a = (x8 - (W1 + W7) * s7) >> 3;
		int32_t x1 = W6 * (s2 + s6) + 4;
		const int32_t x2 = (x1 - (W2 + W6) * s6) >> 3, x3 = (x1 + (W2 - W6) * s2) >> 3;
		x1 = x4a + x6a;
		const int32_t x4 = x4a - x6a, x6 = x5a + x7a, x5 = x5a - x7a;
		int32_t x0 = s0 * 256 + 8192;
		const int32_t x7 = s4 * 256;
		x8 = x0 + x7;
		x0 = x0 - x7;
		const int32_t y7 = x8 + x3, y8 = x8 - x3, y3 = x0 + x2, y0 = x0 - x2;
		const int32_t z2 = ((x4 + x5) * 181 + 128) >> 8, z4 = ((x4 - x5) * 181 + 128) >> 8;
		const int32_t v[8] = {(y7 + x1) >> 14, (y3 + z2) >> 14, (y0 + z4) >> 14, (y8 + x6) >> 14,
		                      (y8 - x6) >> 14, (y0 - z4) >> 14, (y3 - z2) >> 14, (y7 - x1) >> 14};
		uint8_t *d = dst;
		for (int k = 0; k < 8; ++k, d += stride) d[0] = clip255c(bad, add ? d[0] + v[k] : v[k]);
	}
}

/* one half-sample interpolated prediction sample (motioncomp.cpp: copy, (a + b + 1) >> 1 horizontal /
 * vertical, (a + b + c + d + 2) >> 2) at (x, y) of plane p (row stride `stride`, `gap` bytes between
 * horizontal neighbours), with the half flags hx / hy; reads outside [0, w) x [0, h) are clamped and
 * counted (the reference reads outside its frame) */
static inline int mc_px(const uint8_t *p, int stride, int w, int h, int gap, int x, int y, int hx, int hy, uint64_t *oob)
{
	const int x1 = x + gap * hx, y1 = y + hy;
	if (x < 0 || y < 0 || x1 >= w || y1 >= h) {
		(*oob)++;
		x = x < 0 ? 0 : x >= w ? w - 1 : x;
		y = y < 0 ? 0 : y >= h ? h - 1 : y;
	}
	{
		const int xb = x1 < 0 ? 0 : x1 >= w ? w - 1 : x1, yb = y1 < 0 ? 0 : y1 >= h ? h - 1 : y1;
		const int a = p[y * stride + x], b = p[y * stride + xb], c = p[yb * stride + x], d = p[yb * stride + xb];
		if (hx && hy) return (a + b + c + d + 2) >> 2;
		if (hx) return (a + b + 1) >> 1;
		if (hy) return (a + c + 1) >> 1;
		return a;
	}
}

/* the prediction of one direction into (or, avg, averaged with) the MB at (mbx, mby) of cur: frame
 * prediction (one vector, 16 lines) or field prediction (vector i for the lines of parity i, from the
 * reference field field_sel); chroma vector = luma vector / 2 truncated (motioncomp.cpp:499-505) */
static void predict(const m2d_frame_t *ref, const m2d_frame_t *cur, int W, int H, const m2v_mb_t *r, int dir, int avg,
                    uint64_t *oob)
{
	const int field = (r->flags & M2V_REC_FIELD) != 0;
	for (int part = 0; part < (field ? 2 : 1); ++part) {
		const int mvx = r->mv[dir][part][0], mvy = r->mv[dir][part][1];
		const int sel = field ? (r->field_sel >> (2 * dir + part)) & 1 : 0;
		/* field lines: plane rows 2 k + sel of the reference, written to rows 2 k + part */
		const int rs = field ? 2 : 1;                   /* row step in the frame */
		const int lh = field ? 8 : 16, ch = field ? 4 : 8;
		const int fh = field ? H / 2 : H;              /* height of the plane being read (field or frame) */
		for (int j = 0; j < lh; ++j)
			for (int i = 0; i < 16; ++i) {
				const int x = r->mbx * 16 + i + (mvx >> 1);
				const int yf = (field ? r->mby * 8 : r->mby * 16) + j + (mvy >> 1);
				const int v = mc_px(ref->luma + (field ? sel * W : 0), W * rs, W, fh, 1, x, yf, mvx & 1, mvy & 1, oob);
				uint8_t *d = cur->luma + (size_t)(r->mby * 16 + j * rs + (field ? part : 0)) * W + r->mbx * 16 + i;
				*d = (uint8_t)(avg ? (*d + v + 1) >> 1 : v);
			}
		{
			const int cx = mvx / 2, cy = mvy / 2;
			for (int j = 0; j < ch; ++j)
				for (int i = 0; i < 16; ++i) { /* bytes: Cb / Cr interleaved */
					const int x = r->mbx * 16 + i + 2 * (cx >> 1);
					const int yf = (field ? r->mby * 4 : r->mby * 8) + j + (cy >> 1);
					const int v = mc_px(ref->chroma + (field ? sel * W : 0), W * rs, W, fh / 2, 2, x, yf, cx & 1, cy & 1, oob);
					uint8_t *d = cur->chroma + (size_t)(r->mby * 8 + j * rs + (field ? part : 0)) * W + r->mbx * 16 + i;
					*d = (uint8_t)(avg ? (*d + v + 1) >> 1 : v);
				}
		}
	}
}

void m2v_recon_picture_cpu(const m2v_picture_t *pic, const m2d_frame_t *frames, uint64_t *clip_bad, uint64_t *mc_bad)
{
	const int W = pic->width, H = pic->height;
	const m2d_frame_t *cur = &frames[pic->cur];
	for (int k = 0; k < pic->n_mbs; ++k) {
		const m2v_mb_t *r = &pic->mb[k];
		int16_t c[64];
		const int16_t *src = pic->coef + r->coef;
		if (!r->flags) continue;
		if (r->flags & M2V_REC_COPY) {
			m2v_mb_t z;
			if (pic->copy < 0 || pic->copy == pic->cur) continue; /* in place */
			memset(&z, 0, sizeof(z));
			z.mbx = r->mbx;
			z.mby = r->mby;
			predict(&frames[pic->copy], cur, W, H, &z, 0, 0, mc_bad);
			continue;
		}
		if (r->flags & M2V_REC_FWD) predict(&frames[pic->fwd < 0 ? pic->cur : pic->fwd], cur, W, H, r, 0, 0, mc_bad);
		if (r->flags & M2V_REC_BWD)
			predict(&frames[pic->bwd < 0 ? pic->cur : pic->bwd], cur, W, H, r, 1, (r->flags & M2V_REC_FWD) != 0, mc_bad);
		{
			const int dct_field = (r->flags & M2V_REC_DCT_FIELD) != 0, add = !(r->flags & M2V_REC_INTRA);
			uint8_t *luma = cur->luma + (size_t)r->mby * 16 * W + (size_t)r->mbx * 16;
			uint8_t *chroma = cur->chroma + (size_t)r->mby * 8 * W + (size_t)r->mbx * 16;
			for (int i = 0; i < 6; ++i) {
				if (!(r->cbp & (1 << (5 - i)))) continue;
				memcpy(c, src, sizeof(c));
				src += 64;
				if (i < 4) {
					/* LUMA_BLOCK_OFFSET (mpeg2.cpp:1120) */
					const size_t off = !dct_field ? (size_t)((i & 1) + ((i & 2) ? W : 0)) * 8
					                              : (size_t)(i & 1) * 8 + ((i & 2) ? (size_t)W : 0);
					idct_block(c, luma + off, W << dct_field, 1, add, clip_bad);
				} else {
					idct_block(c, chroma + (i - 4), W, 2, add, clip_bad);
				}
			}
		}
	}
}

/* ------------------------------------------------------------------ m2d_func_table_t */
static mpeg2_dec_t *CTX(void *p) { return (mpeg2_dec_t *)p; }

static int hdr_dummy(void *a, void *b)
{
	(void)a;
	(void)b;
	return 0;
}

extern int m2dec_host_cpu_ok; /* cpucheck.c */

static int api_init(void *ctx, int dummy, int (*cb)(void *, void *), void *arg)
{
	mpeg2_dec_t *m = CTX(ctx);
	(void)dummy;
	if (!m || !m2dec_host_cpu_ok) return -1;
	memset(m, 0, sizeof(*m));
	pthread_once(&lut_once, build_luts);
	m->header_callback = cb ? cb : hdr_dummy;
	m->header_callback_arg = arg;
	set_default_state(m);
	m->qmat[0] = m2v_default_intra_qmat;
	m->qmat[1] = m2v_default_intra_qmat; /* replaced by the first sequence header */
	m->prev_intra = 0;
	m->copy_src = -1;
	dec_bits_open(&m->stream_i, NULL);
	return 0;
}

static dec_bits *api_stream_pos(void *ctx)
{
	return &CTX(ctx)->stream_i;
}

/* mpeg2.cpp:1632-1651 */
static int api_get_info(void *ctx, m2d_info_t *info)
{
	mpeg2_dec_t *m = CTX(ctx);
	if (!m || !info) return -1;
	info->src_width = (int16_t)((m->hsize + 15) & ~15);
	info->src_height = (int16_t)((m->vsize + 15) & ~15);
	info->disp_width = (int16_t)m->disp_w;
	info->disp_height = (int16_t)m->disp_h;
	info->frame_num = 3;
	info->crop[0] = 0;
	info->crop[1] = (int16_t)(info->src_width - m->hsize);
	info->crop[2] = 0;
	info->crop[3] = (int16_t)(info->src_height - m->vsize);
	info->additional_size = 0;
	return 0;
}

/* mpeg2.cpp:111-128 */
static int api_set_frames(void *ctx, int n, m2d_frame_t *frames, uint8_t *work, int work_len)
{
	mpeg2_dec_t *m = CTX(ctx);
	(void)work;
	(void)work_len;
	if (!m || (unsigned)n > M2V_MAX_FRAMES || !frames) return -1;
	m->num = n;
	memcpy(m->frames, frames, sizeof(m2d_frame_t) * (size_t)n);
	for (int i = 0; i < n; ++i)
		if (!frames[i].luma || ((uintptr_t)frames[i].luma & 15) || !frames[i].chroma || ((uintptr_t)frames[i].chroma & 15))
			return -1;
	m->index = -1;
	m->pic_open = 0;
	if (m->gpu && m2v_hip_set_frames(m->gpu, n, frames, m->fw, m->mbmax_y * 16) < 0) return -1;
	return 0;
}

/* m2d_decode_data (mpeg2.cpp:1583-1604) */
static int api_decode_picture(void *ctx)
{
	mpeg2_dec_t *m = CTX(ctx);
	if (!m) return -1;
	m->coding_type = 0;
	for (;;) {
		h264_bits_t b;
		int err = 0;
		const int code = next_unit(m);
		if (code < 0) {
			picture_close(m); /* (an unfinished last picture: what was decoded of it) */
			return -1;
		}
		hb_init(&b, m->unit, m->unit_len);
		if (code == 0) {
			if (picture_header(m, &b) < 0) return -1;
		} else if (code < 0xb0) {
			if (!m->num) return -1; /* no frames */
			err = slice(m, &b, code);
			if (err == 1 && picture_close(m) < 0) return -1;
		} else if (code == 0xb3) {
			sequence_header(m, &b);
		} else if (code == 0xb5) {
			extension(m, &b);
		}
		/* 0xb2 user data, 0xb8 GOP header, 0xb7 sequence end, system codes: nothing to do */
		if (err == 1) {
			m->pictures++;
			return 1;
		}
	}
}

static void frame_info(const mpeg2_dec_t *m, m2d_frame_t *f, int idx)
{
	*f = m->frames[idx];
	f->width = (int16_t)m->hsize; /* stride = horizontal_size_value (reference quirk) */
	f->height = (int16_t)m->vsize;
}

/* mpeg2.cpp:1543-1573 */
static int api_peek(void *ctx, m2d_frame_t *frame, int is_end)
{
	mpeg2_dec_t *m = CTX(ctx);
	int idx, r;
	if (!m || !frame) return -1;
	if (m->coding_type == M2V_B) idx = m->index;
	else if (is_end && 0 < m->out_state && m->out_state < 4) idx = m->ref[1];
	else idx = m->ref[0];
	frame_info(m, frame, idx < 0 ? 0 : idx);
	if (m->coding_type != M2V_B) {
		const int s = m->out_state >> 1;
		r = s == 0 ? 0 : s == 1 ? is_end != 0 : s == 2 ? 1 : 0;
	} else {
		r = m->out_state & 1;
	}
	/* a frame handed out: its picture into the caller's memory now */
	if (r > 0 && m->gpu && m2v_hip_sync(m->gpu, idx < 0 ? 0 : idx) < 0) return -1;
	return r;
}

static int api_get(void *ctx, m2d_frame_t *frame, int is_end)
{
	mpeg2_dec_t *m = CTX(ctx);
	const int r = api_peek(ctx, frame, is_end);
	if (r > 0) {
		if (m->coding_type == M2V_B) m->out_state &= ~1;
		else m->out_state -= 2;
	}
	return r;
}

static const m2d_func_table_t m2d_func_ = {
	sizeof(mpeg2_dec_t),
	api_init,
	api_stream_pos,
	api_get_info,
	api_set_frames,
	api_decode_picture,
	api_peek,
	api_get,
};

const m2d_func_table_t * const m2d_func = &m2d_func_;

/* extra C ABI: release the heap a context owns (the reference's context owns none); CLIP255C
 * domain violations seen by a context (checks that no output depends on reference UB) */
void m2dec_amd_m2v_release(void *ctx)
{
	mpeg2_dec_t *m = CTX(ctx);
	if (!m) return;
	free(m->unit);
	m->unit = NULL;
	m->unit_cap = 0;
	free(m->pic.mb);
	free(m->pic.coef);
	m->pic.mb = NULL;
	m->pic.coef = NULL;
	m->pic.n_mbs = 0;
	m->coef_cap = 0;
	if (m->gpu) m2v_hip_destroy(m->gpu);
	m->gpu = NULL;
}

/* reconstruct on the gfx950 GPU instead of the CPU (call after init, before the first sequence
 * header); -1 if no usable device: the context then keeps the CPU reconstruction */
int m2dec_amd_m2v_use_gpu(void *ctx, int device)
{
	mpeg2_dec_t *m = CTX(ctx);
	if (!m || m->gpu) return -1;
	m->gpu = m2v_hip_create(device);
	if (!m->gpu) {
		fprintf(stderr, "m2dec_amd: no gfx950 device for the MPEG-2 reconstruction\n");
		return -1;
	}
	m->gpu_device = device;
	return 0;
}

uint64_t m2dec_amd_m2v_mc_out_of_frame(const void *ctx)
{
	return ctx ? ((const mpeg2_dec_t *)ctx)->mc_out_of_frame : 0;
}

uint64_t m2dec_amd_m2v_clip_violations(const void *ctx)
{
	return ctx ? ((const mpeg2_dec_t *)ctx)->clip_out_of_domain : 0;
}

/* probes of the block-level paths for the reference's own unit tests (m2dec.cpp:142-217,
 * mpeg2.cpp:1743-1798): the decoder state is a fresh context (m2d_mb_set_default) */
int m2dec_amd_m2v_intra_dc(const uint8_t *bits, size_t n, int cc, int dc_precision, int pred, int *value)
{
	mpeg2_dec_t m;
	h264_bits_t b;
	int bad = 0;
	pthread_once(&lut_once, build_luts);
	memset(&m, 0, sizeof(m));
	m.dc_scale = 3 - dc_precision;
	m.dc_max = (1 << (8 + dc_precision)) - 1;
	m.dc_pred[0] = m.dc_pred[1] = m.dc_pred[2] = (int16_t)pred;
	hb_init(&b, bits, n);
	*value = intra_dc(&m, &b, cc, &bad);
	return bad ? -1 : (int)((b.p - bits) * 8 - (size_t)b.bits); /* bits consumed */
}

int m2dec_amd_m2v_intra_ac(const uint8_t *bits, size_t n, int mpeg2, int intra_vlc_format, int alternate_scan,
                           int q_scale, const uint8_t *qmat, int dc, int16_t coef[64])
{
	static const uint8_t flat16[64] = {
		16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
		16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
		16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16};
	mpeg2_dec_t m;
	h264_bits_t b;
	pthread_once(&lut_once, build_luts);
	memset(&m, 0, sizeof(m));
	m.mpeg2 = mpeg2;
	m.intra_vlc_format = intra_vlc_format;
	m.scan = m2v_scan[alternate_scan & 1];
	m.q_scale = q_scale;
	m.qmat[0] = qmat ? qmat : flat16;
	m.coef[0] = (int16_t)dc;
	hb_init(&b, bits, n);
	if (intra_ac(&m, &b) < 0) return -1;
	memcpy(coef, m.coef, sizeof(m.coef));
	return (int)((b.p - bits) * 8 - (size_t)b.bits);
}
