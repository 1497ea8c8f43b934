/* Bit writer, NAL packaging and CABAC encoder for the synthetic stream generator (spec 7.2, 9.3.4). */
#ifndef H264GEN_BITWRITER_H
#define H264GEN_BITWRITER_H
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
	uint8_t *b;
	size_t cap, n; /* bytes completed */
	uint32_t acc;  /* pending bits (MSB first) */
	int na;        /* number of pending bits (< 8) */
} bw_t;

static inline void bw_init(bw_t *w)
{
	memset(w, 0, sizeof(*w));
	w->cap = 1 << 16;
	w->b = (uint8_t *)malloc(w->cap);
}

static inline void bw_reset(bw_t *w)
{
	w->n = 0;
	w->acc = 0;
	w->na = 0;
}

static inline void bw_byte(bw_t *w, uint8_t v)
{
	if (w->n == w->cap) {
		w->cap *= 2;
		w->b = (uint8_t *)realloc(w->b, w->cap);
	}
	w->b[w->n++] = v;
}

static inline void bw_bit(bw_t *w, int v)
{
	w->acc = (w->acc << 1) | (uint32_t)(v & 1);
	if (++w->na == 8) {
		bw_byte(w, (uint8_t)w->acc);
		w->acc = 0;
		w->na = 0;
	}
}

static inline void bw_bits(bw_t *w, uint32_t v, int n)
{
	for (int i = n - 1; i >= 0; --i) bw_bit(w, (int)((v >> i) & 1));
}

static inline void bw_ue(bw_t *w, uint32_t v)
{
	uint32_t x = v + 1;
	int len = 31 - __builtin_clz(x);
	bw_bits(w, 0, len);
	bw_bits(w, x, len + 1);
}

static inline void bw_se(bw_t *w, int v)
{
	bw_ue(w, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v));
}

static inline void bw_te(bw_t *w, int v, int range)
{
	if (range == 1) bw_bit(w, !v);
	else bw_ue(w, (uint32_t)v);
}

static inline int bw_aligned(const bw_t *w) { return w->na == 0; }

static inline void bw_trailing(bw_t *w)
{
	bw_bit(w, 1);
	while (w->na) bw_bit(w, 0);
}

/* Annex B: start code, NAL header, RBSP with emulation prevention (7.4.1) */
static inline void nal_emit(bw_t *out, int ref_idc, int type, const bw_t *rbsp)
{
	int zeros = 0;
	bw_byte(out, 0);
	bw_byte(out, 0);
	bw_byte(out, 0);
	bw_byte(out, 1);
	bw_byte(out, (uint8_t)((ref_idc << 5) | type));
	for (size_t i = 0; i < rbsp->n; ++i) {
		uint8_t v = rbsp->b[i];
		if (zeros >= 2 && v <= 3) {
			bw_byte(out, 3);
			zeros = 0;
		}
		bw_byte(out, v);
		zeros = (v == 0) ? zeros + 1 : 0;
	}
}

/* ------------------------------------------------------------------ CABAC encoder (9.3.4.2 - 9.3.4.6) */
typedef struct {
	bw_t *w;
	uint32_t low, range;
	int outstanding;
	int first;
	uint8_t st[1024]; /* (pStateIdx << 1) | valMPS */
} cenc_t;

void cenc_init_ctx(cenc_t *e, int slice_type_i, int cabac_init_idc, int qp);
void cenc_start(cenc_t *e, bw_t *w);
void cenc_decision(cenc_t *e, int ctx, int bin);
void cenc_bypass(cenc_t *e, int bin);
void cenc_terminate(cenc_t *e, int bin); /* bin 1 flushes */

#endif
