/* CABAC arithmetic encoder (ITU-T H.264 9.3.4.2 - 9.3.4.6); context init per 9.3.1.1. */
#include "bitwriter.h"
#include "h264_spec_tables.h"

void cenc_init_ctx(cenc_t *e, int is_i, int cabac_init_idc, int qp)
{
	int tab = is_i ? 0 : 1 + cabac_init_idc;
	for (int i = 0; i < H264_NUM_CTX; ++i) {
		int m = h264_cabac_init_mn[tab][i][0], n = h264_cabac_init_mn[tab][i][1];
		int pre = ((m * (qp < 0 ? 0 : (qp > 51 ? 51 : qp))) >> 4) + n;
		if (pre < 1) pre = 1;
		if (pre > 126) pre = 126;
		if (pre <= 63) e->st[i] = (uint8_t)((63 - pre) << 1);
		else e->st[i] = (uint8_t)(((pre - 64) << 1) | 1);
	}
	/* ctx 276 (end_of_slice / I_PCM) is the terminate context: not adaptive */
}

void cenc_start(cenc_t *e, bw_t *w)
{
	e->w = w;
	e->low = 0;
	e->range = 510;
	e->outstanding = 0;
	e->first = 1;
}

static void put_bit(cenc_t *e, int b)
{
	if (e->first) e->first = 0;
	else bw_bit(e->w, b);
	while (e->outstanding > 0) {
		bw_bit(e->w, 1 - b);
		e->outstanding--;
	}
}

static void renorm(cenc_t *e)
{
	while (e->range < 256) {
		if (e->low < 256) {
			put_bit(e, 0);
		} else if (e->low >= 512) {
			e->low -= 512;
			put_bit(e, 1);
		} else {
			e->low -= 256;
			e->outstanding++;
		}
		e->range <<= 1;
		e->low <<= 1;
	}
}

void cenc_decision(cenc_t *e, int ctx, int bin)
{
	int s = e->st[ctx] >> 1, mps = e->st[ctx] & 1;
	uint32_t lps = h264_range_lps[s][(e->range >> 6) & 3];
	e->range -= lps;
	if (bin != mps) {
		e->low += e->range;
		e->range = lps;
		if (s == 0) mps = 1 - mps;
		s = h264_trans_idx_lps[s];
	} else {
		if (s < 62) s++;
	}
	e->st[ctx] = (uint8_t)((s << 1) | mps);
	renorm(e);
}

void cenc_bypass(cenc_t *e, int bin)
{
	e->low <<= 1;
	if (bin) e->low += e->range;
	if (e->low >= 1024) {
		put_bit(e, 1);
		e->low -= 1024;
	} else if (e->low < 512) {
		put_bit(e, 0);
	} else {
		e->low -= 512;
		e->outstanding++;
	}
}

void cenc_terminate(cenc_t *e, int bin)
{
	e->range -= 2;
	if (bin) {
		e->low += e->range;
		/* EncodeFlush (9.3.4.5) */
		e->range = 2;
		renorm(e);
		put_bit(e, (e->low >> 9) & 1);
		bw_bits(e->w, ((e->low >> 7) & 3) | 1, 2);
	} else {
		renorm(e);
	}
}
