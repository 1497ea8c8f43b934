/*
 * Record traces: parse a whole stream once on the host and keep every picture's records
 * (include/m2d_recon.h) in one contiguous buffer, in decoding order, plus the output order.
 *
 * A trace is what the GPU replay (m2dec_amd_hip_replay_*) uploads once and then reconstructs
 * repeatedly with the records resident in HBM — the measurement of the reconstruction hot path
 * without the host parse (bench.py).  Capturing uses the same parser and driver as decoding
 * (m2dec_amd_decode_stream) with a back end that stores records instead of reconstructing.
 */
#include <stdlib.h>
#include <string.h>
#include "m2dec_amd.h"

struct m2dec_amd_trace {
	int width, height, nslots;
	int npics, cap;
	m2dec_amd_trace_pic_t *pics;
	uint8_t *buf;
	size_t len, bcap;
	int nout;
	int *order; /* output order: picture indices */
	int crop[4];
};

typedef struct {
	m2dec_amd_trace_t *t;
	m2d_frame_t frames[64];
	int nframes;
	int slot_pic[64];
	m2r_picture_t pic;
	uint8_t *arena;
	size_t arena_size;
	int failed;
} capture_t;

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

static int cap_set_frames(void *self, int n, const m2d_frame_t *frames, int width, int height)
{
	capture_t *c = (capture_t *)self;
	if (n > 64) n = 64;
	memcpy(c->frames, frames, sizeof(m2d_frame_t) * (size_t)n);
	c->nframes = n;
	c->t->width = width;
	c->t->height = height;
	if (n > c->t->nslots) c->t->nslots = n;
	for (int i = 0; i < 64; ++i) c->slot_pic[i] = -1;
	return 0;
}

static m2r_picture_t *cap_acquire(void *self, int wm, int hm)
{
	capture_t *c = (capture_t *)self;
	size_t n = (size_t)wm * hm;
	size_t need = al256(n * sizeof(m2r_mb_t)) + al256(n * sizeof(m2r_deblock_t)) + al256(256 * sizeof(m2r_slice_t)) +
	              al256(n * sizeof(m2r_inter_t)) + al256(n * 416 * sizeof(int16_t));
	uint8_t *p;
	if (need > c->arena_size) {
		free(c->arena);
		c->arena = (uint8_t *)malloc(need);
		c->arena_size = c->arena ? need : 0;
		if (!c->arena) return NULL;
	}
	p = c->arena;
	memset(&c->pic, 0, sizeof(c->pic));
	c->pic.width_mbs = wm;
	c->pic.height_mbs = hm;
	c->pic.mb = (m2r_mb_t *)p; p += al256(n * sizeof(m2r_mb_t));
	c->pic.dbk = (m2r_deblock_t *)p; p += al256(n * sizeof(m2r_deblock_t));
	c->pic.slice = (m2r_slice_t *)p; p += al256(256 * sizeof(m2r_slice_t));
	c->pic.inter = (m2r_inter_t *)p; p += al256(n * sizeof(m2r_inter_t));
	c->pic.coef = (int16_t *)p;
	c->pic.cap_slices = 256;
	c->pic.cap_inter = (int)n;
	c->pic.cap_coef = (int)(n * 416);
	return &c->pic;
}

static int append(m2dec_amd_trace_t *t, const void *src, size_t n, uint64_t *off)
{
	size_t need = al256(t->len) + n;
	if (need > t->bcap) {
		size_t nc = t->bcap ? t->bcap : ((size_t)1 << 24);
		uint8_t *nb;
		while (nc < need) nc *= 2;
		nb = (uint8_t *)realloc(t->buf, nc);
		if (!nb) return -1;
		t->buf = nb;
		t->bcap = nc;
	}
	t->len = al256(t->len);
	*off = t->len;
	if (n) memcpy(t->buf + t->len, src, n);
	t->len += n;
	return 0;
}

static int cap_submit(void *self, m2r_picture_t *pic)
{
	capture_t *c = (capture_t *)self;
	m2dec_amd_trace_t *t = c->t;
	m2dec_amd_trace_pic_t *tp;
	size_t n = (size_t)pic->width_mbs * pic->height_mbs;
	if (t->npics == t->cap) {
		int nc = t->cap ? t->cap * 2 : 64;
		m2dec_amd_trace_pic_t *np = (m2dec_amd_trace_pic_t *)realloc(t->pics, sizeof(*np) * (size_t)nc);
		if (!np) return -1;
		t->pics = np;
		t->cap = nc;
	}
	tp = &t->pics[t->npics];
	memset(tp, 0, sizeof(*tp));
	tp->slot = pic->slot;
	tp->width_mbs = pic->width_mbs;
	tp->height_mbs = pic->height_mbs;
	tp->n_inter = pic->n_inter;
	tp->n_coef = pic->n_coef;
	tp->n_slices = pic->n_slices;
	tp->n_intra = pic->n_intra;
	tp->deblock = pic->deblock;
	if (append(t, pic->mb, n * sizeof(m2r_mb_t), &tp->off_mb) < 0 ||
	    append(t, pic->dbk, n * sizeof(m2r_deblock_t), &tp->off_dbk) < 0 ||
	    append(t, pic->slice, (size_t)pic->n_slices * sizeof(m2r_slice_t), &tp->off_slice) < 0 ||
	    append(t, pic->inter, (size_t)pic->n_inter * sizeof(m2r_inter_t), &tp->off_inter) < 0 ||
	    append(t, pic->coef, (size_t)pic->n_coef * sizeof(int16_t), &tp->off_coef) < 0)
		return -1;
	tp->record_bytes = (int64_t)(n * (sizeof(m2r_mb_t) + sizeof(m2r_deblock_t)) + (size_t)pic->n_slices * sizeof(m2r_slice_t) +
	                             (size_t)pic->n_inter * sizeof(m2r_inter_t) + (size_t)pic->n_coef * sizeof(int16_t));
	/* algorithmic MC input: one reference byte per predicted sample per list */
	for (int i = 0; i < pic->n_inter; ++i)
		for (int l = 0; l < 2; ++l)
			for (int b8 = 0; b8 < 4; ++b8)
				if (pic->inter[i].slot[l][b8] >= 0) tp->ref_bytes += 64 + 32;
	tp->frame_bytes = (int64_t)n * 384;
	if (pic->slot >= 0 && pic->slot < 64) c->slot_pic[pic->slot] = t->npics;
	t->npics++;
	return 0;
}

static int cap_sync(void *self, int slot)
{
	(void)self;
	(void)slot;
	return 0;
}

static void cap_destroy(void *self) { (void)self; }

static void cap_on_frame(void *arg, const m2d_frame_t *f)
{
	capture_t *c = (capture_t *)arg;
	m2dec_amd_trace_t *t = c->t;
	int slot = -1;
	for (int i = 0; i < c->nframes; ++i)
		if (c->frames[i].luma == f->luma) slot = i;
	if (slot < 0 || c->slot_pic[slot] < 0) {
		c->failed = 1;
		return;
	}
	if ((t->nout & 255) == 0) {
		int *no = (int *)realloc(t->order, sizeof(int) * (size_t)(t->nout + 256));
		if (!no) {
			c->failed = 1;
			return;
		}
		t->order = no;
	}
	t->order[t->nout++] = c->slot_pic[slot];
	for (int i = 0; i < 4; ++i) t->crop[i] = f->crop[i];
}

int m2dec_amd_trace_capture(const uint8_t *data, size_t len, m2dec_amd_trace_t **out)
{
	capture_t c;
	m2r_backend_t be;
	int n;
	memset(&c, 0, sizeof(c));
	memset(&be, 0, sizeof(be));
	c.t = (m2dec_amd_trace_t *)calloc(1, sizeof(m2dec_amd_trace_t));
	if (!c.t) return -1;
	for (int i = 0; i < 64; ++i) c.slot_pic[i] = -1;
	be.self = &c;
	be.set_frames = cap_set_frames;
	be.acquire = cap_acquire;
	be.submit = cap_submit;
	be.sync_frame = cap_sync;
	be.destroy = cap_destroy;
	be.bind = NULL;
	be.flush = NULL;
	n = m2dec_amd_decode_stream(data, len, &be, 0, cap_on_frame, &c, NULL);
	free(c.arena);
	if (n < 0 || c.failed) {
		m2dec_amd_trace_free(c.t);
		return -1;
	}
	*out = c.t;
	return c.t->npics;
}

int m2dec_amd_trace_info(const m2dec_amd_trace_t *t, int *npics, int *width, int *height, int *nslots, int *nout)
{
	if (!t) return -1;
	if (npics) *npics = t->npics;
	if (width) *width = t->width;
	if (height) *height = t->height;
	if (nslots) *nslots = t->nslots;
	if (nout) *nout = t->nout;
	return 0;
}

const m2dec_amd_trace_pic_t *m2dec_amd_trace_pictures(const m2dec_amd_trace_t *t) { return t ? t->pics : NULL; }
const uint8_t *m2dec_amd_trace_records(const m2dec_amd_trace_t *t, size_t *len)
{
	if (!t) return NULL;
	if (len) *len = t->len;
	return t->buf;
}
const int *m2dec_amd_trace_output_order(const m2dec_amd_trace_t *t) { return t ? t->order : NULL; }
int m2dec_amd_trace_crop(const m2dec_amd_trace_t *t, int crop[4])
{
	if (!t) return -1;
	for (int i = 0; i < 4; ++i) crop[i] = t->crop[i];
	return 0;
}

void m2dec_amd_trace_free(m2dec_amd_trace_t *t)
{
	if (!t) return;
	free(t->pics);
	free(t->buf);
	free(t->order);
	free(t);
}
