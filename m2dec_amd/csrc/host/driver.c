/*
 * M2Decoder for any m2d_func_table_t (src/app/m2decoder.h:33-223 + the reread / skip logic of
 * src/app/h264dec.cpp:66-86, 181-186): codec tables h264d_func / m2d_func, the Frames pool sized in
 * the header callback (SetFrames, m2decoder.h:54-80; frames.h: luma and chroma allocated separately,
 * 16-byte aligned), the output loop with the DPB "emptify" option (decode / decode_residual,
 * m2decoder.h:132-157) and `-f` skip-to-keyframe with the SPS / PPS replay (skip_frames,
 * m2decoder.h:96-131).  Used by the h264dec CLI for both codecs.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "m2dec_amd.h"
#include "h264_dec.h"
#include "h265_dec.h"

#define MAX_HDR 256

typedef struct {
	const m2d_func_table_t *func;
	void *ctx;
	int h264;
	int h265;
	const uint8_t *data;
	size_t len, pos;
	/* -f: headers replayed before the key frame (header_data_list_t), then a null sentinel */
	const uint8_t *hdr[MAX_HDR + 1];
	int hdr_len[MAX_HDR + 1];
	int nhdr, hdr_head;
	/* Frames (frames.h) */
	uint8_t *mem[64][2];
	m2d_frame_t frames[64];
	int nframes;
	size_t luma_len;
	uint8_t *second;
	size_t second_len;
	int failed;
	m2dec_hold_t *hold; /* H.265: frames the caller still reads after get (m2dec_amd_decode_h265_held) */
} drv_t;

static int reread(void *arg)
{
	drv_t *v = (drv_t *)arg;
	if (v->hdr_head < v->nhdr) {
		if (v->hdr[v->hdr_head]) {
			dec_bits_set_data(v->func->stream_pos(v->ctx), v->hdr[v->hdr_head], (size_t)v->hdr_len[v->hdr_head], 0);
			v->hdr_head++;
			return 0;
		}
		v->nhdr = v->hdr_head = 0; /* the sentinel: the header replay ends */
		return -1;
	}
	if (v->pos < v->len) {
		/* (the reference passes the whole input length here even after a skip; the remainder is meant) */
		dec_bits_set_data(v->func->stream_pos(v->ctx), v->data + v->pos, v->len - v->pos, 0);
		v->pos = v->len;
		return 0;
	}
	return -1;
}

/* Frame memory kept across decodes, process-wide.  A frame-sized malloc is fresh zero pages, so the first copy of a
 * picture into it takes ~760 page faults per 1080p frame (~0.4 ms, serial in the thread that syncs the picture):
 * the H.265 output tail of the r176 timeline.  A process decoding stream after stream takes the same buffers back
 * (by exact size; at most POOL_CAP bytes are parked, the oldest sizes go first).  The decoders write every sample
 * of a picture before it is output or referenced, as with a fresh buffer. */
#define POOL_MAX 256
#define POOL_CAP ((size_t)1 << 30)
static pthread_mutex_t pool_mu = PTHREAD_MUTEX_INITIALIZER;
static struct {
	uint8_t *p;
	size_t n;
} pool[POOL_MAX];
static int pool_n;
static size_t pool_bytes;

static uint8_t *pool_take(size_t n)
{
	pthread_mutex_lock(&pool_mu);
	for (int i = pool_n - 1; i >= 0; --i)
		if (pool[i].n == n) {
			uint8_t *p = pool[i].p;
			memmove(&pool[i], &pool[i + 1], (size_t)(pool_n - 1 - i) * sizeof(pool[0]));
			--pool_n;
			pool_bytes -= n;
			pthread_mutex_unlock(&pool_mu);
			return p;
		}
	pthread_mutex_unlock(&pool_mu);
	return (uint8_t *)malloc(n);
}

static int pool_on(void)
{
	static int on = -1; /* M2DEC_AMD_FRAME_POOL=0: every decode mallocs and frees its own frames */
	if (on < 0) {
		const char *e = getenv("M2DEC_AMD_FRAME_POOL");
		on = !(e && e[0] == '0');
	}
	return on;
}

static void pool_give(uint8_t *p, size_t n)
{
	if (!p) return;
	if (n > POOL_CAP || !pool_on()) {
		free(p);
		return;
	}
	pthread_mutex_lock(&pool_mu);
	while (pool_n && (pool_n == POOL_MAX || pool_bytes + n > POOL_CAP)) { /* the oldest go */
		free(pool[0].p);
		pool_bytes -= pool[0].n;
		memmove(&pool[0], &pool[1], (size_t)(pool_n - 1) * sizeof(pool[0]));
		--pool_n;
	}
	pool[pool_n].p = p;
	pool[pool_n].n = n;
	++pool_n;
	pool_bytes += n;
	pthread_mutex_unlock(&pool_mu);
}

static void frames_free(drv_t *v)
{
	if (v->hold) m2dec_hold_wait_idle(v->hold); /* (nobody reads the frames any more) */
	for (int i = 0; i < v->nframes; ++i) {
		pool_give(v->mem[i][0], v->luma_len + 15);
		pool_give(v->mem[i][1], (v->luma_len >> 1) + 15);
	}
	free(v->second);
	v->second = NULL;
	v->nframes = 0;
}

/* M2Decoder::SetFrames (m2decoder.h:54-80) */
static int header_cb(void *arg, void *id)
{
	drv_t *v = (drv_t *)arg;
	m2d_info_t info;
	int width, height, bufnum;
	size_t luma_len;
	v->func->get_info(v->ctx, &info);
	width = (info.src_width + 15) & ~15;
	height = (info.src_height + 15) & ~15;
	luma_len = (size_t)width * (size_t)height;
	/* m2decoder.h:59-66: +16 for H.264 / H.265; at most 64 (H.264) or MAX_FRAME_NUM 16 */
	bufnum = info.frame_num + ((v->h264 || v->h265) ? 16 : 0);
	if (bufnum > (v->h264 ? 64 : 16)) bufnum = v->h264 ? 64 : 16;
	if (v->nframes && bufnum <= v->nframes && luma_len <= v->luma_len &&
	    (size_t)(info.additional_size ? info.additional_size : 1) <= v->second_len) {
		for (int i = 0; i < v->nframes; ++i) v->frames[i].id = id;
		return 0;
	}
	frames_free(v);
	fprintf(stderr, "%d x %d x %d\n", info.src_width - info.crop[0] - info.crop[1],
	        info.src_height - info.crop[2] - info.crop[3], info.frame_num);
	v->luma_len = luma_len;
	v->second_len = info.additional_size ? (size_t)info.additional_size : 1;
	v->second = (uint8_t *)calloc(1, v->second_len);
	for (int i = 0; i < bufnum; ++i) {
		v->mem[i][0] = pool_take(luma_len + 15);
		v->mem[i][1] = pool_take((luma_len >> 1) + 15);
		memset(&v->frames[i], 0, sizeof(v->frames[i]));
		v->frames[i].luma = (uint8_t *)(((uintptr_t)v->mem[i][0] + 15) & ~(uintptr_t)15);
		v->frames[i].chroma = (uint8_t *)(((uintptr_t)v->mem[i][1] + 15) & ~(uintptr_t)15);
		v->frames[i].id = id;
	}
	v->nframes = bufnum;
	if (!v->second || v->func->set_frames(v->ctx, bufnum, v->frames, v->second, info.additional_size) < 0) v->failed = 1;
	return 0;
}

/* M2Decoder::is_h264frame_head (m2decoder.h:214-222) */
static int h264_frame_head(const uint8_t *p, long n, int *key, int *hdr)
{
	int t;
	if (n < 2) return 0;
	t = p[0] & 31;
	*key = (t == 5);
	*hdr = (t == 7) || (t == 8);
	return (p[1] & 128) && (t == 5 || t == 1);
}

/* M2Decoder::skip_frames (m2decoder.h:96-131): returns the frames skipped up to the key frame, and the
 * key frame's byte offset in *skipped_bytes (-1: no key frame) */
static int skip_frames(drv_t *v, int skip_frm, long *skipped_bytes)
{
	long pos = 0;
	int skipped = 0, skipped_key = 0;
	const uint8_t *key_at = NULL;
	while (pos < (long)v->len) {
		const int rb = m2d_next_start_code(v->data + pos, (int)((long)v->len - pos));
		int key = 0, hdr = 0;
		if (rb < 0) break;
		pos += rb;
		if (h264_frame_head(v->data + pos, (long)v->len - pos, &key, &hdr)) {
			if (key) {
				key_at = v->data + pos - 3;
				skipped_key = skipped;
			}
			if (skip_frm < ++skipped) break;
		} else if (hdr && v->nhdr < MAX_HDR) {
			const int size = m2d_next_start_code(v->data + pos, (int)((long)v->len - pos));
			v->hdr[v->nhdr] = v->data + pos - 3;
			v->hdr_len[v->nhdr] = size;
			v->nhdr++;
		}
	}
	/* decode the collected headers (each decode_picture call sees them, then the sentinel) */
	while (v->nhdr > v->hdr_head) {
		v->hdr[v->nhdr] = NULL;
		v->hdr_len[v->nhdr] = 0;
		v->nhdr++;
		v->func->decode_picture(v->ctx);
	}
	if (key_at) {
		*skipped_bytes = key_at - v->data;
		return skipped_key;
	}
	*skipped_bytes = -1;
	return -1;
}

int m2dec_amd_decode_table(const m2d_func_table_t *func, int h264, const uint8_t *data, size_t len, int dpb,
                           int emptify, int skip, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                           int *last_error)
{
	return m2dec_amd_decode_table2(func, h264, data, len, dpb, emptify, skip, NULL, -1, on_frame, arg, last_error);
}

/* the checks of the calling thread's last m2d_func decode (m2dec_amd_m2v_last_checks) */
static __thread uint64_t t_m2v_clip, t_m2v_mc;

void m2dec_amd_m2v_last_checks(uint64_t *clip_violations, uint64_t *mc_out_of_frame)
{
	if (clip_violations) *clip_violations = t_m2v_clip;
	if (mc_out_of_frame) *mc_out_of_frame = t_m2v_mc;
}

static int decode_core(const m2d_func_table_t *func, int h264, const uint8_t *data, size_t len, int dpb, int emptify,
                       int skip, const m2r_backend_t *backend, int parse_threads, int m2v_device,
                       void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error);

static int decode_core265(const uint8_t *data, size_t len, const h265r_backend_t *be, int device, int emptify,
                          void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, m2dec_hold_t *hold,
                          int *last_error);

/* H.265 through h265d_func (M2Decoder with MODE_H265, m2decoder.h:180-182): the back end `be` (borrowed;
 * NULL: the gfx950 one on `device`) */
int m2dec_amd_decode_h265(const uint8_t *data, size_t len, const h265r_backend_t *be, int device, int emptify,
                          void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error)
{
	return decode_core265(data, len, be, device, emptify, on_frame, arg, NULL, last_error);
}

/* the same with `hold`: on_frame may keep reading a frame after it returns until it releases it from `hold`;
 * the decoder does not write that frame (sync_frame waits) nor frees it meanwhile.  Only for a back end that
 * writes the caller's frames inside sync_frame alone (the gfx950 one: NULL, or one with `stage`) */
int m2dec_amd_decode_h265_held(const uint8_t *data, size_t len, const h265r_backend_t *be, int device,
                               void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, m2dec_hold_t *hold,
                               int *last_error)
{
	return decode_core265(data, len, be, device, 0, on_frame, arg, hold, last_error);
}

static int decode_loop(drv_t *v, int emptify, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg);

static int decode_core265(const uint8_t *data, size_t len, const h265r_backend_t *be, int device, int emptify,
                          void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, m2dec_hold_t *hold,
                          int *last_error)
{
	drv_t v;
	int err;
	memset(&v, 0, sizeof(v));
	v.hold = hold;
	v.func = h265d_func;
	v.h265 = 1;
	v.data = data;
	v.len = len;
	v.ctx = calloc(1, h265d_func->context_size);
	if (!v.ctx) return -1;
	h265d_func->init(v.ctx, -1, header_cb, &v);
	if (be) m2dec_amd_h265_set_backend(v.ctx, be);
	else m2dec_amd_h265_set_device(v.ctx, device);
	h265_set_hold(v.ctx, hold);
	dec_bits_set_callback(h265d_func->stream_pos(v.ctx), reread, &v);
	err = decode_loop(&v, emptify, on_frame, arg);
	if (last_error) *last_error = err;
	if (be) m2dec_amd_h265_set_backend(v.ctx, NULL); /* borrowed */
	m2dec_amd_h265_release(v.ctx);
	free(v.ctx);
	frames_free(&v);
	return err;
}

/* h264dec.cpp:251-257 over M2Decoder::decode / decode_residual (m2decoder.h:132-157) */
static int decode_loop(drv_t *v, int emptify, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg)
{
	const m2d_func_table_t *func = v->func;
	m2d_frame_t frm;
	int err = -1;
	for (;;) {
		while (func->peek_decoded_frame(v->ctx, &frm, 0) <= 0) {
			err = func->decode_picture(v->ctx);
			if (v->failed) err = -1;
			if (err < 0) {
				while (func->peek_decoded_frame(v->ctx, &frm, 1) > 0) {
					if (on_frame) on_frame(arg, &frm);
					func->get_decoded_frame(v->ctx, &frm, 1);
				}
				return err;
			}
		}
		do {
			func->get_decoded_frame(v->ctx, &frm, 0);
			if (on_frame) on_frame(arg, &frm);
		} while (emptify && 0 < func->peek_decoded_frame(v->ctx, &frm, 0));
		err = func->decode_picture(v->ctx);
		if (v->failed) err = -1;
		if (err < 0) {
			while (0 < func->peek_decoded_frame(v->ctx, &frm, 1)) {
				if (on_frame) on_frame(arg, &frm);
				func->get_decoded_frame(v->ctx, &frm, 1);
			}
			return err;
		}
	}
}

static int decode_core(const m2d_func_table_t *func, int h264, const uint8_t *data, size_t len, int dpb, int emptify,
                       int skip, const m2r_backend_t *backend, int parse_threads, int m2v_device,
                       void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error)
{
	drv_t v;
	m2d_frame_t frm;
	int err = -1;
	memset(&v, 0, sizeof(v));
	v.func = func;
	v.h264 = h264;
	v.data = data;
	v.len = len;
	v.ctx = calloc(1, func->context_size);
	if (!v.ctx) return -1;
	func->init(v.ctx, dpb, header_cb, &v);
	if (h264 && backend) m2dec_amd_h264_set_backend(v.ctx, backend);
	if (h264 && parse_threads >= 0) m2dec_amd_h264_set_parse_threads(v.ctx, parse_threads);
	if (!h264 && m2v_device >= 0 && m2dec_amd_m2v_use_gpu(v.ctx, m2v_device) < 0) { /* (asked for: no host fallback) */
		free(v.ctx);
		if (last_error) *last_error = -1;
		return -3;
	}
	dec_bits_set_callback(func->stream_pos(v.ctx), reread, &v);
	if (skip) {
		long skipped_bytes = 0;
		const int n = skip_frames(&v, skip, &skipped_bytes);
		if (skipped_bytes > 0) v.pos = (size_t)skipped_bytes;
		fprintf(stderr, "Skip %d frames(%ld bytes).\n", n, skipped_bytes);
	}
	/* h264dec.cpp:251-257 over M2Decoder::decode / decode_residual */
	for (;;) {
		while (func->peek_decoded_frame(v.ctx, &frm, 0) <= 0) {
			err = func->decode_picture(v.ctx);
			if (v.failed) err = -1;
			if (err < 0) {
				while (func->peek_decoded_frame(v.ctx, &frm, 1) > 0) {
					if (on_frame) on_frame(arg, &frm);
					func->get_decoded_frame(v.ctx, &frm, 1);
				}
				goto done;
			}
		}
		do {
			func->get_decoded_frame(v.ctx, &frm, 0);
			if (on_frame) on_frame(arg, &frm);
		} while (emptify && 0 < func->peek_decoded_frame(v.ctx, &frm, 0));
		err = func->decode_picture(v.ctx);
		if (v.failed) err = -1;
		if (err < 0) {
			while (0 < func->peek_decoded_frame(v.ctx, &frm, 1)) {
				if (on_frame) on_frame(arg, &frm);
				func->get_decoded_frame(v.ctx, &frm, 1);
			}
			break;
		}
	}
done:
	if (last_error) *last_error = err;
	if (h264 && backend) m2dec_amd_h264_set_backend(v.ctx, NULL); /* borrowed: the caller destroys it */
	if (h264) {
		m2dec_amd_h264_release(v.ctx);
	} else {
		t_m2v_clip = m2dec_amd_m2v_clip_violations(v.ctx);
		t_m2v_mc = m2dec_amd_m2v_mc_out_of_frame(v.ctx);
		m2dec_amd_m2v_release(v.ctx);
	}
	free(v.ctx);
	frames_free(&v);
	return err;
}

int m2dec_amd_decode_table2(const m2d_func_table_t *func, int h264, const uint8_t *data, size_t len, int dpb,
                            int emptify, int skip, const m2r_backend_t *backend, int parse_threads,
                            void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error)
{
	return decode_core(func, h264, data, len, dpb, emptify, skip, backend, parse_threads, -1, on_frame, arg, last_error);
}

int m2dec_amd_decode_m2v(const uint8_t *data, size_t len, int device, int emptify,
                         void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error)
{
	return decode_core(m2d_func, 0, data, len, -1, emptify, 0, NULL, -1, device, on_frame, arg, last_error);
}
