#include <stddef.h>
/*
 * h264d_func — the reference's m2d_func_table_t for H.264 (h264.cpp:12057-12068), backed by the
 * m2dec_amd host parser + a reconstruction back end (the gfx950 HIP back end by default).
 *
 *   init                  h264.cpp:446-464
 *   get_info              h264.cpp:505-525
 *   set_frames            h264.cpp:647-661
 *   decode_picture        h264.cpp:663-693  (returns 1 per picture, -1 error, -2 end of data)
 *   peek/get_decoded_frame h264.cpp:817-867
 *
 * Extra C-ABI entry points (include/m2dec_amd.h): back-end selection, release, and a driver that
 * mirrors src/app/h264dec.cpp + m2decoder.h so tests and bench.py can decode a whole stream.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "h264_dec.h"
#include "m2dec_amd.h"

static int hdr_dummy(void *a, void *b)
{
	(void)a;
	(void)b;
	return 0;
}

static double mono_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------ caller context = handle
 * The reference's context is plain caller memory: M2Decoder allocates context_size bytes
 * (m2decoder.h:184) and frees them with delete[] (m2decoder.h:43-50) without any release call, and
 * SetFrames deletes the frames inside the header callback (m2decoder.h:68-77).  This decoder owns
 * worker threads' work, GPU buffers and pinned memory, so none of it may live in, or point into,
 * that memory.  The caller's context_size bytes hold only a handle; the state (h264_dec_t) is
 * library memory kept in a process registry:
 *   - nothing the library runs between API calls (pool workers, pipe_drive, GPU copies) touches
 *     caller memory: frames reach the caller's buffers only inside peek / get (sync_frame copies out
 *     of the back end's own staging), so dropping frames or the context at any time is safe;
 *   - a state whose context the caller dropped is reclaimed by the registry: when init() is called
 *     on the same context address again (the caller reuses the memory), or when a new context
 *     would bring the registry over M2DEC_AMD_MAX_CONTEXTS (default 8) — then the least recently
 *     used state that is done with its stream goes first: decode_picture returned -2 AND a later
 *     peek / get found the DPB empty (M2Decoder::decode drains it with peek / get after -2,
 *     m2decoder.h:136-141, so a state is never taken out from under that loop).  A live stream is
 *     never evicted for being idle unless M2DEC_AMD_IDLE_EVICT_S is set (opt-in: states not called
 *     for that many seconds become reclaimable too).  A state is never reclaimed during a call on it.
 *     Calls on a reclaimed context fail without looping the reference's drivers: decode_picture
 *     returns -1, peek / get return 0 (no frame), stream_pos returns an empty reader.
 *   - m2dec_amd_h264_release() still frees a context at once (optional). */
typedef struct {
	uint64_t magic;
	uint64_t gen;
	h264_dec_t *st;
} h264_handle_t;

#define H264_HANDLE_MAGIC 0x6d32646563616d64ull /* "m2decamd" */

static pthread_mutex_t reg_mu = PTHREAD_MUTEX_INITIALIZER;
static h264_dec_t *reg_head;
static int reg_count;
static uint64_t reg_gen;
static long reg_evicted;

static void state_destroy(h264_dec_t *d);

static int env_int(const char *name, int def)
{
	const char *e = getenv(name);
	return e && *e ? atoi(e) : def;
}

/* registry lookup of a caller context; counts the call in (leave() counts it out) */
static h264_dec_t *enter(void *ctx)
{
	const h264_handle_t *h = (const h264_handle_t *)ctx;
	h264_dec_t *d;
	if (!h || h->magic != H264_HANDLE_MAGIC) return NULL;
	pthread_mutex_lock(&reg_mu);
	for (d = reg_head; d; d = d->reg_next)
		if (d == h->st && d->gen == h->gen && d->owner == ctx) break;
	if (d) {
		d->in_call++;
		d->last_call = mono_s();
	}
	pthread_mutex_unlock(&reg_mu);
	if (!d) {
		static int warned;
		if (!__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED))
			fprintf(stderr, "m2dec_amd: call on a context that was released or reclaimed (not initialised, "
			                "dropped, or evicted over M2DEC_AMD_MAX_CONTEXTS)\n");
	}
	return d;
}

static void leave(h264_dec_t *d)
{
	pthread_mutex_lock(&reg_mu);
	d->in_call--;
	pthread_mutex_unlock(&reg_mu);
}

h264_dec_t *h264_state(void *ctx)
{
	h264_dec_t *d = enter(ctx);
	if (d) leave(d);
	return d;
}

/* States to reclaim before registering a context at `ctx` (registry mutex held): those initialised
 * on the same address (its memory is being reused: that context is gone), then LRU ones over the
 * cap.  They are unlinked here and destroyed by the caller outside the mutex. */
static int reclaim_victims(const void *ctx, h264_dec_t **out, int max)
{
	const int cap = env_int("M2DEC_AMD_MAX_CONTEXTS", 8);
	const int idle_on = getenv("M2DEC_AMD_IDLE_EVICT_S") && *getenv("M2DEC_AMD_IDLE_EVICT_S");
	const double idle = (double)env_int("M2DEC_AMD_IDLE_EVICT_S", 0), now = mono_s();
	int n = 0;
	for (h264_dec_t **pp = &reg_head; *pp && n < max;) {
		h264_dec_t *d = *pp;
		if (d->owner == ctx && !d->in_call) {
			*pp = d->reg_next;
			reg_count--;
			out[n++] = d;
		} else {
			if (d->owner == ctx) d->owner = NULL; /* (in a call on another thread: orphaned, reclaimed later) */
			pp = &d->reg_next;
		}
	}
	/* hard ceiling: at twice the cap, a state idle for M2DEC_AMD_HARD_IDLE_S (default 10 s) goes
	 * too, whatever M2DEC_AMD_IDLE_EVICT_S says: a context its caller dropped mid-stream without release (and
	 * whose memory is never reused for an init) would otherwise hold its frames, back end and pinned arenas
	 * for the life of the process */
	const double hard_idle = (double)env_int("M2DEC_AMD_HARD_IDLE_S", 10);
	while (reg_count >= cap && n < max) {
		h264_dec_t **best = NULL;
		const int hard = reg_count >= 2 * cap;
		for (h264_dec_t **pp = &reg_head; *pp; pp = &(*pp)->reg_next) {
			const h264_dec_t *d = *pp;
			if (d->in_call || !((d->finished && d->drained) || !d->owner || (idle_on && now - d->last_call >= idle) ||
			                    (hard && now - d->last_call >= hard_idle)))
				continue;
			if (!best || d->last_call < (*best)->last_call) best = pp;
		}
		if (!best) {
			static int warned;
			if (reg_count >= 2 * cap && !__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED))
				fprintf(stderr, "m2dec_amd: %d live decoder contexts, over twice M2DEC_AMD_MAX_CONTEXTS=%d and none "
				                "idle for M2DEC_AMD_HARD_IDLE_S=%.0f s (contexts dropped without release?)\n",
				        reg_count, cap, hard_idle);
			break;
		}
		h264_dec_t *d = *best;
		*best = d->reg_next;
		reg_count--;
		reg_evicted++;
		out[n++] = d;
	}
	return n;
}

extern int m2dec_host_cpu_ok; /* cpucheck.c */

static int api_init(void *ctx, int dpb_max, int (*cb)(void *, void *), void *arg)
{
	h264_handle_t *h = (h264_handle_t *)ctx;
	h264_dec_t *victims[64], *d;
	int nv;
	if (!ctx || !m2dec_host_cpu_ok) return -1;
	pthread_mutex_lock(&reg_mu);
	nv = reclaim_victims(ctx, victims, 64);
	pthread_mutex_unlock(&reg_mu);
	for (int i = 0; i < nv; ++i) state_destroy(victims[i]);
	d = (h264_dec_t *)calloc(1, sizeof(h264_dec_t));
	if (!d) {
		memset(h, 0, sizeof(*h));
		return -1;
	}
	d->stream = &d->stream_i;
	d->header_callback = cb ? cb : hdr_dummy;
	d->header_callback_arg = arg;
	d->dpb_max_arg = dpb_max;
	h264_dpb_init(&d->dpb, dpb_max);
	dec_bits_open(d->stream, m2d_load_bytes_skip03);
	for (int i = 0; i < 16; ++i) d->refs[1][i].col = (int16_t)i;
	d->curr_col = 16;
	d->sh.first_mb = -1;
	d->parse_threads = -1; /* default: decided when the back end is created */
	d->stats = getenv("M2DEC_AMD_ASYNC_STATS") != NULL;
	d->owner = ctx;
	d->last_call = mono_s();
	pthread_mutex_lock(&reg_mu);
	d->gen = ++reg_gen;
	d->reg_next = reg_head;
	reg_head = d;
	reg_count++;
	pthread_mutex_unlock(&reg_mu);
	h->magic = H264_HANDLE_MAGIC;
	h->gen = d->gen;
	h->st = d;
	return 0;
}

static dec_bits *api_stream_pos(void *ctx)
{
	static dec_bits gone; /* a reclaimed context: a reader with no data */
	h264_dec_t *d = h264_state(ctx);
	return d ? d->stream : &gone;
}

static int api_get_info(void *ctx, m2d_info_t *info)
{
	h264_dec_t *d = enter(ctx);
	const h264_sps_t *s;
	if (!d) return -1;
	if (!info) {
		leave(d);
		return -1;
	}
	/* the reference reads the SPS of the current slice's PPS (h264.cpp:511) */
	s = &d->sps[d->pps[d->sh.pps_id].sps_id];
	if (!s->valid) s = &d->sps[d->active_sps];
	info->src_width = (int16_t)s->width;
	info->src_height = (int16_t)s->height;
	info->disp_width = (int16_t)s->width;
	info->disp_height = (int16_t)s->height;
	info->frame_num = (int16_t)(s->num_ref_frames + 1);
	for (int i = 0; i < 4; ++i) info->crop[i] = (int16_t)s->crop[i];
	info->additional_size = 16; /* parser state lives in the library's state / back end, not the caller's work buffer */
	leave(d);
	return 0;
}

static int ensure_backend(h264_dec_t *d)
{
	if (!d->have_backend) {
		if (m2dec_amd_hip_backend_create(&d->backend, d->device) < 0) {
			fprintf(stderr, "m2dec_amd: HIP reconstruction back end unavailable (no gfx950 device / HIP runtime); "
			                "install an explicit back end with m2dec_amd_h264_set_backend() for CPU checking\n");
			return -1;
		}
		d->have_backend = 1;
		if (d->parse_threads < 0) { /* default for the product path: parse ahead on the pool */
			const char *e = getenv("M2DEC_AMD_PARSE_THREADS");
			d->parse_threads = e ? atoi(e) : m2d_cpu_share(); /* the CPU share (cpushare.c); profiles/r48*_threads.txt: 14-20 within noise, 12 ~8 % lower */
		}
	}
	if (d->parse_threads > 0 && !d->as && h264_async_start(d, d->parse_threads) < 0) return -1;
	return 0;
}

static int alloc_geometry(h264_dec_t *d, int w, int h)
{
	int mb_w = w >> 4, mb_h = h >> 4, n = mb_w * mb_h;
	if (mb_w <= 0 || mb_h <= 0) return -1;
	if (d->mb_w == mb_w && d->mb_h == mb_h && d->mbi) return 0;
	free(d->mbi);
	d->mbi = (h264_mbinfo_t *)calloc((size_t)n, sizeof(h264_mbinfo_t));
	for (int i = 0; i < 17; ++i) {
		free(d->colpic[i].mb);
		d->colpic[i].mb = (h264_colmb_t *)calloc(H264_COL_ENTRIES(n), sizeof(h264_colmb_t));
		memset(d->colpic[i].map_col_frameidx, 0, sizeof(d->colpic[i].map_col_frameidx));
		if (!d->colpic[i].mb) return -1;
	}
	if (!d->mbi) return -1;
	d->mb_w = mb_w;
	d->mb_h = mb_h;
	d->n_mbs = n;
	return 0;
}

static int set_frames_st(h264_dec_t *d, int n, m2d_frame_t *frames, uint8_t *work)
{
	const h264_sps_t *s;
	if (n < 3 || n > H264D_MAX_FRAME_NUM || !frames || !work) return -1;
	d->num_frames = n;
	memcpy(d->frames, frames, sizeof(m2d_frame_t) * (size_t)n);
	memset(d->lru, 0, sizeof(d->lru));
	s = &d->sps[d->active_sps];
	if (alloc_geometry(d, s->width, s->height) < 0) return -1;
	if (ensure_backend(d) < 0) return -1;
	if (d->backend.set_frames(d->backend.self, n, d->frames, s->width, s->height) < 0) return -1;
	d->frames_ready = 1;
	return 0;
}

static int api_set_frames(void *ctx, int n, m2d_frame_t *frames, uint8_t *work, int work_len)
{
	h264_dec_t *d = enter(ctx);
	int r;
	(void)work_len;
	if (!d) return -1;
	r = set_frames_st(d, n, frames, work);
	leave(d);
	return r;
}

/* one slice NAL */
static int read_slice(h264_dec_t *d, int nal_unit_type, int nal_ref_idc)
{
	const h264_sps_t *s;
	int prev_first = d->in_picture ? d->sh.first_mb : -1;
	int err;
	if (d->as && d->in_picture) {
		/* parse-ahead: a slice whose first_mb is not above the previous one starts the next picture
		 * (h264.cpp:1427-1430): close the current one, and read this NAL again next time */
		h264_bits_t b;
		hb_init(&b, d->nal + 1, d->nal_len - 1);
		if ((int)hb_ue(&b) <= prev_first) {
			d->nal_replay = 1;
			return h264_async_close(d);
		}
	}
	hb_init(&d->bs, d->nal + 1, d->nal_len - 1);
	d->slice_rbsp = d->nal + 1;
	d->slice_rbsp_end = d->nal + d->nal_len;
	{
		/* bit position of the rbsp_stop_one_bit */
		size_t len = d->nal_len - 1;
		const uint8_t *p = d->slice_rbsp;
		d->slice_rbsp_bits = len ? (len - 1) * 8 + (size_t)(7 - __builtin_ctz(p[len - 1])) : 0;
	}
	err = h264_slice_header(d, &d->bs, nal_unit_type, nal_ref_idc);
	if (err < 0) return err;
	if (d->in_picture && d->sh.first_mb <= prev_first) return -2; /* h264.cpp:1427-1430 */
	s = &d->sps[d->active_sps];
	if (!d->lookahead && !d->frames_ready) return -1;
	if (d->lookahead && ((s->width >> 4) != d->mb_w || (s->height >> 4) != d->mb_h) && h264_async_sps(d) < 0)
		return -1; /* new geometry: the co-located stores are reallocated, no job may still use them */
	if (alloc_geometry(d, s->width, s->height) < 0) return -1;
	if (!d->in_picture) {
		if (h264_picture_begin(d) < 0) return -1;
	}
	if (d->lookahead) return h264_async_add_slice(d) < 0 ? -1 : 0;
	if (d->as) return 0; /* API context of the pipeline: the lookahead context parses the slice data */
	err = h264_slice_data(d);
	if (err < 0) return err;
	if (err == 1) return h264_picture_finish(d);
	return 0;
}

/* The NAL loop of decode_picture (h264.cpp:663-693): returns 1 per picture, -1 on error, -2 at the
 * end of the data.  Run on the API context (headers, DPB, frame slots, back-end submission) and, in
 * the parse-ahead pipeline, on the lookahead context (headers, slice-data jobs), which stays up to
 * a few dozen pictures ahead and hands every NAL it finished over to the API context. */
int h264_decode_loop(h264_dec_t *d)
{
	for (;;) {
		/* NALs come from the lookahead context (re-evaluated per NAL: the pipeline starts inside the
		 * header callback of an SPS) */
		const int queued = d->as && !d->lookahead;
		int type, ref_idc, err = 0, r;
		r = queued ? h264_async_nal_next(d) : h264_nal_next(d);
		if (r < 0) {
			if (r == -3) return -1; /* the lookahead context failed before this point */
			if (d->as && d->in_picture) return h264_async_close(d); /* the last picture */
			return -2;
		}
		if (d->nal_len == 0) continue;
		type = d->nal[0] & 31;
		ref_idc = (d->nal[0] >> 5) & 3;
		if (d->as && d->in_picture && type >= 6 && type <= 9) {
			/* SEI / SPS / PPS / AUD after a picture's slices start the next access unit (7.4.1.2.3) */
			d->nal_replay = 1;
			return h264_async_close(d);
		}
		/* the header callback may free the caller's frames (m2decoder.h:68-77): every closed picture is
		 * bound first, so that sync_frame can still deliver it from the back end's own staging */
		if (queued && type == 7 && h264_async_drain(d, -1) < 0) return -1;
		switch (type) {
		case 1:
		case 5:
			err = read_slice(d, type, ref_idc);
			if (err != 0) return err;
			break;
		case 7: {
			h264_bits_t b;
			int id;
			hb_init(&b, d->nal + 1, d->nal_len - 1);
			id = h264_parse_sps(d, &b);
			if (id < 0) return id;
			if (!d->in_picture) d->active_sps = id;
			if (d->lookahead) {
				h264_async_la_sps(d); /* pictures after it wait for the API context's callback */
			} else {
				d->header_callback(d->header_callback_arg, d->stream->id);
				if (d->as) h264_async_api_sps(d);
			}
			break;
		}
		case 8: {
			h264_bits_t b;
			hb_init(&b, d->nal + 1, d->nal_len - 1);
			err = h264_parse_pps(d, &b, d->nal_len - 1);
			if (err < 0) return err;
			break;
		}
		default:
			break;
		}
		if (d->lookahead && h264_async_push_nal(d) < 0) return -1;
	}
}

static int api_decode_picture(void *ctx)
{
	h264_dec_t *d = enter(ctx);
	int r;
	if (!d) return -1;
	if (d->fault) { /* a frame could not be delivered (deliver): the stream is broken */
		leave(d);
		return -1;
	}
	d->eos = 0;
	if (d->as) h264_async_resume(d);
	r = h264_decode_loop(d);
	d->finished = r == -2;
	d->drained = 0;
	if (d->finished) h264_async_trim(d);
	leave(d);
	return r;
}

static int deliver(h264_dec_t *d, int idx, m2d_frame_t *frame)
{
	double t0 = 0, t1 = 0;
	if (idx < 0) {
		if (d->finished) d->drained = 1; /* the caller has every frame of its stream */
		return 0;
	}
	if (d->stats) t0 = mono_s();
	/* a failure here (a submission / bind error, a device fault) delivers no frame and fails the next
	 * decode_picture: peek returning -1 would spin M2Decoder's `while (peek(ctx, &frm, 1))` drain
	 * (m2decoder.h:138) forever */
	if (d->as && h264_async_drain(d, idx) < 0) { /* the picture in that slot is parsed and submitted */
		d->fault = 1;
		return 0;
	}
	if (d->stats) t1 = mono_s();
	/* the frame's copy out of the device is still running: let the lookahead dispatch more parse jobs
	 * meanwhile (one picture's headers per step, ~0.1 ms at 1080p), then wait */
	if (d->as && d->have_backend && d->backend.ready)
		while (!d->backend.ready(d->backend.self, idx) && h264_async_pump_step(d)) {
		}
	/* (sync_frame copies the picture into the caller's frame, on this thread, inside this call) */
	if (d->have_backend && d->backend.sync_frame(d->backend.self, idx) < 0) {
		d->fault = 1;
		return 0;
	}
	if (d->stats) {
		d->t_drain += t1 - t0;
		d->t_sync += mono_s() - t1;
	}
	*frame = d->frames[idx];
	return 1;
}

static int api_peek(void *ctx, m2d_frame_t *frame, int bypass)
{
	h264_dec_t *d = enter(ctx);
	int r;
	if (!d) return 0; /* reclaimed: no frame (a -1 would keep `while (peek(ctx, &f, 1))` loops going) */
	r = frame ? deliver(d, h264_dpb_peek(&d->dpb, bypass), frame) : -1;
	leave(d);
	return r;
}

static int api_get(void *ctx, m2d_frame_t *frame, int bypass)
{
	h264_dec_t *d = enter(ctx);
	int r;
	if (!d) return 0;
	r = frame ? deliver(d, h264_dpb_pop(&d->dpb, bypass), frame) : -1;
	leave(d);
	return r;
}

static const m2d_func_table_t h264d_func_ = {
	sizeof(h264_handle_t),
	api_init,
	api_stream_pos,
	api_get_info,
	api_set_frames,
	api_decode_picture,
	api_peek,
	api_get,
};

const m2d_func_table_t * const h264d_func = &h264d_func_;

/* ------------------------------------------------------------------ extra C ABI */
int m2dec_amd_h264_set_backend2(void *ctx, const m2r_backend_t *be, size_t be_size)
{
	h264_dec_t *d;
	if (be && (be_size < offsetof(m2r_backend_t, bind) || be_size > sizeof(m2r_backend_t))) return -1;
	d = enter(ctx);
	if (!d) return -1;
	h264_async_records_wait(d); /* (the old back end may still upload job records) */
	if (!be) { /* detach a borrowed back end without destroying it */
		d->have_backend = 0;
	} else {
		if (d->have_backend && d->backend.destroy) d->backend.destroy(d->backend.self);
		/* a caller built against an older m2r_backend_t passes its smaller size: the members it does
		 * not know (bind) stay NULL, so its back end gets pictures in API order */
		memset(&d->backend, 0, sizeof(d->backend));
		memcpy(&d->backend, be, be_size);
		d->have_backend = 1;
	}
	leave(d);
	return 0;
}

int m2dec_amd_h264_set_backend(void *ctx, const m2r_backend_t *be)
{
	return m2dec_amd_h264_set_backend2(ctx, be, sizeof(m2r_backend_t));
}

int m2dec_amd_abi_version(void) { return M2DEC_AMD_ABI_VERSION; }
size_t m2dec_amd_stats_size(void) { return sizeof(m2dec_amd_stats_t); }

int m2dec_amd_h264_set_parse_threads(void *ctx, int threads)
{
	h264_dec_t *d = enter(ctx);
	int r = -1;
	if (!d) return -1;
	if (!d->as) { /* before the first set_frames */
		d->parse_threads = threads < 0 ? 0 : threads;
		r = 0;
	}
	leave(d);
	return r;
}

int m2dec_amd_h264_set_device(void *ctx, int device)
{
	h264_dec_t *d = enter(ctx);
	if (!d) return -1;
	d->device = device;
	leave(d);
	return 0;
}

static void state_destroy(h264_dec_t *d)
{
	const int stats = d->stats;
	const double t0 = mono_s();
	if (stats) fprintf(stderr, "deliver: drain %.3f s, sync_frame %.3f s\n", d->t_drain, d->t_sync);
	h264_async_stop(d);
	const double t1 = mono_s();
	if (d->have_backend && d->backend.destroy) d->backend.destroy(d->backend.self);
	d->have_backend = 0;
	const double t2 = mono_s();
	free(d->mbi);
	for (int i = 0; i < 17; ++i) free(d->colpic[i].mb);
	free(d->nal);
	free(d);
	if (stats)
		fprintf(stderr, "state_destroy: pipeline %.2f ms, back end %.2f ms, heap %.2f ms\n", 1e3 * (t1 - t0),
		        1e3 * (t2 - t1), 1e3 * (mono_s() - t2));
}

void m2dec_amd_h264_release(void *ctx)
{
	h264_handle_t *h = (h264_handle_t *)ctx;
	h264_dec_t *d = NULL;
	if (!h || h->magic != H264_HANDLE_MAGIC) return;
	pthread_mutex_lock(&reg_mu);
	for (h264_dec_t **pp = &reg_head; *pp; pp = &(*pp)->reg_next)
		if (*pp == h->st && (*pp)->gen == h->gen && !(*pp)->in_call) {
			d = *pp;
			*pp = d->reg_next;
			reg_count--;
			break;
		}
	pthread_mutex_unlock(&reg_mu);
	h->magic = 0;
	if (d) state_destroy(d);
}

int m2dec_amd_h264_registry(int *contexts, long *evicted)
{
	pthread_mutex_lock(&reg_mu);
	if (contexts) *contexts = reg_count;
	if (evicted) *evicted = reg_evicted;
	pthread_mutex_unlock(&reg_mu);
	return 0;
}

/* ------------------------------------------------------------------ stream driver (h264dec.cpp + m2decoder.h) */
typedef struct {
	void *ctx;               /* the caller-side context (a handle, h264d_func->context_size bytes) */
	h264_dec_t *d;           /* its state, for the driver's statistics */
	const uint8_t *data;
	size_t len;
	size_t pos;
	int outbuf;
	uint8_t *frame_mem;
	m2d_frame_t frames[H264D_MAX_FRAME_NUM];
	int nframes;
	size_t luma_len;
	uint8_t work[64];
	int extra;               /* frames beyond the decoder's need (held by the caller meanwhile) */
	size_t frame_size;       /* frame_mem: a block of the frame pool (fpool_take) */
	m2dec_hold_t *hold;
	int failed;
	double setup_s;
	double t_last;           /* on_frame of the last frame returned */
	void (*on_frame)(void *arg, const m2d_frame_t *f);
	void *arg;
} driver_t;

static void emit(driver_t *v, const m2d_frame_t *f)
{
	if (v->on_frame) v->on_frame(v->arg, f);
	v->t_last = mono_s();
}

static int drv_reread(void *arg)
{
	driver_t *v = (driver_t *)arg;
	if (v->pos < v->len) {
		dec_bits_set_data(h264d_func->stream_pos(v->ctx), v->data + v->pos, v->len - v->pos, 0);
		v->pos = v->len;
		return 0;
	}
	return -1;
}

/* Frame memory of the stream driver outlives a stream (bench steps, a service decoding stream after
 * stream): fresh memory costs page faults.  The frames are plain caller memory — the back end never
 * writes them asynchronously (sync_frame copies into them inside peek / get), so a block can go back
 * to the pool as soon as no MD5 thread reads it. */
static pthread_mutex_t fpool_mu = PTHREAD_MUTEX_INITIALIZER;
static struct {
	uint8_t *mem;
	size_t size;
} fpool[16];

static uint8_t *fpool_take(size_t need, size_t *size)
{
	uint8_t *m = NULL;
	pthread_mutex_lock(&fpool_mu);
	for (int i = 0; i < 16 && !m; ++i)
		if (fpool[i].mem && fpool[i].size >= need) {
			m = fpool[i].mem;
			*size = fpool[i].size;
			fpool[i].mem = NULL;
		}
	pthread_mutex_unlock(&fpool_mu);
	if (!m) {
		m = (uint8_t *)aligned_alloc(4096, need);
		*size = need;
	}
	return m;
}

static void fpool_give(uint8_t *m, size_t size)
{
	if (!m) return;
	pthread_mutex_lock(&fpool_mu);
	for (int i = 0; i < 16; ++i)
		if (!fpool[i].mem) {
			fpool[i].mem = m;
			fpool[i].size = size;
			m = NULL;
			break;
		}
	pthread_mutex_unlock(&fpool_mu);
	free(m);
}

/* M2Decoder::SetFrames, m2decoder.h:54-80 */
static int drv_header(void *arg, void *id)
{
	driver_t *v = (driver_t *)arg;
	m2d_info_t info;
	int w, h, bufnum;
	size_t luma_len;
	(void)id;
	if (h264d_func->get_info(v->ctx, &info) < 0) {
		v->failed = 1;
		return -1;
	}
	w = (info.src_width + 15) & ~15;
	h = (info.src_height + 15) & ~15;
	luma_len = (size_t)w * (size_t)h;
	bufnum = v->outbuf + info.frame_num + 16 + v->extra;
	if (bufnum > H264D_MAX_FRAME_NUM) bufnum = H264D_MAX_FRAME_NUM;
	if (v->frame_mem && bufnum <= v->nframes && luma_len <= v->luma_len) return 0;
	if (v->hold) m2dec_hold_wait_idle(v->hold); /* nobody reads the old frames any more */
	fpool_give(v->frame_mem, v->frame_size);
	v->frame_mem = fpool_take(((luma_len * 3 / 2 + 4095) & ~(size_t)4095) * (size_t)bufnum, &v->frame_size);
	if (!v->frame_mem) {
		v->failed = 1;
		return -1;
	}
	{
		size_t fsz = (luma_len * 3 / 2 + 4095) & ~(size_t)4095;
		for (int i = 0; i < bufnum; ++i) {
			memset(&v->frames[i], 0, sizeof(v->frames[i]));
			v->frames[i].luma = v->frame_mem + fsz * (size_t)i;
			v->frames[i].chroma = v->frames[i].luma + luma_len;
		}
	}
	v->nframes = bufnum;
	v->luma_len = luma_len;
	{
		const double t0 = mono_s();
		if (h264d_func->set_frames(v->ctx, bufnum, v->frames, v->work, info.additional_size) < 0) v->failed = 1;
		v->setup_s += mono_s() - t0;
		if (v->d->stats) fprintf(stderr, "set_frames: %d frames, %.3f s\n", bufnum, mono_s() - t0);
	}
	return 0;
}

int m2dec_amd_decode_stream(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device,
                            void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, m2dec_amd_stats_t *stats)
{
	return m2dec_amd_decode_stream2(data, len, backend, device, -1, on_frame, arg, stats);
}

int m2dec_amd_decode_stream3(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                             int parse_threads, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                             m2dec_amd_stats_t *stats);

int m2dec_amd_decode_stream2(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                             void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, m2dec_amd_stats_t *stats)
{
	return m2dec_amd_decode_stream3(data, len, backend, device, dpb, -1, on_frame, arg, stats);
}

/* parse_threads: -1 the context's default, else m2dec_amd_h264_set_parse_threads(threads) */
int m2dec_amd_decode_stream3(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                             int parse_threads, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                             m2dec_amd_stats_t *stats)
{
	return h264_decode_stream_held(data, len, backend, device, dpb, parse_threads, 0, NULL, on_frame, NULL, arg, stats);
}

/* the stream driver; `hold`: on_frame may keep reading a frame after it returns until it releases it
 * from `hold` (the frame is not reused meanwhile), with `extra` more frames than the decoder needs;
 * on_end (optional): called after the last frame, before the held frames are waited for */
int h264_decode_stream_held(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                            int parse_threads, int extra, m2dec_hold_t *hold,
                            void (*on_frame)(void *arg, const m2d_frame_t *f), void (*on_end)(void *arg), void *arg,
                            m2dec_amd_stats_t *stats)
{
	driver_t v;
	void *ctx = calloc(1, h264d_func->context_size);
	h264_dec_t *d;
	m2d_frame_t frm;
	int err = 0, n = 0;
	if (!ctx) return -1;
	memset(&v, 0, sizeof(v));
	v.ctx = ctx;
	v.data = data;
	v.len = len;
	v.on_frame = on_frame;
	v.arg = arg;
	v.extra = extra;
	v.hold = hold;
	if (h264d_func->init(ctx, dpb, drv_header, &v) < 0 || !(d = h264_state(ctx))) {
		free(ctx);
		return -1;
	}
	v.d = d;
	d->hold = hold;
	d->device = device;
	if (backend) m2dec_amd_h264_set_backend(ctx, backend);
	if (parse_threads >= 0) m2dec_amd_h264_set_parse_threads(ctx, parse_threads);
	dec_bits_set_callback(h264d_func->stream_pos(ctx), drv_reread, &v);
	const double t_start = mono_s();
	v.t_last = t_start;
	/* h264dec.cpp:251-257 + M2Decoder::decode / decode_residual (m2decoder.h:132-157) */
	for (;;) {
		err = 0;
		while (h264d_func->peek_decoded_frame(ctx, &frm, 0) <= 0) {
			err = h264d_func->decode_picture(ctx);
			if (v.failed) { err = -1; break; }
			if (err < 0) {
				while (h264d_func->peek_decoded_frame(ctx, &frm, 1) > 0) {
					emit(&v, &frm);
					n++;
					h264d_func->get_decoded_frame(ctx, &frm, 1);
				}
				goto done;
			}
		}
		h264d_func->get_decoded_frame(ctx, &frm, 0);
		if (d->stats && n == 0) fprintf(stderr, "first frame out: %.3f s\n", mono_s() - t_start);
		emit(&v, &frm);
		n++;
		err = h264d_func->decode_picture(ctx);
		if (err < 0) {
			while (h264d_func->peek_decoded_frame(ctx, &frm, 1) > 0) {
				emit(&v, &frm);
				n++;
				h264d_func->get_decoded_frame(ctx, &frm, 1);
			}
			break;
		}
	}
done:
	if (on_end) on_end(arg);
	if (d->stats) fprintf(stderr, "stream: %d frames, %.3f s\n", n, mono_s() - t_start);
	if (stats && !backend && d->have_backend) {
		m2dec_amd_hip_timing_t t;
		if (m2dec_amd_hip_backend_timing(&d->backend, &t) == 0) {
			stats->kernel_us = t.picture_us;
			stats->kernel_launches = t.kernel_launches;
			stats->alg_bytes = t.frame_bytes + t.ref_bytes + t.record_bytes;
			stats->h2d_us = t.h2d_us;
			stats->d2h_us = t.d2h_us;
			stats->d2h_bytes = t.d2h_bytes;
			stats->host_copy_us = t.host_copy_us;
		}
	}
	if (stats) {
		long par, fb;
		stats->parse_cpu_s = h264_async_parse_seconds(d, &par, &fb);
		stats->slice_par_pictures = par;
		stats->slice_par_fallbacks = fb;
	}
	if (stats) {
		stats->frames_out = n;
		stats->pictures = (int)d->pictures;
		stats->last_error = err;
		stats->ahead = (int)d->ahead_submits;
		stats->t_start = t_start;
		stats->t_end = v.t_last;
		stats->setup_s = v.setup_s;
	}
	if (backend) m2dec_amd_h264_set_backend(ctx, NULL); /* borrowed: the caller destroys it */
	{
		const double t0 = mono_s();
		m2dec_amd_h264_release(ctx);
		if (stats) stats->teardown_s = mono_s() - t0;
	}
	free(ctx);
	if (hold) m2dec_hold_wait_idle(hold);
	fpool_give(v.frame_mem, v.frame_size);
	return (err == -2) ? n : -1;
}

/* ------------------------------------------------------------------ held frames */
void m2dec_hold_init(m2dec_hold_t *h)
{
	memset(h, 0, sizeof(*h));
	pthread_mutex_init(&h->mu, NULL);
	pthread_cond_init(&h->cv, NULL);
}

void m2dec_hold_destroy(m2dec_hold_t *h)
{
	pthread_mutex_destroy(&h->mu);
	pthread_cond_destroy(&h->cv);
}

int m2dec_hold_busy(const m2dec_hold_t *h, const uint8_t *luma)
{
	for (int i = 0; i < h->n; ++i)
		if (h->luma[i] == luma) return h->cnt[i] > 0;
	return 0;
}

void m2dec_hold_add(m2dec_hold_t *h, const uint8_t *luma)
{
	pthread_mutex_lock(&h->mu);
	int i = 0;
	while (i < h->n && h->luma[i] != luma) ++i;
	if (i == h->n && h->n < 64) {
		h->luma[i] = luma;
		h->cnt[i] = 0;
		h->n++;
	}
	if (i < h->n) h->cnt[i]++;
	pthread_mutex_unlock(&h->mu);
}

void m2dec_hold_release(m2dec_hold_t *h, const uint8_t *luma)
{
	pthread_mutex_lock(&h->mu);
	for (int i = 0; i < h->n; ++i)
		if (h->luma[i] == luma && h->cnt[i] > 0) {
			h->cnt[i]--;
			break;
		}
	pthread_cond_broadcast(&h->cv);
	pthread_mutex_unlock(&h->mu);
}

void m2dec_hold_wait_idle(m2dec_hold_t *h)
{
	pthread_mutex_lock(&h->mu);
	for (;;) {
		int busy = 0;
		for (int i = 0; i < h->n; ++i) busy |= h->cnt[i] > 0;
		if (!busy) break;
		pthread_cond_wait(&h->cv, &h->mu);
	}
	h->n = 0; /* (frame memory may be reallocated: forget the addresses) */
	pthread_mutex_unlock(&h->mu);
}
