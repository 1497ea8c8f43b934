/*
 * Throughput drivers over the unchanged h264d_func decode path (the same loop as h264dec -O,
 * h264dec.cpp:251-257 + m2decoder.h:132-157, see m2dec_amd_decode_stream2):
 *
 *   m2dec_amd_decode_stream_md5   one stream; every output frame is copied out of the caller's frame
 *                                 buffer and its FileWriterMd5 line (filewrite.h:99-124) computed on
 *                                 helper threads, so MD5 overlaps the parse of the next pictures;
 *   m2dec_amd_decode_streams_md5  n independent streams, one host thread (and one decoder context)
 *                                 each, sharing one GPU — the within-GPU form of SURVEY.md §8e's
 *                                 stream sharding.
 *
 * Decoder contexts are independent (all state in the context, const global tables), as in the
 * reference (h264.h:435-446), so the threads share nothing but the device.
 */
#define _GNU_SOURCE /* pthread_setname_np */
#include <pthread.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include "h264_dec.h"
#include "h265_dec.h"
#include "m2dec_amd.h"

/* M2DEC_AMD_THREAD_CPU=1: a driver thread prints its CPU time when it ends (tools/thread_cpu.py reads it: an
 * exited thread is gone from /proc/self/task) */
static void thread_cpu_report(const char *name)
{
	static int on = -1;
	if (on < 0) on = getenv("M2DEC_AMD_THREAD_CPU") && atoi(getenv("M2DEC_AMD_THREAD_CPU"));
	if (on) {
		struct timespec ts;
		clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
		fprintf(stderr, "thread-cpu %s %.3f\n", name, 1e3 * ts.tv_sec + 1e-6 * ts.tv_nsec);
	}
}

#define MD5_RING 64        /* frames queued or being hashed (all streams of a pipe) */
#define MD5_EXTRA 40       /* frames a stream's decoder gets beyond its need (held by queued MD5s meanwhile) */
#define MD5_BATCH 16       /* frames one thread hashes together (m2dec_amd_frames_md5 lanes) */
#define MD5_MIN_BATCH 8    /* a batch costs about the same CPU time for 2 or 16 frames: a thread waits for
                              this many (or MD5_WAIT_S after the oldest was queued, or the end) */
#define MD5_WAIT_S 0.004
/* the shared pipe of several concurrent streams: frames arrive ~4x as fast, so full 16-frame batches cost half
 * the CPU time per frame of 8-frame ones (8 streams 2142 vs 2059 fps, profiles/r131_ab_md5_streams.txt) */
#define MD5_MIN_BATCH_STREAMS 16
#define MD5_WAIT_S_STREAMS 0.008
#define MD5_THREADS_MAX 16
#define MD5_THREADS 16     /* one stream: a 16-frame batch of 1080p takes one core ~6.5 ms on the box's EPYC
                              9575F, one frame alone 3.3 ms (tools/md5_batch_bench.py, profiles/r85_md5_batch.txt);
                              most threads only work in tail mode (below); M2DEC_AMD_MD5_THREADS */
/* tail mode once at most this many parse workers are busy: one stream 12 (c3 medians 28.83 vs 29.21 and 29.77 vs
 * 30.97 ms against 4 on two boxes, profiles/r137_ab_md5_tail_busy.txt; 16 = always: 30.15 ms), the shared pipe of
 * concurrent streams 4 (their pool stays busy until near the end) */
#define MD5_TAIL_PARSE_BUSY 12
#define MD5_TAIL_TAKE 2
#define MD5_TAIL_PARSE_BUSY_STREAMS 4
#define MD5_BIG_FRAME ((size_t)6 << 20) /* frames above this (4K) are not batched short of min_batch */

/* one stream's MD5 threads: MD5_THREADS, at most the process's CPU share (cpushare.c) */
static int md5_threads_default(void)
{
	const int s = m2d_cpu_share();
	return s < MD5_THREADS ? s : MD5_THREADS;
}

/* The MD5 threads hash the decoder's frame buffers in place: on_frame holds the frame (the decoder
 * does not reuse it until it is released, h264_dec.h m2dec_hold_t) and queues it; no copy on the
 * caller's thread.  One pipe may serve several streams (m2dec_amd_decode_streams_md5): their frames
 * share the 16 lanes of a batch, which a single stream fills only at its end. */
struct md5_pipe;
typedef struct {
	struct md5_pipe *pipe;
	m2dec_hold_t hold;
	char *md5s;
	int max;
	int n;                   /* frames delivered */
	int ended;               /* md5_on_end ran */
	double t_done;           /* the last MD5 line written */
} md5_stream_t;

typedef struct md5_pipe {
	pthread_mutex_t mu;
	pthread_cond_t cv_job, cv_free;
	m2d_frame_t frm[MD5_RING];
	md5_stream_t *of[MD5_RING];
	int idx[MD5_RING];       /* output frame number of the job in slot k */
	double t_queued[MD5_RING];
	int state[MD5_RING];     /* 0 free, 1 queued, 2 being hashed */
	int head, next;          /* slots filled / taken by a hashing thread, in order */
	int quit;                /* no more frames (every stream ended) */
	int streams, ended;      /* streams using the pipe / past their last frame: hash at once */
	int stats;
	int delay_us;            /* M2DEC_AMD_MD5_DELAY_US (tests) */
	int min_batch;           /* frames a thread waits for (M2DEC_AMD_MD5_MIN_BATCH, default MD5_MIN_BATCH) */
	int tail_mode;           /* M2DEC_AMD_MD5_TAIL (default 1) */
	int tail_busy;           /* tail mode at most this many busy parse workers (M2DEC_AMD_MD5_TAIL_BUSY) */
	int tail_take;           /* frames a thread takes together in tail mode (M2DEC_AMD_MD5_TAIL_TAKE, 1-3) */
	double wait_s;           /* ... or this long after the oldest was queued (M2DEC_AMD_MD5_WAIT_US) */
	double t_wait;           /* callers: waiting for a free queue slot */
	double t_hash;           /* MD5 threads: time hashing */
	long batches;
	pthread_t th[MD5_THREADS_MAX];
	int nth;
} md5_pipe_t;

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* a free thread takes every queued frame (up to MD5_BATCH) and hashes them side by side */
static void *md5_worker(void *arg)
{
	pthread_setname_np(pthread_self(), "m2d-md5");
	md5_pipe_t *p = (md5_pipe_t *)arg;
	pthread_mutex_lock(&p->mu);
	for (;;) {
		while (p->next == p->head && !p->quit) pthread_cond_wait(&p->cv_job, &p->mu);
		if (p->next == p->head) break;
		m2d_place_self(); /* (numa.c) */
		/* tail mode: the parse pool is (nearly) out of work — a stream's last pictures are being parsed or
		 * coming out: hash one frame at once, alone — 3.3 ms instead of a batch's 6.5 ms after the stream's
		 * last output (a batch taken as the last 2-4 pictures parse ends last: r98).  While the pool is
		 * busy, batches keep the MD5 CPU time small. */
		int tail = 0;
		for (;;) { /* (the tail test is redone on every wake: the parse pool may finish while a thread waits) */
			tail = p->tail_mode && m2dec_parse_busy() <= p->tail_busy;
			if (tail || p->quit || p->ended || p->head - p->next >= p->min_batch) break;
			double left = p->t_queued[p->next % MD5_RING] + p->wait_s - now_s();
			if (left <= 0) break;
			if (p->tail_mode && left > 5e-4) left = 5e-4;
			struct timespec ts;
			clock_gettime(CLOCK_REALTIME, &ts);
			ts.tv_nsec += (long)(left * 1e9);
			ts.tv_sec += ts.tv_nsec / 1000000000L;
			ts.tv_nsec %= 1000000000L;
			pthread_cond_timedwait(&p->cv_job, &p->mu, &ts);
		}
		/* frames per thread: in tail mode one each (the threads still hashing finish within ~3 ms and take
		 * the rest; a thread that took all queued frames alone ran 6.7 ms past the last frame: r97), more
		 * only when the queue outnumbers the threads.  Outside the tail, a batch short of min_batch (the wait
		 * timed out) of large frames goes one frame per thread too: any batch of 2-16 costs about twice one
		 * frame's time on the 16-lane kernel (6.3-6.5 ms for 1080p on the box, profiles/r128_md5_batch.txt),
		 * and for a 4K frame (12.4 MB, ~13 ms alone) a 3-frame batch taken while the parse was still busy
		 * ran 25 ms and ended the C5 decode (profiles/r127_timeline_c5.txt) */
		const int queued = p->head - p->next;
		const size_t fbytes = (size_t)p->frm[p->next % MD5_RING].width * (size_t)p->frm[p->next % MD5_RING].height * 3 / 2;
		int share = tail ? (queued + p->nth - 1) / p->nth
		                 : ((queued < p->min_batch && fbytes > MD5_BIG_FRAME) ? 1 : MD5_BATCH);
		/* tail: up to tail_take frames side by side on one core (md5.c stitched chains: 2 frames of 1080p in
		 * 3.13 ms, 3 in 3.39 ms against 3.24 ms for one on the box's host, profiles/r141_md5host.txt), so the
		 * tail's frames need a third to half of the cores.  c3 median decode 29.00 vs 30.68 ms with pairs;
		 * 4K frames stay one per thread (C5 47.5 vs 45.9 ms with pairs, profiles/r141_ab_tail_take_*.txt) */
		if (tail && share < p->tail_take && fbytes <= MD5_BIG_FRAME)
			share = queued < p->tail_take ? queued : p->tail_take;
		if (p->next == p->head) continue; /* (another thread took them) */
		m2d_frame_t f[MD5_BATCH];
		md5_stream_t *sof[MD5_BATCH];
		int ks[MD5_BATCH], ix[MD5_BATCH], n = 0;
		while (n < share && n < MD5_BATCH && p->next < p->head) {
			const int k = p->next % MD5_RING;
			p->next++;
			p->state[k] = 2;
			f[n] = p->frm[k];
			sof[n] = p->of[k];
			ix[n] = p->idx[k];
			ks[n++] = k;
		}
		pthread_mutex_unlock(&p->mu);
		if (p->delay_us) usleep((useconds_t)p->delay_us); /* (tests: MD5 slower than the decoder) */
		char lines[MD5_BATCH][35];
		m2d_cpu_enter(); /* (cpushare.c: within the busy-thread slots the parse leaves free) */
		const double th = now_s();
		m2d_tl('H', n, n ? ix[0] : -1);
		m2dec_amd_frames_md5(f, n, lines);
		m2d_tl('h', n, n ? ix[0] : -1);
		m2d_cpu_leave();
		const double th1 = now_s();
		const double t = now_s();
		pthread_mutex_lock(&p->mu);
		p->t_hash += th1 - th;
		p->batches++;
		for (int j = 0; j < n; ++j) {
			if (ix[j] < sof[j]->max) memcpy(sof[j]->md5s + (size_t)ix[j] * 35, lines[j], 35);
			if (t > sof[j]->t_done) sof[j]->t_done = t;
			p->state[ks[j]] = 0;
		}
		/* (last: once its holds are released a stream may return and its md5_stream_t is gone) */
		for (int j = 0; j < n; ++j) m2dec_hold_release(&sof[j]->hold, f[j].luma);
		pthread_cond_broadcast(&p->cv_free);
	}
	pthread_mutex_unlock(&p->mu);
	thread_cpu_report("m2d-md5");
	return NULL;
}

/* on_frame of the stream driver: hold the frame, queue its MD5 */
static void md5_on_frame(void *arg, const m2d_frame_t *f)
{
	md5_stream_t *s = (md5_stream_t *)arg;
	md5_pipe_t *p = s->pipe;
	const double t0 = p->stats ? now_s() : 0;
	m2dec_hold_add(&s->hold, f->luma);
	pthread_mutex_lock(&p->mu);
	while (p->state[p->head % MD5_RING]) pthread_cond_wait(&p->cv_free, &p->mu);
	const int k = p->head % MD5_RING;
	if (p->stats) p->t_wait += now_s() - t0;
	p->frm[k] = *f;
	p->of[k] = s;
	m2d_tl('O', s->n, 0);
	p->idx[k] = s->n++;
	p->t_queued[k] = now_s();
	p->state[k] = 1;
	p->head++;
	pthread_cond_broadcast(&p->cv_job);
	pthread_mutex_unlock(&p->mu);
}

/* a stream's last frame was queued: hash what is left at once */
static void md5_on_end(void *arg)
{
	md5_stream_t *s = (md5_stream_t *)arg;
	md5_pipe_t *p = s->pipe;
	pthread_mutex_lock(&p->mu);
	if (!s->ended) {
		s->ended = 1;
		p->ended++;
		if (p->ended >= p->streams) p->quit = 1;
	}
	pthread_cond_broadcast(&p->cv_job);
	pthread_mutex_unlock(&p->mu);
}

static int pipe_open(md5_pipe_t *p, int streams, int threads)
{
	memset(p, 0, sizeof(*p));
	pthread_mutex_init(&p->mu, NULL);
	pthread_cond_init(&p->cv_job, NULL);
	pthread_cond_init(&p->cv_free, NULL);
	if (getenv("M2DEC_AMD_MD5_DELAY_US")) p->delay_us = atoi(getenv("M2DEC_AMD_MD5_DELAY_US"));
	p->min_batch = streams > 1 ? MD5_MIN_BATCH_STREAMS : MD5_MIN_BATCH;
	p->wait_s = streams > 1 ? MD5_WAIT_S_STREAMS : MD5_WAIT_S;
	if (getenv("M2DEC_AMD_MD5_MIN_BATCH")) p->min_batch = atoi(getenv("M2DEC_AMD_MD5_MIN_BATCH")); /* tuning */
	if (getenv("M2DEC_AMD_MD5_WAIT_US")) p->wait_s = 1e-6 * atoi(getenv("M2DEC_AMD_MD5_WAIT_US"));
	if (p->min_batch < 1) p->min_batch = 1;
	if (p->min_batch > MD5_BATCH) p->min_batch = MD5_BATCH;
	p->stats = getenv("M2DEC_AMD_ASYNC_STATS") != NULL;
	p->tail_mode = getenv("M2DEC_AMD_MD5_TAIL") ? atoi(getenv("M2DEC_AMD_MD5_TAIL")) != 0 : 1;
	p->tail_take = getenv("M2DEC_AMD_MD5_TAIL_TAKE") ? atoi(getenv("M2DEC_AMD_MD5_TAIL_TAKE")) : MD5_TAIL_TAKE;
	if (p->tail_take < 1) p->tail_take = 1;
	if (p->tail_take > 3) p->tail_take = 3;
	p->tail_busy = getenv("M2DEC_AMD_MD5_TAIL_BUSY") ? atoi(getenv("M2DEC_AMD_MD5_TAIL_BUSY"))
	                                                 : (streams > 1 ? MD5_TAIL_PARSE_BUSY_STREAMS : MD5_TAIL_PARSE_BUSY);
	p->streams = streams;
	for (; p->nth < threads && p->nth < MD5_THREADS_MAX; ++p->nth)
		if (pthread_create(&p->th[p->nth], NULL, md5_worker, p) != 0) break;
	if (!p->nth) {
		pthread_mutex_destroy(&p->mu);
		pthread_cond_destroy(&p->cv_job);
		pthread_cond_destroy(&p->cv_free);
		return -1;
	}
	return 0;
}

static void pipe_close(md5_pipe_t *p)
{
	pthread_mutex_lock(&p->mu);
	p->quit = 1; /* (already set by the last md5_on_end unless a decode failed early) */
	pthread_cond_broadcast(&p->cv_job);
	pthread_mutex_unlock(&p->mu);
	for (int i = 0; i < p->nth; ++i) pthread_join(p->th[i], NULL);
	if (p->stats)
		fprintf(stderr, "md5: caller waits %.3f s, %d frames in %ld batches, hashing %.3f s (%d threads)\n", p->t_wait,
		        p->head, p->batches, p->t_hash, p->nth);
	pthread_mutex_destroy(&p->mu);
	pthread_cond_destroy(&p->cv_job);
	pthread_cond_destroy(&p->cv_free);
}

/* one stream through the shared pipe p: decode, MD5 lines into md5s; returns frames or < 0 */
static int stream_md5(md5_pipe_t *p, const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                      int parse_threads, char *md5s, int max, m2dec_amd_stats_t *stats)
{
	md5_stream_t s;
	m2dec_amd_stats_t st;
	int r;
	memset(&s, 0, sizeof(s));
	s.pipe = p;
	s.md5s = md5s;
	s.max = max;
	m2dec_hold_init(&s.hold);
	memset(&st, 0, sizeof(st));
	const char *ex = getenv("M2DEC_AMD_MD5_EXTRA"); /* (tests: fewer spare frames -> the decoder waits on holds) */
	m2d_tl('D', 0, 0);
	r = h264_decode_stream_held(data, len, backend, device, dpb, parse_threads, ex ? atoi(ex) : MD5_EXTRA, &s.hold,
	                            md5_on_frame, md5_on_end, &s, &st);
	md5_on_end(&s); /* (a decode that failed early did not reach on_end: do not hold the pipe up) */
	m2dec_hold_wait_idle(&s.hold); /* every queued MD5 of this stream is written */
	m2dec_hold_destroy(&s.hold);
	pthread_mutex_lock(&p->mu);
	if (s.t_done > st.t_end) st.t_end = s.t_done; /* delivered = its MD5 line written */
	pthread_mutex_unlock(&p->mu);
	st.hold_waits = s.hold.waits;
	m2d_tl('d', s.n, 0);
	if (stats) *stats = st;
	return r < 0 ? r : s.n;
}

static int decode_md5(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                      int parse_threads, int md5_threads, char *md5s, int max, m2dec_amd_stats_t *stats);

int m2dec_amd_decode_stream_md5(const uint8_t *data, size_t len, int device, int dpb, char *md5s, int max,
                                m2dec_amd_stats_t *stats)
{
	const char *e = getenv("M2DEC_AMD_MD5_THREADS");
	return decode_md5(data, len, NULL, device, dpb, -1, e && atoi(e) > 0 ? atoi(e) : md5_threads_default(), md5s, max, stats);
}

int m2dec_amd_decode_stream_md5_backend(const uint8_t *data, size_t len, const m2r_backend_t *backend, int parse_threads,
                                        int md5_threads, char *md5s, int max, m2dec_amd_stats_t *stats)
{
	return decode_md5(data, len, backend, 0, -1, parse_threads, md5_threads, md5s, max, stats);
}

/* ---- H.265 and MPEG-2 through the MD5 pipe (m2dec_amd_decode_h265_md5 / _m2v_md5): their frame LRUs
 * know no holds, so each delivered frame is copied into one of the driver's buffers and hashed there */
#define H265_MD5_RING 24 /* copies in flight: queued or being hashed */
typedef struct {
	md5_stream_t *s;
	uint8_t *buf[H265_MD5_RING];
	size_t bytes;
	int next;
	int failed;
} h265_md5_t;

/* the gfx950 H.265 back end writes the caller's frames only inside sync_frame, which waits for their holds:
 * the frame is hashed in place (m2dec_amd_decode_h265_held) */
static void h265_md5_in_place(void *arg, const m2d_frame_t *f)
{
	h265_md5_t *h = (h265_md5_t *)arg;
	md5_on_frame(h->s, f);
}

static void h265_md5_on_frame(void *arg, const m2d_frame_t *f)
{
	h265_md5_t *h = (h265_md5_t *)arg;
	const size_t ls = (size_t)f->width * (size_t)f->height, bytes = ls * 3 / 2;
	uint8_t *b;
	if (h->failed) return;
	if (bytes != h->bytes) { /* (a new geometry: every queued copy hashed first) */
		m2dec_hold_wait_idle(&h->s->hold);
		for (int i = 0; i < H265_MD5_RING; ++i) {
			free(h->buf[i]);
			h->buf[i] = NULL;
		}
		h->bytes = bytes;
	}
	if (!h->buf[h->next] && !(h->buf[h->next] = (uint8_t *)malloc(bytes))) {
		h->failed = 1;
		return;
	}
	b = h->buf[h->next];
	h->next = (h->next + 1) % H265_MD5_RING;
	pthread_mutex_lock(&h->s->hold.mu); /* the buffer's previous frame is hashed */
	while (m2dec_hold_busy(&h->s->hold, b)) pthread_cond_wait(&h->s->hold.cv, &h->s->hold.mu);
	pthread_mutex_unlock(&h->s->hold.mu);
	{
		void *to[2] = {b, b + ls};
		const void *from[2] = {f->luma, f->chroma};
		const size_t len[2] = {ls, ls / 2};
		m2dec_par_memcpy(M2DEC_CREW_SYNC, 2, to, from, len); /* (parcopy.c) */
	}
	{
		m2d_frame_t c = *f;
		c.luma = b;
		c.chroma = b + ls;
		md5_on_frame(h->s, &c);
	}
}

static int copy_md5(int codec, const uint8_t *data, size_t len, const h265r_backend_t *be, int device, char *md5s,
                    int max, int *last_error)
{
	md5_pipe_t p;
	md5_stream_t s;
	h265_md5_t h;
	int err = 0, r;
	const char *e = getenv("M2DEC_AMD_MD5_THREADS");
	if (pipe_open(&p, 1, e && atoi(e) > 0 ? atoi(e) : md5_threads_default()) < 0) return -1;
	memset(&s, 0, sizeof(s));
	s.pipe = &p;
	s.md5s = md5s;
	s.max = max;
	m2dec_hold_init(&s.hold);
	memset(&h, 0, sizeof(h));
	h.s = &s;
	const char *ip = getenv("M2DEC_AMD_H265_MD5_IN_PLACE"); /* (A/B: 0 = copy every frame first) */
	if (codec == 265 && (!be || be->stage) && !(ip && atoi(ip) == 0))
		r = m2dec_amd_decode_h265_held(data, len, be, device, h265_md5_in_place, &h, &s.hold, &err);
	else if (codec == 265) r = m2dec_amd_decode_h265(data, len, be, device, 0, h265_md5_on_frame, &h, &err);
	else r = m2dec_amd_decode_m2v(data, len, device, 0, h265_md5_on_frame, &h, &err);
	md5_on_end(&s);
	m2dec_hold_wait_idle(&s.hold); /* every queued MD5 is written */
	m2dec_hold_destroy(&s.hold);
	pipe_close(&p);
	for (int i = 0; i < H265_MD5_RING; ++i) free(h.buf[i]);
	if (last_error) *last_error = err;
	return h.failed || r == -3 ? -1 : s.n;
}

int m2dec_amd_decode_h265_md5(const uint8_t *data, size_t len, const h265r_backend_t *be, int device, char *md5s, int max,
                              int *last_error)
{
	return copy_md5(265, data, len, be, device, md5s, max, last_error);
}

int m2dec_amd_decode_m2v_md5(const uint8_t *data, size_t len, int device, char *md5s, int max, int *last_error)
{
	return copy_md5(2, data, len, NULL, device, md5s, max, last_error);
}

static int decode_md5(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                      int parse_threads, int md5_threads, char *md5s, int max, m2dec_amd_stats_t *stats)
{
	md5_pipe_t p;
	int r;
	if (pipe_open(&p, 1, md5_threads) < 0) return -1;
	r = stream_md5(&p, data, len, backend, device, dpb, parse_threads, md5s, max, stats);
	pipe_close(&p);
	return r;
}

typedef struct {
	md5_pipe_t *pipe;
	const uint8_t *data;
	size_t len;
	int device;
	char *md5s;
	int max;
	int result;
} stream_job_t;

static void *stream_worker(void *arg)
{
	pthread_setname_np(pthread_self(), "m2d-stream");
	stream_job_t *j = (stream_job_t *)arg;
	/* parse-ahead workers a stream may occupy in the shared pool (M2DEC_AMD_STREAM_PARSE_THREADS) */
	const char *e = getenv("M2DEC_AMD_STREAM_PARSE_THREADS");
	/* profiles/r59_sweep_e2e.txt: 8 streams, 3 -> ~1440, 8 -> ~1490 fps; at most the CPU share (cpushare.c) */
	const int pt = e && atoi(e) > 0 ? atoi(e) : (m2d_cpu_share() < 8 ? m2d_cpu_share() : 8);
	j->result = stream_md5(j->pipe, j->data, j->len, NULL, j->device, -1, pt, j->md5s, j->max, NULL);
	thread_cpu_report("m2d-stream");
	return NULL;
}

/* n streams, one host thread and decoder context each, one MD5 pipe for all of them */
int m2dec_amd_decode_streams_md5(int n, const uint8_t *const *datas, const size_t *lens, int device, char *const *md5s,
                                 const int *max, int *frames)
{
	stream_job_t *jobs;
	pthread_t *th;
	md5_pipe_t pipe;
	int ok = 0;
	if (n <= 0) return -1;
	{
		const char *m = getenv("M2DEC_AMD_STREAM_MD5_THREADS"); /* MD5 threads of the shared pipe */
		int mt = m && atoi(m) > 0 ? atoi(m) : (n + 1) / 2 + 1;
		if (!(m && atoi(m) > 0) && mt > m2d_cpu_share()) mt = m2d_cpu_share();
		if (pipe_open(&pipe, n, mt) < 0) return -1;
	}
	jobs = (stream_job_t *)calloc((size_t)n, sizeof(*jobs));
	th = (pthread_t *)calloc((size_t)n, sizeof(*th));
	if (!jobs || !th) {
		free(jobs);
		free(th);
		pipe_close(&pipe);
		return -1;
	}
	for (int i = 0; i < n; ++i) {
		jobs[i].pipe = &pipe;
		jobs[i].data = datas[i];
		jobs[i].len = lens[i];
		jobs[i].device = device;
		jobs[i].md5s = md5s[i];
		jobs[i].max = max[i];
		jobs[i].result = -1;
		if (pthread_create(&th[i], NULL, stream_worker, &jobs[i]) != 0) {
			for (int k = i; k < n; ++k) { /* (streams never started end now) */
				pthread_mutex_lock(&pipe.mu);
				pipe.ended++;
				if (pipe.ended >= pipe.streams) pipe.quit = 1;
				pthread_cond_broadcast(&pipe.cv_job);
				pthread_mutex_unlock(&pipe.mu);
			}
			n = i;
			ok = -1;
			break;
		}
	}
	for (int i = 0; i < n; ++i) {
		pthread_join(th[i], NULL);
		if (frames) frames[i] = jobs[i].result;
		if (jobs[i].result < 0) ok = -1;
	}
	pipe_close(&pipe);
	free(jobs);
	free(th);
	return ok;
}

/* ---------------------------------------------------------------- host-parse measurement back end */
/* A back end that keeps no pixels: acquire hands out one record arena, submit / sync do nothing.
 * Decoding through it times the host side alone (parse, or the parse-ahead pipeline). */
typedef struct {
	m2r_picture_t pic;
	uint8_t *mem;
	size_t size;
} null_be_t;

static int null_set_frames(void *self, int n, const m2d_frame_t *frames, int w, int h)
{
	(void)self; (void)n; (void)frames; (void)w; (void)h;
	return 0;
}

static m2r_picture_t *null_acquire(void *self, int wm, int hm)
{
	null_be_t *b = (null_be_t *)self;
	const int n = wm * hm;
	const size_t need = (size_t)n * (sizeof(m2r_mb_t) + sizeof(m2r_deblock_t) + sizeof(m2r_inter_t) + 416 * sizeof(int16_t)) +
	                    256 * sizeof(m2r_slice_t) + 64;
	if (need > b->size) {
		free(b->mem);
		b->mem = (uint8_t *)malloc(need);
		b->size = b->mem ? need : 0;
		if (!b->mem) return NULL;
	}
	uint8_t *p = b->mem;
	memset(&b->pic, 0, sizeof(b->pic));
	b->pic.width_mbs = wm;
	b->pic.height_mbs = hm;
	b->pic.mb = (m2r_mb_t *)p; p += (size_t)n * sizeof(m2r_mb_t);
	b->pic.dbk = (m2r_deblock_t *)p; p += (size_t)n * sizeof(m2r_deblock_t);
	b->pic.slice = (m2r_slice_t *)p; p += 256 * sizeof(m2r_slice_t);
	b->pic.inter = (m2r_inter_t *)p; p += (size_t)n * sizeof(m2r_inter_t);
	b->pic.coef = (int16_t *)p;
	b->pic.cap_slices = 256;
	b->pic.cap_inter = n;
	b->pic.cap_coef = n * 416;
	return &b->pic;
}

static int null_submit(void *self, m2r_picture_t *pic)
{
	(void)self; (void)pic;
	return 0;
}

static int null_sync(void *self, int slot)
{
	(void)self; (void)slot;
	return 0;
}

static void null_destroy(void *self)
{
	null_be_t *b = (null_be_t *)self;
	free(b->mem);
	free(b);
}

int m2dec_amd_null_backend_create(m2r_backend_t *out)
{
	null_be_t *b = (null_be_t *)calloc(1, sizeof(null_be_t));
	if (!b || !out) {
		free(b);
		return -1;
	}
	out->self = b;
	out->set_frames = null_set_frames;
	out->acquire = null_acquire;
	out->submit = null_submit;
	out->sync_frame = null_sync;
	out->destroy = null_destroy;
	out->bind = NULL;
	out->flush = NULL;
	out->ready = NULL;
	out->records_busy = NULL;
	return 0;
}
