/*
 * Parse-ahead pipeline: the slice data of several pictures parsed at once on worker threads, behind
 * the unchanged h264d_func API ("pipelining parse n+1 with GPU recon n").
 *
 * What stays on the caller's thread, in stream order: NAL scanning, SPS/PPS, every slice header
 * (POC, reference lists, weights, marking syntax), the reference marking / co-located store swap /
 * DPB insertion of a finished picture (they need only the headers), and every call into the back
 * end (acquire / submit / sync_frame), in decode order.
 *
 * What moves to the workers: h264_slice_data (CABAC/CAVLC, MV prediction, direct, bS -> records)
 * and the deblock edge resolution of a whole picture.  A job is one picture: for each of its slices
 * a copy of the decoder context right after that slice's header (60 KB) and a copy of its RBSP;
 * the worker runs the slices in order on a private context, carrying the few fields the slice
 * parser accumulates across slices, into a private MB-info array and a private record arena.
 *
 * Cross-picture dependencies of the slice data: a B slice reads the co-located store of its
 * refs[1][0] (spatial and temporal direct, h264.cpp:9777 / 9848), written by an earlier picture's
 * parse -> the job waits for that writer job.  A store is recycled by the marking swap
 * (h264.cpp:10970-10984) -> a job that writes it is dispatched only after every earlier job that
 * read or wrote it has finished.
 *
 * Picture boundaries: the synchronous parser knows a picture is complete when its last MB is
 * parsed; here the caller's thread sees only headers, so a picture is closed when the next
 * picture's first slice arrives (first_mb not above the previous slice's, the reference's own
 * test, h264.cpp:1427-1430) or at the end of the data.  decode_picture still returns 1 once per
 * picture and the DPB output order is unchanged; a frame is handed out (peek / get) only after its
 * picture was parsed and submitted, and sync_frame has waited for its reconstruction.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "h264_dec.h"

#define AS_MAX 32 /* jobs alive (collecting + dispatched + free) */

typedef struct h264_job {
	int nsl, capsl;
	h264_dec_t **snap;        /* [nsl] decoder context right after each slice header */
	uint8_t **rbsp;           /* [nsl] slice RBSP copies (16 zero bytes of padding) */
	h264_mbinfo_t *mbi;       /* private neighbour state */
	size_t mbi_n;
	m2r_picture_t pic;        /* private record arena */
	uint8_t *arena;
	size_t arena_size;
	int slot, col_store;
	int nonref;               /* no slice has nal_ref_idc: its co-located store is never read ... */
	h264_colmb_t *priv_col;   /* ... so it writes this private one (no ordering against other jobs) */
	size_t priv_n;
	long deps[8];             /* seq of the jobs whose parse must finish first (jobs are recycled:
	                             never keep a pointer past its submission) */
	int ndeps;
	long seq;
	int taken, done, err;     /* guarded by the pipeline mutex */
	h264_dec_t *w;            /* worker context */
} h264_job_t;

struct h264_async {
	pthread_mutex_t mu;
	pthread_cond_t cv_work, cv_done;
	pthread_t th[16];
	int nth, quit, depth;
	h264_job_t *fifo[AS_MAX]; /* dispatched, not yet submitted: [tail, head) */
	long head, tail;
	h264_job_t *queue[AS_MAX]; /* dispatched; [qtail, qhead) holds every job not yet taken */
	long qhead, qtail;
	h264_job_t *cur;          /* the picture being collected */
	h264_job_t *free_jobs[AS_MAX];
	int nfree;
	long seq;
	long col_last[17];        /* seq of the last dispatched job that reads or writes store i */
	h264_job_t *col_writer[17]; /* dispatched, unsubmitted job writing store i */
};

static int job_arena(h264_job_t *j, int wm, int hm)
{
	const int n = wm * hm;
	const size_t need = (size_t)n * (sizeof(m2r_mb_t) + sizeof(m2r_deblock_t) + sizeof(m2r_inter_t) + 416 * sizeof(int16_t)) +
	                    256 * sizeof(m2r_slice_t) + 64;
	if (need > j->arena_size) {
		free(j->arena);
		j->arena = (uint8_t *)malloc(need);
		j->arena_size = j->arena ? need : 0;
		if (!j->arena) return -1;
	}
	uint8_t *p = j->arena;
	m2r_picture_t *pic = &j->pic;
	memset(pic, 0, sizeof(*pic));
	pic->width_mbs = wm;
	pic->height_mbs = hm;
	pic->mb = (m2r_mb_t *)p; p += (size_t)n * sizeof(m2r_mb_t);
	pic->dbk = (m2r_deblock_t *)p; p += (size_t)n * sizeof(m2r_deblock_t);
	pic->slice = (m2r_slice_t *)p; p += 256 * sizeof(m2r_slice_t);
	pic->inter = (m2r_inter_t *)p; p += (size_t)n * sizeof(m2r_inter_t);
	pic->coef = (int16_t *)p;
	pic->cap_slices = 256;
	pic->cap_inter = n;
	pic->cap_coef = n * 416;
	if ((size_t)n > j->mbi_n) {
		free(j->mbi);
		j->mbi = (h264_mbinfo_t *)malloc(sizeof(h264_mbinfo_t) * (size_t)n);
		j->mbi_n = j->mbi ? (size_t)n : 0;
		if (!j->mbi) return -1;
	}
	return 0;
}

static void job_clear(h264_job_t *j)
{
	for (int i = 0; i < j->nsl; ++i) {
		free(j->snap[i]);
		free(j->rbsp[i]);
	}
	j->nsl = 0;
	j->ndeps = 0;
	j->taken = 0;
	j->done = 0;
	j->err = 0;
}

static void job_free(h264_job_t *j)
{
	if (!j) return;
	job_clear(j);
	free(j->snap);
	free(j->rbsp);
	free(j->mbi);
	free(j->priv_col);
	free(j->arena);
	free(j->w);
	free(j);
}

/* ---------------------------------------------------------------- worker */
static void job_run(h264_job_t *j)
{
	h264_dec_t *w = j->w;
	int mbs = 0, slice_num = 0, slice_rec = 0, last_firstline = 0, ret = 0;
	int8_t idc[1024], alpha[1024], beta[1024];
	const int n = j->snap[0]->n_mbs;
	for (int i = 0; i < n; ++i) {
		j->mbi[i].type = -1;
		j->mbi[i].slice = -1;
	}
	last_firstline = j->snap[0]->last_firstline;
	for (int k = 0; k < j->nsl; ++k) {
		const h264_dec_t *s = j->snap[k];
		const ptrdiff_t off = j->rbsp[k] - s->slice_rbsp;
		memcpy(w, s, sizeof(*w));
		w->mbi = j->mbi;
		w->pic = &j->pic;
		if (j->nonref) w->colpic[w->curr_col].mb = j->priv_col;
		w->mbs_decoded = mbs;
		w->slice_num = slice_num;
		w->slice_rec = slice_rec;
		w->last_firstline = last_firstline;
		memcpy(w->slice_idc, idc, (size_t)slice_num);
		memcpy(w->slice_alpha, alpha, (size_t)slice_num);
		memcpy(w->slice_beta, beta, (size_t)slice_num);
		/* the bit reader and RBSP bounds pointed into the caller's NAL buffer: rebase onto the copy */
		w->bs.p += off;
		w->bs.end += off;
		w->slice_rbsp += off;
		w->slice_rbsp_end += off;
		ret = h264_slice_data(w);
		if (ret < 0) {
			j->err = 1;
			return;
		}
		mbs = w->mbs_decoded;
		slice_rec = w->slice_rec;
		last_firstline = w->last_firstline;
		memcpy(idc + slice_num, w->slice_idc + slice_num, (size_t)(w->slice_num - slice_num));
		memcpy(alpha + slice_num, w->slice_alpha + slice_num, (size_t)(w->slice_num - slice_num));
		memcpy(beta + slice_num, w->slice_beta + slice_num, (size_t)(w->slice_num - slice_num));
		slice_num = w->slice_num;
	}
	if (ret != 1) { /* the picture's MBs were not all coded (the synchronous parser would stop too) */
		j->err = 1;
		return;
	}
	h264_picture_resolve_deblock(w);
}

/* 1: every job j waits for has finished parsing (0: not yet); a dependency no longer in the fifo was
 * submitted, hence finished.  *err collects their errors.  Caller holds the mutex. */
static int deps_ready(const struct h264_async *as, const h264_job_t *j, int *err)
{
	for (int i = 0; i < j->ndeps; ++i)
		for (long k = as->tail; k < as->head; ++k) {
			const h264_job_t *o = as->fifo[k % AS_MAX];
			if (o->seq != j->deps[i]) continue;
			if (!o->done) return 0;
			*err |= o->err;
		}
	return 1;
}

/* Workers take the oldest queued job whose dependencies have finished, so a B picture waiting for
 * its co-located P does not hold a worker while later P pictures could be parsed. */
static void *worker(void *arg)
{
	struct h264_async *as = (struct h264_async *)arg;
	pthread_mutex_lock(&as->mu);
	for (;;) {
		h264_job_t *j = NULL;
		int dep_err = 0;
		for (;;) {
			while (as->qtail < as->qhead && as->queue[as->qtail % AS_MAX]->taken) as->qtail++;
			for (long k = as->qtail; k < as->qhead && !j; ++k) {
				h264_job_t *c = as->queue[k % AS_MAX];
				dep_err = 0;
				if (!c->taken && deps_ready(as, c, &dep_err)) j = c;
			}
			if (j || (as->quit && as->qtail == as->qhead)) break;
			pthread_cond_wait(&as->cv_work, &as->mu);
		}
		if (!j) break;
		j->taken = 1;
		pthread_mutex_unlock(&as->mu);
		if (dep_err) j->err = 1;
		else job_run(j);
		pthread_mutex_lock(&as->mu);
		j->done = 1;
		pthread_cond_broadcast(&as->cv_done);
		pthread_cond_broadcast(&as->cv_work); /* jobs waiting on this one may be ready */
	}
	pthread_mutex_unlock(&as->mu);
	return NULL;
}

/* ---------------------------------------------------------------- caller's thread */
int h264_async_start(h264_dec_t *d, int threads)
{
	struct h264_async *as;
	if (threads <= 0) return 0;
	if (threads > 16) threads = 16;
	as = (struct h264_async *)calloc(1, sizeof(*as));
	if (!as) return -1;
	pthread_mutex_init(&as->mu, NULL);
	pthread_cond_init(&as->cv_work, NULL);
	pthread_cond_init(&as->cv_done, NULL);
	as->depth = threads + 2;
	{
		const char *e = getenv("M2DEC_AMD_PARSE_DEPTH"); /* tuning: pictures in flight past the oldest */
		if (e && atoi(e) > 0) as->depth = atoi(e) < AS_MAX - 2 ? atoi(e) : AS_MAX - 2;
	}
	for (int i = 0; i < 17; ++i) as->col_last[i] = -1;
	for (int i = 0; i < threads; ++i) {
		if (pthread_create(&as->th[i], NULL, worker, as) != 0) break;
		as->nth++;
	}
	if (!as->nth) {
		free(as);
		return -1;
	}
	d->as = as;
	return 0;
}

static h264_job_t *job_get(struct h264_async *as)
{
	h264_job_t *j;
	if (as->nfree) return as->free_jobs[--as->nfree];
	j = (h264_job_t *)calloc(1, sizeof(*j));
	if (!j) return NULL;
	j->w = (h264_dec_t *)malloc(sizeof(h264_dec_t));
	if (!j->w) {
		free(j);
		return NULL;
	}
	return j;
}

static void job_put(struct h264_async *as, h264_job_t *j)
{
	job_clear(j);
	if (as->nfree < AS_MAX) as->free_jobs[as->nfree++] = j;
	else job_free(j);
}

/* copy a finished job's records into the back end's arena and submit it (decode order) */
static int submit_oldest(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	h264_job_t *j = as->fifo[as->tail % AS_MAX];
	m2r_picture_t *dst;
	const m2r_picture_t *src = &j->pic;
	int n, err;
	pthread_mutex_lock(&as->mu);
	while (!j->done) pthread_cond_wait(&as->cv_done, &as->mu);
	as->tail++; /* workers scan [tail, head) under the mutex */
	pthread_mutex_unlock(&as->mu);
	for (int i = 0; i < 17; ++i)
		if (as->col_writer[i] == j) as->col_writer[i] = NULL;
	err = j->err;
	if (!err) {
		n = src->width_mbs * src->height_mbs;
		dst = d->backend.acquire(d->backend.self, src->width_mbs, src->height_mbs);
		if (!dst || dst->cap_slices < src->n_slices || dst->cap_inter < src->n_inter || dst->cap_coef < src->n_coef) {
			err = 1;
		} else {
			dst->slot = src->slot;
			dst->n_inter = src->n_inter;
			dst->n_coef = src->n_coef;
			dst->n_slices = src->n_slices;
			dst->n_intra = src->n_intra;
			dst->deblock = src->deblock;
			memcpy(dst->mb, src->mb, sizeof(m2r_mb_t) * (size_t)n);
			memcpy(dst->dbk, src->dbk, sizeof(m2r_deblock_t) * (size_t)n);
			memcpy(dst->slice, src->slice, sizeof(m2r_slice_t) * (size_t)src->n_slices);
			memcpy(dst->inter, src->inter, sizeof(m2r_inter_t) * (size_t)src->n_inter);
			memcpy(dst->coef, src->coef, sizeof(int16_t) * (size_t)src->n_coef);
			err = d->backend.submit(d->backend.self, dst) < 0;
		}
	}
	job_put(as, j);
	return err ? -1 : 0;
}

/* submit every dispatched job up to and including the newest one that writes `slot` (-1: all) */
int h264_async_drain(h264_dec_t *d, int slot)
{
	struct h264_async *as = d->as;
	long upto = -1;
	if (!as) return 0;
	for (long i = as->tail; i < as->head; ++i)
		if (slot < 0 || as->fifo[i % AS_MAX]->slot == slot) upto = i;
	while (as->tail <= upto)
		if (submit_oldest(d) < 0) return -1;
	return 0;
}

/* a slice header was parsed into d: open the picture's job if needed, append the slice */
int h264_async_add_slice(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	h264_job_t *j = as->cur;
	if (!j) {
		j = job_get(as);
		if (!j || job_arena(j, d->mb_w, d->mb_h) < 0) return -1;
		j->slot = d->curr_idx;
		j->pic.slot = d->curr_idx;
		j->col_store = d->curr_col;
		as->cur = j;
	}
	if (j->nsl == j->capsl) {
		int cap = j->capsl ? 2 * j->capsl : 4;
		h264_dec_t **s = (h264_dec_t **)realloc(j->snap, sizeof(*s) * (size_t)cap);
		uint8_t **r;
		if (!s) return -1;
		j->snap = s;
		r = (uint8_t **)realloc(j->rbsp, sizeof(*r) * (size_t)cap);
		if (!r) return -1;
		j->rbsp = r;
		j->capsl = cap;
	}
	{
		const size_t len = (size_t)(d->slice_rbsp_end - d->slice_rbsp);
		h264_dec_t *snap = (h264_dec_t *)malloc(sizeof(h264_dec_t));
		uint8_t *rb = (uint8_t *)calloc(1, len + 32);
		if (!snap || !rb) {
			free(snap);
			free(rb);
			return -1;
		}
		memcpy(snap, d, sizeof(*snap));
		memcpy(rb, d->slice_rbsp, len);
		j->snap[j->nsl] = snap;
		j->rbsp[j->nsl] = rb;
		j->nsl++;
	}
	return 0;
}

/* the picture being collected is complete (the next picture started, or end of data): marking /
 * DPB on this thread, slice data to the workers */
int h264_async_close(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	h264_job_t *j = as->cur;
	if (!j) return -1;
	as->cur = NULL;
	j->seq = as->seq++;
	/* a non-reference picture is never anyone's refs[1][0]: its co-located store is dead data */
	j->nonref = 1;
	for (int k = 0; k < j->nsl; ++k) j->nonref &= (j->snap[k]->sh.nal_ref_idc == 0);
	if (j->nonref && (size_t)j->snap[0]->n_mbs > j->priv_n) {
		free(j->priv_col);
		j->priv_col = (h264_colmb_t *)malloc(sizeof(h264_colmb_t) * (size_t)j->snap[0]->n_mbs);
		j->priv_n = j->priv_col ? (size_t)j->snap[0]->n_mbs : 0;
		if (!j->priv_col) return -1;
	}
	/* co-located stores this picture reads (B slices) -> wait for their writers */
	for (int k = 0; k < j->nsl; ++k) {
		const h264_dec_t *s = j->snap[k];
		if (s->sh.slice_type != 1) continue;
		const int c = s->refs[1][0].col;
		if (c < 0 || c >= 17) continue;
		h264_job_t *wj = as->col_writer[c];
		int seen = 0;
		for (int i = 0; i < j->ndeps; ++i) seen |= wj && (j->deps[i] == wj->seq);
		if (wj && !seen && j->ndeps < 8) j->deps[j->ndeps++] = wj->seq;
		if (as->col_last[c] < j->seq) as->col_last[c] = j->seq;
	}
	/* the store this picture writes: every earlier job that read or wrote it must have finished */
	if (!j->nonref) {
		const long last = as->col_last[j->col_store];
		pthread_mutex_lock(&as->mu);
		for (long i = as->tail; i < as->head; ++i) {
			h264_job_t *o = as->fifo[i % AS_MAX];
			if (o->seq <= last)
				while (!o->done) pthread_cond_wait(&as->cv_done, &as->mu);
		}
		pthread_mutex_unlock(&as->mu);
		as->col_last[j->col_store] = j->seq;
		as->col_writer[j->col_store] = j;
	}
	/* marking, store swap, DPB insertion (headers only) */
	d->pic = NULL;
	if (h264_picture_mark(d) < 0) return -1;
	/* dispatch */
	pthread_mutex_lock(&as->mu);
	as->fifo[as->head % AS_MAX] = j;
	as->head++;
	as->queue[as->qhead % AS_MAX] = j;
	as->qhead++;
	pthread_cond_signal(&as->cv_work);
	pthread_mutex_unlock(&as->mu);
	/* bounded depth; then hand over whatever is already finished, in order */
	while (as->head - as->tail > as->depth)
		if (submit_oldest(d) < 0) return -1;
	for (;;) {
		int ready;
		if (as->tail == as->head) break;
		pthread_mutex_lock(&as->mu);
		ready = as->fifo[as->tail % AS_MAX]->done;
		pthread_mutex_unlock(&as->mu);
		if (!ready) break;
		if (submit_oldest(d) < 0) return -1;
	}
	return 1;
}

void h264_async_stop(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	if (!as) return;
	pthread_mutex_lock(&as->mu);
	as->quit = 1;
	pthread_cond_broadcast(&as->cv_work);
	pthread_mutex_unlock(&as->mu);
	for (int i = 0; i < as->nth; ++i) pthread_join(as->th[i], NULL);
	for (long i = as->tail; i < as->head; ++i) job_free(as->fifo[i % AS_MAX]);
	job_free(as->cur);
	for (int i = 0; i < as->nfree; ++i) job_free(as->free_jobs[i]);
	pthread_mutex_destroy(&as->mu);
	pthread_cond_destroy(&as->cv_work);
	pthread_cond_destroy(&as->cv_done);
	free(as);
	d->as = NULL;
}
