/*
 * Large host copies spread over small process-wide thread crews (m2dec_par_memcpy).
 *
 * Two serial stages of the decode path move megabytes per picture on one thread: the submission copy of a
 * picture's records into the back end's pinned arena (h264_async.c copy_submit, ~4.5 MB at 1080p: the
 * submitting thread is the path's one serial stage, submissions go in decoding order) and the copy of a
 * finished frame from pinned staging into the caller's frame inside peek / get (runtime.hip be_sync,
 * 3.1 MB at 1080p, on the API thread, once per output frame: the API thread's loop bounds the stream's end,
 * profiles/r89_timeline.txt).  On one core each is ~0.07 / 0.25 ms; cut into 256 KB pieces that the crew
 * and the caller take from a shared counter they run at several cores' bandwidth.  Each stage has its own
 * crew (M2DEC_CREW_SUBMIT, M2DEC_CREW_SYNC) so the two never wait for each other; a second caller of the
 * same crew (another decoder context) copies on its own thread.  M2DEC_AMD_COPY_CREW = threads per crew
 * (default 3, 0: plain memcpy).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "h264_dec.h"

#define PAR_CREW 3
#define PAR_MIN (512 << 10)
#define PAR_PIECE (256 << 10)

typedef struct {
	pthread_mutex_t mu, one;
	pthread_cond_t cv_go, cv_done;
	uint8_t *dst[4];
	const uint8_t *src[4];
	size_t off[5];          /* the copies of one call: their start offsets in the joint range */
	int ncopies;
	size_t total;
	long gen;               /* a new call */
	int busy;               /* crew members still in the current call */
	size_t next;            /* next piece's offset (atomic) */
	int started;
} par_crew_t;

static par_crew_t g_crews[M2DEC_CREWS];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void par_pieces(par_crew_t *c)
{
	for (;;) {
		const size_t o = __atomic_fetch_add(&c->next, (size_t)PAR_PIECE, __ATOMIC_RELAXED);
		if (o >= c->total) return;
		const size_t end = o + PAR_PIECE < c->total ? o + PAR_PIECE : c->total;
		for (int k = 0; k < c->ncopies; ++k) { /* a piece may span the end of one copy and the start of the next */
			const size_t a = o > c->off[k] ? o : c->off[k], b = end < c->off[k + 1] ? end : c->off[k + 1];
			if (a < b) memcpy(c->dst[k] + (a - c->off[k]), c->src[k] + (a - c->off[k]), b - a);
		}
	}
}

static void *crew_main(void *arg)
{
	par_crew_t *c = (par_crew_t *)arg;
	long seen = 0;
	pthread_setname_np(pthread_self(), "m2d-copy");
	pthread_mutex_lock(&c->mu);
	for (;;) {
		while (c->gen == seen) pthread_cond_wait(&c->cv_go, &c->mu);
		seen = c->gen;
		pthread_mutex_unlock(&c->mu);
		m2d_place_self(); /* (numa.c) */
		par_pieces(c);
		pthread_mutex_lock(&c->mu);
		if (--c->busy == 0) pthread_cond_signal(&c->cv_done);
	}
	return NULL;
}

static void crews_start(void)
{
	const char *e = getenv("M2DEC_AMD_COPY_CREW");
	/* (a share below 8 CPUs: one helper, below 4: none; cpushare.c) */
	const int n = e ? atoi(e) : (m2d_cpu_share() >= 8 ? PAR_CREW : (m2d_cpu_share() >= 4 ? 1 : 0));
	for (int w = 0; w < M2DEC_CREWS; ++w) {
		par_crew_t *c = &g_crews[w];
		pthread_mutex_init(&c->mu, NULL);
		pthread_mutex_init(&c->one, NULL);
		pthread_cond_init(&c->cv_go, NULL);
		pthread_cond_init(&c->cv_done, NULL);
		for (int i = 0; i < n && i < 8; ++i) {
			pthread_t t;
			if (pthread_create(&t, NULL, crew_main, c) != 0) break;
			pthread_detach(t);
			c->started++;
		}
	}
}

void m2dec_par_memcpy(int crew, int n, void *const *dst, const void *const *src, const size_t *len)
{
	size_t total = 0;
	for (int k = 0; k < n; ++k) total += len[k];
	pthread_once(&g_once, crews_start);
	par_crew_t *c = &g_crews[crew < 0 || crew >= M2DEC_CREWS ? 0 : crew];
	if (total < PAR_MIN || !c->started || pthread_mutex_trylock(&c->one) != 0) {
		for (int k = 0; k < n; ++k)
			if (len[k]) memcpy(dst[k], src[k], len[k]);
		return;
	}
	pthread_mutex_lock(&c->mu);
	c->ncopies = n;
	c->off[0] = 0;
	for (int k = 0; k < n; ++k) {
		c->dst[k] = (uint8_t *)dst[k];
		c->src[k] = (const uint8_t *)src[k];
		c->off[k + 1] = c->off[k] + len[k];
	}
	c->total = total;
	c->next = 0;
	c->busy = c->started;
	c->gen++;
	pthread_cond_broadcast(&c->cv_go);
	pthread_mutex_unlock(&c->mu);
	par_pieces(c);
	pthread_mutex_lock(&c->mu);
	while (c->busy) pthread_cond_wait(&c->cv_done, &c->mu);
	pthread_mutex_unlock(&c->mu);
	pthread_mutex_unlock(&c->one);
}
