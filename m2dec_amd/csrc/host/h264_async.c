/*
 * Parse-ahead pipeline: the slice data of many pictures parsed at once on worker threads, behind
 * the unchanged h264d_func API ("pipelining parse n+1 with GPU recon n").
 *
 * Two decoder contexts run the same NAL loop (h264_decode_loop) on the caller's thread:
 *
 *   the lookahead context L   reads the stream, parses SPS / PPS / slice headers, does the reference
 *                             marking and the co-located store swap, and turns every picture into a
 *                             job (its slice data to be parsed on a worker).  It names pictures by
 *                             virtual frame ids, not frame slots, so it does not depend on the
 *                             caller's output calls and can run up to `depth` pictures ahead of the
 *                             API.  Every NAL it has finished goes into a queue for A.
 *   the API context A         consumes that NAL queue: headers again, the header callback
 *                             (set_frames), frame-slot LRU (find_empty_frame, h264.cpp:924-962),
 *                             marking, DPB insertion and output bumping — exactly the state the
 *                             reference's synchronous decoder has at each decode_picture / peek / get
 *                             call, whatever order the caller uses them in.  At each picture it
 *                             closes, A records the virtual-id -> slot translation of that picture's
 *                             job; the job's records are translated when they are submitted.
 *
 * Before this split the API context also created the jobs, so parse-ahead could never get further
 * ahead than the DPB output lag (peek/get must wait for the bumped picture): 3-4 pictures in flight.
 *
 * The parser compares frame_idx values only for equality (bS motion tests, the co-located reference
 * map of temporal direct, the record ref slots), so virtual ids (unique among live pictures, reused
 * as late as possible) give the same records as frame slots.
 *
 * A job is one picture: for each of its slices a copy of L right after that slice's header (60 KB)
 * and a copy of its RBSP; the worker runs the slices in order on a private context, carrying the
 * few fields the slice parser accumulates across slices, into a private MB-info array and a private
 * record arena.
 *
 * Cross-picture dependencies of the slice data: a B slice reads the co-located store of its
 * refs[1][0] (spatial and temporal direct, h264.cpp:9777 / 9848), written by an earlier picture's
 * parse -> the job waits for that writer job.  A store is recycled by the marking swap
 * (h264.cpp:10970-10984) -> a job that writes it is dispatched only after every earlier job that
 * read or wrote it has finished.
 *
 * Picture boundaries: the synchronous parser knows a picture is complete when its last MB is
 * parsed; here the header-level loop sees only headers, so a picture is closed when the next
 * picture's first slice arrives (first_mb not above the previous slice's, the reference's own
 * test, h264.cpp:1427-1430), at a SEI / SPS / PPS / AUD NAL, or at the end of the data.
 * decode_picture still returns 1 once per picture and the DPB output order is unchanged; a frame
 * is handed out (peek / get) only after its picture was parsed and submitted, and sync_frame has
 * waited for its reconstruction.
 *
 * The stream is read ahead of decode_picture by up to `depth` pictures, so stream_pos() points
 * past the picture decode_picture last returned.
 *
 * Decode ahead (back ends with bind, m2d_recon.h): a parsed picture is submitted at once, named by
 * its virtual id (the back end keeps one picture buffer per id), instead of waiting for the API
 * context to give it a frame slot.  Without it the GPU could never run ahead of the caller's output
 * calls: a B picture is bumped out right after it is decoded, and sync_frame on it drained the
 * device before the next picture was even submitted (one picture in flight).  The API context's
 * close binds the buffer to the slot; a picture waits (is submitted in API order) when the previous
 * picture of its virtual id is not bound yet, or when an SPS the API context has not run the header
 * callback for lies before it.
 */
#define _GNU_SOURCE /* pthread_setname_np */
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <string.h>
#include <time.h>
#include "h264_dec.h"

#define AS_MAX 64 /* jobs dispatched and not yet submitted */

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct h264_job {
	int nsl, capsl;
	int nkeep;                /* snap / rbsp entries allocated (kept across pictures: no malloc, page
	                             faults or heap trims on the lookahead's per-picture path) */
	h264_dec_t **snap;        /* [nsl] lookahead context right after each slice header */
	uint8_t **rbsp;           /* [nsl] slice RBSP copies (32 zero bytes of padding) */
	size_t *rbsp_cap;         /* [nkeep] their capacities */
	h264_mbinfo_t *mbi;       /* private neighbour state */
	size_t mbi_n;
	m2r_picture_t pic;        /* private record arena (frame ids are virtual until submission) */
	uint8_t *arena;           /* laid out as m2r_arena_layout() */
	size_t arena_size;
	int arena_pinned;         /* the arena is pinned host memory (m2dec_amd_pinned_alloc) */
	int ext_busy;             /* submitted as M2R_PIC_EXTERNAL: the back end may still read the arena */
	int vid;                  /* virtual frame id of the picture (lookahead context) */
	int slot;                 /* frame slot (API context; -1 until A closed the picture) */
	int poc;                  /* consistency check between the two contexts */
	int8_t map[64];           /* virtual id -> frame slot, as of the API context's close */
	long sps_nal;             /* NAL index of the last SPS the lookahead read before this picture */
	int submitted, bound;     /* records handed to the back end / its buffer bound to `slot` */
	int sub_err;              /* its submission failed (decode ahead: nothing to bind) */
	int col_store;
	long col_dep;             /* seq of the job writing the co-located store this (single-slice B) picture
	                             reads, if it may start while that one is still parsing (-1: no) */
	int col_early;            /* started so: direct prediction waits for the writer's rows (job_run) */
	uint64_t refmask;         /* virtual ids any slice of the picture may read (every in-use entry of its
	                             reference lists, known at dispatch: pipe_drive's early submission) */
	int nonref;               /* no slice has nal_ref_idc: its co-located store is never read ... */
	h264_colmb_t *priv_col;   /* ... so it writes this private one (no ordering against other jobs) */
	size_t priv_n;
	long deps[8];             /* seq of the jobs whose parse must finish first (jobs are recycled:
	                             never keep a pointer past its submission) */
	/* slice-parallel parse (job_run_par): per slice a private context and a private view of the
	 * record arena; slices are taken from sl_next by the job's worker and idle workers */
	h264_dec_t **sw;
	m2r_picture_t *spic;
	int *sret;
	int capsw;
	int sl_next, sl_done;     /* guarded by the pipeline mutex */
	int ndeps;
	long seq;
	int taken, done, err;     /* guarded by the pipeline mutex */
	h264_dec_t *w;            /* worker context */
} h264_job_t;

typedef struct {
	uint8_t *buf;
	size_t cap, len;
} nal_ent_t;

struct h264_async {
	pthread_mutex_t *mu;      /* the parse pool's mutex (g_parse.mu): it guards every pipeline's job state */
	pthread_cond_t cv_done;
	struct h264_async *pnext; /* the pool's list of pipelines */
	h264_dec_t *api;          /* the API context (library memory: the caller's context is only a handle) */
	int nth;                  /* pool workers this pipeline may occupy at once */
	int running;              /* pool workers inside one of its jobs or slices */
	int quit, depth;
	h264_job_t *fifo[AS_MAX]; /* dispatched, not yet submitted: [tail, head); job seq s at fifo[s % AS_MAX] */
	long head, tail;          /* tail: oldest job not retired (submitted, and bound when decoding ahead) */
	long sub;                 /* next job to submit: [tail, sub) submitted */
	long bnd;                 /* decode ahead: next job to bind: [tail, bnd) bound */
	int ahead;                /* decode ahead: the back end has bind (M2R_PIC_VIRTUAL submissions) */
	int ext;                  /* decode ahead, and the back end takes M2R_PIC_EXTERNAL pictures: job arenas
	                             are pinned and uploaded from where the workers wrote them (no record copy) */
	int driving;              /* decode ahead: a thread is inside pipe_drive (back-end calls are serial) */
	int held;                 /* decode ahead: submitted since the last back-end flush */
	int sub_err;
	int ahead_all;            /* M2DEC_AMD_AHEAD_ALL (tests): the API context closes a picture only after the
	                             pipe_drive submitted it, so every picture goes ahead whatever the thread timing */
	long la_sps_nal;          /* NAL index of the last SPS the lookahead context read (-1: none) */
	long api_sps_nal;         /* NAL index of the last SPS whose header callback the API context ran */
	h264_job_t *queue[AS_MAX]; /* dispatched; [qtail, qhead) holds every job not yet taken */
	long qhead, qtail;
	h264_job_t *cur;          /* the picture the lookahead context is collecting */
	h264_job_t *free_jobs[AS_MAX];
	int nfree;
	long seq;                 /* jobs dispatched by the lookahead context */
	long a_seq;               /* pictures closed by the API context: jobs [tail, a_seq) may be submitted */
	long col_last[17];        /* seq of the last dispatched job that reads or writes store i */
	long col_writer[17];      /* seq of the last dispatched job writing store i (-1: none) */
	/* lookahead context and its NAL hand-over queue (ring, [nq_tail, nq_head)) */
	h264_dec_t *la;
	int la_done, la_err;
	nal_ent_t *nq;
	long nq_head, nq_tail, nq_cap;
	int8_t vmap[64];          /* API context: virtual id -> frame slot */
	/* co-located store buffers taken out of the lookahead's stores (h264_colpic_t.mb) while jobs
	 * still used them: free once every job dispatched before `unmap_seq` was submitted */
	struct {
		h264_colmb_t *mb;
		long unmap_seq;
	} spare[64];
	int nspare;
	size_t col_n;             /* MBs per store buffer */
	/* M2DEC_AMD_ASYNC_STATS: where the caller's thread spends its time (seconds) */
	int stats;
	double t0, t_col_wait, t_done_wait, t_copy, t_submit, t_slice, t_parse, t_la;
	/* pictures whose slices are being parsed in parallel (slices left to take: sl_next < nsl) */
	h264_job_t *par[16];
	int npar;
	int slice_par;            /* M2DEC_AMD_SLICE_PAR (default 1): slices of a picture on several workers */
	long n_par, n_par_fallback; /* pictures parsed slice-parallel / re-parsed sequentially after a try */
	long n_early;             /* reference pictures submitted ahead of older jobs (early_ok) */
};

/* The parse pool: one set of worker threads per process, shared by every decoder's pipeline (a
 * decoder context owns no thread, so a context the caller drops leaves none behind, and N streams
 * decoded at once do not oversubscribe the host with N private pools).  Workers take the oldest
 * ready job (or a slice of a picture parsed slice-parallel) of any pipeline, round robin over the
 * pipelines, each pipeline capped at its own `nth` workers at a time.  Threads are created on
 * demand (up to the largest `nth` asked for) and live for the process. */
#define POOL_MAX 64
static struct {
	pthread_mutex_t mu;
	pthread_cond_t cv_work;
	pthread_t th[POOL_MAX];
	int nth;
	struct h264_async *pipes; /* registered pipelines */
	struct h264_async *rr;    /* the pipeline to look at first next time */
} g_parse = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, {0}, 0, NULL, NULL};

static void pipe_drive(struct h264_async *as);
static int g_col_pipe = 1; /* M2DEC_AMD_COL_PIPE: co-located row pipelining (deps_ready) */
static int g_early = 1;    /* M2DEC_AMD_EARLY: parsed reference pictures submitted ahead of older B pictures */
static int g_nonref_delay_us; /* M2DEC_AMD_NONREF_DELAY_US (tests): non-reference pictures finish late */
static int g_col_delay_us; /* M2DEC_AMD_COL_PIPE_DELAY_US (tests: anchors slowed down, readers start early) */
static int job_ext_idle(struct h264_async *as, h264_job_t *j, int wait);

/* page-locked bytes held by job arenas of the process (in use and pooled): M2DEC_AMD_ASYNC_STATS */
static long long g_pinned_bytes;

static void arena_free(h264_job_t *j)
{
	if (j->arena_pinned) {
		m2dec_amd_pinned_free(j->arena);
		__atomic_fetch_sub(&g_pinned_bytes, (long long)j->arena_size, __ATOMIC_RELAXED);
	} else {
		free(j->arena);
	}
	j->arena = NULL;
	j->arena_size = 0;
	j->arena_pinned = 0;
}

/* the job's record arena for a wm x hm picture (pinned when the pipeline uploads from it: `pinned`) */
static int job_arena(h264_job_t *j, int wm, int hm, int pinned)
{
	const int n = wm * hm;
	const m2r_arena_layout_t l = m2r_arena_layout(n);
	if (l.size > j->arena_size || (pinned && !j->arena_pinned)) {
		arena_free(j);
		if (pinned && (j->arena = (uint8_t *)m2dec_amd_pinned_alloc(l.size))) {
			j->arena_pinned = 1;
			__atomic_fetch_add(&g_pinned_bytes, (long long)l.size, __ATOMIC_RELAXED);
		} else {
			j->arena = (uint8_t *)malloc(l.size);
		}
		if (!j->arena) return -1;
		j->arena_size = l.size;
	}
	uint8_t *p = j->arena;
	m2r_picture_t *pic = &j->pic;
	memset(pic, 0, sizeof(*pic));
	pic->width_mbs = wm;
	pic->height_mbs = hm;
	pic->mb = (m2r_mb_t *)(p + l.mb);
	pic->dbk = (m2r_deblock_t *)(p + l.dbk);
	pic->slice = (m2r_slice_t *)(p + l.slice);
	pic->inter = (m2r_inter_t *)(p + l.inter);
	pic->coef = (int16_t *)(p + l.coef);
	pic->cap_slices = M2R_ARENA_SLICES;
	pic->cap_inter = n;
	pic->cap_coef = n * M2R_COEF_PER_MB;
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
	j->nsl = 0;
	j->ndeps = 0;
	j->taken = 0;
	j->done = 0;
	j->err = 0;
	j->slot = -1;
	j->submitted = 0;
	j->bound = 0;
	j->sub_err = 0;
}

static void job_free(h264_job_t *j)
{
	if (!j) return;
	job_clear(j);
	for (int i = 0; i < j->nkeep; ++i) {
		free(j->snap[i]);
		free(j->rbsp[i]);
	}
	free(j->snap);
	free(j->rbsp);
	free(j->rbsp_cap);
	free(j->mbi);
	free(j->priv_col);
	for (int i = 0; i < j->capsw; ++i) free(j->sw[i]);
	free(j->sw);
	free(j->spic);
	free(j->sret);
	arena_free(j);
	free(j->w);
	free(j);
}

/* Jobs (each with a record arena of ~1 KB per MB) outlive a pipeline: a context's jobs go back to a
 * process-wide pool when it stops or reaches the end of its stream, and the next context takes them —
 * no allocation or page faults while decoding, no frees when a context goes.  Mutex: g_parse.mu. */
#define JOB_POOL_MAX 320 /* r101: 96 freed most of eight concurrent streams' jobs at every stream end, and the
                            * next streams pinned their arenas again (hipHostMalloc, ~2 ms each, on the
                            * lookahead's thread): 8 streams 1000 fps, 1490 with unpinned arenas */
static h264_job_t *g_jobs[JOB_POOL_MAX];
static long g_jobs_new; /* jobs created (each pins its arena on first use): M2DEC_AMD_ASYNC_STATS */
static int g_njobs;
static long long g_pool_pinned; /* page-locked bytes of the pooled jobs' arenas */
static h264_job_t *pool_take(int i);

/* the pool is bounded by the page-locked bytes it keeps, not only by its job count: at ~8.5 MB per
 * 1080p job and ~27 MB per 4K job, 320 pooled jobs would keep up to 8.6 GB locked.  The bound is what the
 * process's pipelines had in flight at their peak (so the next streams of the same workload find every job
 * they need pinned already: r5, a fixed 2 GB under the eight concurrent 1080p streams' 2.8 GB peak re-pinned
 * ~90 jobs per pass, 8 streams 1156 fps vs 1812 before the cap), at least 2 GB, at most
 * M2DEC_AMD_POOL_PINNED_MAX_MB (default 8192).  M2DEC_AMD_POOL_PINNED_MB fixes it instead. */
static long long g_inuse_peak; /* page-locked bytes of jobs outside the pool, most seen (g_parse.mu) */
static long long pool_pinned_cap(void)
{
	static long long fixed = -2, hard = -1;
	if (fixed == -2) {
		const char *e = getenv("M2DEC_AMD_POOL_PINNED_MB");
		fixed = e && *e ? atoll(e) << 20 : -1;
		const char *h = getenv("M2DEC_AMD_POOL_PINNED_MAX_MB");
		hard = (h && *h ? atoll(h) : 8192) << 20;
	}
	if (fixed >= 0) return fixed;
	const long long base = (long long)2048 << 20;
	const long long want = g_inuse_peak > base ? g_inuse_peak : base;
	return want < hard ? want : hard;
}

static void job_release(h264_job_t *j) /* (mutex held; the back end no longer reads its arena) */
{
	if (!j) return;
	job_clear(j);
	const long long pin = j->arena_pinned ? (long long)j->arena_size : 0;
	{
		const long long inuse = __atomic_load_n(&g_pinned_bytes, __ATOMIC_RELAXED) - g_pool_pinned;
		if (inuse > g_inuse_peak) g_inuse_peak = inuse;
	}
	if (pin > pool_pinned_cap()) {
		job_free(j);
		return;
	}
	/* the pool is ordered oldest first: over the count or the pinned bytes, the oldest pooled jobs go (a 4K
	 * stream after 1080p ones keeps its own jobs, not the 1080p ones it will not take) */
	while (g_njobs && (g_njobs >= JOB_POOL_MAX || g_pool_pinned + pin > pool_pinned_cap())) job_free(pool_take(0));
	g_jobs[g_njobs++] = j;
	g_pool_pinned += pin;
}

static h264_job_t *pool_take(int i) /* (mutex held; keeps the pool's order) */
{
	h264_job_t *j = g_jobs[i];
	memmove(&g_jobs[i], &g_jobs[i + 1], sizeof(g_jobs[0]) * (size_t)(g_njobs - 1 - i));
	g_njobs--;
	if (j->arena_pinned) g_pool_pinned -= (long long)j->arena_size;
	return j;
}

/* Free every pooled job (their page-locked arenas included): m2dec_amd_release_pools().  Jobs in use by live
 * pipelines are untouched. */
void h264_async_pool_release(void)
{
	pthread_mutex_lock(&g_parse.mu);
	while (g_njobs) job_free(pool_take(g_njobs - 1));
	pthread_mutex_unlock(&g_parse.mu);
}

long long h264_async_pinned_bytes(long long *pooled)
{
	if (pooled) {
		pthread_mutex_lock(&g_parse.mu);
		*pooled = g_pool_pinned;
		pthread_mutex_unlock(&g_parse.mu);
	}
	return __atomic_load_n(&g_pinned_bytes, __ATOMIC_RELAXED);
}

/* ---------------------------------------------------------------- worker */
/* the reference summary of a parsed picture's motion records (M2R_PIC_REFS), formed by the worker while
 * they are in its cache */
static void pic_refs(m2r_picture_t *p)
{
	uint64_t m = 0;
	int nb = 0;
	for (int i = 0; i < p->n_inter; ++i) {
		const int8_t *s = &p->inter[i].slot[0][0];
		for (int k = 0; k < 8; ++k) {
			nb += s[k] >= 0;
			m |= (uint64_t)(s[k] >= 0) << (s[k] & 63);
		}
	}
	p->ref_blocks = nb;
	p->ref_slots = m;
	p->flags |= M2R_PIC_REFS;
}

static void job_run_slices(h264_job_t *j);

/* a picture's slices in order on this worker, with the co-located row pipelining around them */
static void job_run(h264_job_t *j)
{
	h264_dec_t *w = j->w;
	const h264_dec_t *s0 = j->snap[0];
	const int n = s0->n_mbs;
	int *pub = NULL;
	const int *sub = NULL;
	if (j->nsl == 1 && !j->nonref) pub = h264_col_progress(s0->colpic[s0->curr_col].mb, n);
	if (j->col_early) sub = h264_col_progress(s0->colpic[s0->refs[1][0].col].mb, n);
	w->col_pub = pub;
	w->col_sub = sub;
	w->col_pub_delay_us = g_col_delay_us;
	job_run_slices(j);
	if (pub) __atomic_store_n(pub, j->err ? -1 : H264_COL_FINAL(n), __ATOMIC_RELEASE);
	if (sub) { /* the writer's outcome decides this picture's (as a finished dependency's error would) */
		int v, spins = 0;
		while ((v = __atomic_load_n(sub, __ATOMIC_ACQUIRE)) >= 0 && v != H264_COL_FINAL(n))
			if (++spins < 64) __builtin_ia32_pause();
			else sched_yield();
		if (v < 0 || w->col_sub_fail) j->err = 1;
	}
	j->col_early = 0;
}

static void job_run_slices(h264_job_t *j)
{
	h264_dec_t *w = j->w;
	int mbs = 0, coded = 0, slice_num = 0, slice_rec = 0, last_firstline = 0, ret = 0;
	w->par_first_mb = 0;
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
		{
			int *pub = w->col_pub;
			const int *sub = w->col_sub;
			const int ok = k ? w->col_sub_ok : 0, fail = k ? w->col_sub_fail : 0, delay = w->col_pub_delay_us;
			memcpy(w, s, sizeof(*w));
			w->col_pub = pub; /* (job_run's, kept across the slices) */
			w->col_pub_delay_us = delay;
			w->col_sub = sub;
			w->col_sub_ok = ok;
			w->col_sub_fail = fail;
		}
		w->par_first_mb = 0;
		w->mbi = j->mbi;
		w->pic = &j->pic;
		if (j->nonref) w->colpic[w->curr_col].mb = j->priv_col;
		w->mbs_decoded = mbs;
		w->mbs_coded = coded;
		w->slice_num = slice_num;
		w->slice_rec = slice_rec;
		w->last_firstline = last_firstline;
		memcpy(w->slice_idc, idc, (size_t)slice_num);
		memcpy(w->slice_alpha, alpha, (size_t)slice_num);
		memcpy(w->slice_beta, beta, (size_t)slice_num);
		/* the bit reader and RBSP bounds pointed into the lookahead's NAL buffer: rebase onto the copy */
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
		coded = w->mbs_coded;
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

/* Slice-parallel parse of one picture.  The slices of a picture are
 * independent for the slice-data parse: intra / motion prediction and the CABAC / CAVLC contexts never
 * read an MB of another slice (availability stops at the slice), so slice k runs on its own context
 * with its own MB range, writing its records into the picture arena from MB first_mb(k) on (coefficients
 * from first_mb(k) * 416, inter records from first_mb(k): the arena holds the worst case of every MB)
 * and its slice record at index k.  Afterwards: the records are packed in slice order (offsets in the
 * MB records moved with them), the MB-edge bS toward an earlier slice (skipped during the parse,
 * par_first_mb) is computed, and the per-slice deblock parameters are gathered for
 * h264_picture_resolve_deblock.  The records equal the sequential parse's up to where the
 * coefficients / inter records sit.  A picture whose slices do not tile it exactly in order (the
 * sequential parse's picture-complete test) is parsed again sequentially.  Returns 0, or -1 when
 * job_run must take over. */
static void slice_run(h264_job_t *j, int k)
{
	const h264_dec_t *s = j->snap[k];
	h264_dec_t *w = j->sw[k];
	m2r_picture_t *pk = &j->spic[k];
	const ptrdiff_t off = j->rbsp[k] - s->slice_rbsp;
	const int first = s->sh.first_mb;
	*pk = j->pic;
	pk->n_slices = k;
	pk->n_inter = first;
	pk->n_coef = first * 416;
	pk->n_intra = 0;
	memcpy(w, s, sizeof(*w));
	w->col_pub = NULL; /* (multi-slice pictures neither publish nor start early: job_run) */
	w->col_sub = NULL;
	w->par_first_mb = first;
	w->mbi = j->mbi;
	w->pic = pk;
	if (j->nonref) w->colpic[w->curr_col].mb = j->priv_col;
	w->mbs_decoded = 0;
	w->slice_num = k;
	w->bs.p += off;
	w->bs.end += off;
	w->slice_rbsp += off;
	w->slice_rbsp_end += off;
	j->sret[k] = h264_slice_data(w);
}

static int job_run_par(struct h264_async *as, h264_job_t *j)
{
	const int nsl = j->nsl, n = j->snap[0]->n_mbs;
	if (j->pic.n_slices || j->pic.n_inter || j->pic.n_coef || j->pic.n_intra || nsl > 16) return -1;
	for (int k = 1; k < nsl; ++k)
		if (j->snap[k]->sh.first_mb <= j->snap[k - 1]->sh.first_mb) return -1;
	if (j->snap[0]->sh.first_mb != 0 || j->snap[nsl - 1]->sh.first_mb >= n) return -1;
	if (nsl > j->capsw) {
		h264_dec_t **sw = (h264_dec_t **)realloc(j->sw, sizeof(*sw) * (size_t)nsl);
		if (!sw) return -1;
		j->sw = sw;
		for (int k = j->capsw; k < nsl; ++k) j->sw[k] = NULL;
		j->capsw = nsl;
		free(j->spic);
		free(j->sret);
		j->spic = (m2r_picture_t *)malloc(sizeof(m2r_picture_t) * (size_t)nsl);
		j->sret = (int *)malloc(sizeof(int) * (size_t)nsl);
		if (!j->spic || !j->sret) { /* (keep sw[] and capsw consistent for job_free) */
			free(j->spic);
			free(j->sret);
			j->spic = NULL;
			j->sret = NULL;
			for (int k = 0; k < j->capsw; ++k) free(j->sw[k]);
			free(j->sw);
			j->sw = NULL;
			j->capsw = 0;
			return -1;
		}
	}
	for (int k = 0; k < nsl; ++k) {
		if (!j->sw[k]) j->sw[k] = (h264_dec_t *)malloc(sizeof(h264_dec_t));
		if (!j->sw[k]) return -1;
	}
	for (int i = 0; i < n; ++i) {
		j->mbi[i].type = -1;
		j->mbi[i].slice = -1;
	}
	/* offer the slices to idle workers; this worker takes them too, and waits for the rest */
	pthread_mutex_lock(as->mu);
	if (as->npar >= 16) {
		pthread_mutex_unlock(as->mu);
		return -1;
	}
	j->sl_next = 0;
	j->sl_done = 0;
	as->par[as->npar++] = j;
	pthread_cond_broadcast(&g_parse.cv_work);
	while (j->sl_next < nsl) {
		const int k = j->sl_next++;
		if (j->sl_next == nsl)
			for (int i = 0; i < as->npar; ++i)
				if (as->par[i] == j) as->par[i] = as->par[--as->npar];
		pthread_mutex_unlock(as->mu);
		slice_run(j, k);
		pthread_mutex_lock(as->mu);
		j->sl_done++;
	}
	{
		const double tw = now_s();
		const int waits = j->sl_done < nsl;
		if (waits) m2d_cpu_primary(-1); /* (not busy while the helpers finish: cpushare.c) */
		while (j->sl_done < nsl) pthread_cond_wait(&as->cv_done, as->mu);
		as->t_parse -= now_s() - tw; /* the worker's job time counts parse work only */
		pthread_mutex_unlock(as->mu);
		if (waits) m2d_cpu_primary(1);
	}

	/* every slice parsed exactly its MB range, in order, the last one ending the picture */
	for (int k = 0; k < nsl; ++k) {
		const int first = j->snap[k]->sh.first_mb, end = k + 1 < nsl ? j->snap[k + 1]->sh.first_mb : n;
		if (j->sret[k] != (k + 1 == nsl ? 1 : 0) || j->sw[k]->mbs_decoded != end - first) return -1;
	}
	/* pack the coefficient pool and the inter records in slice order */
	{
		m2r_picture_t *pic = &j->pic;
		int ncoef = 0, ninter = 0, nintra = 0;
		for (int k = 0; k < nsl; ++k) {
			const m2r_picture_t *pk = &j->spic[k];
			const int first = j->snap[k]->sh.first_mb, end = k + 1 < nsl ? j->snap[k + 1]->sh.first_mb : n;
			const int cb = first * 416, ib = first;
			const int nc = pk->n_coef - cb, ni = pk->n_inter - ib;
			if (ncoef != cb) memmove(pic->coef + ncoef, pic->coef + cb, sizeof(int16_t) * (size_t)nc);
			if (ninter != ib) memmove(pic->inter + ninter, pic->inter + ib, sizeof(m2r_inter_t) * (size_t)ni);
			for (int a = first; a < end; ++a) {
				m2r_mb_t *r = &pic->mb[a];
				r->coef -= (uint32_t)(cb - ncoef);
				if (r->kind == M2R_MB_INTER) r->inter -= (uint32_t)(ib - ninter);
			}
			ncoef += nc;
			ninter += ni;
			nintra += pk->n_intra;
		}
		pic->n_coef = ncoef;
		pic->n_inter = ninter;
		pic->n_intra = nintra;
		pic->n_slices = nsl;
	}
	/* the picture-level context: the last slice's, with every slice's deblock parameters */
	{
		h264_dec_t *w = j->sw[nsl - 1];
		w->pic = &j->pic;
		w->par_first_mb = 0;
		for (int k = 0; k < nsl - 1; ++k) {
			w->slice_idc[k] = j->sw[k]->slice_idc[k];
			w->slice_alpha[k] = j->sw[k]->slice_alpha[k];
			w->slice_beta[k] = j->sw[k]->slice_beta[k];
		}
		w->slice_num = nsl;
		w->mbs_decoded = n;
		for (int k = 1; k < nsl; ++k) {
			const int first = j->snap[k]->sh.first_mb, mw = w->mb_w;
			/* MBs with the left or top neighbour in an earlier slice: the MB row from the slice's first MB */
			for (int a = first; a < n && a < first + mw; ++a)
				if (((a % mw) != 0 && a - 1 < first) || (a >= mw && a - mw < first)) h264_fix_bs(w, a);
		}
		h264_picture_resolve_deblock(w);
	}
	return 0;
}

/* 1: every job j waits for has finished parsing (0: not yet); a dependency no longer in the fifo was
 * submitted, hence finished.  *err collects their errors.  Caller holds the mutex. */
/* Co-located row pipelining.  A B picture reads the co-located motion of its refPicList1[0] only at
 * its own MB position (direct prediction), and a single-slice picture stores its co-located motion in
 * raster order.  So the B picture may start as soon as the picture writing that store has started: the
 * writer publishes the MBs stored so far in the store buffer's progress word (store_col), and direct
 * prediction of MB addr waits until that word passes addr (col_wait).  Without it each B picture waited
 * for the whole parse of its anchor: the pool idled at the start of the stream (only I / P pictures
 * runnable) and at its end (the last B pictures behind the last anchors), ~7 of 26 ms in r99.  The
 * writer is running whenever a reader waits on it (it was taken first, and it waits on nothing itself
 * or, a B reference, only on running writers in turn), so waits end.  M2DEC_AMD_COL_PIPE=0: off. */

static int deps_ready(const struct h264_async *as, const h264_job_t *j, int *err, int *early)
{
	*early = 0;
	for (int i = 0; i < j->ndeps; ++i) {
		const long s = j->deps[i];
		if (s < as->tail || s >= as->head) continue;
		const h264_job_t *o = as->fifo[s % AS_MAX];
		if (!o->done) {
			if (g_col_pipe && s == j->col_dep && o->taken && o->nsl == 1 && !o->nonref) {
				*early = 1;
				continue;
			}
			return 0;
		}
		*err |= o->err;
	}
	return 1;
}

static int g_parse_prio = 20; /* M2DEC_AMD_PARSE_PRIO (read when the pool starts): pick_job's window */

/* A ready job (or a slice to help with) of pipeline `as`, marked taken; NULL if none.  Mutex held. */
static h264_job_t *pick_job(struct h264_async *as, h264_job_t **slice_of, int *slice_k, int *dep_err)
{
	*slice_of = NULL;
	/* a slice of a picture parsed slice-parallel first: that picture is already under way */
	if (as->npar) {
		h264_job_t *pj = as->par[0];
		*slice_k = pj->sl_next++;
		if (pj->sl_next == pj->nsl) as->par[0] = as->par[--as->npar];
		*slice_of = pj;
		return NULL;
	}
	/* a taken job leaves the queue at once (its entry is cleared): once finished and retired it is
	 * recycled for a later picture, and a stale entry would hand that one out half built */
	while (as->qtail < as->qhead && !as->queue[as->qtail % AS_MAX]) as->qtail++;
	/* Reference pictures within g_parse_prio (20) jobs of the oldest queued one first (the oldest such), then
	 * the oldest ready job.  The oldest-first order alone feeds the in-order submission evenly but starts
	 * the stream's last anchors late, and the B pictures waiting for them leave workers idle for ~8 ms
	 * (profiles/r96_timeline.txt); anchors first without a bound (a window of 64) parse the B pictures,
	 * and with them the submission, late (profiles/r86_timeline.txt).  An anchor parsed about one round
	 * of the pool ahead of the oldest job is done when its B pictures come up (tools/parse_sched_sim.py;
	 * profiles/r97_ab_window.txt, r99: windows 0 / 12 / 20 / 32 / 64 -> median 32.7 / 31.7-33.2 / 32.0-32.5 /
	 * 33.3 / 33.7 ms).
	 * M2DEC_AMD_PARSE_PRIO = the window (0: oldest first). */
	const long window_end = as->qtail + g_parse_prio;
	for (int pass = g_parse_prio ? 0 : 1; pass < 2; ++pass)
		for (long k = as->qtail; k < as->qhead && (pass || k < window_end); ++k) {
			h264_job_t *c = as->queue[k % AS_MAX];
			*dep_err = 0;
			int early;
			if (c && (pass || !c->nonref) && deps_ready(as, c, dep_err, &early)) {
				c->taken = 1;
				c->col_early = early;
				as->queue[k % AS_MAX] = NULL;
				if (c->nsl == 1 && !c->nonref) /* (its readers may start from now on: they see this) */
					__atomic_store_n(h264_col_progress(c->snap[0]->colpic[c->col_store].mb, c->snap[0]->n_mbs), 0,
					                 __ATOMIC_RELAXED);
				return c;
			}
		}
	return NULL;
}

/* pool workers driving pipelines after their jobs, wall and thread CPU time (M2DEC_AMD_ASYNC_STATS) */
static long long g_drive_ns, g_drive_cpu_ns, g_job_cpu_ns;

/* pool workers inside a job or slice, all pipelines (m2dec_parse_busy: the MD5 pipe's tail mode) */
static int g_parse_running;

int m2dec_parse_busy(void) { return __atomic_load_n(&g_parse_running, __ATOMIC_RELAXED); }

/* Pool workers take the oldest queued job whose dependencies have finished, so a B picture waiting
 * for its co-located P does not hold a worker while later P pictures could be parsed; pipelines are
 * served round robin.  A finished job may let its pipeline submit: the worker drives it. */
static void *pool_worker(void *arg)
{
	pthread_setname_np(pthread_self(), "m2d-parse");
	(void)arg;
	pthread_mutex_lock(&g_parse.mu);
	for (;;) {
		struct h264_async *as = NULL, *first = g_parse.rr ? g_parse.rr : g_parse.pipes;
		h264_job_t *j = NULL, *pj = NULL;
		int k = 0, dep_err = 0;
		for (struct h264_async *p = first; p && !j && !pj;) {
			if (!p->quit && p->running < p->nth) {
				j = pick_job(p, &pj, &k, &dep_err);
				if (j || pj) as = p;
			}
			p = p->pnext ? p->pnext : g_parse.pipes;
			if (p == first) break;
		}
		if (!as) {
			pthread_cond_wait(&g_parse.cv_work, &g_parse.mu);
			m2d_place_self(); /* (numa.c: near the GPU once a device back end exists) */
			continue;
		}
		g_parse.rr = as->pnext;
		as->running++;
		__atomic_fetch_add(&g_parse_running, 1, __ATOMIC_RELAXED);
		pthread_mutex_unlock(&g_parse.mu);
		m2d_cpu_primary(1); /* (cpushare.c: MD5 batches use the slots the parse leaves free) */
		if (pj) {
			const double ts = now_s();
			slice_run(pj, k);
			m2d_cpu_primary(-1);
			const double te = now_s();
			pthread_mutex_lock(&g_parse.mu);
			as->t_parse += te - ts;
			pj->sl_done++;
		} else {
			const double tp = now_s(); /* (two clock reads per picture: the parse time is always kept) */
			struct timespec jc0;
			if (as->stats) clock_gettime(CLOCK_THREAD_CPUTIME_ID, &jc0);
			m2d_tl('P', j->seq, j->snap[0]->sh.slice_type);
			if (dep_err) {
				j->err = 1;
				if (j->nsl == 1 && !j->nonref) /* (a reader may have started on this writer: release it) */
					__atomic_store_n(h264_col_progress(j->snap[0]->colpic[j->col_store].mb, j->snap[0]->n_mbs), -1,
					                 __ATOMIC_RELEASE);
			} else if (!(as->slice_par && j->nsl > 1)) job_run(j);
			else if (job_run_par(as, j) < 0) {
				job_run(j);
				__atomic_fetch_add(&as->n_par_fallback, 1, __ATOMIC_RELAXED);
			} else {
				__atomic_fetch_add(&as->n_par, 1, __ATOMIC_RELAXED);
			}
			if (!j->err) pic_refs(&j->pic);
			if (g_nonref_delay_us && j->nonref) usleep((useconds_t)g_nonref_delay_us);
			if (as->stats) {
				struct timespec jc1;
				clock_gettime(CLOCK_THREAD_CPUTIME_ID, &jc1);
				__atomic_fetch_add(&g_job_cpu_ns, (long long)(jc1.tv_sec - jc0.tv_sec) * 1000000000LL + (jc1.tv_nsec - jc0.tv_nsec),
				                   __ATOMIC_RELAXED);
			}
			m2d_cpu_primary(-1);
			pthread_mutex_lock(&g_parse.mu);
			const double te = now_s();
			m2d_tl('p', j->seq, j->snap[0]->sh.slice_type);
			as->t_parse += te - tp;
			if (as->stats > 1)
				fprintf(stderr, "job %ld type %d slices %d: start %.1f ms, parse %.2f ms\n", j->seq,
				        j->snap[0]->sh.slice_type, j->nsl, 1e3 * (tp - as->t0), 1e3 * (te - tp));
			j->done = 1;
			pthread_cond_broadcast(&g_parse.cv_work); /* jobs waiting on this one may be ready */
		}
		as->running--;
		__atomic_fetch_sub(&g_parse_running, 1, __ATOMIC_RELAXED);
		pthread_cond_broadcast(&as->cv_done);
		if (j) {
			if (as->stats) { /* (process-wide: `as` may be gone once the drive returns) */
				struct timespec c0, c1;
				const double w0 = now_s();
				clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
				pipe_drive(as);
				clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
				__atomic_fetch_add(&g_drive_ns, (long long)(1e9 * (now_s() - w0)), __ATOMIC_RELAXED);
				__atomic_fetch_add(&g_drive_cpu_ns, (long long)(c1.tv_sec - c0.tv_sec) * 1000000000LL + (c1.tv_nsec - c0.tv_nsec),
				                   __ATOMIC_RELAXED);
			} else {
				pipe_drive(as);
			}
		}
	}
	return NULL;
}

/* Process exit with contexts still decoding (a caller that drops its decoders, m2decoder.h:39-50, and
 * returns from main): the detached workers would go on parsing and driving back ends while the static
 * destructors tear down the HIP runtime and the back ends' process pools under them.  So the first
 * worker's creation registers this: every pipeline stops taking work, and exit waits (bounded) until no
 * worker is inside a job or a back-end call; the idle workers then sleep on cv_work through exit. */
static void pool_atexit(void)
{
	struct timespec ts;
	pthread_mutex_lock(&g_parse.mu);
	for (struct h264_async *p = g_parse.pipes; p; p = p->pnext) p->quit = 1;
	clock_gettime(CLOCK_REALTIME, &ts);
	ts.tv_sec += 2;
	for (;;) {
		struct h264_async *busy = NULL;
		for (struct h264_async *p = g_parse.pipes; p && !busy; p = p->pnext)
			if (p->running || p->driving) busy = p;
		if (!busy || pthread_cond_timedwait(&busy->cv_done, &g_parse.mu, &ts) != 0) break;
	}
	pthread_mutex_unlock(&g_parse.mu);
}

/* at least n pool workers (mutex held) */
static int pool_grow(int n)
{
	if (n > POOL_MAX) n = POOL_MAX;
	if (g_parse.nth == 0 && n > 0) {
		const char *c = getenv("M2DEC_AMD_COL_PIPE");
		if (c) g_col_pipe = atoi(c) != 0;
		if (getenv("M2DEC_AMD_EARLY")) g_early = atoi(getenv("M2DEC_AMD_EARLY")) != 0;
		if (getenv("M2DEC_AMD_NONREF_DELAY_US")) g_nonref_delay_us = atoi(getenv("M2DEC_AMD_NONREF_DELAY_US"));
		if (getenv("M2DEC_AMD_COL_PIPE_DELAY_US")) g_col_delay_us = atoi(getenv("M2DEC_AMD_COL_PIPE_DELAY_US"));
		const char *e = getenv("M2DEC_AMD_PARSE_PRIO");
		if (e) g_parse_prio = atoi(e) < 0 ? 0 : atoi(e);
		atexit(pool_atexit);
	}
	while (g_parse.nth < n) {
		pthread_attr_t at;
		pthread_attr_init(&at);
		pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
		const int e = pthread_create(&g_parse.th[g_parse.nth], &at, pool_worker, NULL);
		pthread_attr_destroy(&at);
		if (e != 0) break;
		g_parse.nth++;
	}
	return g_parse.nth;
}

/* ---------------------------------------------------------------- start / stop */

static void la_free(h264_dec_t *la)
{
	if (!la) return;
	free(la->mbi);
	for (int i = 0; i < 17; ++i) free(la->colpic[i].mb);
	free(la->nal);
	free(la);
}

/* Called from the first set_frames (inside the SPS header callback, on the API context's NAL loop):
 * the lookahead context starts as a copy of the API context at this stream position; from the next
 * NAL on, the API context reads NALs only from the lookahead's queue. */
int h264_async_start(h264_dec_t *d, int threads)
{
	struct h264_async *as;
	h264_dec_t *la;
	if (threads <= 0) return 0;
	if (threads > POOL_MAX) threads = POOL_MAX;
	as = (struct h264_async *)calloc(1, sizeof(*as));
	la = (h264_dec_t *)malloc(sizeof(h264_dec_t));
	if (!as || !la) {
		free(as);
		free(la);
		return -1;
	}
	memcpy(la, d, sizeof(*la));
	la->mbi = NULL;
	la->mbi_cap = 0;
	la->mb_w = la->mb_h = la->n_mbs = 0; /* alloc_geometry: own MB info and co-located stores */
	for (int i = 0; i < 17; ++i) la->colpic[i].mb = NULL;
	la->nal = NULL;
	la->nal_cap = 0;
	la->nal_len = 0;
	la->nal_replay = 0;
	la->have_backend = 0;
	la->pic = NULL;
	la->lookahead = 1;
	la->vid_next = 0;
	la->as = as;
	as->la = la;
	as->nq_cap = 256;
	as->nq = (nal_ent_t *)calloc((size_t)as->nq_cap, sizeof(nal_ent_t));
	if (!as->nq) goto fail;
	for (int i = 0; i < 64; ++i) as->vmap[i] = -1;
	as->mu = &g_parse.mu;
	as->api = d;
	pthread_cond_init(&as->cv_done, NULL);
	as->depth = 3 * threads + 12; /* (16 workers: the cap, 60 pictures; profiles/r59_knobs.txt) */
	{
		const char *e = getenv("M2DEC_AMD_PARSE_DEPTH"); /* tuning: pictures the lookahead runs ahead */
		if (e && atoi(e) > 0) as->depth = atoi(e);
	}
	if (as->depth > AS_MAX - 4) as->depth = AS_MAX - 4;
	for (int i = 0; i < 17; ++i) as->col_last[i] = as->col_writer[i] = -1;
	as->la_sps_nal = -1;
	as->ahead = d->have_backend && d->backend.bind && !getenv("M2DEC_AMD_NO_AHEAD");
	as->ext = as->ahead && d->backend.records_busy && !(getenv("M2DEC_AMD_EXTERNAL") && atoi(getenv("M2DEC_AMD_EXTERNAL")) == 0);
	as->stats = getenv("M2DEC_AMD_ASYNC_STATS") ? atoi(getenv("M2DEC_AMD_ASYNC_STATS")) : 0;
	as->slice_par = !getenv("M2DEC_AMD_SLICE_PAR") || atoi(getenv("M2DEC_AMD_SLICE_PAR")) != 0;
	as->t0 = now_s();
	as->api_sps_nal = -1;
	as->ahead_all = getenv("M2DEC_AMD_AHEAD_ALL") && atoi(getenv("M2DEC_AMD_AHEAD_ALL"));
	pthread_mutex_lock(&g_parse.mu);
	{
		/* the pool is sized for the host share, not per pipeline: M2DEC_AMD_POOL_THREADS, default the process's
		 * CPU share (cpushare.c: affinity ∩ cgroup quota ÷ the node's GPU ranks; 16 on the GPU box,
		 * profiles/r48*_threads.txt), at least what a pipeline asks for */
		const char *e = getenv("M2DEC_AMD_POOL_THREADS");
		const int want = e && atoi(e) > 0 ? atoi(e) : m2d_cpu_slots() > 0 ? m2d_cpu_slots() : m2d_cpu_share();
		pool_grow(want > threads ? want : threads);
	}
	as->nth = g_parse.nth < threads ? g_parse.nth : threads;
	if (as->nth <= 0) {
		pthread_mutex_unlock(&g_parse.mu);
		pthread_cond_destroy(&as->cv_done);
		goto fail;
	}
	as->pnext = g_parse.pipes;
	g_parse.pipes = as;
	pthread_mutex_unlock(&g_parse.mu);
	d->as = as;
	return 0;
fail:
	free(as->nq);
	free(as);
	free(la);
	return -1;
}

/* CPU seconds the workers spent parsing slice data so far (0 without parse-ahead), and the pictures
 * parsed slice-parallel / re-parsed sequentially after a slice-parallel try */
double h264_async_parse_seconds(h264_dec_t *d, long *par, long *par_fallback)
{
	struct h264_async *as = d->as;
	double t;
	*par = *par_fallback = 0;
	if (!as) return 0.0;
	pthread_mutex_lock(as->mu);
	t = as->t_parse;
	*par = as->n_par;
	*par_fallback = as->n_par_fallback;
	pthread_mutex_unlock(as->mu);
	return t;
}

/* Wait until the back end reads no job arena of this pipeline any more (before the jobs leave it, or
 * the back end is replaced).  Caller's thread; no worker or driver of the pipeline may run. */
void h264_async_records_wait(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	h264_job_t *busy[2 * AS_MAX];
	int n = 0;
	if (!as || !as->ext) return;
	pthread_mutex_lock(as->mu);
	while (as->driving) pthread_cond_wait(&as->cv_done, as->mu);
	as->driving = 1; /* (no back-end call of a pool worker meanwhile; job_get runs on this thread) */
	for (long i = as->tail; i < as->head; ++i)
		if (as->fifo[i % AS_MAX]->ext_busy) busy[n++] = as->fifo[i % AS_MAX];
	for (int i = 0; i < as->nfree; ++i)
		if (as->free_jobs[i]->ext_busy) busy[n++] = as->free_jobs[i];
	pthread_mutex_unlock(as->mu);
	for (int i = 0; i < n; ++i) (void)job_ext_idle(as, busy[i], 1);
	pthread_mutex_lock(as->mu);
	as->driving = 0;
	pthread_cond_broadcast(&as->cv_done);
	pthread_mutex_unlock(as->mu);
}

void h264_async_stop(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	if (!as) return;
	if (as->stats)
		fprintf(stderr, "async: %ld jobs, depth %d; caller: lookahead %.3f s (col-store waits %.3f s, slice copies "
		                "%.3f s), oldest-done waits %.3f s, record copies %.3f s, back-end submit %.3f s; workers "
		                "parse %.3f s; jobs created so far in the process %ld; early submissions %ld; page-locked job "
		                "arenas %.1f MB (pooled %.1f MB); co-located row waits in the process %.3f s; workers driving in the process %.3f s (CPU %.3f s), job CPU %.3f s\n",
		        as->seq, as->depth, as->t_la, as->t_col_wait, as->t_slice, as->t_done_wait, as->t_copy, as->t_submit,
		        as->t_parse, g_jobs_new, as->n_early, (double)__atomic_load_n(&g_pinned_bytes, __ATOMIC_RELAXED) / 1e6,
		        (double)g_pool_pinned / 1e6, 1e-9 * (double)h264_col_spin_ns(), 1e-9 * (double)__atomic_load_n(&g_drive_ns, __ATOMIC_RELAXED),
		        1e-9 * (double)__atomic_load_n(&g_drive_cpu_ns, __ATOMIC_RELAXED),
		        1e-9 * (double)__atomic_load_n(&g_job_cpu_ns, __ATOMIC_RELAXED));
	/* no pool worker starts anything of this pipeline any more; wait for the ones inside it */
	pthread_mutex_lock(as->mu);
	as->quit = 1;
	while (as->running || as->driving) pthread_cond_wait(&as->cv_done, as->mu);
	for (struct h264_async **pp = &g_parse.pipes; *pp; pp = &(*pp)->pnext)
		if (*pp == as) {
			*pp = as->pnext;
			break;
		}
	if (g_parse.rr == as) g_parse.rr = NULL;
	pthread_mutex_unlock(as->mu);
	/* (no worker or driver of this pipeline runs now: the back end is ours to wait on, outside the pool's
	 * mutex) jobs another context may take next must not be read by this back end any more */
	h264_async_records_wait(d);
	pthread_mutex_lock(as->mu);
	for (long i = as->tail; i < as->head; ++i) job_release(as->fifo[i % AS_MAX]);
	job_release(as->cur);
	for (int i = 0; i < as->nfree; ++i) job_release(as->free_jobs[i]);
	pthread_mutex_unlock(as->mu);
	for (long i = 0; i < as->nq_cap; ++i) free(as->nq[i].buf);
	for (int i = 0; i < as->nspare; ++i) free(as->spare[i].mb);
	free(as->nq);
	la_free(as->la);
	pthread_cond_destroy(&as->cv_done);
	free(as);
	d->as = NULL;
}

/* The stream ended (decode_picture returned -2): the retired jobs (record arenas of about 1 KB per MB
 * each) go back to the process pool, the co-located spares are freed.  A context the caller drops at
 * the end of its stream then holds little host memory until the registry reclaims it.  (The lookahead context's co-located stores stay: temporal / spatial
 * direct of a continuation reads them.) */
void h264_async_trim(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	int idle;
	if (!as) return;
	pthread_mutex_lock(as->mu);
	{
		int keep = 0;
		for (int i = 0; i < as->nfree; ++i) {
			h264_job_t *j = as->free_jobs[i];
			if (job_ext_idle(as, j, 0)) job_release(j);
			else as->free_jobs[keep++] = j; /* (still uploading: job_get or stop takes it later) */
		}
		as->nfree = keep;
	}
	idle = as->head == as->tail;
	pthread_mutex_unlock(as->mu);
	if (idle) { /* no job may still read a spare (the lookahead runs on this thread) */
		for (int i = 0; i < as->nspare; ++i) free(as->spare[i].mb);
		as->nspare = 0;
	}
}

/* the back end no longer reads job j's arena (wait = 0: never blocks; wait = 1: see records_busy) */
static int job_ext_idle(struct h264_async *as, h264_job_t *j, int wait)
{
	const m2r_backend_t *be = &as->api->backend;
	if (j->ext_busy && !(be->records_busy && be->records_busy(be->self, j->arena, wait) != 0)) j->ext_busy = 0;
	return !j->ext_busy;
}

static h264_job_t *job_get(struct h264_async *as, size_t need)
{
	h264_job_t *j;
	/* (the newest retired jobs may still be uploading: take the first one that is not) */
	for (int i = 0; i < as->nfree; ++i)
		if (job_ext_idle(as, as->free_jobs[i], 0)) {
			j = as->free_jobs[i];
			as->free_jobs[i] = as->free_jobs[--as->nfree];
			return j;
		}
	if (g_njobs) {
		/* the newest pooled job whose arena already fits this geometry (pinned if the pipeline uploads from it):
		 * a 4K stream after 1080p ones otherwise re-pins a pooled 1080p job's arena (~27 MB, several ms on
		 * the lookahead's thread) for each job it takes */
		for (int i = g_njobs - 1; i >= 0; --i)
			if (g_jobs[i]->arena_size >= need && (!as->ext || g_jobs[i]->arena_pinned)) return pool_take(i);
		return pool_take(g_njobs - 1);
	}
	j = (h264_job_t *)calloc(1, sizeof(*j));
	if (!j) return NULL;
	g_jobs_new++;
	j->slot = -1;
	j->w = (h264_dec_t *)malloc(sizeof(h264_dec_t));
	if (!j->w) {
		free(j);
		return NULL;
	}
	return j;
}

/* (mutex held; the caller drives the pipeline, so it may wait on the back end: records_busy) */
static void job_put(struct h264_async *as, h264_job_t *j)
{
	job_clear(j);
	if (as->nfree < AS_MAX) {
		as->free_jobs[as->nfree++] = j;
		return;
	}
	/* full: free a job whose arena the back end no longer reads (a just-retired job's upload may still
	 * read its pinned records) — an idle free one in j's place, else j once its upload is done */
	if (j->ext_busy)
		for (int i = 0; i < as->nfree; ++i)
			if (job_ext_idle(as, as->free_jobs[i], 0)) {
				h264_job_t *o = as->free_jobs[i];
				as->free_jobs[i] = j;
				j = o;
				break;
			}
	(void)job_ext_idle(as, j, 1);
	job_free(j);
}

/* ---------------------------------------------------------------- API context: submission */
/* Submission is in decode order ([tail, sub) submitted, [tail, bnd) bound).
 *
 * Without bind (back ends that only take frame slots) it runs on the caller's thread: a job goes to
 * the back end once the API context closed it, its virtual ids translated to the frame slots of
 * that moment (j->map), and retires at once.
 *
 * With bind (decode ahead) pipe_drive makes every back-end call but sync_frame: it submits each
 * parsed job as it is, virtual ids naming the back end's picture buffers, as soon as the rules below
 * allow — possibly long before the API context reaches it — and binds closed jobs' buffers to the
 * frame slots the API context chose, in order.  It runs mostly on the pool worker that finished a
 * job, so the record copies and the HIP calls stay off the caller's thread; the caller's thread
 * closes pictures and, to hand a frame out, waits until its job is bound (h264_async_drain) before
 * sync_frame. */

/* records into the back end's arena (virtual ids as they are, or translated to slots) + submit */
static int copy_submit(h264_dec_t *d, h264_job_t *j, int virt)
{
	struct h264_async *as = d->as;
	const m2r_picture_t *src = &j->pic;
	const int n = src->width_mbs * src->height_mbs;
	double t1 = as->stats ? now_s() : 0;
	m2d_tl('A', j->seq, 0);
	m2r_picture_t *dst = d->backend.acquire(d->backend.self, src->width_mbs, src->height_mbs);
	m2d_tl('a', j->seq, 0);
	if (!dst || dst->cap_slices < src->n_slices || dst->cap_inter < src->n_inter || dst->cap_coef < src->n_coef) return 1;
	dst->slot = virt ? (j->vid & 63) : j->slot;
	dst->flags = virt ? M2R_PIC_VIRTUAL : 0;
	dst->n_inter = src->n_inter;
	dst->n_coef = src->n_coef;
	dst->n_slices = src->n_slices;
	dst->n_intra = src->n_intra;
	dst->deblock = src->deblock;
	if (src->flags & M2R_PIC_REFS) {
		dst->flags |= M2R_PIC_REFS;
		dst->ref_blocks = src->ref_blocks;
		dst->ref_slots = src->ref_slots;
		if (!virt) {
			dst->ref_slots = 0;
			for (int v = 0; v < 64; ++v)
				if (((src->ref_slots >> v) & 1) && j->map[v] >= 0) dst->ref_slots |= 1ull << (j->map[v] & 63);
		}
	}
	if (virt && as->ext && j->arena_pinned && d->backend.records_busy) {
		/* the back end uploads the job's own (pinned) records: nothing to copy; the job is not reused
		 * until records_busy says the upload is done (job_get) */
		dst->flags |= M2R_PIC_EXTERNAL;
		dst->mb = src->mb;
		dst->dbk = src->dbk;
		dst->slice = src->slice;
		dst->inter = src->inter;
		dst->coef = src->coef;
		j->ext_busy = 1;
	} else if (virt) {
		memcpy(dst->slice, src->slice, sizeof(m2r_slice_t) * (size_t)src->n_slices);
		void *const to[4] = {dst->mb, dst->dbk, dst->inter, dst->coef};
		const void *const from[4] = {src->mb, src->dbk, src->inter, src->coef};
		const size_t len[4] = {sizeof(m2r_mb_t) * (size_t)n, sizeof(m2r_deblock_t) * (size_t)n,
		                       sizeof(m2r_inter_t) * (size_t)src->n_inter, sizeof(int16_t) * (size_t)src->n_coef};
		m2dec_par_memcpy(M2DEC_CREW_SUBMIT, 4, to, from, len);
	} else {
		memcpy(dst->slice, src->slice, sizeof(m2r_slice_t) * (size_t)src->n_slices);
		memcpy(dst->mb, src->mb, sizeof(m2r_mb_t) * (size_t)n);
		memcpy(dst->dbk, src->dbk, sizeof(m2r_deblock_t) * (size_t)n);
		for (int i = 0; i < src->n_inter; ++i) {
			const m2r_inter_t *si = &src->inter[i];
			m2r_inter_t *di = &dst->inter[i];
			memcpy(di->mv, si->mv, sizeof(di->mv));
			memcpy(di->refidx, si->refidx, sizeof(di->refidx));
			for (int k = 0; k < 8; ++k) {
				const int v = (&si->slot[0][0])[k];
				(&di->slot[0][0])[k] = (int8_t)(v < 0 ? -1 : j->map[v & 63]);
			}
		}
		memcpy(dst->coef, src->coef, sizeof(int16_t) * (size_t)src->n_coef);
	}
	if (as->stats) {
		const double t2 = now_s();
		as->t_copy += t2 - t1;
		t1 = t2;
	}
	m2d_tl('C', j->seq, 0);
	int err = d->backend.submit(d->backend.self, dst) < 0;
	if (!err && !virt && d->backend.flush) err = d->backend.flush(d->backend.self) < 0; /* (in API order: one at a time) */
	if (as->stats) as->t_submit += now_s() - t1;
	return err;
}

/* ---- without bind: the caller's thread */
static int submit_next(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	h264_job_t *j = as->fifo[as->sub % AS_MAX];
	const double t0 = as->stats ? now_s() : 0;
	int err;
	pthread_mutex_lock(as->mu);
	while (!j->done) pthread_cond_wait(&as->cv_done, as->mu);
	pthread_mutex_unlock(as->mu);
	if (as->stats) as->t_done_wait += now_s() - t0;
	err = j->err || copy_submit(d, j, 0);
	pthread_mutex_lock(as->mu);
	as->sub++;
	as->tail++; /* workers scan [tail, head) under the mutex */
	job_put(as, j);
	pthread_mutex_unlock(as->mu);
	return err ? -1 : 0;
}

/* ---- decode ahead */
/* a parsed job the API context has not closed yet may go to the back end now: no header callback
 * (set_frames) the API context has not run yet lies before it, and the previous picture of its
 * virtual buffer is bound (so the back end orders the overwrite after that copy-out).  Mutex held. */
static int ahead_ok(const struct h264_async *as, const h264_job_t *j)
{
	if (j->err || j->sps_nal > as->api_sps_nal) return 0;
	for (long i = as->tail; i < j->seq; ++i) {
		const h264_job_t *o = as->fifo[i % AS_MAX];
		if (o->vid == j->vid && !o->bound) return 0;
	}
	return 1;
}

/* Early submission (M2DEC_AMD_EARLY).  Submission is in decode order, and the pool finishes the
 * reference pictures (I / P) well before the B pictures decoded before them (anchors first in pick_job,
 * B pictures are longer): the r105 timeline had the stream's last anchors parsed at 15-17 ms but submitted
 * at 21-23 ms behind their B pictures, so the device ran the anchor chain P52 -> P55 -> P58 after the
 * parse had ended.  A parsed reference picture j may go to the back end before older unsubmitted jobs
 * when (mutex held):
 *   - ahead_ok: no header callback pending before it, the previous picture of its virtual buffer bound;
 *   - RAW: the newest job before it writing each buffer it may read (refmask) was submitted;
 *   - WAR: no older unsubmitted job may read its buffer's previous content (their refmasks, known at
 *     dispatch, so unparsed jobs count too).
 * The back end then sees every reference before its readers and every reader of a buffer's old content
 * before its overwrite, as with decode order; its device-side ordering (row flags by launch sequence,
 * WAR events, in-launch war / war_writer) only needs that.  Binding stays in decode order. */
static int early_ok(const struct h264_async *as, const h264_job_t *j)
{
	if (!j->done || j->err || j->submitted || j->nonref || !ahead_ok(as, j)) return 0;
	const int v = j->vid & 63;
	uint64_t need = j->refmask;
	for (long i = j->seq - 1; i >= as->tail; --i) {
		const h264_job_t *o = as->fifo[i % AS_MAX];
		const int ov = o->vid & 63;
		if (!o->submitted) {
			if ((o->refmask >> v) & 1) return 0;         /* reads the buffer's old content */
			if ((need >> ov) & 1) return 0;              /* the reference is not on the device yet */
		}
		need &= ~(1ull << ov);                           /* (older writers of that buffer: overwritten) */
	}
	return 1;
}

/* Decode ahead: make every step the state allows — bind the oldest closed, submitted job (and retire
 * what is bound), or submit the next parsed job that is closed or allowed ahead.  There is no
 * submitter thread: whoever changes what is possible (a pool worker that finished a job, the API
 * context closing a picture or running a header callback, a thread about to wait for a bind) calls
 * this, and the first one in does the back-end calls (serially) until nothing is left; the others
 * return at once — the state is re-checked under the mutex before the driver leaves, so no step is
 * lost.  Mutex held on entry and on return. */
static void pipe_drive(struct h264_async *as)
{
	h264_dec_t *d = as->api;
	if (!as->ahead || as->driving || as->quit) return;
	as->driving = 1;
	while (!as->quit) { /* (a context being released stops after the back-end call under way) */
		if (as->bnd < as->sub && as->bnd < as->a_seq) {
			h264_job_t *j = as->fifo[as->bnd % AS_MAX];
			const int skip = j->sub_err, vid = j->vid & 63, slot = j->slot;
			pthread_mutex_unlock(as->mu);
			m2d_tl('B', vid, slot);
			const int err = !skip && d->backend.bind(d->backend.self, vid, slot) < 0;
			m2d_tl('b', vid, slot);
			pthread_mutex_lock(as->mu);
			j->bound = 1;
			as->sub_err += err;
			as->bnd++;
			while (as->tail < as->bnd) {
				h264_job_t *o = as->fifo[as->tail % AS_MAX];
				as->tail++;
				job_put(as, o);
			}
			pthread_cond_broadcast(&as->cv_done);
			continue;
		}
		if (as->sub < as->head && as->fifo[as->sub % AS_MAX]->submitted) { /* (went early) */
			as->sub++;
			continue;
		}
		if (as->sub < as->head) {
			h264_job_t *j = as->fifo[as->sub % AS_MAX];
			if (j->done && (as->sub < as->a_seq || ahead_ok(as, j))) {
				const int ahead = as->sub >= as->a_seq;
				pthread_mutex_unlock(as->mu);
				if (as->stats > 1 && j->err) fprintf(stderr, "job %ld: parse error, not submitted\n", j->seq);
				m2d_tl('S', j->seq, 0);
				const int err = j->err || copy_submit(d, j, 1);
				m2d_tl('s', j->seq, 0);
				pthread_mutex_lock(as->mu);
				j->sub_err = err;
				j->submitted = 1;
				as->sub_err += err;
				as->held |= !err && d->backend.flush != NULL;
				as->sub++;
				d->ahead_submits += ahead && !err;
				pthread_cond_broadcast(&as->cv_done);
				continue;
			}
		}
		if (g_early) {
			h264_job_t *e = NULL;
			for (long i = as->sub + 1; i < as->head && i < as->sub + 32 && !e; ++i)
				if (early_ok(as, as->fifo[i % AS_MAX])) e = as->fifo[i % AS_MAX];
			if (e) {
				pthread_mutex_unlock(as->mu);
				m2d_tl('S', e->seq, 1);
				const int err = copy_submit(d, e, 1);
				m2d_tl('s', e->seq, 1);
				pthread_mutex_lock(as->mu);
				e->sub_err = err;
				e->submitted = 1;
				as->sub_err += err;
				as->held |= !err && d->backend.flush != NULL;
				d->ahead_submits += !err;
				as->n_early += !err;
				pthread_cond_broadcast(&as->cv_done);
				continue;
			}
		}
		if (as->held) {
			/* nothing more to do for now: let the back end launch what it holds (it may keep them while the
			 * device is busy, returning 1: the next drive asks again, and a bind launches them anyway) */
			pthread_mutex_unlock(as->mu);
			const int r = d->backend.flush(d->backend.self);
			pthread_mutex_lock(as->mu);
			as->sub_err += r < 0;
			if (r > 0) break;
			as->held = 0;
			continue;
		}
		break;
	}
	as->driving = 0;
	pthread_cond_broadcast(&as->cv_done);
}

/* a submission or bind failed since the last call: report it once (mutex held) */
static int take_error(struct h264_async *as)
{
	const int e = as->sub_err;
	as->sub_err = 0;
	return e ? -1 : 0;
}

/* every closed job up to and including the newest one that writes `slot` (-1: all) is submitted —
 * and, decoding ahead, bound to its slot */
int h264_async_drain(h264_dec_t *d, int slot)
{
	struct h264_async *as = d->as;
	long upto = -1;
	if (!as) return 0;
	if (!as->ahead) {
		for (long i = as->tail; i < as->a_seq; ++i)
			if (slot < 0 || as->fifo[i % AS_MAX]->slot == slot) upto = i;
		while (as->sub <= upto)
			if (submit_next(d) < 0) return -1;
		return 0;
	}
	const double t0 = as->stats ? now_s() : 0;
	pthread_mutex_lock(as->mu);
	for (long i = as->tail; i < as->a_seq; ++i)
		if (slot < 0 || as->fifo[i % AS_MAX]->slot == slot) upto = i;
	while (as->bnd <= upto) {
		pipe_drive(as);
		if (as->bnd > upto) break;
		/* waiting for the pool: keep the lookahead dispatching meanwhile (this is the caller's thread) */
		pthread_mutex_unlock(as->mu);
		const int stepped = h264_async_pump_step(d);
		pthread_mutex_lock(as->mu);
		if (stepped) continue;
		if (as->bnd > upto) break;
		pthread_cond_wait(&as->cv_done, as->mu);
	}
	const int err = take_error(as);
	pthread_mutex_unlock(as->mu);
	if (as->stats) as->t_done_wait += now_s() - t0;
	return err;
}

/* without bind: submit, in order and without waiting, closed jobs whose parse finished.  Decoding
 * ahead pipe_drive does that; report its errors */
static int submit_ready(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	if (as->ahead) {
		pthread_mutex_lock(as->mu);
		const int err = take_error(as);
		pthread_mutex_unlock(as->mu);
		return err;
	}
	for (;;) {
		int ready;
		if (as->sub >= as->a_seq) return 0;
		pthread_mutex_lock(as->mu);
		ready = as->fifo[as->sub % AS_MAX]->done;
		pthread_mutex_unlock(as->mu);
		if (!ready) return 0;
		if (submit_next(d) < 0) return -1;
	}
}

/* the API context ran the header callback of the SPS it just read: pictures after it may go ahead */
void h264_async_api_sps(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	pthread_mutex_lock(as->mu);
	as->api_sps_nal = as->nq_tail - 1;
	pipe_drive(as);
	pthread_mutex_unlock(as->mu);
}

/* ---------------------------------------------------------------- lookahead context */
/* run the lookahead until `until_nal` (the queue holds a NAL) or, else, until it is `depth` pictures
 * ahead of the API context / out of job slots / at the end of the data */
static void pump(h264_dec_t *d, int until_nal)
{
	struct h264_async *as = d->as;
	const double t0 = as->stats ? now_s() : 0;
	while (!as->la_done) {
		if (until_nal) {
			if (as->nq_head > as->nq_tail) break;
		} else if (as->seq - as->a_seq >= as->depth) {
			break;
		}
		/* job slots: submit what the API context closed before dispatching more */
		if (as->ahead) {
			int full;
			pthread_mutex_lock(as->mu);
			while (as->head - as->tail >= AS_MAX - 2 && as->tail < as->a_seq) {
				pipe_drive(as);
				if (as->head - as->tail < AS_MAX - 2) break;
				pthread_cond_wait(&as->cv_done, as->mu);
			}
			full = as->head - as->tail >= AS_MAX - 2;
			pthread_mutex_unlock(as->mu);
			if (full) break;
		} else {
			while (as->head - as->tail >= AS_MAX - 2 && as->sub < as->a_seq)
				if (submit_next(d) < 0) {
					as->la_done = as->la_err = 1;
					break;
				}
			if (as->head - as->tail >= AS_MAX - 2) break;
		}
		const int r = h264_decode_loop(as->la);
		if (r == -2) as->la_done = 1;
		else if (r < 0) as->la_done = as->la_err = 1;
	}
	if (as->stats) as->t_la += now_s() - t0;
}

/* One step of the lookahead (one picture's headers + dispatch), if it may run now: the caller's thread
 * calls this while it waits inside peek / get — for a bind (h264_async_drain) or for a frame's copy out
 * of the device (h264_api.c deliver) — so that the lookahead keeps dispatching parse jobs while the
 * caller is blocked on the device (before, it only ran inside decode_picture: while the caller waited
 * for a frame the parse pool ran dry, profiles/r81_timeline.txt).  Returns 1 if it made a step. */
int h264_async_pump_step(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	if (!as || as->la_done || as->seq - as->a_seq >= as->depth) return 0;
	pthread_mutex_lock(as->mu);
	const int full = as->head - as->tail >= AS_MAX - 2;
	pthread_mutex_unlock(as->mu);
	if (full) return 0;
	const double t0 = as->stats ? now_s() : 0;
	const long before = as->seq;
	const int r = h264_decode_loop(as->la);
	if (r == -2) as->la_done = 1;
	else if (r < 0) as->la_done = as->la_err = 1;
	if (as->stats) as->t_la += now_s() - t0;
	return as->seq != before || r >= 0;
}

/* the lookahead context finished a NAL: hand it to the API context (buffers are swapped, not copied) */
int h264_async_push_nal(h264_dec_t *la)
{
	struct h264_async *as = la->as;
	if (as->nq_head - as->nq_tail == as->nq_cap) {
		const long cap = 2 * as->nq_cap;
		nal_ent_t *q = (nal_ent_t *)calloc((size_t)cap, sizeof(nal_ent_t));
		if (!q) return -1;
		for (long i = 0; i < as->nq_cap; ++i) q[(as->nq_tail + i) % cap] = as->nq[(as->nq_tail + i) % as->nq_cap];
		free(as->nq);
		as->nq = q;
		as->nq_cap = cap;
	}
	nal_ent_t *e = &as->nq[as->nq_head % as->nq_cap];
	uint8_t *b = e->buf;
	const size_t c = e->cap;
	e->buf = la->nal;
	e->cap = la->nal_cap;
	e->len = la->nal_len;
	la->nal = b;
	la->nal_cap = c;
	la->nal_len = 0;
	as->nq_head++;
	return 0;
}

/* a new decode_picture call: a lookahead that stopped at the end of the data may read again (the
 * caller's refill callback can have more data now); one that failed stays stopped */
void h264_async_resume(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	if (as->la_done && !as->la_err) {
		as->la_done = 0;
		as->la->eos = 0;
	}
}

/* API context: the next NAL (0), end of data (-1), or the lookahead failed before this point (-3) */
int h264_async_nal_next(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	if (d->nal_replay) {
		d->nal_replay = 0;
		return 0;
	}
	if (as->nq_head == as->nq_tail) pump(d, 1);
	if (as->nq_head == as->nq_tail) return as->la_err ? -3 : -1;
	nal_ent_t *e = &as->nq[as->nq_tail % as->nq_cap];
	uint8_t *b = d->nal;
	const size_t c = d->nal_cap;
	d->nal = e->buf;
	d->nal_cap = e->cap;
	d->nal_len = e->len;
	e->buf = b;
	e->cap = c;
	e->len = 0;
	as->nq_tail++;
	return 0;
}

/* lookahead: it read an SPS (the API context runs the header callback there: set_frames) */
void h264_async_la_sps(h264_dec_t *la)
{
	la->as->la_sps_nal = la->as->nq_head;
}

/* lookahead: wait until every dispatched job has finished (before its co-located stores are
 * reallocated for a new picture size) */
int h264_async_sps(h264_dec_t *la)
{
	struct h264_async *as = la->as;
	pthread_mutex_lock(as->mu);
	/* (a job below the tail is retired — and its object maybe recycled: do not look at it again) */
	for (long i = as->tail; i < as->head; ++i)
		while (i >= as->tail && !as->fifo[i % AS_MAX]->done) pthread_cond_wait(&as->cv_done, as->mu);
	pthread_mutex_unlock(as->mu);
	return 0;
}

/* lookahead: a slice header was parsed into la: open the picture's job if needed, append the slice */
int h264_async_add_slice(h264_dec_t *la)
{
	struct h264_async *as = la->as;
	h264_job_t *j = as->cur;
	const double ts = as->stats ? now_s() : 0;
	if (!j) {
		pthread_mutex_lock(as->mu); /* (pipe_drive recycles jobs) */
		j = job_get(as, m2r_arena_layout(la->mb_w * la->mb_h).size);
		pthread_mutex_unlock(as->mu);
		if (!j || job_arena(j, la->mb_w, la->mb_h, as->ext) < 0) return -1;
		j->vid = la->curr_idx;
		j->slot = -1;
		j->sps_nal = as->la_sps_nal;
		j->pic.slot = la->curr_idx;
		j->col_store = la->curr_col;
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
		{
			size_t *c = (size_t *)realloc(j->rbsp_cap, sizeof(*c) * (size_t)cap);
			if (!c) return -1;
			j->rbsp_cap = c;
		}
		j->capsl = cap;
	}
	{
		const size_t len = (size_t)(la->slice_rbsp_end - la->slice_rbsp);
		const int k = j->nsl;
		if (k == j->nkeep) { /* a new entry (kept with the job from then on) */
			j->snap[k] = (h264_dec_t *)malloc(sizeof(h264_dec_t));
			j->rbsp[k] = NULL;
			j->rbsp_cap[k] = 0;
			if (!j->snap[k]) return -1;
			j->nkeep++;
		}
		if (j->rbsp_cap[k] < len + 32) {
			const size_t cap = (len + 32) + (len + 32) / 4; /* room for the next pictures' sizes */
			free(j->rbsp[k]);
			j->rbsp[k] = (uint8_t *)malloc(cap);
			j->rbsp_cap[k] = j->rbsp[k] ? cap : 0;
			if (!j->rbsp[k]) return -1;
		}
		h264_dec_t *snap = j->snap[k];
		uint8_t *rb = j->rbsp[k];
		memcpy(snap, la, sizeof(*snap));
		memcpy(rb, la->slice_rbsp, len);
		memset(rb + len, 0, 32);
		j->snap[j->nsl] = snap;
		j->rbsp[j->nsl] = rb;
		j->nsl++;
	}
	if (as->stats) as->t_slice += now_s() - ts;
	return 0;
}

/* a store buffer no job can still use (a spare unmapped before every unsubmitted job), or a new one */
static h264_colmb_t *col_spare_get(struct h264_async *as, int n_mbs, long tail)
{
	if (as->col_n != (size_t)n_mbs) { /* new geometry (no job in flight, h264_async_sps) */
		for (int i = 0; i < as->nspare; ++i) free(as->spare[i].mb);
		as->nspare = 0;
		as->col_n = (size_t)n_mbs;
	}
	for (int i = 0; i < as->nspare; ++i)
		if (as->spare[i].unmap_seq <= tail) {
			h264_colmb_t *b = as->spare[i].mb;
			as->spare[i] = as->spare[--as->nspare];
			return b;
		}
	return (h264_colmb_t *)calloc(H264_COL_ENTRIES(n_mbs), sizeof(h264_colmb_t));
}

/* lookahead: the picture being collected is complete: marking in the lookahead context, slice
 * data to the workers */
static int la_close(h264_dec_t *la)
{
	struct h264_async *as = la->as;
	h264_job_t *j = as->cur;
	if (!j) return -1;
	as->cur = NULL;
	j->seq = as->seq;
	j->poc = j->snap[0]->sh.poc;
	/* a non-reference picture is never anyone's refs[1][0]: its co-located store is dead data */
	j->nonref = 1;
	j->refmask = 0;
	for (int k = 0; k < j->nsl; ++k) {
		const h264_dec_t *sk = j->snap[k];
		j->nonref &= (sk->sh.nal_ref_idc == 0);
		for (int l = 0; l < 2; ++l)
			for (int i = 0; i < 16; ++i)
				if (sk->refs[l][i].in_use && sk->refs[l][i].frame_idx >= 0) j->refmask |= 1ull << (sk->refs[l][i].frame_idx & 63);
	}
	if (j->nonref && (size_t)j->snap[0]->n_mbs > j->priv_n) {
		free(j->priv_col);
		j->priv_col = (h264_colmb_t *)malloc(sizeof(h264_colmb_t) * (size_t)j->snap[0]->n_mbs);
		j->priv_n = j->priv_col ? (size_t)j->snap[0]->n_mbs : 0;
		if (!j->priv_col) return -1;
	}
	/* co-located stores this picture reads (B slices) -> wait for their writers */
	j->col_dep = -1;
	for (int k = 0; k < j->nsl; ++k) {
		const h264_dec_t *s = j->snap[k];
		if (s->sh.slice_type != 1) continue;
		const int c = s->refs[1][0].col;
		if (c < 0 || c >= 17) continue;
		const long ws = as->col_writer[c];
		int seen = 0;
		for (int i = 0; i < j->ndeps; ++i) seen |= (j->deps[i] == ws);
		if (ws >= 0 && !seen && j->ndeps < 8) j->deps[j->ndeps++] = ws; /* (finished or retired: no wait) */
		if (j->nsl == 1) j->col_dep = ws;
		if (as->col_last[c] < j->seq) as->col_last[c] = j->seq;
	}
	/* the store this picture writes: if an earlier job that reads or writes its buffer is still
	 * unsubmitted, the picture writes a fresh buffer instead (its snapshots are re-pointed) and the
	 * old one waits in the spare list until those jobs are submitted */
	if (!j->nonref) {
		const int c = j->col_store;
		const long last = as->col_last[c];
		long tail;
		pthread_mutex_lock(as->mu); /* (pipe_drive moves the tail) */
		tail = as->tail;
		pthread_mutex_unlock(as->mu);
		if (last >= tail) {
			const double tw = as->stats ? now_s() : 0;
			h264_colmb_t *nb = col_spare_get(as, la->n_mbs, tail);
			if (nb) {
				if (as->nspare < 64) {
					as->spare[as->nspare].mb = la->colpic[c].mb;
					as->spare[as->nspare].unmap_seq = j->seq;
					as->nspare++;
				} else {
					free(nb); /* spare list full: wait as before */
					nb = NULL;
				}
			}
			if (nb) {
				la->colpic[c].mb = nb;
				for (int k = 0; k < j->nsl; ++k) j->snap[k]->colpic[c].mb = nb;
			} else {
				m2d_tl('W', j->seq, (int)last);
				pthread_mutex_lock(as->mu);
				for (long i = as->tail; i < as->head && i <= last; ++i) /* (jobs seq = fifo index) */
					while (i >= as->tail && !as->fifo[i % AS_MAX]->done) pthread_cond_wait(&as->cv_done, as->mu);
				pthread_mutex_unlock(as->mu);
				m2d_tl('w', j->seq, 0);
			}
			if (as->stats) as->t_col_wait += now_s() - tw;
		}
		as->col_last[c] = j->seq;
		as->col_writer[c] = j->seq;
	}
	/* marking, store swap (headers only) */
	la->pic = NULL;
	if (h264_picture_mark(la) < 0) return -1;
	/* dispatch */
	m2d_tl('Q', j->seq, (int)(as->seq - as->a_seq));
	pthread_mutex_lock(as->mu);
	as->fifo[as->head % AS_MAX] = j;
	as->head++;
	as->seq++;
	as->queue[as->qhead % AS_MAX] = j;
	as->qhead++;
	pthread_cond_broadcast(&g_parse.cv_work);
	pthread_mutex_unlock(as->mu);
	return 1;
}

/* API context: the picture is complete (the same boundary the lookahead saw): marking, DPB, the
 * job's frame-id translation; keep the lookahead ahead and hand over whatever is already parsed */
static int api_close(h264_dec_t *d)
{
	struct h264_async *as = d->as;
	h264_job_t *j;
	while (as->a_seq >= as->head && !as->la_done) pump(d, 0); /* (never: the lookahead closed it first) */
	if (as->a_seq >= as->head) return -1;
	j = as->fifo[as->a_seq % AS_MAX];
	if (j->poc != d->sh.poc) {
		fprintf(stderr, "m2dec_amd: parse-ahead lost step (picture %ld: poc %d vs %d)\n", as->a_seq, j->poc, d->sh.poc);
		return -1;
	}
	d->pic = NULL;
	if (h264_picture_mark(d) < 0) return -1;
	as->vmap[j->vid & 63] = (int8_t)d->curr_idx;
	memcpy(j->map, as->vmap, sizeof(j->map));
	pthread_mutex_lock(as->mu);
	if (as->ahead && as->ahead_all)
		while (!j->submitted && !(j->done && j->err)) {
			pipe_drive(as);
			if (j->submitted) break;
			pthread_cond_wait(&as->cv_done, as->mu);
		}
	j->slot = d->curr_idx;
	as->a_seq++;
	pipe_drive(as); /* (decode ahead: bind it, and submit what that allows) */
	pthread_mutex_unlock(as->mu);
	pump(d, 0);
	if (submit_ready(d) < 0) return -1;
	return 1;
}

int h264_async_close(h264_dec_t *d)
{
	return d->lookahead ? la_close(d) : api_close(d);
}
