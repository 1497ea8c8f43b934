/*
 * M2DEC_AMD_TIMELINE=path: a host-side event timeline of the decode pipeline (diagnostics, off by
 * default).  Events are {CLOCK_MONOTONIC ns, kind, a, b}, appended lock-free to a process-wide array
 * and written to `path` as CSV at exit; tools/timeline.py lines them up with a rocprofv3 kernel /
 * copy trace of the same run (same clock).  Kinds (upper case: begin, lower case: end):
 *   P/p parse job (a = job seq, b = slice type)   S/s record copy + submit (a = job seq)
 *   L   k_picture launch (a = pictures, b = stream) B/b bind (a = virtual id, b = frame slot)
 *   Y/y sync_frame (a = slot)                      H/h MD5 batch (a = frames)
 *   O   frame handed to the writer (a = index)     D/d one decode_stream_md5 call
 */
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <pthread.h>
#include "h264_dec.h"

typedef struct {
	int64_t t;
	int32_t kind, a, b;
} tl_ev_t;

#define TL_CAP (1 << 20)
static tl_ev_t *g_ev;
static atomic_long g_n;
static const char *g_path;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void tl_dump(void)
{
	FILE *f = fopen(g_path, "w");
	long n = atomic_load(&g_n);
	if (!f) return;
	if (n > TL_CAP) n = TL_CAP;
	fprintf(f, "t_ns,kind,a,b\n");
	for (long i = 0; i < n; ++i)
		if (g_ev[i].kind) fprintf(f, "%lld,%c,%d,%d\n", (long long)g_ev[i].t, (char)g_ev[i].kind, g_ev[i].a, g_ev[i].b);
	fclose(f);
}

static void tl_init(void)
{
	g_path = getenv("M2DEC_AMD_TIMELINE");
	if (!g_path || !*g_path) {
		g_path = NULL;
		return;
	}
	g_ev = (tl_ev_t *)calloc(TL_CAP, sizeof(tl_ev_t));
	if (!g_ev) {
		g_path = NULL;
		return;
	}
	atexit(tl_dump);
}

void m2d_tl(int kind, long a, long b)
{
	pthread_once(&g_once, tl_init);
	if (!g_path) return;
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	const long i = atomic_fetch_add_explicit(&g_n, 1, memory_order_relaxed);
	if (i >= TL_CAP) return;
	g_ev[i].t = (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
	g_ev[i].a = (int32_t)a;
	g_ev[i].b = (int32_t)b;
	g_ev[i].kind = kind;
}
