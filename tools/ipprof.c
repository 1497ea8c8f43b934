/* Cycle-sampling profile of the H.264 / H.265 host parse (null back end), for hosts without a perf tool:
 * perf_event_open sampling of the instruction pointer every PERIOD cycles, reported as offsets into
 * libm2dec_amd.so (resolve them with addr2line -f -i -e m2dec_amd/lib/libm2dec_amd.so).
 *   tools/ipprof.c <stream.264|stream.265> [reps] [bm] > samples.txt      (lines: "offset count"; bm: sample branch
 *   misses instead of cycles; an H.265 stream is parsed on the caller's thread: M2DEC_AMD_H265_THREADS=0) */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <linux/perf_event.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>
#include "m2dec_amd.h"

#define PAGES 64 /* data pages of the ring (a power of 2; stays under the unprivileged mlock limit) */
#define PERIOD 100000
#define MAXOFF (1 << 24)

static uint32_t hist[MAXOFF];

/* H.265: a back end whose calls do nothing (only the parser is sampled) */
static int n265_frames(void *self, int n, const m2d_frame_t *f, int w, int h) { (void)self; (void)n; (void)f; (void)w; (void)h; return 0; }
static int n265_submit(void *self, const h265r_picture_t *p) { (void)self; (void)p; return 0; }
static int n265_sync(void *self, int slot) { (void)self; (void)slot; return 0; }
static void n265_destroy(void *self) { (void)self; }
static long other;

static void drain(struct perf_event_mmap_page *mp, uintptr_t base)
{
	const size_t pg = (size_t)sysconf(_SC_PAGESIZE), size = PAGES * pg;
	unsigned char *data = (unsigned char *)mp + pg;
	uint64_t head = __atomic_load_n(&mp->data_head, __ATOMIC_ACQUIRE), tail = mp->data_tail;
	while (tail < head) {
		struct perf_event_header h;
		unsigned char rec[64];
		for (size_t k = 0; k < sizeof h; ++k) ((unsigned char *)&h)[k] = data[(tail + k) % size];
		if (h.size > sizeof rec || h.size < sizeof h) break;
		for (size_t k = 0; k < h.size; ++k) rec[k] = data[(tail + k) % size];
		if (h.type == PERF_RECORD_SAMPLE) {
			uint64_t ip;
			memcpy(&ip, rec + sizeof h, 8);
			if (ip >= base && ip - base < MAXOFF) hist[ip - base]++;
			else other++;
		}
		tail += h.size;
	}
	__atomic_store_n(&mp->data_tail, tail, __ATOMIC_RELEASE);
}

int main(int argc, char **argv)
{
	FILE *f = fopen(argv[1], "rb");
	if (!f) return 1;
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	fseek(f, 0, SEEK_SET);
	unsigned char *d = malloc((size_t)n);
	if (fread(d, 1, (size_t)n, f) != (size_t)n) return 1;
	fclose(f);
	const int reps = argc > 2 ? atoi(argv[2]) : 3;
	Dl_info di;
	if (!dladdr((void *)m2dec_amd_decode_stream3, &di)) return 1;
	const uintptr_t base = (uintptr_t)di.dli_fbase;
	struct perf_event_attr a;
	memset(&a, 0, sizeof a);
	a.type = PERF_TYPE_HARDWARE;
	a.size = sizeof a;
	const int bm = argc > 3 && !strcmp(argv[3], "bm");
	a.config = bm ? PERF_COUNT_HW_BRANCH_MISSES : PERF_COUNT_HW_CPU_CYCLES;
	a.sample_period = bm ? PERIOD / 50 : PERIOD;
	a.sample_type = PERF_SAMPLE_IP;
	a.disabled = 1;
	a.exclude_kernel = 1;
	a.exclude_hv = 1;
	const int fd = (int)syscall(__NR_perf_event_open, &a, 0, -1, -1, 0);
	if (fd < 0) { perror("perf_event_open"); return 1; }
	const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
	struct perf_event_mmap_page *mp = mmap(NULL, (PAGES + 1) * pg, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
	if (mp == MAP_FAILED) { perror("mmap"); return 1; }
	const int h265 = strlen(argv[1]) > 4 && !strcmp(argv[1] + strlen(argv[1]) - 4, ".265");
	if (h265) setenv("M2DEC_AMD_H265_THREADS", "0", 1);
	for (int r = 0; r < reps && h265; ++r) {
		h265r_backend_t be;
		memset(&be, 0, sizeof be);
		be.set_frames = n265_frames;
		be.submit = n265_submit;
		be.sync_frame = n265_sync;
		be.destroy = n265_destroy;
		int last = 0;
		ioctl(fd, PERF_EVENT_IOC_ENABLE, 0);
		const int fr = m2dec_amd_decode_h265(d, (size_t)n, &be, 0, 0, NULL, NULL, &last);
		ioctl(fd, PERF_EVENT_IOC_DISABLE, 0);
		drain(mp, base);
		fprintf(stderr, "rep %d: %d (last %d)\n", r, fr, last);
	}
	for (int r = 0; r < reps && !h265; ++r) {
		m2r_backend_t be;
		m2dec_amd_null_backend_create(&be);
		/* (one pass of the stream fits the ring: ~13k samples of 16 bytes at PERIOD) */
		ioctl(fd, PERF_EVENT_IOC_ENABLE, 0);
		const int fr = m2dec_amd_decode_stream3(d, (size_t)n, &be, 0, -1, 0, NULL, NULL, NULL);
		ioctl(fd, PERF_EVENT_IOC_DISABLE, 0);
		drain(mp, base);
		be.destroy(be.self);
		fprintf(stderr, "rep %d: %d frames\n", r, fr);
	}
	fprintf(stderr, "samples outside the library: %ld\n", other);
	for (int i = 0; i < MAXOFF; ++i)
		if (hist[i]) printf("%x %u\n", i, hist[i]);
	return 0;
}
