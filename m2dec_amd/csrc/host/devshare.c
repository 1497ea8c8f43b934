/*
 * The device-wide workgroup budget shared by every process that decodes on one GPU.
 *
 * Why (DESIGN §5 "Forward-progress invariant"): a decode-path k_picture launch has workgroups that spin on
 * row-progress words written by EARLIER launches of the same process, possibly queued on another HIP stream,
 * and the hardware may dispatch a later launch first.  The launches are therefore admitted against a budget
 * equal to the device's resident capacity for k_picture: all admitted launches fit on the device together,
 * every wait points at an earlier admitted launch, so the oldest unfinished one always runs.  The reference
 * runs one decoder process per stream (test.sh:2, `parallel src/app/h264dec -O` = one process per core), so
 * the budget has to be the DEVICE's, not the process's: two processes with private budgets could together
 * fill the device with spinners whose producers never get a slot.
 *
 * So the budget lives in a small shared-memory segment named after the GPU's PCI bus id and the owner
 * (/dev/shm/m2dec_amd.budget.<bus id>.u<uid>, mode 0600; M2DEC_AMD_SHARE_GROUP=1: .g<gid>, 0660, for several
 * users of one group on one GPU).  Each process holds one lease {pid, start time, units, contexts}; the
 * segment's total is the sum of the leases.  A robust process-shared mutex guards it (a holder that dies
 * inside the critical section leaves EOWNERDEAD: the next locker recomputes the total from the leases).
 * Liveness (round 6): each lease holder keeps an open-file-description write lock on one byte of
 * the segment file per lease (F_OFD_SETLK at offset sizeof(seg_t) + lease index).  The kernel drops it when the
 * holder dies, in any PID namespace, so a lease whose byte nobody locks is dead (a pid check would misread
 * processes of another namespace sharing /dev/shm); a dead lease is reclaimed when a reservation does not fit:
 * its launches died with their process (the driver tears down a dead process's queues).
 *
 * The segment is validated on open (magic, layout version, capacity = this device's, every lease within the
 * capacity, total = the sum of the leases) and its total on every reservation.  A segment that fails (corrupted,
 * another layout version, or every lease held by a live process) is refused LOUDLY: the back end does not
 * start, rather than silently falling back to a private budget that brings back the cross-process starvation
 * hazard.  M2DEC_AMD_SHARE=0 is the explicit opt-out (a process-local budget).
 *
 * Units: k_picture's workgroups cost ceil(M2D_SHARE_UNITS_PER_CU / resident-per-CU) units each and the
 * capacity is M2D_SHARE_UNITS_PER_CU x CUs, so contexts whose occupancy differs (LDS per picture width)
 * share one account (the runtime computes the cost per context, not a single smallest capacity).
 *
 * Host code only, no HIP: the CPU test (tests/test_devshare_cpu.py) forks processes against a segment.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include "devshare.h"

#define SHARE_MAGIC 0x6d326462u /* "m2db" */
#define SHARE_VERSION 3
#define SHARE_LEASES 256

typedef struct {
	int32_t pid;
	int32_t units;    /* workgroup units this process holds now */
	int32_t contexts; /* live decode-path back ends of this process on the device */
	int32_t wait_ms;  /* CLOCK_MONOTONIC ms (| 1) of this process's last reservation that did not fit; 0: none */
	uint64_t start;   /* /proc/<pid>/stat start time (diagnostics) */
} lease_t;

typedef struct {
	uint32_t magic, version;
	pthread_mutex_t mu;
	int32_t cap;          /* units */
	int32_t total;        /* sum of the leases' units */
	int64_t reclaimed;    /* units taken back from dead processes (diagnostics) */
	lease_t lease[SHARE_LEASES];
} seg_t;

struct m2d_share {
	seg_t *seg;
	int fd;            /* the segment file, kept open for the lease byte locks */
	int idx;           /* this process's lease */
	int32_t pid;
	uint64_t start;
	int32_t cap;       /* the capacity this process opened with */
	char path[200];
	int exited;             /* process exit dropped the lease; the mapping stays for threads still running */
	int32_t local_used;     /* after exit: reservations are accounted here, within cap */
	struct m2d_share *next; /* open handles of this process (closed at exit) */
};

static pthread_mutex_t g_open_mu = PTHREAD_MUTEX_INITIALIZER;
static m2d_share_t *g_open;

static int32_t now_ms(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (int32_t)((uint32_t)((uint64_t)ts.tv_sec * 1000u + (uint64_t)ts.tv_nsec / 1000000u) | 1u);
}

static uint64_t proc_start(int pid)
{
	char p[64], buf[1024];
	snprintf(p, sizeof p, "/proc/%d/stat", pid);
	int fd = open(p, O_RDONLY | O_CLOEXEC);
	if (fd < 0) return 0;
	ssize_t n = read(fd, buf, sizeof buf - 1);
	close(fd);
	if (n <= 0) return 0;
	buf[n] = 0;
	/* field 22 (starttime), counted after the ")" that closes the command name */
	char *s = strrchr(buf, ')');
	if (!s) return 0;
	int field = 2;
	for (; *s && field < 22; ++s)
		if (*s == ' ') ++field;
	return strtoull(s, NULL, 10);
}

static off_t lease_byte(int i) { return (off_t)sizeof(seg_t) + i; }

/* the holder of lease i is alive iff some open file description holds the write lock on its byte */
static int lease_dead(int fd, const lease_t *l, int i)
{
	if (l->pid <= 0) return 1;
	struct flock fl;
	memset(&fl, 0, sizeof fl);
	fl.l_type = F_WRLCK;
	fl.l_whence = SEEK_SET;
	fl.l_start = lease_byte(i);
	fl.l_len = 1;
	if (fcntl(fd, F_OFD_GETLK, &fl) < 0) return kill(l->pid, 0) < 0 && errno == ESRCH; /* (no OFD locks: pid) */
	return fl.l_type == F_UNLCK;
}

static int lease_lock(int fd, int i, int type)
{
	struct flock fl;
	memset(&fl, 0, sizeof fl);
	fl.l_type = (short)type;
	fl.l_whence = SEEK_SET;
	fl.l_start = lease_byte(i);
	fl.l_len = 1;
	return fcntl(fd, F_OFD_SETLK, &fl);
}

/* the layout is this version's and every field is within its range: 0 ok, else why not */
static const char *seg_check(const seg_t *g, int cap)
{
	if (__atomic_load_n(&g->magic, __ATOMIC_ACQUIRE) != SHARE_MAGIC) return "bad magic";
	if (g->version != SHARE_VERSION) return "another layout version (another m2dec_amd build decodes on this GPU)";
	if (g->cap != cap) return "capacity differs from this device's";
	int64_t sum = 0;
	for (int i = 0; i < SHARE_LEASES; ++i) {
		const lease_t *l = &g->lease[i];
		if (l->pid < 0 || l->units < 0 || l->units > g->cap || l->contexts < 0 || (!l->pid && (l->units || l->contexts)))
			return "a lease out of range";
		sum += l->units;
	}
	if (g->total != sum || g->total < 0 || g->total > g->cap) return "total is not the sum of the leases";
	return NULL;
}

static void recount(seg_t *g)
{
	int32_t t = 0;
	for (int i = 0; i < SHARE_LEASES; ++i) t += g->lease[i].units;
	g->total = t;
}

static int lock(seg_t *g)
{
	int r = pthread_mutex_lock(&g->mu);
	if (r == EOWNERDEAD) { /* the holder died inside: the leases are the truth */
		recount(g);
		pthread_mutex_consistent(&g->mu);
		r = 0;
	}
	return r;
}

/* reclaim the leases of processes that are gone; returns the units freed */
static int sweep(int fd, seg_t *g, int self)
{
	int freed = 0;
	for (int i = 0; i < SHARE_LEASES; ++i) {
		lease_t *l = &g->lease[i];
		if (i == self || l->pid == 0) continue;
		if (lease_dead(fd, l, i)) {
			freed += l->units;
			memset(l, 0, sizeof *l);
		}
	}
	if (freed) {
		g->reclaimed += freed;
		recount(g);
	}
	return freed;
}

static void seg_init(seg_t *g, int cap)
{
	memset(g, 0, sizeof *g);
	pthread_mutexattr_t at;
	pthread_mutexattr_init(&at);
	pthread_mutexattr_setpshared(&at, PTHREAD_PROCESS_SHARED);
	pthread_mutexattr_setrobust(&at, PTHREAD_MUTEX_ROBUST);
	pthread_mutex_init(&g->mu, &at);
	pthread_mutexattr_destroy(&at);
	g->cap = cap;
	g->version = SHARE_VERSION;
	__atomic_store_n(&g->magic, SHARE_MAGIC, __ATOMIC_RELEASE);
}

static seg_t *map_fd(int fd)
{
	void *p = mmap(NULL, sizeof(seg_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
	return p == MAP_FAILED ? NULL : (seg_t *)p;
}

/* Publish an initialised segment atomically: build it under a private name, then link() it to the final name
 * (fails if another process published first: then use theirs).  *fd_out: the open file (kept for the lease
 * locks).  *why: M2D_SHARE_UNAVAILABLE (no shared memory here) or M2D_SHARE_REFUSED (a file that is not a
 * valid segment of this version: checked by the caller under the lock). */
static seg_t *open_seg(const char *path, int cap, int mode, int *fd_out, int *why)
{
	*why = M2D_SHARE_UNAVAILABLE;
	for (int attempt = 0; attempt < 50; ++attempt) {
		int fd = open(path, O_RDWR | O_CLOEXEC);
		if (fd >= 0) {
			struct stat sb;
			seg_t *g = NULL;
			if (fstat(fd, &sb) == 0 && (size_t)sb.st_size >= sizeof(seg_t)) g = map_fd(fd);
			if (!g || __atomic_load_n(&g->magic, __ATOMIC_ACQUIRE) != SHARE_MAGIC) {
				if (g) munmap(g, sizeof(seg_t));
				close(fd);
				*why = M2D_SHARE_REFUSED; /* (a half-published segment is never visible: link() publishes) */
				return NULL;
			}
			*fd_out = fd;
			return g;
		}
		if (errno != ENOENT) {
			if (errno == EACCES) *why = M2D_SHARE_REFUSED; /* (someone else's file under our name) */
			return NULL;
		}
		char tmp[240];
		snprintf(tmp, sizeof tmp, "%s.%d.tmp", path, (int)getpid());
		int tfd = open(tmp, O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, (mode_t)mode);
		if (tfd < 0) return NULL;
		(void)fchmod(tfd, (mode_t)mode); /* (the umask does not widen or narrow it) */
		if (ftruncate(tfd, sizeof(seg_t)) != 0) {
			close(tfd);
			unlink(tmp);
			return NULL;
		}
		seg_t *g = map_fd(tfd);
		if (!g) {
			close(tfd);
			unlink(tmp);
			return NULL;
		}
		seg_init(g, cap);
		const int linked = link(tmp, path) == 0;
		const int link_errno = errno;
		unlink(tmp);
		if (linked) {
			*fd_out = tfd;
			return g;
		}
		munmap(g, sizeof(seg_t));
		close(tfd);
		if (link_errno != EEXIST) return NULL;
		/* lost the race: open theirs */
	}
	return NULL;
}

m2d_share_t *m2d_share_open(const char *key, int cap_units, int *why)
{
	int dummy;
	if (!why) why = &dummy;
	*why = M2D_SHARE_UNAVAILABLE;
	if (!key || cap_units <= 0) return NULL;
	m2d_share_t *s = (m2d_share_t *)calloc(1, sizeof *s);
	if (!s) return NULL;
	const char *dir = getenv("M2DEC_AMD_SHARE_DIR");
	if (!dir) dir = access("/dev/shm", W_OK) == 0 ? "/dev/shm" : "/tmp";
	const char *gm = getenv("M2DEC_AMD_SHARE_GROUP"); /* opt-in: the processes of one group share the budget */
	const int group = gm && atoi(gm);
	snprintf(s->path, sizeof s->path, "%s/m2dec_amd.budget.%s.%c%u", dir, key, group ? 'g' : 'u',
	         group ? (unsigned)getgid() : (unsigned)getuid());
	for (char *c = s->path + strlen(dir) + 1; *c; ++c)
		if (*c == '/') *c = '_';
	s->pid = (int32_t)getpid();
	s->start = proc_start(s->pid);
	s->idx = -1;
	s->fd = -1;
	s->cap = cap_units;
	seg_t *g = NULL;
	const char *bad = NULL;
	for (int attempt = 0; attempt < 50 && !g; ++attempt) {
		g = open_seg(s->path, cap_units, group ? 0660 : 0600, &s->fd, why);
		if (!g) break;
		if (lock(g) != 0) {
			munmap(g, sizeof(seg_t));
			close(s->fd);
			g = NULL;
			break;
		}
		if (g->magic != SHARE_MAGIC) { /* retired by its last user between our open and lock: open anew */
			pthread_mutex_unlock(&g->mu);
			munmap(g, sizeof(seg_t));
			close(s->fd);
			g = NULL;
			continue;
		}
		if ((bad = seg_check(g, cap_units)) != NULL) {
			pthread_mutex_unlock(&g->mu);
			munmap(g, sizeof(seg_t));
			close(s->fd);
			g = NULL;
			*why = M2D_SHARE_REFUSED;
			break;
		}
	}
	if (!g) {
		if (*why == M2D_SHARE_REFUSED)
			fprintf(stderr, "m2dec_amd: REFUSING the shared workgroup budget %s: %s.  A private budget would let another "
			        "process's waiting workgroups starve this one's (DESIGN.md §5); remove the file if no decoder uses it, "
			        "or set M2DEC_AMD_SHARE=0 to run with a process-local budget\n",
			        s->path, bad ? bad : "not a valid segment (or not ours)");
		free(s);
		return NULL;
	}
	s->seg = g;
	/* our lease: one left by this very process (a second open), else a free or dead one */
	for (int pass = 0; pass < 2 && s->idx < 0; ++pass) {
		for (int i = 0; i < SHARE_LEASES; ++i) {
			lease_t *l = &g->lease[i];
			if (pass == 0 ? (l->pid == s->pid && l->start == s->start) : l->pid == 0) {
				s->idx = i;
				break;
			}
		}
		if (s->idx < 0 && pass == 0) sweep(s->fd, g, -1);
	}
	if (s->idx >= 0 && lease_lock(s->fd, s->idx, F_WRLCK) < 0 && errno != EINVAL &&
	    g->lease[s->idx].pid != s->pid) { /* (this process's other handle holds the byte of its own lease) */
		s->idx = -1; /* a free entry whose byte a live holder still locks: the table is not trustworthy */
	}
	if (s->idx >= 0 && g->lease[s->idx].pid != s->pid) {
		lease_t *l = &g->lease[s->idx];
		memset(l, 0, sizeof *l);
		l->pid = s->pid;
		l->start = s->start;
	}
	pthread_mutex_unlock(&g->mu);
	if (s->idx < 0) {
		fprintf(stderr, "m2dec_amd: REFUSING the shared workgroup budget %s: all %d leases are held by live processes\n",
		        s->path, SHARE_LEASES);
		*why = M2D_SHARE_REFUSED;
		munmap(g, sizeof(seg_t));
		close(s->fd);
		free(s);
		return NULL;
	}
	*why = 0;
	pthread_mutex_lock(&g_open_mu);
	s->next = g_open;
	g_open = s;
	pthread_mutex_unlock(&g_open_mu);
	return s;
}

int m2d_share_try(m2d_share_t *s, int units, int *total, int *procs)
{
	if (__atomic_load_n(&s->exited, __ATOMIC_ACQUIRE)) { /* after exit: this process's own account, within cap */
		if (__atomic_add_fetch(&s->local_used, units, __ATOMIC_ACQ_REL) <= s->cap) return 1;
		__atomic_sub_fetch(&s->local_used, units, __ATOMIC_ACQ_REL);
		return 0;
	}
	seg_t *g = s->seg;
	if (lock(g) != 0) return 0;
	if (g->total < 0 || g->total > g->cap || g->cap != s->cap || g->lease[s->idx].pid != s->pid) {
		pthread_mutex_unlock(&g->mu);
		fprintf(stderr, "m2dec_amd: the shared workgroup budget %s is corrupted (cap %d, total %d): refusing to launch\n",
		        s->path, g->cap, g->total);
		return -1;
	}
	int ok = 0;
	for (int pass = 0; pass < 2; ++pass) {
		if (g->total + units <= g->cap) {
			g->lease[s->idx].units += units;
			g->total += units;
			ok = 1;
			break;
		}
		if (pass == 0 && !sweep(s->fd, g, s->idx)) break;
	}
	g->lease[s->idx].wait_ms = ok ? 0 : now_ms(); /* (m2d_share_others_waiting) */
	if (total) *total = g->total;
	if (procs) { /* processes holding units now (diagnostics: the concurrency the budget saw) */
		int np = 0;
		for (int i = 0; i < SHARE_LEASES; ++i) np += g->lease[i].pid && g->lease[i].units > 0;
		*procs = np;
	}
	pthread_mutex_unlock(&g->mu);
	return ok;
}

void m2d_share_release(m2d_share_t *s, int units)
{
	if (__atomic_load_n(&s->exited, __ATOMIC_ACQUIRE)) {
		__atomic_sub_fetch(&s->local_used, units, __ATOMIC_ACQ_REL); /* (units taken before exit were never local:
		                                                                 the account may go negative, never above cap) */
		return;
	}
	seg_t *g = s->seg;
	if (units <= 0 || lock(g) != 0) return;
	lease_t *l = &g->lease[s->idx];
	if (units > l->units) units = l->units;
	l->units -= units;
	g->total -= units;
	pthread_mutex_unlock(&g->mu);
}

/* 1 when another process's reservation did not fit within the last 100 ms (it retries every 50 us while it
 * waits): this process's reaper then returns completed launches' units at once.  Lock-free read. */
int m2d_share_others_waiting(m2d_share_t *s)
{
	if (__atomic_load_n(&s->exited, __ATOMIC_ACQUIRE)) return 0;
	const seg_t *g = s->seg;
	const int32_t now = now_ms();
	for (int i = 0; i < SHARE_LEASES; ++i) {
		if (i == s->idx) continue;
		const int32_t w = __atomic_load_n(&g->lease[i].wait_ms, __ATOMIC_RELAXED);
		if (w && (int32_t)((uint32_t)now - (uint32_t)w) < 100) return 1;
	}
	return 0;
}

int m2d_share_contexts(m2d_share_t *s, int delta)
{
	if (__atomic_load_n(&s->exited, __ATOMIC_ACQUIRE)) return 1;
	seg_t *g = s->seg;
	if (lock(g) != 0) return 1;
	g->lease[s->idx].contexts += delta;
	if (g->lease[s->idx].contexts < 0) g->lease[s->idx].contexts = 0;
	int n = 0;
	for (int i = 0; i < SHARE_LEASES; ++i)
		if (g->lease[i].pid && (i == s->idx || !lease_dead(s->fd, &g->lease[i], i))) n += g->lease[i].contexts;
	pthread_mutex_unlock(&g->mu);
	return n;
}

int m2d_share_state(m2d_share_t *s, int *cap, int *total, int *mine, int *procs, long *reclaimed)
{
	seg_t *g = s->seg;
	if (lock(g) != 0) return -1;
	int np = 0;
	for (int i = 0; i < SHARE_LEASES; ++i)
		if (g->lease[i].pid && g->lease[i].units) ++np;
	if (cap) *cap = g->cap;
	if (total) *total = g->total;
	if (mine) *mine = g->lease[s->idx].units;
	if (procs) *procs = np;
	if (reclaimed) *reclaimed = (long)g->reclaimed;
	pthread_mutex_unlock(&g->mu);
	return 0;
}

int m2d_share_cap(const m2d_share_t *s)
{
	return s->seg->cap;
}

/* drop this process's lease; the last live user retires the segment (magic cleared under the lock, so an
 * opener that mapped it meanwhile opens anew) and removes its file, so nothing is left in /dev/shm */
static void share_drop(m2d_share_t *s, int unmap)
{
	seg_t *g = s->seg;
	if (lock(g) == 0) {
		lease_t *l = &g->lease[s->idx];
		g->total -= l->units;
		memset(l, 0, sizeof *l);
		int live = 0;
		for (int i = 0; i < SHARE_LEASES; ++i)
			live += g->lease[i].pid != 0 && i != s->idx && !lease_dead(s->fd, &g->lease[i], i);
		if (!live) {
			g->magic = 0;
			unlink(s->path);
		}
		(void)lease_lock(s->fd, s->idx, F_UNLCK);
		pthread_mutex_unlock(&g->mu);
	}
	if (unmap) {
		munmap(g, sizeof(seg_t));
		close(s->fd);
	}
}

void m2d_share_close(m2d_share_t *s)
{
	if (!s) return;
	pthread_mutex_lock(&g_open_mu);
	for (m2d_share_t **p = &g_open; *p; p = &(*p)->next)
		if (*p == s) {
			*p = s->next;
			break;
		}
	pthread_mutex_unlock(&g_open_mu);
	share_drop(s, 1);
	free(s);
}

/* process exit: the runtime keeps its per-device handles for the life of the process.  The lease goes (its
 * units back to the other processes, the file removed by the last user) but the handle and its mapping stay:
 * library threads still running through exit (the budget reaper) keep using them, and any reservation after
 * this point is granted without touching the segment (the process is leaving) */
__attribute__((destructor)) static void share_exit(void)
{
	pthread_mutex_lock(&g_open_mu);
	m2d_share_t *s = g_open;
	g_open = NULL;
	pthread_mutex_unlock(&g_open_mu);
	for (; s; s = s->next) {
		__atomic_store_n(&s->exited, 1, __ATOMIC_RELEASE);
		share_drop(s, 0);
	}
}

/* ---- C-ABI for tests and diagnostics (include/m2dec_amd.h) */
void *m2dec_amd_share_open(const char *key, int cap_units) { return m2d_share_open(key, cap_units, NULL); }
void *m2dec_amd_share_open2(const char *key, int cap_units, int *why) { return m2d_share_open(key, cap_units, why); }
int m2dec_amd_share_path(void *s, char *out, int n)
{
	if (!s || !out || n <= 0) return -1;
	snprintf(out, (size_t)n, "%s", ((m2d_share_t *)s)->path);
	return 0;
}
int m2dec_amd_share_try(void *s, int units) { return s ? m2d_share_try((m2d_share_t *)s, units, NULL, NULL) : 0; }
void m2dec_amd_share_release(void *s, int units)
{
	if (s) m2d_share_release((m2d_share_t *)s, units);
}
int m2dec_amd_share_state(void *s, int *cap, int *total, int *mine, int *procs, long *reclaimed)
{
	return s ? m2d_share_state((m2d_share_t *)s, cap, total, mine, procs, reclaimed) : -1;
}
void m2dec_amd_share_close(void *s) { m2d_share_close((m2d_share_t *)s); }
int m2dec_amd_share_others_waiting(void *s) { return s ? m2d_share_others_waiting((m2d_share_t *)s) : 0; }
