/*
 * Placement of the library's own threads near the GPU a process decodes on.
 *
 * C4 / C5 at 8 GPUs run one process per GPU (bench.py under torchrun, or test.sh's decoder processes on
 * several cards).  Each process's host work — the parse pool, the MD5 helpers, the copy crews, the H.265
 * parse-ahead workers — reads the bitstream, writes the pinned record arenas the GPU uploads from, and hashes
 * the pinned staging buffers the GPU copies frames into.  Those buffers are first touched by these threads, so
 * running them on the CPUs of the GPU's NUMA node keeps the host memory of every DMA on the node the GPU's
 * PCIe root sits on, and keeps two GPUs' processes off each other's caches.
 *
 * The node comes from sysfs: /sys/bus/pci/devices/<bus id>/numa_node (the id hipDeviceGetPCIBusId gives), its
 * CPUs from /sys/devices/system/node/node<n>/cpulist, intersected with the CPUs this process may use
 * (sched_getaffinity: a container's or a launcher's cpuset wins).  An unknown node (-1, no sysfs), an empty
 * intersection, or the placement not asked for (M2DEC_AMD_NUMA=1) leaves the threads where they are.  The caller's own threads are never
 * moved: each library thread applies the placement to itself (m2d_place_self) when it starts and whenever the
 * placement changed since it last looked.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "h264_dec.h"

static pthread_mutex_t g_place_mu = PTHREAD_MUTEX_INITIALIZER;
static cpu_set_t g_place;
static int g_place_gen;      /* 0: no placement */
static int g_place_node = -1;
static __thread int t_gen;   /* the placement this thread applied */

static int read_line(const char *path, char *buf, size_t n)
{
	FILE *f = fopen(path, "r");
	if (!f) return -1;
	const int ok = fgets(buf, (int)n, f) != NULL;
	fclose(f);
	return ok ? 0 : -1;
}

/* "0-15,64-79" -> set */
static int parse_cpulist(const char *s, cpu_set_t *set)
{
	CPU_ZERO(set);
	int any = 0;
	while (*s && *s != '\n') {
		while (*s == ',' || *s == ' ') s++;
		if (!isdigit((unsigned char)*s)) break;
		char *e;
		long a = strtol(s, &e, 10), b = a;
		s = e;
		if (*s == '-') {
			b = strtol(s + 1, &e, 10);
			s = e;
		}
		for (long c = a; c <= b && c < CPU_SETSIZE; ++c) {
			CPU_SET((int)c, set);
			any = 1;
		}
	}
	return any ? 0 : -1;
}

/* keep one hardware thread per physical core (the lowest CPU of each core_cpus_list / thread_siblings_list):
 * M2DEC_AMD_NUMA_SMT=1 — two parse workers on the sibling threads of one core each run ~40 % slower */
static void one_per_core(const char *root, cpu_set_t *set)
{
	cpu_set_t keep;
	CPU_ZERO(&keep);
	for (int c = 0; c < CPU_SETSIZE; ++c) {
		if (!CPU_ISSET(c, set)) continue;
		char path[512], buf[1024];
		cpu_set_t sib;
		snprintf(path, sizeof path, "%s/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", root, c);
		if (read_line(path, buf, sizeof buf) < 0 || parse_cpulist(buf, &sib) < 0) {
			CPU_SET(c, &keep);
			continue;
		}
		int first = -1;
		for (int k = 0; k < CPU_SETSIZE && first < 0; ++k)
			if (CPU_ISSET(k, &sib) && CPU_ISSET(k, set)) first = k;
		if (first == c) CPU_SET(c, &keep);
	}
	if (CPU_COUNT(&keep)) *set = keep;
}

/* the GPU's NUMA node (or -1) and the CPUs to run on: the node's CPUs the process may use, else all it may use */
int m2d_numa_cpus(const char *root, const char *bus_id, cpu_set_t *out)
{
	char path[512], buf[4096], id[64];
	cpu_set_t allowed, node;
	CPU_ZERO(&allowed);
	if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) CPU_ZERO(&allowed);
	*out = allowed;
	if (!root) root = "";
	/* sysfs names PCI devices in lower case, with the domain */
	snprintf(id, sizeof id, "%s", bus_id ? bus_id : "");
	for (char *c = id; *c; ++c) *c = (char)tolower((unsigned char)*c);
	snprintf(path, sizeof path, "%s/sys/bus/pci/devices/%s/numa_node", root, id);
	if (read_line(path, buf, sizeof buf) < 0) return -1;
	const int n = atoi(buf);
	if (n < 0) return -1;
	snprintf(path, sizeof path, "%s/sys/devices/system/node/node%d/cpulist", root, n);
	if (read_line(path, buf, sizeof buf) < 0 || parse_cpulist(buf, &node) < 0) return -1;
	cpu_set_t both;
	CPU_AND(&both, &node, &allowed);
	if (CPU_COUNT(&both) == 0) return n; /* (the process may not use that node: stay where it may) */
	const char *smt = getenv("M2DEC_AMD_NUMA_SMT");
	if (smt && atoi(smt)) one_per_core(root, &both);
	*out = both;
	return n;
}

void m2d_place_device(const char *bus_id)
{
	/* opt-in (M2DEC_AMD_NUMA=1; bench.py sets it for its ranks when it runs on several GPUs): on the one-GPU box
	 * the unbound threads measured steadier — NUMA off 2036 / 2048 / 2046 fps, bound to the node 2084 / 2007 /
	 * 1451 (profiles/r121_ab_place.txt) */
	const char *e = getenv("M2DEC_AMD_NUMA");
	if (!e || !atoi(e)) return;
	cpu_set_t set;
	const int node = m2d_numa_cpus(getenv("M2DEC_AMD_SYSFS_ROOT"), bus_id, &set);
	pthread_mutex_lock(&g_place_mu);
	if (!g_place_gen && node >= 0) { /* the first device this process decodes on places its threads */
		g_place = set;
		g_place_node = node;
		g_place_gen = 1;
		if (getenv("M2DEC_AMD_DEBUG"))
			fprintf(stderr, "m2dec_amd: library threads on NUMA node %d (%d CPUs) for GPU %s\n", node, CPU_COUNT(&set), bus_id);
	}
	pthread_mutex_unlock(&g_place_mu);
}

void m2d_place_self(void)
{
	const int gen = __atomic_load_n(&g_place_gen, __ATOMIC_ACQUIRE);
	if (gen == t_gen) return;
	cpu_set_t set;
	pthread_mutex_lock(&g_place_mu);
	set = g_place;
	pthread_mutex_unlock(&g_place_mu);
	t_gen = gen;
	(void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

/* ---- C-ABI for tests and diagnostics */
int m2dec_amd_numa_cpus(const char *sysfs_root, const char *pci_bus_id, int *cpus, int max, int *node)
{
	cpu_set_t set;
	const int n = m2d_numa_cpus(sysfs_root, pci_bus_id, &set);
	if (node) *node = n;
	int k = 0;
	for (int c = 0; c < CPU_SETSIZE && k < max; ++c)
		if (CPU_ISSET(c, &set)) cpus[k++] = c;
	return k;
}

int m2dec_amd_numa_node(void)
{
	pthread_mutex_lock(&g_place_mu);
	const int n = g_place_gen ? g_place_node : -1;
	pthread_mutex_unlock(&g_place_mu);
	return n;
}
