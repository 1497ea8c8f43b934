/*
 * Host runtime of the gfx950 reconstruction back end: the picture scheduler, the m2r_backend_t
 * behind h264d_func (decode path), and the trace replay used by bench.py.
 *
 * Picture scheduler.  A picture is ONE launch, k_picture (inter workers + one workgroup per MB row:
 * intra, then deblocking).  Pictures depend on each other only through frame slots:
 *   - read-after-write : NOT a stream wait.  The inter workers poll the reference pictures' row
 *                        flags on the device, so a picture's motion compensation starts while its
 *                        references are still being deblocked further down;
 *   - write-after-read : a picture overwrites its destination slot only after every picture that
 *                        read the slot's previous content has finished (and after that content's
 *                        own writer and device-to-host copy): stream event waits.
 * Pictures are dealt round-robin over NSTREAMS HIP streams (one hardware queue each with the
 * default GPU_MAX_HW_QUEUES=4), each owning its scratch words and hand-off records; the frame pool,
 * the row flags and the error word are shared.  Every wait points at an earlier launch, so the
 * oldest unfinished picture can always run.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <atomic>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>
#include "recon_internal.h"
#include "m2dec_amd.h"
#include "devshare.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "m2dec_amd HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -1; } } while (0)

extern "C" void m2d_tl(int kind, long a, long b); /* timeline.c (M2DEC_AMD_TIMELINE diagnostics) */
extern "C" void m2d_place_device(const char *bus_id); /* numa.c: the library's threads near this GPU */
/* parcopy.c: a large host copy spread over a thread crew (h264_dec.h; declared here, C linkage) */
extern "C" void m2dec_par_memcpy(int crew, int n, void *const *dst, const void *const *src, const size_t *len);
enum { M2DEC_CREW_SYNC_ = 1 }; /* = M2DEC_CREW_SYNC (h264_dec.h) */

namespace {

static double wall_s()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int dbg_knob(const char *name)
{
	const char *v = getenv(name);
	return v && atoi(v);
}

const int NSTREAMS = 8; /* most launch streams of a decoder context (arrays); g_nstreams of them are used */
/* launch streams in use: one hardware queue each, the copy stream another — more streams than queues
 * share a queue and serialise their launches.  4 when the runtime has at least 5 queues (at 1080p 4 x 2
 * pictures fill the workgroup budget: profiles/r95_ab_prio_streams.txt), else 3 (HIP's default
 * GPU_MAX_HW_QUEUES=4); M2DEC_AMD_STREAMS = 1..8.  The runtime reads GPU_MAX_HW_QUEUES once, when it
 * starts, and offers no query for it: the value in the environment when the library first uses HIP is taken
 * as what the runtime got.  The library never sets it (a caller's HIP configuration is the caller's): a
 * process that wants 4 launch streams calls m2dec_amd_configure_queues() before anything uses HIP, as the
 * h264dec CLI and bench.py do. */
static int nstreams()
{
	static int n = 0;
	if (!n) {
		const char *e = getenv("M2DEC_AMD_STREAMS");
		const char *q = getenv("GPU_MAX_HW_QUEUES");
		/* one hardware queue per launch stream + one for the copy stream: 4 launch streams from 5 queues (with
		 * the per-picture grids 5 and 6 streams fit the budget too: A/Bs r104 / r105 within noise, 30.1-32.3
		 * ms per c3 decode for 4, 5 and 6) */
		int v = e ? atoi(e) : (q && atoi(q) >= 5 ? 4 : 3);
		n = v < 1 ? 1 : (v > NSTREAMS ? NSTREAMS : v);
	}
	return n;
}

const int BMAX = 4; /* at most this many pictures per decode-path launch: the back end holds submitted
                     * pictures back until the decoder flushes (the end of a burst of submits) or it holds
                     * max_held, so that pictures parsed together run in one launch */

/* Forward-progress invariant of the decode path.  A picture's workgroups spin on its references' row
 * flags, written by EARLIER launches that may sit on other HIP streams (hardware queues), and the
 * hardware may dispatch a later launch first.  If the spinning workgroups of later launches could fill
 * every workgroup slot of the device, an earlier launch would never get its workgroups dispatched.
 * So every decode-path launch in this process (all decoder contexts, all their streams) first
 * reserves its workgroup count from a device-wide budget equal to the resident-workgroup capacity of
 * k_picture (occupancy x CUs); the reservation is returned when the launch completes.  All reserved
 * launches fit on the device together, and every wait points at an earlier launch, which holds a
 * reservation too — so the oldest unfinished launch always runs.  (A replay k_batch launch is one
 * kernel whose waits point at lower block indices: in-order dispatch inside a launch.) */
struct SlotBudget {
	std::mutex mu;
	bool ready = false;
	int cap_units = 0;  /* the device's budget: M2D_SHARE_UNITS_PER_CU x CUs (devshare.h) */
	int used_local = 0; /* process-local account, when no shared segment could be opened */
	bool refused = false; /* the device's segment exists but is invalid: this process does not launch (devshare.c) */
	m2d_share_t *share = nullptr; /* the device's cross-process budget (devshare.c), normally */
	int max_procs = 0, max_total = 0; /* diagnostics: the most processes / units seen holding the budget */
	std::deque<std::pair<hipEvent_t, int>> pend; /* completion event of a launch, its units */
	std::vector<hipEvent_t> pool;
	/* with the shared budget, units go back as soon as their launch completes, by a reaper thread: another
	 * process may be waiting for them while this one makes no further launch (a test driver idle while its child
	 * decodes) */
	std::condition_variable cv;
	bool reaper_on = false;

	/* once per device: the capacity in units and the shared segment keyed by the PCI bus id
	 * (M2DEC_AMD_SHARE=0: a process-local budget, which is safe only while this is the one process
	 * decoding on the device) */
	void setup_locked(int dev)
	{
		if (ready) return;
		ready = true;
		int cus = 0;
		if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 1;
		cap_units = M2D_SHARE_UNITS_PER_CU * cus;
		const char *e = getenv("M2DEC_AMD_SHARE");
		char bus[64] = {0};
		if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, dev) != hipSuccess) bus[0] = 0;
		if (bus[0]) m2d_place_device(bus); /* (numa.c: the library's threads near this GPU) */
		if (!e || atoi(e)) {
			int why = M2D_SHARE_UNAVAILABLE;
			if (bus[0]) share = m2d_share_open(bus, cap_units, &why);
			if (share) cap_units = std::min(cap_units, m2d_share_cap(share));
			else if (why == M2D_SHARE_REFUSED) refused = true; /* (reported by devshare.c: no decode on a private budget) */
			else fprintf(stderr, "m2dec_amd: no shared workgroup budget for device %d (%s): process-local budget\n", dev, bus);
		}
	}
	void setup(int dev)
	{
		std::lock_guard<std::mutex> lk(mu);
		setup_locked(dev);
	}

	/* 1 taken, 0 not now, -1 never (a refused or corrupted segment) */
	int take(int units)
	{
		if (refused) return -1;
		if (share) {
			int total = 0, procs = 0;
			const int r = m2d_share_try(share, units, &total, &procs);
			if (r < 0) {
				refused = true;
				return -1;
			}
			const bool ok = r != 0;
			max_procs = std::max(max_procs, procs);
			if (ok) max_total = std::max(max_total, total);
			return ok ? 1 : 0;
		}
		if (used_local + units > cap_units) return 0;
		used_local += units;
		max_procs = 1;
		max_total = std::max(max_total, used_local);
		return 1;
	}
	void give(int units)
	{
		if (share) m2d_share_release(share, units);
		else used_local -= units;
	}
	void retire()
	{
		for (size_t i = 0; i < pend.size();) {
			if (hipEventQuery(pend[i].first) == hipSuccess) {
				give(pend[i].second);
				pool.push_back(pend[i].first);
				pend.erase(pend.begin() + (long)i);
			} else {
				++i;
			}
		}
	}

	/* reserve `units` (a launch's workgroups x the context's cost per workgroup, or the whole budget for a
	 * bigger launch); returns the units reserved.  Waits for this process's oldest launch when its own launches
	 * hold the budget, else (other processes', or a launch of this process between reserve and registered)
	 * polls */
	int reserve(int units)
	{
		std::unique_lock<std::mutex> lk(mu);
		const int want = std::min(units, cap_units);
		double t_wait = 0;
		for (;;) {
			retire();
			const int tk = take(want);
			if (tk < 0) return -1;
			if (tk) break;
			if (const char *lp = getenv("M2DEC_AMD_BUDGET_LOG")) { /* diagnostics: a reservation waiting long */
				const double now = wall_s();
				if (t_wait == 0) t_wait = now;
				else if (now - t_wait > 0.5) {
					int cap = 0, total = 0, mine = 0, procs = 0;
					long rec = 0;
					if (share) m2d_share_state(share, &cap, &total, &mine, &procs, &rec);
					if (FILE *f = fopen(lp, "a")) {
						fprintf(f, "pid %d: reserve %d units waits %.1f s: shared %d cap %d total %d mine %d procs %d pend %zu used_local %d\n",
						        (int)getpid(), want, now - t_wait, share != nullptr, cap, total, mine, procs, pend.size(), used_local);
						fclose(f);
					}
					t_wait = now;
				}
			}
			if (!pend.empty()) {
				hipEvent_t e = pend.front().first;
				lk.unlock();
				(void)hipEventSynchronize(e);
				lk.lock();
				continue;
			}
			lk.unlock();
			std::this_thread::sleep_for(std::chrono::microseconds(50));
			lk.lock();
		}
		return want;
	}

	hipEvent_t event()
	{
		std::lock_guard<std::mutex> lk(mu);
		hipEvent_t e = nullptr;
		if (!pool.empty()) {
			e = pool.back();
			pool.pop_back();
		} else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
			e = nullptr;
		}
		return e;
	}

	/* the launch's completion event is recorded: it returns `n` units once it fires */
	void registered(hipEvent_t e, int n)
	{
		std::lock_guard<std::mutex> lk(mu);
		pend.emplace_back(e, n);
		if (share && !reaper_on) {
			reaper_on = true;
			std::thread th([this] { reap(); });
			(void)pthread_setname_np(th.native_handle(), "m2d-reaper");
			th.detach();
		}
		cv.notify_one();
	}

	/* the reaper: while another process waits for units, returns the units of completed launches, polling the
	 * pending launches' events every 100 us (hipEventQuery); sleeps on the condition variable while nothing is
	 * pending or nobody else waits.  Not
	 * hipEventSynchronize: a thread blocked in it holds up other threads' HIP calls on that launch's stream
	 * (the first reaper serialised every submission behind the previous picture's completion: the end-to-end
	 * C3 decode fell from 31 to 72 ms, one picture per launch) */
	void reap()
	{
		std::unique_lock<std::mutex> lk(mu);
		std::vector<hipEvent_t> snap, done;
		for (;;) {
			cv.wait(lk, [this] { return !pend.empty(); });
			/* nobody else waiting: this process's own reservations retire what completed (retire()); the reaper
			 * only looks again in 2 ms — its event queries contend with the decode threads' HIP calls (r123: 8
			 * concurrent streams ~10 % slower with the reaper polling every 100 us) */
			if (!m2d_share_others_waiting(share)) {
				cv.wait_for(lk, std::chrono::milliseconds(2));
				continue;
			}
			/* the queries outside the mutex: the submitting threads reserve under it */
			snap.clear();
			for (auto &p : pend) snap.push_back(p.first);
			lk.unlock();
			done.clear();
			for (hipEvent_t e : snap)
				if (hipEventQuery(e) == hipSuccess) done.push_back(e);
			lk.lock();
			for (hipEvent_t e : done)
				for (size_t i = 0; i < pend.size(); ++i)
					if (pend[i].first == e) {
						give(pend[i].second);
						pool.push_back(e);
						pend.erase(pend.begin() + (long)i);
						break;
					}
			if (pend.empty()) continue;
			lk.unlock();
			std::this_thread::sleep_for(std::chrono::microseconds(100));
			lk.lock();
		}
	}

	void cancel(int n)
	{
		std::lock_guard<std::mutex> lk(mu);
		give(n);
	}

	/* decode-path back ends alive on the device, all processes (delta: this process's change) */
	int contexts(int delta, int local)
	{
		std::lock_guard<std::mutex> lk(mu);
		return share ? m2d_share_contexts(share, delta) : local;
	}
};

/* per device ordinal; never destroyed: a static array's destructors would run at process exit and destroy the
 * condition variable the reaper thread still waits on, and pthread_cond_destroy waits for its waiters — an
 * exit that never ends (the round-5 GPU runs' harness hang: every picture decoded, the process never exited) */
SlotBudget *const g_budget = new SlotBudget[16];

/* M2DEC_AMD_SHARE_REPORT=1: at exit, what each device's budget saw (tests/test_gpu_cli.py's concurrent-process
 * case prints it: the overlap the decoding processes had) */
__attribute__((destructor)) static void budget_report()
{
	if (!getenv("M2DEC_AMD_SHARE_REPORT")) return;
	for (int d = 0; d < 16; ++d)
		if (g_budget[d].ready)
			fprintf(stderr, "m2dec_amd budget: device %d shared %d, max processes %d, max units %d / %d\n", d,
			        g_budget[d].share != nullptr, g_budget[d].max_procs, g_budget[d].max_total, g_budget[d].cap_units);
}
std::atomic<int> g_live_backends[16]; /* decode-path back ends alive per device in this process (several pictures
                                       * per launch only for a lone stream: concurrent streams already fill the
                                       * budget) */

/* Streams and events outlive a decoder context too (creating a stream and the ~160 events of a back
 * end costs ~10 ms): released ones are kept per device and handed to the next context. */
struct HipPool {
	std::mutex mu;
	std::vector<hipStream_t> streams[16];
	std::vector<hipEvent_t> events[16][2]; /* [dev][timing] */

	hipError_t stream(int dev, hipStream_t *s)
	{
		{
			std::lock_guard<std::mutex> lk(mu);
			if (!streams[dev & 15].empty()) {
				*s = streams[dev & 15].back();
				streams[dev & 15].pop_back();
				return hipSuccess;
			}
		}
		return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
	}
	void put_stream(int dev, hipStream_t s)
	{
		if (!s) return;
		(void)hipStreamSynchronize(s);
		std::lock_guard<std::mutex> lk(mu);
		streams[dev & 15].push_back(s);
	}
	hipError_t event(int dev, bool timing, hipEvent_t *e)
	{
		{
			std::lock_guard<std::mutex> lk(mu);
			auto &v = events[dev & 15][timing];
			if (!v.empty()) {
				*e = v.back();
				v.pop_back();
				return hipSuccess;
			}
		}
		return timing ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableTiming);
	}
	void put_event(int dev, bool timing, hipEvent_t e)
	{
		if (!e) return;
		(void)hipEventSynchronize(e);
		std::lock_guard<std::mutex> lk(mu);
		events[dev & 15][timing].push_back(e);
	}
};
HipPool g_pool;

/* Device buffers outlive a decoder context as well: the picture buffers (64 x 1.5 W H, 200 MB at
 * 1080p), the hand-off records and the progress words are handed to the next context of the same
 * geometry instead of hipFree + hipMalloc (several ms per context at 1080p).  Exact-size match; at
 * most 4 GiB kept per process, least recently given out first. */
const size_t kPoolDevBytes = (size_t)4 << 30;
struct DevPool {
	std::mutex mu;
	struct Block {
		int dev;
		void *p;
		size_t n;
	};
	std::vector<Block> blocks; /* oldest given first */
	size_t kept = 0;

	hipError_t take(int dev, void **p, size_t n)
	{
		{
			std::lock_guard<std::mutex> lk(mu);
			for (size_t i = blocks.size(); i-- > 0;)
				if (blocks[i].dev == dev && blocks[i].n == n) {
					*p = blocks[i].p;
					kept -= n;
					blocks.erase(blocks.begin() + (long)i);
					return hipSuccess;
				}
		}
		return hipMalloc(p, n);
	}
	/* over the cap, the OLDEST blocks go, not the one given: a 4K stream after 1080p ones keeps its own
	 * buffers (the 1080p ones it will not take are what leaves) */
	void give(int dev, void *p, size_t n)
	{
		if (!p) return;
		std::vector<void *> drop;
		{
			std::lock_guard<std::mutex> lk(mu);
			if (n <= kPoolDevBytes) {
				while (!blocks.empty() && kept + n > kPoolDevBytes) {
					drop.push_back(blocks.front().p);
					kept -= blocks.front().n;
					blocks.erase(blocks.begin());
				}
				blocks.push_back({dev, p, n});
				kept += n;
				p = nullptr;
			}
		}
		for (void *q : drop) (void)hipFree(q);
		if (p) (void)hipFree(p);
	}
} g_dev;

/* Host ranges page-locked for the life of the process (m2dec_amd_hip_pin: the stream driver's pooled
 * frame memory).  set_frames does not register frames inside them again — a new stream reuses the
 * pool's frames without ~0.15 ms of pinning per frame. */
struct PinCache {
	std::mutex mu;
	std::vector<std::pair<const uint8_t *, size_t>> ranges;
	bool covers(const uint8_t *p, size_t n)
	{
		std::lock_guard<std::mutex> lk(mu);
		for (auto &r : ranges)
			if (p >= r.first && p + n <= r.first + r.second) return true;
		return false;
	}
} g_pins;
const int NEVENTS = 4096; /* recycled sync events: far more than the pictures a dependency can span */

struct RecPtrs {
	const m2r_mb_t *mb;
	const m2r_deblock_t *dbk;
	const m2r_slice_t *sl;
	const m2r_inter_t *it;
	const int16_t *coef;
};

/* per-picture launch description */
struct PicJob {
	RecPtrs r;
	int slot, n_inter, n_intra, deblock;
	uint64_t refs; /* bit per reference slot read by k_inter */
};

struct Sched {
	int dev = 0;
	int W = 0, H = 0, Wmb = 0, Hmb = 0, nslots = 0;
	size_t fsz = 0;
	uint8_t *frames = nullptr; /* device frame pool [nslots] x fsz */
	hipStream_t st[NSTREAMS] = {}; /* per in-flight index: uploads, k_picture, downloads */
	int *prog = nullptr;       /* [NSTREAMS] x (completion counters [2 BMAX], scratch [BMAX][SCR_WORDS]) */
	PictureArgs *pargs = nullptr; /* [NSTREAMS][BMAX] kernel arguments of the decode-path launches */
	uint8_t *hand = nullptr;   /* [NSTREAMS * BMAX][hand_bytes()] hand-off records */
	int *err = nullptr;
	unsigned long long *rowflag = nullptr; /* [ROWFLAG_N][Hmb]: ROWFLAG(seq, MB columns final) per picture row */
	int seq = 0;               /* pictures launched */
	SlotSeq slot_seq;          /* seq + 1 of the picture held by each slot */
	int inter_grid = 80;       /* persistent inter workers per picture (5/16 of the CUs) */
	int row_wgs = 16;          /* row-pair workgroups of a P / B picture (pairs taken from a queue); r133 sweep on
	                            * the round-5 kernels: 8 / 12 / 16 / 20 / 24 -> replay ~6800 / 7640 / 7745 / 7615 /
	                            * 7590 fps, c3 decode median 30.06 (12) vs 29.49 ms (16), profiles/r133_sweep_replay_grid.txt */
	int rr = 0;
	int pics_fit = 1;          /* pictures per decode-path launch that keep NSTREAMS launches within the budget */
	int resident_per_cu = 0;   /* k_picture workgroups resident per CU at this geometry */
	int wg_units = 0;          /* budget units per k_picture workgroup (SlotBudget, devshare.h) */
	int cap_wg = 0;            /* k_picture workgroups the device holds at once at this geometry */
	hipEvent_t busy[NSTREAMS] = {}; /* recorded behind each decode-path launch on the stream (its own event) */
	bool busy_set[NSTREAMS] = {};
	hipEvent_t ev[NEVENTS] = {};
	int ev_next = 0;
	hipEvent_t slot_write[64] = {};
	std::vector<hipEvent_t> readers[64];
	size_t lds_set = 0;
	m2dec_amd_hip_timing_t tm;

	int init(int device)
	{
		dev = device;
		memset(&tm, 0, sizeof(tm));
		CHECK(hipSetDevice(dev));
		for (int k = 0; k < nstreams(); ++k) {
			CHECK(g_pool.stream(dev, &st[k])); /* (the rest stay null) */
			CHECK(g_pool.event(dev, false, &busy[k]));
		}
		CHECK(hipMalloc(&err, 16)); /* [0] a failed hand-off, [1] a reported slow one (the sync events: next_event) */
		CHECK(hipMemset(err, 0, 16));
		if (const char *e = getenv("M2DEC_AMD_SPIN_REPORT")) /* (tests: force the slow-wait path) */
			if (atoi(e) > 0 && m2dec_amd_hip_set_spin_report((unsigned)atoi(e)) < 0) return -1;
		memset(&slot_seq, 0, sizeof(slot_seq));
		int cus = 0;
		if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
			inter_grid = cus * 5 / 16; /* 80 on MI355X (sweep at 4 waves per SIMD: 64 -> 80 +3 %, 96+ slower) */
		if (const char *g = getenv("M2DEC_AMD_INTER_WG")) /* tuning knob: inter workers per picture */
			if (atoi(g) > 0) inter_grid = atoi(g);
		if (const char *g = getenv("M2DEC_AMD_ROW_WG")) /* tuning knob: row-pair workgroups of a P / B picture */
			if (atoi(g) > 0) row_wgs = atoi(g);
		return 0;
	}

	/* (re)size the frame pool and per-stream scratch */
	int configure(int width, int height, int n)
	{
		CHECK(hipSetDevice(dev));
		for (auto &s : st)
			if (s) CHECK(hipStreamSynchronize(s));
		size_t nfsz = ((size_t)width * height * 3 / 2 + 4095) & ~(size_t)4095;
		if (frames && (nfsz != fsz || n > nslots)) {
			g_dev.give(dev, frames, fsz * (size_t)nslots);
			frames = nullptr;
		}
		if (!frames) {
			CHECK(g_dev.take(dev, (void **)&frames, nfsz * (size_t)n));
			CHECK(hipMemsetAsync(frames, 0, nfsz * (size_t)n, st[0])); /* (a pooled buffer holds another stream's pictures) */
			nslots = n;
		}
		if (prog && (width / 16 != Wmb || height / 16 != Hmb)) {
			batch_free();
			g_dev.give(dev, prog, prog_bytes());
			g_dev.give(dev, hand, hand_bytes() * NSTREAMS * BMAX);
			g_dev.give(dev, rowflag, rowflag_bytes());
			prog = nullptr;
			hand = nullptr;
			rowflag = nullptr;
		}
		W = width;
		H = height;
		Wmb = width / 16;
		Hmb = height / 16;
		fsz = nfsz;
		if (!prog) {
			CHECK(g_dev.take(dev, (void **)&prog, prog_bytes()));
			if (!pargs) CHECK(hipMalloc(&pargs, sizeof(PictureArgs) * NSTREAMS * BMAX));
			CHECK(g_dev.take(dev, (void **)&hand, hand_bytes() * NSTREAMS * BMAX));
			CHECK(g_dev.take(dev, (void **)&rowflag, rowflag_bytes()));
		}
		CHECK(hipMemsetAsync(rowflag, 0, rowflag_bytes(), st[0]));
		/* the I-picture hand-off words carry a tag derived from seq, which restarts here: no word of an
		 * earlier picture (or decoder) may be left holding a tag a new picture will use */
		CHECK(hipMemsetAsync(hand, 0, hand_bytes() * NSTREAMS * BMAX, st[0]));
		if (bt.hand) CHECK(hipMemsetAsync(bt.hand, 0, hand_bytes() * (size_t)bt.cap, st[0]));
		CHECK(hipStreamSynchronize(st[0]));
		seq = 0;
		memset(&slot_seq, 0, sizeof(slot_seq));
		for (int i = 0; i < 64; ++i) {
			slot_write[i] = nullptr;
			readers[i].clear();
		}
		size_t lds = m2r_deblock_lds_bytes(W, Wmb);
		if (lds > 65536 && lds > lds_set) {
			CHECK(hipFuncSetAttribute((const void *)k_batch, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
			CHECK(hipFuncSetAttribute((const void *)k_picture, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
			lds_set = lds;
		}
		{
			/* resident-workgroup capacity of k_picture at THIS picture size (its LDS sets the occupancy): the
			 * cost of one of its workgroups in the device budget, and the capacity this context plans with.
			 * Per context: another context's geometry (a 4K one before a 1080p one) changes neither. */
			int per_cu = 0, cus = 0;
			CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_picture, 256, lds));
			CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
			per_cu = std::max(1, per_cu);
			g_budget[dev & 15].setup(dev);
			if (g_budget[dev & 15].refused) return -1; /* (devshare.c printed why) */
			resident_per_cu = per_cu;
			wg_units = (M2D_SHARE_UNITS_PER_CU + per_cu - 1) / per_cu;
			cap_wg = std::max(1, std::min(per_cu * std::max(1, cus), g_budget[dev & 15].cap_units / wg_units));
			/* pictures per launch such that a launch on each stream fits the budget at once: a reserve
			 * that has to wait would stall the thread driving the pipeline (a parse worker) */
			pics_fit = std::max(1, std::min(BMAX, cap_wg / (nstreams() * picture_blocks_dp(inter_grid, row_wgs, Hmb, true))));
			if (dbg_knob("M2DEC_AMD_DEBUG"))
				fprintf(stderr, "k_picture: %d workgroups resident (%d per CU, %d units each), %d pictures per launch fit\n",
				        cap_wg, per_cu, wg_units, pics_fit);
		}
		return 0;
	}

	size_t hand_bytes() const { return (size_t)Hmb * Wmb * (HBI_BYTES + HBD_BYTES) + (size_t)Hmb * NSEG(Wmb) * 8 * HBP_BYTES; }
	size_t stream_words() const { return 2 * BMAX + (size_t)BMAX * SCR_WORDS(Hmb, Wmb); }
	size_t prog_bytes() const { return sizeof(int) * stream_words() * NSTREAMS; }
	size_t rowflag_bytes() const { return sizeof(unsigned long long) * ROWFLAG_N * (size_t)Hmb; }

	hipEvent_t next_event()
	{
		if (!ev[ev_next] && g_pool.event(dev, false, &ev[ev_next]) != hipSuccess) return nullptr;
		hipEvent_t e = ev[ev_next];
		ev_next = (ev_next + 1) % NEVENTS;
		return e;
	}

	/* pick a stream for a picture writing `slot`; enqueue its write-after-read / write-after-write
	 * waits.  Read-after-write on the reference slots is NOT a stream wait: k_inter polls the
	 * references' row flags on the device, so it overlaps their deblocking. */
	int begin(int slot, uint64_t refs)
	{
		const int k = pick();
		return waits(k, slot, refs) < 0 ? -1 : k;
	}

	/* the stream of the next launch: the first idle one after the last pick, else round robin */
	int pick()
	{
		const int n = nstreams();
		int k = rr;
		for (int i = 0; i < n; ++i) {
			const int c = (rr + i) % n;
			if (idle(c)) {
				k = c;
				break;
			}
		}
		rr = (k + 1) % n;
		return k;
	}

	/* no decode-path launch of this context still runs on stream k */
	bool idle(int k) { return !busy_set[k] || hipEventQuery(busy[k]) == hipSuccess; }

	bool any_idle()
	{
		for (int k = 0; k < nstreams(); ++k)
			if (idle(k)) return true;
		return false;
	}

	int mark_busy(int k)
	{
		CHECK(hipEventRecord(busy[k], st[k]));
		busy_set[k] = true;
		return 0;
	}

	/* on stream k, before a picture writing `slot` (launched in a later call on k): the waits for the
	 * launches that read or wrote the slot's previous content (pictures of the same launch are ordered on
	 * the device instead: war / war_writer) */
	int waits(int k, int slot, uint64_t refs)
	{
		(void)refs;
		hipStream_t s = st[k];
		for (hipEvent_t e : readers[slot]) CHECK(hipStreamWaitEvent(s, e, 0));
		if (slot_write[slot]) CHECK(hipStreamWaitEvent(s, slot_write[slot], 0));
		if (dbg_knob("M2DEC_AMD_RAW"))
			for (int i = 0; i < 64; ++i)
				if (((refs >> i) & 1) && slot_write[i]) CHECK(hipStreamWaitEvent(st[k], slot_write[i], 0));
		if (dbg_knob("M2DEC_AMD_SYNC")) CHECK(hipDeviceSynchronize());
		return 0;
	}

	/* n (<= BMAX) pictures in decode order = one k_picture launch on stream k (waits() done for each);
	 * tev (optional): [0] recorded after it; inter_done: the event after which the pictures' reference
	 * reads are over.  Inside the launch a picture that overwrites a slot an earlier one of the launch
	 * read or wrote waits for it on the device (war / war_writer on the completion counters), as in a
	 * replay batch; workgroups are dispatched in block order, so every such wait points backwards. */
	int launch_multi(int k, const PicJob *jobs, int n, hipEvent_t *tev, hipEvent_t *inter_done, hipEvent_t *tstart = nullptr,
	                 bool slot_waits = false)
	{
		if (n < 1 || n > BMAX) return -1;
		hipStream_t s = st[k];
		PictureArgs ha[BMAX];
		if (dbg_knob("M2DEC_AMD_DEBUG")) fprintf(stderr, "launch_multi: stream %d, %d pictures, seq %d\n", k, n, seq);
		int *words = prog + (size_t)k * stream_words();
		int last_writer[64];
		int rd[64][BMAX], nrd[64];
		for (int i = 0; i < 64; ++i) last_writer[i] = -1, nrd[i] = 0;
		for (int p = 0; p < n; ++p) {
			const PicJob &j = jobs[p];
			PictureArgs &a = ha[p];
			memset(&a, 0, sizeof(a));
			a.mbs = j.r.mb;
			a.inters = j.r.it;
			a.slices = j.r.sl;
			a.pool = j.r.coef;
			a.dbk = j.r.dbk;
			a.frames = frames;
			a.fsz = fsz;
			a.W = W;
			a.H = H;
			a.Wmb = Wmb;
			a.Hmb = Hmb;
			a.slot = j.slot;
			a.seq = seq++;
			a.n_inter = j.n_inter;
			a.n_intra = j.n_intra;
			a.inter_workers = inter_grid;
			a.row_wgs = row_wgs;
			a.scratch = words + 2 * BMAX + (size_t)p * SCR_WORDS(Hmb, Wmb);
			a.hbi = hand + ((size_t)k * BMAX + p) * hand_bytes();
			a.hbd = a.hbi + (size_t)Hmb * Wmb * HBI_BYTES;
			a.hbp = a.hbd + (size_t)Hmb * Wmb * HBD_BYTES;
			a.rowflag = rowflag;
			a.err = err;
			a.ss = slot_seq;
			a.fin = words;
			a.pidx = p;
			a.didx = p;
			a.n_war = nrd[j.slot];
			for (int i = 0; i < a.n_war; ++i) a.war[i] = rd[j.slot][i];
			a.war_writer = last_writer[j.slot];
			nrd[j.slot] = 0;
			last_writer[j.slot] = p;
			for (int r = 0; r < 64; ++r)
				if ((j.refs >> r) & 1) rd[r][nrd[r]++] = p;
			slot_seq.s[j.slot] = a.seq + 1;
			tm.inter_launches += j.n_inter ? 1 : 0;
			tm.intra_launches += j.n_intra ? 1 : 0;
			tm.deblock_launches++;
		}
		hoist_intra(ha, n);
		int nb = 0; /* the launch's workgroups: each picture's own (picture_blocks_dp), in dispatch order */
		for (int p = 0; p < n; ++p) {
			ha[p].blk0 = nb;
			ha[p].nblk = picture_blocks_dp(inter_grid, row_wgs, Hmb, ha[p].n_inter != 0);
			nb += ha[p].nblk;
		}
		CHECK(hipMemsetAsync(words, 0, sizeof(int) * (2 * BMAX + (size_t)n * SCR_WORDS(Hmb, Wmb)), s));
		/* the arguments go to device memory (pageable source: staged by the copy call) */
		CHECK(hipMemcpyAsync(pargs + (size_t)k * BMAX, ha, sizeof(PictureArgs) * n, hipMemcpyHostToDevice, s));
		/* slot_waits: the pictures' write-after-read / -write waits go in here, after the copies — a copy behind a
		 * wait on another stream's launch can hold this thread until that launch completes (round-5 H.265
		 * trace: a 4 MB record upload behind such waits returned after 8-10 ms) */
		if (slot_waits)
			for (int p = 0; p < n; ++p)
				if (waits(k, jobs[p].slot, jobs[p].refs) < 0) return -1;
		{
			/* the device-wide workgroup budget (SlotBudget): reserve, launch, register the release */
			SlotBudget &bg = g_budget[dev & 15];
			hipEvent_t done = bg.event();
			if (!done) return -1;
			const int held = bg.reserve(nb * std::max(1, wg_units));
			if (held < 0) return -1; /* (a refused / corrupted shared budget: reported by devshare.c) */
			if (tstart) CHECK(hipEventRecord(*tstart, s)); /* (decode path: TimingSlot e[3], the kernel's start) */
			hipLaunchKernelGGL(k_picture, dim3(nb), dim3(256), m2r_deblock_lds_bytes(W, Wmb), s,
			                   (const PictureArgs *)(pargs + (size_t)k * BMAX), n);
			if (hipGetLastError() != hipSuccess || hipEventRecord(done, s) != hipSuccess) {
				bg.cancel(held);
				fprintf(stderr, "m2dec_amd: k_picture launch failed\n");
				return -1;
			}
			bg.registered(done, held);
		}
		*inter_done = next_event();
		CHECK(hipEventRecord(*inter_done, s));
		if (tev) CHECK(hipEventRecord(tev[0], s));
		return 0;
	}

	int launch(int k, const PicJob &j, hipEvent_t *tev, hipEvent_t *inter_done)
	{
		return launch_multi(k, &j, 1, tev, inter_done);
	}

	/* ---- batch launches (trace replay): one k_batch per run of pictures, slot reuse ordered on the
	 * device (PictureArgs.war / war_writer), everything on stream 0 */
	struct Batch {
		int cap = 0;                 /* pictures */
		int *words = nullptr;        /* [2 cap] completion counters, then [cap][SCR_WORDS] scratch */
		uint8_t *hand = nullptr;     /* [cap][hand_bytes] */
		static const int NB = 4;
		PictureArgs *d_args[NB] = {}, *h_args[NB] = {};
		hipEvent_t used[NB] = {};
		int next = 0;
	} bt;

	int batch_reserve(int cap)
	{
		if (cap <= bt.cap) return 0;
		batch_free();
		CHECK(hipMalloc(&bt.words, sizeof(int) * ((size_t)2 * cap + (size_t)cap * SCR_WORDS(Hmb, Wmb))));
		CHECK(hipMalloc(&bt.hand, hand_bytes() * (size_t)cap));
		CHECK(hipMemset(bt.hand, 0, hand_bytes() * (size_t)cap)); /* tags: see the geometry setup */
		for (int i = 0; i < Batch::NB; ++i) {
			CHECK(hipMalloc(&bt.d_args[i], sizeof(PictureArgs) * cap));
			CHECK(hipHostMalloc((void **)&bt.h_args[i], sizeof(PictureArgs) * cap, hipHostMallocDefault));
			CHECK(hipEventCreateWithFlags(&bt.used[i], hipEventDisableTiming));
		}
		bt.cap = cap;
		return 0;
	}

	void batch_free()
	{
		if (bt.words) (void)hipFree(bt.words);
		if (bt.hand) (void)hipFree(bt.hand);
		for (int i = 0; i < Batch::NB; ++i) {
			if (bt.d_args[i]) (void)hipFree(bt.d_args[i]);
			if (bt.h_args[i]) (void)hipHostFree(bt.h_args[i]);
			if (bt.used[i]) (void)hipEventDestroy(bt.used[i]);
			bt.d_args[i] = bt.h_args[i] = nullptr;
			bt.used[i] = nullptr;
		}
		bt.words = nullptr;
		bt.hand = nullptr;
		bt.cap = 0;
	}

	/* Dispatch order inside a batch.  Workgroups are dispatched in block order, so a picture starts
	 * only once every earlier picture's blocks are resident.  An intra-only picture reads no
	 * reference: it only has to follow the pictures that read its slot's previous content and that
	 * content's writer.  Move each one up to right after those (its seq, and so every reference
	 * relation, stays in decode order), so that an I picture — the longest wavefront of a GOP —
	 * overlaps the previous GOP's tail instead of starting after it.  Every wait still points at a
	 * lower dispatch position: no deadlock.  a[] is in decode order on entry, dispatch order on exit. */
	void hoist_intra(PictureArgs *a, int n)
	{
		if (getenv("M2DEC_AMD_NO_HOIST")) return;
		std::vector<int> order(n), pos(n);
		for (int i = 0; i < n; ++i) order[i] = i;
		for (int p = 0; p < n; ++p) {
			if (a[p].n_inter) continue;
			for (int i = 0; i < n; ++i) pos[order[i]] = i;
			int e = 0;
			for (int i = 0; i < a[p].n_war; ++i) e = std::max(e, pos[a[p].war[i]] + 1);
			if (a[p].war_writer >= 0) e = std::max(e, pos[a[p].war_writer] + 1);
			const int cur = pos[p];
			if (e >= cur) continue;
			order.erase(order.begin() + cur);
			order.insert(order.begin() + e, p);
		}
		for (int i = 0; i < n; ++i) pos[order[i]] = i;
		std::vector<PictureArgs> b(a, a + n);
		for (int i = 0; i < n; ++i) {
			PictureArgs &d = a[i];
			d = b[order[i]];
			d.pidx = i;
			for (int k = 0; k < d.n_war; ++k) d.war[k] = pos[d.war[k]];
			if (d.war_writer >= 0) d.war_writer = pos[d.war_writer];
		}
	}

	/* launch up to n pictures as one k_batch on stream 0 (fewer if a slot's readers would exceed
	 * WAR_MAX); capture: verification copy-out area [n][fsz] or null.  Returns the pictures taken. */
	int launch_batch(const PicJob *jobs, int n, uint8_t *capture)
	{
		if (n > bt.cap) return -1;
		hipStream_t s = st[0];
		const int idx = bt.next;
		bt.next = (bt.next + 1) % Batch::NB;
		CHECK(hipEventSynchronize(bt.used[idx])); /* its host / device argument arrays are free again */
		PictureArgs *ha = bt.h_args[idx];
		int last_writer[64];
		std::vector<int> rd[64];
		for (int i = 0; i < 64; ++i) last_writer[i] = -1;
		int taken = 0;
		for (int p = 0; p < n; ++p) {
			const PicJob &j = jobs[p];
			if ((int)rd[j.slot].size() > WAR_MAX) break;
			PictureArgs &a = ha[p];
			memset(&a, 0, sizeof(a));
			a.mbs = j.r.mb;
			a.inters = j.r.it;
			a.slices = j.r.sl;
			a.pool = j.r.coef;
			a.dbk = j.r.dbk;
			a.frames = frames;
			a.fsz = fsz;
			a.W = W;
			a.H = H;
			a.Wmb = Wmb;
			a.Hmb = Hmb;
			a.slot = j.slot;
			a.seq = seq++;
			a.n_inter = j.n_inter;
			a.n_intra = j.n_intra;
			a.inter_workers = inter_grid;
			a.row_wgs = row_wgs;
		a.row_wgs = row_wgs;
			a.scratch = bt.words + 2 * (size_t)bt.cap + (size_t)p * SCR_WORDS(Hmb, Wmb);
			a.hbi = bt.hand + (size_t)p * hand_bytes();
			a.hbd = a.hbi + (size_t)Hmb * Wmb * HBI_BYTES;
			a.hbp = a.hbd + (size_t)Hmb * Wmb * HBD_BYTES;
			a.rowflag = rowflag;
			a.err = err;
			a.ss = slot_seq;
			a.fin = bt.words;
			a.pidx = p;
			a.didx = p;
			a.n_war = (int)rd[j.slot].size();
			for (int i = 0; i < a.n_war; ++i) a.war[i] = rd[j.slot][i];
			a.war_writer = last_writer[j.slot];
			a.capture = capture ? capture + (size_t)p * fsz : nullptr;
			rd[j.slot].clear();
			last_writer[j.slot] = p;
			for (int r = 0; r < 64; ++r)
				if ((j.refs >> r) & 1) rd[r].push_back(p);
			slot_seq.s[j.slot] = a.seq + 1;
			tm.inter_launches += j.n_inter ? 1 : 0;
			tm.intra_launches += j.n_intra ? 1 : 0;
			tm.deblock_launches++;
			taken++;
		}
		if (!taken) return -1;
		hoist_intra(ha, taken);
		CHECK(hipMemcpyAsync(bt.d_args[idx], ha, sizeof(PictureArgs) * taken, hipMemcpyHostToDevice, s));
		CHECK(hipMemsetAsync(bt.words, 0, sizeof(int) * (2 * (size_t)bt.cap + (size_t)taken * SCR_WORDS(Hmb, Wmb)), s));
		const int bpp = picture_blocks(inter_grid, Hmb);
		hipLaunchKernelGGL(k_batch, dim3(bpp * taken), dim3(256), m2r_deblock_lds_bytes(W, Wmb), s, (const PictureArgs *)bt.d_args[idx], bpp);
		CHECK(hipGetLastError());
		CHECK(hipEventRecord(bt.used[idx], s));
		return taken;
	}

	/* after everything that touches the picture's slot on stream k was enqueued (incl. any copy) */
	int end(int k, const PicJob &j, hipEvent_t inter_done)
	{
		hipEvent_t w = next_event();
		CHECK(hipEventRecord(w, st[k]));
		for (int r = 0; r < 64; ++r)
			if ((j.refs >> r) & 1) readers[r].push_back(inter_done);
		readers[j.slot].clear();
		slot_write[j.slot] = w;
		return 0;
	}

	int sync_all()
	{
		CHECK(hipSetDevice(dev));
		for (auto &s : st)
			if (s) CHECK(hipStreamSynchronize(s));
		return 0;
	}

	bool stall_told = false;
	int check_err()
	{
		int e[2] = {0, 0};
		CHECK(hipMemcpy(e, err, sizeof(e), hipMemcpyDeviceToHost));
		if (e[1] && !stall_told) {
			stall_told = true;
			fprintf(stderr, "m2dec_amd: device %d: a wavefront hand-off waited past the report threshold (code %d; the GPU "
			        "is shared with other work?) — waited on, the decode goes on\n", dev, e[1]);
		}
		if (e[0]) {
			fprintf(stderr, "m2dec_amd: wavefront hand-off failed (err=%d)\n", e[0]);
			return -1;
		}
		return 0;
	}

	void destroy()
	{
		(void)hipSetDevice(dev);
		for (auto &s : st)
			if (s) (void)hipStreamSynchronize(s);
		batch_free();
		for (auto &s : st)
			if (s) (void)hipStreamSynchronize(s);
		for (auto &e : ev) {
			g_pool.put_event(dev, false, e);
			e = nullptr;
		}
		for (auto &e : busy) {
			if (e) g_pool.put_event(dev, false, e);
			e = nullptr;
		}
		g_dev.give(dev, frames, fsz * (size_t)nslots);
		if (prog) g_dev.give(dev, prog, prog_bytes());
		if (hand) g_dev.give(dev, hand, hand_bytes() * NSTREAMS * BMAX);
		if (rowflag) g_dev.give(dev, rowflag, rowflag_bytes());
		if (pargs) (void)hipFree(pargs);
		if (err) (void)hipFree(err);
		frames = nullptr;
		prog = nullptr;
		hand = nullptr;
		rowflag = nullptr;
		for (auto &s : st) {
			g_pool.put_stream(dev, s);
			s = nullptr;
		}
	}
};

uint64_t refs_of(const m2r_inter_t *it, int n)
{
	uint64_t m = 0;
	for (int i = 0; i < n; ++i)
		for (int l = 0; l < 2; ++l)
			for (int b = 0; b < 4; ++b)
				if (it[i].slot[l][b] >= 0) m |= 1ull << (it[i].slot[l][b] & 63);
	return m;
}

int64_t ref_bytes_of(const m2r_inter_t *it, int n)
{
	/* algorithmic MC input: one reference byte per predicted sample per list */
	int64_t s = 0;
	for (int i = 0; i < n; ++i)
		for (int l = 0; l < 2; ++l)
			for (int b = 0; b < 4; ++b)
				if (it[i].slot[l][b] >= 0) s += 64 + 32;
	return s;
}

/* pinned host memory for the parser's record arenas (h264_async.c job_arena: uploaded in place,
 * M2R_PIC_EXTERNAL); portable, so any device's back end may read it.  NULL without a device. */
extern "C" void *m2dec_amd_pinned_alloc(size_t n)
{
	void *p = nullptr;
	if (hipHostMalloc(&p, n, hipHostMallocPortable) != hipSuccess) return nullptr;
	return p;
}

extern "C" void m2dec_amd_pinned_free(void *p)
{
	if (p) (void)hipHostFree(p);
}

/* ======================================================================== decode-path back end */
const int kSlicesCap = 64;
const int kArenas = NSTREAMS * BMAX + BMAX + 2; /* at most: launched + held pictures, and the one being filled */

struct Arena {
	m2r_picture_t pic;
	uint8_t *host = nullptr, *dev = nullptr;
	size_t size = 0, off_mb = 0, off_dbk = 0, off_slice = 0, off_inter = 0, off_coef = 0;
	hipEvent_t consumed = nullptr; /* the picture's kernels finished reading the device copy */
	bool pending = false;
	bool held = false;             /* submitted, not launched yet */
	const uint8_t *ext = nullptr;  /* M2R_PIC_EXTERNAL: the parser's records the upload reads (else `host`) */
};

/* Pinned record arenas (+ their device twins) outlive a decoder context: a process decoding stream
 * after stream (a transcoding service, bench.py's steps) reuses them instead of pinning 8 MB per
 * arena per stream (~2 ms each on the MI355X host). */
struct ArenaPool {
	struct Block {
		int dev;
		uint8_t *host, *dev_ptr;
		size_t size;
	};
	std::mutex mu;
	std::vector<Block> free_blocks; /* oldest given first */
	size_t kept = 0;

	/* the smallest block that fits (a 1080p context does not take a 4K stream's arenas), newest of those */
	bool take(int dev, size_t need, Arena &a)
	{
		std::lock_guard<std::mutex> lk(mu);
		long best = -1;
		for (size_t i = free_blocks.size(); i-- > 0;)
			if (free_blocks[i].dev == dev && free_blocks[i].size >= need && (best < 0 || free_blocks[i].size < free_blocks[(size_t)best].size))
				best = (long)i;
		if (best < 0) return false;
		const Block bl = free_blocks[(size_t)best];
		free_blocks.erase(free_blocks.begin() + best);
		kept -= bl.size;
		a.host = bl.host;
		a.dev = bl.dev_ptr;
		a.size = bl.size;
		return true;
	}

	/* at most 64 blocks / 2 GiB (page-locked + the same in HBM); over that the OLDEST go, not the one given (r5:
	 * after the 8-stream leg's 64 1080p arenas filled the pool, each 4K decode pinned 6 new 34 MB arenas at
	 * 5-13 ms apiece and freed them at its end: C5 80-105 ms per decode instead of 50) */
	void give(int dev, Arena &a)
	{
		if (!a.host) return;
		const size_t cap = (size_t)2 << 30;
		std::vector<Block> drop;
		{
			std::lock_guard<std::mutex> lk(mu);
			if (a.size <= cap) {
				while (!free_blocks.empty() && (free_blocks.size() >= 64 || kept + a.size > cap)) {
					drop.push_back(free_blocks.front());
					kept -= free_blocks.front().size;
					free_blocks.erase(free_blocks.begin());
				}
				free_blocks.push_back({dev, a.host, a.dev, a.size});
				kept += a.size;
				a.host = a.dev = nullptr;
				a.size = 0;
			}
		}
		for (auto &bl : drop) {
			(void)hipHostFree(bl.host);
			(void)hipFree(bl.dev_ptr);
		}
		if (a.host) {
			(void)hipHostFree(a.host);
			(void)hipFree(a.dev);
			a.host = a.dev = nullptr;
			a.size = 0;
		}
	}
};
ArenaPool g_arenas;

struct TimingSlot {
	hipEvent_t e[6]; /* start, uploaded, after the kernel, right before the kernel, (unused), end */
	bool pending = false;
};

/* Pinned staging buffers for the frames on their way to the caller (one NV12 picture each), kept
 * per process: a decoder context takes them as pictures are bound and gives them back when the
 * caller has the frame. */
struct StagePool {
	std::mutex mu;
	std::vector<std::pair<uint8_t *, size_t>> free_blocks; /* oldest given first */
	size_t kept = 0;

	uint8_t *take(size_t need)
	{
		{
			std::lock_guard<std::mutex> lk(mu);
			for (size_t i = free_blocks.size(); i-- > 0;)
				if (free_blocks[i].second == need) {
					uint8_t *p = free_blocks[i].first;
					free_blocks.erase(free_blocks.begin() + (long)i);
					kept -= need;
					return p;
				}
		}
		void *p = nullptr;
		if (hipHostMalloc(&p, need, hipHostMallocDefault) != hipSuccess) return nullptr;
		return (uint8_t *)p;
	}
	/* up to 1 GiB kept for the next contexts; over that the OLDEST blocks go, not the one given */
	void give(uint8_t *p, size_t n)
	{
		if (!p) return;
		const size_t cap = (size_t)1 << 30;
		std::vector<uint8_t *> drop;
		{
			std::lock_guard<std::mutex> lk(mu);
			if (n <= cap) {
				while (!free_blocks.empty() && kept + n > cap) {
					drop.push_back(free_blocks.front().first);
					kept -= free_blocks.front().second;
					free_blocks.erase(free_blocks.begin());
				}
				free_blocks.emplace_back(p, n);
				kept += n;
				p = nullptr;
			}
		}
		for (uint8_t *q : drop) (void)hipHostFree(q);
		if (p) (void)hipHostFree(p);
	}
} g_stage;

/* The caller's frames are plain caller memory (m2decoder.h:54-80 may free them inside the header
 * callback; the destructor frees them without telling the decoder, m2decoder.h:39-46).  So the GPU
 * never writes them: a picture is copied device -> the context's own pinned staging buffer for its
 * slot (asynchronously, bind / submit), and staging -> the caller's frame on the caller's thread
 * inside sync_frame, i.e. inside peek / get_decoded_frame.  Between API calls nothing in flight
 * points into caller memory. */
const size_t kStgTail = 64;

/* up to 3 ranges per picture x BMAX pictures, copied by k_upload (blockIdx.y = range) */
struct UploadList {
	const uint8_t *src[3 * 4];
	uint8_t *dst[3 * 4];
	size_t bytes[3 * 4];
	int n;
	void add(const uint8_t *s_, uint8_t *d_, size_t b_)
	{
		src[n] = s_;
		dst[n] = d_;
		bytes[n] = b_;
		++n;
	}
};

/* 16 bytes per thread where source and destination are 16-byte aligned (the arena regions are), the tail bytewise */
__global__ __launch_bounds__(256) void k_upload(UploadList ul)
{
	const int r = blockIdx.y;
	const uint8_t *src = ul.src[r];
	uint8_t *dst = ul.dst[r];
	const size_t bytes = ul.bytes[r];
	const bool al = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
	const size_t n16 = al ? bytes / 16 : 0;
	const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
	for (size_t i = t; i < n16; i += stride) ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
	for (size_t i = n16 * 16 + t; i < bytes; i += stride) dst[i] = src[i];
}

/* M2DEC_AMD_KCOPY=0: the records go up by hipMemcpyAsync (SDMA) as before round 5 (read per back end) */
static bool kcopy_knob()
{
	const char *e = getenv("M2DEC_AMD_KCOPY");
	return e && *e ? atoi(e) != 0 : true;
}
/* The frame goes down by k_upload writing the pinned staging buffer over the host link instead of an SDMA copy
 * while more than one decoder context of this process is live on the device: 8 concurrent c3 streams 2120 vs
 * 2007 fps, but one c3 decode 30.5 vs 29.6 ms and C5 46.7 vs 44.2 ms (the SDMA engine writes host memory faster
 * than the CUs do; profiles/r131_ab_kd2h.txt).  M2DEC_AMD_KCOPY_D2H=0 never, =1 always (read per back end) */
static int kcopy_d2h_knob()
{
	const char *e = getenv("M2DEC_AMD_KCOPY_D2H");
	return e && *e ? atoi(e) : 2;
}
static bool kcopy_d2h(int mode, int dev)
{
	if (mode == 2) return g_live_backends[dev & 15].load(std::memory_order_relaxed) > 1;
	return mode != 0;
}
/* The error word reaches the host by a synchronous 4-byte hipMemcpy per frame (on the null stream, which the
 * non-blocking decode streams do not wait for).  M2DEC_AMD_ERR_SYNC=0 copies it behind the frame on the
 * picture's stream into the staging buffer's tail instead — measured 15 % slower on 8 concurrent streams (1539
 * vs 1813 fps, 1.2 CPU-ms more per frame, profiles/r125_ab_streams_err.txt): a 4-byte D2H per frame on the
 * copy engines costs more than the synchronous read */
static bool err_sync()
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("M2DEC_AMD_ERR_SYNC");
		v = e && *e ? atoi(e) != 0 : 1;
	}
	return v != 0;
}

struct HipBackend {
	Sched sc;
	hipStream_t copy = nullptr; /* decode ahead: bind's copies out of the picture buffers */
	m2d_frame_t frames[64];
	int nframes = 0;
	/* staging: [0, 64) caller slots; [64, 128) decode ahead, picture buffer (virtual id) i - 64 copied out right
	 * behind its kernel, before the API context binds it to a slot (be_bind then moves the buffer to the slot) */
	uint8_t *stg[128];         /* staging buffer holding / receiving index i's picture (null: none) */
	size_t stg_size = 0;       /* picture bytes per staging buffer (1.5 W H); the buffer has kStgTail more: the
	                            * error word as of the copy (read after the copy's event, no hipMemcpy) */
	hipEvent_t slot_ev[128];   /* the copy into stg[i] is complete */
	hipEvent_t d2h_ev[128][2]; /* timing: start / end of that copy */
	bool slot_pending[128];    /* stg[i] holds a picture not yet copied to the caller's frame */
	int prestaged = 0;         /* [64, 128) entries holding a picture (at most kPrestageMax) */
	Arena ar[kArenas];
	int next = 0;
	/* submitted pictures not launched yet (decode order); launched together by be_flush */
	struct Held {
		Arena *a;
		PicJob j;
		bool virt;
		size_t rec_bytes;
		int64_t ref_bytes;
	} held[BMAX];
	int nheld = 0;
	int limit = 1;        /* pictures per launch of this context (fixed at set_frames) */
	int narenas = 2 * NSTREAMS; /* record arenas in use: NSTREAMS * limit + limit + 2 (fixed at set_frames) */
	bool hold = true;    /* flush holds pictures while every stream is busy (M2DEC_AMD_HOLD=0: never) */
	int max_held = BMAX; /* M2DEC_AMD_PICS_PER_LAUNCH; also bounded by the budget (Sched::pics_fit: 2 at
	                      * 1080p and 4K) and 1 while other decode-path back ends are alive.  r67 A/B on c3,
	                      * median of 10 decodes: 1 -> 45.1 ms, 2 -> 42.6, 3 -> 41.3, 4 -> 43.3 */
	TimingSlot tr[16];
	int tr_next = 0;
	bool timing = true;
	bool kcopy = true; /* records up by k_upload (M2DEC_AMD_KCOPY) */
	int kd2h = 2;      /* frames down: 0 SDMA, 1 k_upload, 2 k_upload while several back ends live (M2DEC_AMD_KCOPY_D2H) */
	bool prestage = true; /* decode ahead: copy-out right behind the kernel (M2DEC_AMD_PRESTAGE) */
	/* guards Arena::held / pending / ext: records_busy reads them from any thread while the decoder's
	 * serial calls (acquire, submit, flush, bind) change them */
	std::mutex arena_mu;
};

int launch_held(HipBackend *b);

/* decode ahead: pictures copied out to staging right behind their kernels, on the launch's own stream
 * (M2DEC_AMD_PRESTAGE=0: at bind, on the copy stream, as before round 6), at most kPrestageMax of a back end at a
 * time (pinned memory: 32 x 3 MB at 1080p).  Interleaved A/Bs (r158): C5 46.2 -> 43.4 ms per decode, c3 29.0 ms
 * both ways; on the shared copy stream instead (r140, r156) the copies waiting for their kernels held up the binds'
 * copies of frames the caller takes first, 1-4 % slower */
static const int kPrestageMax = 32;
static bool prestage_knob()
{
	const char *e = getenv("M2DEC_AMD_PRESTAGE");
	return e && *e ? atoi(e) != 0 : true;
}

void flush_timing(HipBackend *b, TimingSlot &t)
{
	if (!t.pending) return;
	float ms;
	(void)hipEventSynchronize(t.e[5]);
	m2dec_amd_hip_timing_t &tm = b->sc.tm;
	if (hipEventElapsedTime(&ms, t.e[0], t.e[1]) == hipSuccess) tm.h2d_us += ms * 1e3;
	/* the kernel alone: from the event recorded right before it (after the launch's argument copy and the
	 * stream's waits on other launches) to the one after it, so that rocprofv3's kernel duration and this
	 * agree (r114: from the upload's end the interval also held those, 1352 vs 1198 us) */
	if (hipEventElapsedTime(&ms, t.e[3], t.e[2]) == hipSuccess) {
		tm.picture_us += ms * 1e3;
		tm.kernel_launches++;
	}
	t.pending = false;
}

/* slot i's staging buffer goes back to the pool (its copy, if any, is complete) */
void stage_drop(HipBackend *b, int i)
{
	if (i >= 64 && b->stg[i]) b->prestaged--;
	g_stage.give(b->stg[i], b->stg_size + kStgTail);
	b->stg[i] = nullptr;
	b->slot_pending[i] = false;
}

int be_set_frames(void *self, int n, const m2d_frame_t *frames, int width, int height)
{
	HipBackend *b = (HipBackend *)self;
	const double t0 = wall_s();
	if (launch_held(b) < 0) return -1;
	if (b->sc.sync_all() < 0) return -1;
	if (b->copy) CHECK(hipStreamSynchronize(b->copy)); /* every staging copy is complete */
	if (n > 64) n = 64;
	memcpy(b->frames, frames, sizeof(m2d_frame_t) * (size_t)n);
	b->nframes = n;
	const size_t stg = (size_t)width * height * 3 / 2;
	/* pictures bound but not yet handed out keep their staging (they reach the new frames) unless the
	 * picture size changed — the reference would hand out the new, unwritten frames then */
	for (int i = 0; i < 128; ++i)
		if (b->stg[i] && (stg != b->stg_size || (i < 64 && i >= n) || i >= 64)) stage_drop(b, i);
	b->stg_size = stg;
	/* one device picture buffer per virtual id (decode ahead) — a caller slot also names one */
	if (b->sc.configure(width, height, 64) < 0) return -1;
	/* pictures per launch: bounded by the budget (pics_fit) and 1 while other decode-path back ends are
	 * alive (concurrent streams fill the budget already); the arena ring covers what can be in flight
	 * (every arena is one pinned + device allocation: a ring larger than needed churns the pools) */
	const int ctxs = g_budget[b->sc.dev & 15].contexts(0, g_live_backends[b->sc.dev & 15].load(std::memory_order_relaxed));
	b->limit = ctxs > 1 ? 1 : std::min(b->max_held, b->sc.pics_fit);
	if (dbg_knob("M2DEC_AMD_DEBUG"))
		fprintf(stderr, "be_set_frames: %d decode contexts on the device, %d pictures per launch (fit %d, max %d)\n", ctxs,
		        b->limit, b->sc.pics_fit, b->max_held);
	b->narenas = std::min(kArenas, nstreams() * b->limit + b->limit + 2);
	if (b->next >= b->narenas) b->next = 0;
	if (dbg_knob("M2DEC_AMD_ASYNC_STATS")) fprintf(stderr, "be_set_frames: configure %.2f ms\n", 1e3 * (wall_s() - t0));
	return 0;
}

/* enqueue the copy of picture buffer `cur` into slot's staging buffer on stream s (after what s waits for) */
int stage_copy(HipBackend *b, const uint8_t *cur, int slot, hipStream_t s)
{
	if (!b->stg[slot] && !(b->stg[slot] = g_stage.take(b->stg_size + kStgTail))) {
		fprintf(stderr, "m2dec_amd: no pinned staging memory\n");
		return -1;
	}
	if (b->timing) CHECK(hipEventRecord(b->d2h_ev[slot][0], s));
	if (kcopy_d2h(b->kd2h, b->sc.dev)) {
		void *dh = nullptr;
		CHECK(hipHostGetDevicePointer(&dh, b->stg[slot], 0));
		UploadList ul;
		ul.n = 0;
		ul.add(cur, (uint8_t *)dh, b->stg_size);
		hipLaunchKernelGGL(k_upload, dim3(256, 1), dim3(256), 0, s, ul);
		CHECK(hipGetLastError());
	} else {
		CHECK(hipMemcpyAsync(b->stg[slot], cur, b->stg_size, hipMemcpyDeviceToHost, s));
	}
	if (!err_sync()) CHECK(hipMemcpyAsync(b->stg[slot] + b->stg_size, b->sc.err, sizeof(int), hipMemcpyDeviceToHost, s));
	if (b->timing) CHECK(hipEventRecord(b->d2h_ev[slot][1], s));
	CHECK(hipEventRecord(b->slot_ev[slot], s));
	b->slot_pending[slot] = true;
	b->sc.tm.d2h_bytes += (int64_t)b->stg_size;
	return 0;
}

int arena_alloc(Arena &a, int wm, int hm)
{
	size_t n = (size_t)wm * hm;
	/* the parser's job arenas have this layout too: an M2R_PIC_EXTERNAL picture uploads the same way */
	const m2r_arena_layout_t l = m2r_arena_layout((int)n);
	a.off_mb = l.mb;
	a.off_dbk = l.dbk;
	a.off_slice = l.slice;
	a.off_inter = l.inter;
	a.off_coef = l.coef;
	const size_t off = l.size;
	if (a.size < off) {
		int dev = 0;
		CHECK(hipGetDevice(&dev));
		g_arenas.give(dev, a);
		if (!g_arenas.take(dev, off, a)) {
			const double t0 = wall_s();
			CHECK(hipHostMalloc(&a.host, off, hipHostMallocDefault));
			CHECK(hipMalloc(&a.dev, off));
			if (dbg_knob("M2DEC_AMD_ASYNC_STATS")) fprintf(stderr, "arena_alloc: %zu bytes %.2f ms\n", off, 1e3 * (wall_s() - t0));
			a.size = off;
		}
	}
	if (!a.consumed) {
		int dev = 0;
		CHECK(hipGetDevice(&dev));
		CHECK(g_pool.event(dev, false, &a.consumed));
	}
	m2r_picture_t &p = a.pic;
	memset(&p, 0, sizeof(p));
	p.width_mbs = wm;
	p.height_mbs = hm;
	p.mb = (m2r_mb_t *)(a.host + a.off_mb);
	p.dbk = (m2r_deblock_t *)(a.host + a.off_dbk);
	p.slice = (m2r_slice_t *)(a.host + a.off_slice);
	p.inter = (m2r_inter_t *)(a.host + a.off_inter);
	p.coef = (int16_t *)(a.host + a.off_coef);
	p.cap_slices = kSlicesCap;
	p.cap_inter = (int)n;
	p.cap_coef = (int)(n * 416);
	return 0;
}

m2r_picture_t *be_acquire(void *self, int wm, int hm)
{
	HipBackend *b = (HipBackend *)self;
	Arena &a = b->ar[b->next];
	b->next = (b->next + 1) % b->narenas;
	if (a.held && launch_held(b) < 0) return nullptr;
	if (a.pending) {
		/* the host copy is overwritten next: wait until that picture's kernels are done with it */
		if (hipEventSynchronize(a.consumed) != hipSuccess) return nullptr;
		std::lock_guard<std::mutex> lk(b->arena_mu);
		a.pending = false;
		a.ext = nullptr;
	}
	if (arena_alloc(a, wm, hm) < 0) return nullptr;
	return &a.pic;
}

int be_submit(void *self, m2r_picture_t *pic)
{
	HipBackend *b = (HipBackend *)self;
	Sched &sc = b->sc;
	Arena *a = nullptr;
	for (auto &x : b->ar)
		if (&x.pic == pic) a = &x;
	const int n = pic->width_mbs * pic->height_mbs;
	const bool virt = (pic->flags & M2R_PIC_VIRTUAL) != 0;
	/* external records: the parser's arena, in the same layout as ours (checked), uploaded from there */
	const uint8_t *ext = nullptr;
	if (pic->flags & M2R_PIC_EXTERNAL) {
		ext = (const uint8_t *)pic->mb;
		if (!a || (const uint8_t *)pic->dbk != ext + a->off_dbk || (const uint8_t *)pic->slice != ext + a->off_slice ||
		    (const uint8_t *)pic->inter != ext + a->off_inter || (const uint8_t *)pic->coef != ext + a->off_coef) {
			fprintf(stderr, "m2dec_amd: submit: external records not in the arena layout\n");
			return -1;
		}
	}
	if (!a || a->held || pic->width_mbs != sc.Wmb || pic->height_mbs != sc.Hmb || pic->slot < 0 || pic->slot >= sc.nslots ||
	    (!virt && pic->slot >= b->nframes) || pic->n_slices > kSlicesCap || pic->n_inter > n || pic->n_coef > n * 416) {
		fprintf(stderr, "m2dec_amd: submit: picture records rejected (arena %d, slot %d)\n", a ? (int)(a - b->ar) : -1, pic->slot);
		return -1;
	}
	HipBackend::Held &h = b->held[b->nheld++];
	PicJob &j = h.j;
	j.slot = pic->slot;
	j.n_inter = pic->n_inter;
	j.n_intra = pic->n_intra;
	j.deblock = pic->deblock;
	const bool sum = (pic->flags & M2R_PIC_REFS) != 0; /* (the producer summarised inter[]) */
	j.refs = (sum ? pic->ref_slots : refs_of(pic->inter, pic->n_inter)) & ~(1ull << pic->slot);
	j.r.mb = (const m2r_mb_t *)(a->dev + a->off_mb);
	j.r.dbk = (const m2r_deblock_t *)(a->dev + a->off_dbk);
	j.r.sl = (const m2r_slice_t *)(a->dev + a->off_slice);
	j.r.it = (const m2r_inter_t *)(a->dev + a->off_inter);
	j.r.coef = (const int16_t *)(a->dev + a->off_coef);
	h.a = a;
	h.virt = virt;
	h.rec_bytes = n * (sizeof(m2r_mb_t) + sizeof(m2r_deblock_t)) + pic->n_slices * sizeof(m2r_slice_t) +
	              pic->n_inter * sizeof(m2r_inter_t) + pic->n_coef * sizeof(int16_t);
	h.ref_bytes = sum ? (int64_t)pic->ref_blocks * (64 + 32) : ref_bytes_of(pic->inter, pic->n_inter);
	{
		std::lock_guard<std::mutex> lk(b->arena_mu);
		a->ext = ext;
		a->held = true;
	}
	/* a caller slot as the picture buffer (no decode ahead): copied out right behind its kernel, so
	 * launched at once, as is a full hand */
	if (!virt || b->nheld >= b->limit) return launch_held(b);
	return 0;
}

/* m2r_backend_t.flush, called by the decoder when a drive of its pipeline has nothing more to submit.
 * While every stream of this context still runs a launch, held pictures wait (returns 1: the decoder asks
 * again on its next drive — a parse finishing, an API call — and a bind of a held picture's buffer or a
 * full hand launches them anyway), so that pictures submitted meanwhile join them in one launch: the
 * decode path is latency-bound per launch (a 2-picture k_picture takes about as long as a 1-picture one,
 * r83 timeline), so a fuller launch is throughput.  With an idle stream they are launched now.
 * M2DEC_AMD_HOLD=0 launches at every flush (the r4 A/B baseline). */
int be_flush(void *self)
{
	HipBackend *b = (HipBackend *)self;
	if (!b->nheld) return 0;
	if (b->hold && b->nheld < b->limit && !b->sc.any_idle()) return 1;
	return launch_held(b) < 0 ? -1 : 0;
}

/* launch the held pictures as one k_picture on the next stream: their slots' waits, the record uploads,
 * the launch, then per picture the consumed event, the copy-out (caller slot), and the slot bookkeeping */
int launch_held(HipBackend *b)
{
	Sched &sc = b->sc;
	const int n = b->nheld;
	if (!n) return 0;
	b->nheld = 0;
	CHECK(hipSetDevice(sc.dev));
	const int k = sc.pick();
	hipStream_t s = sc.st[k];
	m2d_tl('L', n, k);
	PicJob jobs[BMAX];
	for (int i = 0; i < n; ++i) jobs[i] = b->held[i].j; /* (their slot waits: launch_multi, after the uploads) */
	TimingSlot *ts = nullptr;
	if (b->timing) {
		ts = &b->tr[b->tr_next];
		b->tr_next = (b->tr_next + 1) % 16;
		flush_timing(b, *ts);
		CHECK(hipEventRecord(ts->e[0], s));
	}
	if (b->kcopy) {
		/* the records by one kernel reading the pinned arenas over the host link (k_upload): an SDMA upload queued
		 * behind a copy-out that waits for an earlier picture's kernels can hold this thread for milliseconds
		 * (the H.265 back end measured 8-10 ms; here launches averaged 0.44 ms of waits + uploads in a slow c3
		 * decode against 0.07 in a normal one, the GPU idle 7.6 ms of it) */
		UploadList ul;
		ul.n = 0;
		for (int i = 0; i < n; ++i) {
			const Arena *a = b->held[i].a;
			const m2r_picture_t *pic = &a->pic;
			const uint8_t *src = a->ext ? a->ext : a->host;
			void *dsrc = nullptr;
			CHECK(hipHostGetDevicePointer(&dsrc, (void *)src, 0));
			const uint8_t *ds = (const uint8_t *)dsrc;
			ul.add(ds, a->dev, a->off_slice + pic->n_slices * sizeof(m2r_slice_t));
			if (pic->n_inter) ul.add(ds + a->off_inter, a->dev + a->off_inter, pic->n_inter * sizeof(m2r_inter_t));
			if (pic->n_coef) ul.add(ds + a->off_coef, a->dev + a->off_coef, pic->n_coef * sizeof(int16_t));
		}
		hipLaunchKernelGGL(k_upload, dim3(64, ul.n), dim3(256), 0, s, ul);
		CHECK(hipGetLastError());
	} else {
		for (int i = 0; i < n; ++i) {
			/* mb | dbk | used slices in one copy, then the used inter and coefficient prefixes (m2r_arena_layout) */
			const Arena *a = b->held[i].a;
			const m2r_picture_t *pic = &a->pic;
			const uint8_t *src = a->ext ? a->ext : a->host;
			CHECK(hipMemcpyAsync(a->dev, src, a->off_slice + pic->n_slices * sizeof(m2r_slice_t), hipMemcpyHostToDevice, s));
			if (pic->n_inter) CHECK(hipMemcpyAsync(a->dev + a->off_inter, src + a->off_inter, pic->n_inter * sizeof(m2r_inter_t), hipMemcpyHostToDevice, s));
			if (pic->n_coef) CHECK(hipMemcpyAsync(a->dev + a->off_coef, src + a->off_coef, pic->n_coef * sizeof(int16_t), hipMemcpyHostToDevice, s));
		}
	}
	if (ts) CHECK(hipEventRecord(ts->e[1], s));
	m2d_tl('M', n, k);
	hipEvent_t inter_done;
	if (sc.launch_multi(k, jobs, n, ts ? ts->e + 2 : nullptr, &inter_done, ts ? ts->e + 3 : nullptr, true) < 0) return -1;
	if (sc.mark_busy(k) < 0) return -1;
	m2d_tl('N', n, k);
	const size_t ls = (size_t)sc.W * sc.H;
	for (int i = 0; i < n; ++i) {
		HipBackend::Held &h = b->held[i];
		CHECK(hipEventRecord(h.a->consumed, s));
		std::lock_guard<std::mutex> lk(b->arena_mu);
		h.a->pending = true;
		h.a->held = false;
		if (!h.virt) /* the caller's slot is the picture buffer: copy out right behind the kernel */
			if (stage_copy(b, sc.frames + (size_t)h.j.slot * sc.fsz, h.j.slot, s) < 0) return -1;
	}
	if (ts) {
		CHECK(hipEventRecord(ts->e[5], s));
		ts->pending = true;
	}
	for (int i = 0; i < n; ++i) {
		const HipBackend::Held &h = b->held[i];
		if (sc.end(k, h.j, inter_done) < 0) return -1;
		sc.tm.pictures++;
		sc.tm.record_bytes += (int64_t)h.rec_bytes;
		sc.tm.ref_bytes += h.ref_bytes;
		sc.tm.frame_bytes += (int64_t)(ls * 3 / 2);
	}
	/* decode ahead: each picture out to pinned staging right behind its kernel, before the API context binds it
	 * (r139 timeline: with the copy issued at bind, the API thread waited on every frame's copy in turn — 60 copies
	 * of ~0.3 ms each from the bind to the frame's peek, the last one 6.2 ms after the last kernel) */
	for (int i = 0; i < n; ++i) {
		const HipBackend::Held &h = b->held[i];
		if (!h.virt || b->prestaged >= kPrestageMax || !b->prestage) continue;
		const int v = 64 + h.j.slot;
		if (b->stg[v]) { /* (an earlier picture of this buffer never bound — ahead_ok orders reuse after the bind) */
			if (b->slot_pending[v]) CHECK(hipEventSynchronize(b->slot_ev[v]));
			stage_drop(b, v);
		}
		/* on the launch's own stream, right behind it: on the shared copy stream a copy waiting for its kernel held
		 * up the binds' copies of frames the caller takes first (r156: every copy-ahead setting slower) */
		if (stage_copy(b, sc.frames + (size_t)h.j.slot * sc.fsz, v, s) < 0) return -1;
		b->prestaged++;
		hipEvent_t r = sc.next_event(); /* (a reader of the buffer: its next writer waits for the copy) */
		if (!r) return -1;
		CHECK(hipEventRecord(r, s));
		sc.readers[h.j.slot].push_back(r);
	}
	m2d_tl('l', n, k);
	return 0;
}

/* decode ahead: picture buffer `vid` (its last writer is submitted) is caller frame `slot`.  The copy
 * runs on its own stream behind the writer's completion event; it is a reader of the buffer, so the
 * next picture writing `vid` waits for it (Sched::begin) */
int be_bind(void *self, int vid, int slot)
{
	HipBackend *b = (HipBackend *)self;
	Sched &sc = b->sc;
	/* the picture writing vid may be held: then the held pictures go now (others keep waiting) */
	for (int i = 0; i < b->nheld; ++i)
		if (b->held[i].virt && b->held[i].j.slot == vid) {
			if (launch_held(b) < 0) return -1;
			break;
		}
	if (vid < 0 || vid >= sc.nslots || slot < 0 || slot >= b->nframes || !sc.slot_write[vid]) {
		fprintf(stderr, "m2dec_amd: bind: picture buffer %d (written: %d) to frame %d rejected\n", vid,
		        vid >= 0 && vid < 64 && sc.slot_write[vid] != nullptr, slot);
		return -1;
	}
	CHECK(hipSetDevice(sc.dev));
	if (b->slot_pending[64 + vid]) { /* copied out behind its kernel (launch_held): the slot takes that buffer */
		if (b->stg[slot]) {
			if (b->slot_pending[slot]) CHECK(hipEventSynchronize(b->slot_ev[slot])); /* (a picture never handed out) */
			stage_drop(b, slot);
		}
		const int v = 64 + vid;
		std::swap(b->stg[slot], b->stg[v]);
		std::swap(b->slot_ev[slot], b->slot_ev[v]);
		std::swap(b->d2h_ev[slot][0], b->d2h_ev[v][0]);
		std::swap(b->d2h_ev[slot][1], b->d2h_ev[v][1]);
		b->slot_pending[slot] = true;
		b->slot_pending[v] = false;
		b->prestaged--;
		return 0;
	}
	if (!b->copy) CHECK(g_pool.stream(sc.dev, &b->copy));
	CHECK(hipStreamWaitEvent(b->copy, sc.slot_write[vid], 0));
	if (stage_copy(b, sc.frames + (size_t)vid * sc.fsz, slot, b->copy) < 0) return -1;
	hipEvent_t r = sc.next_event();
	if (!r) return -1;
	CHECK(hipEventRecord(r, b->copy));
	sc.readers[vid].push_back(r);
	return 0;
}

/* the picture of `slot` into the caller's frame: wait for its staging copy, then copy it on this
 * (the caller's) thread */
int be_sync(void *self, int slot)
{
	HipBackend *b = (HipBackend *)self;
	if (slot < 0 || slot >= 64) return -1;
	/* (no flush here: sync_frame runs on the API thread while a pool worker may be inside submit / bind /
	 * flush — those three, acquire and set_frames are the serial back-end calls.  The slot's picture was
	 * launched when it was bound, or when it was submitted without decode ahead.) */
	if (b->slot_pending[slot]) {
		m2d_tl('Y', slot, 0);
		CHECK(hipEventSynchronize(b->slot_ev[slot]));
		m2d_tl('y', slot, 0);
		/* the error word copied behind the picture on its stream (a synchronous hipMemcpy here queues behind
		 * whatever shares the null stream's hardware queue, per frame) */
		if (err_sync()) {
			if (b->sc.check_err() < 0) return -1;
		} else {
			int e;
			memcpy(&e, b->stg[slot] + b->stg_size, sizeof(e));
			if (e) {
				fprintf(stderr, "m2dec_amd: wavefront hand-off failed (err=%d)\n", e);
				return -1;
			}
		}
		if (b->timing) {
			float ms;
			if (hipEventElapsedTime(&ms, b->d2h_ev[slot][0], b->d2h_ev[slot][1]) == hipSuccess) b->sc.tm.d2h_us += ms * 1e3;
		}
		const double t0 = wall_s();
		const m2d_frame_t &f = b->frames[slot];
		const size_t ls = b->stg_size / 3 * 2;
		{ /* (on the API thread, once per output frame: spread over the sync copy crew, parcopy.c) */
			void *const to[2] = {f.luma, f.chroma};
			const void *const from[2] = {b->stg[slot], b->stg[slot] + ls};
			const size_t len[2] = {ls, ls / 2};
			m2dec_par_memcpy(M2DEC_CREW_SYNC_, 2, to, from, len);
		}
		b->sc.tm.host_copy_us += (wall_s() - t0) * 1e6;
		stage_drop(b, slot);
	}
	return 0;
}

/* m2r_backend_t.ready: sync_frame(slot) would not wait (no copy pending, or its event fired) */
int be_ready(void *self, int slot)
{
	HipBackend *b = (HipBackend *)self;
	if (slot < 0 || slot >= 64 || !b->slot_pending[slot]) return 1;
	return hipEventQuery(b->slot_ev[slot]) == hipSuccess;
}

/* m2r_backend_t.records_busy: 1 while an arena's upload may still read the external records at `records`
 * (held, or launched and its consumed event not reached); the arena forgets them once it is reached */
int be_records_busy(void *self, const void *records, int wait)
{
	HipBackend *b = (HipBackend *)self;
	for (auto &a : b->ar) {
		bool held, pending;
		hipEvent_t ev;
		{
			std::lock_guard<std::mutex> lk(b->arena_mu);
			if (a.ext != records) continue;
			held = a.held;
			pending = a.pending;
			ev = a.consumed;
		}
		if (held) {
			if (!wait) return 1;
			if (launch_held(b) < 0) return 1; /* (only while no other call runs: see m2d_recon.h) */
			std::lock_guard<std::mutex> lk(b->arena_mu);
			pending = a.pending;
			ev = a.consumed;
		}
		if (pending) {
			const hipError_t q = wait ? hipEventSynchronize(ev) : hipEventQuery(ev);
			if (q != hipSuccess) return 1;
		}
		std::lock_guard<std::mutex> lk(b->arena_mu);
		if (a.ext == records && !a.held) a.ext = nullptr;
		return a.ext == records;
	}
	return 0;
}

void be_destroy(void *self)
{
	HipBackend *b = (HipBackend *)self;
	const double t0 = wall_s();
	for (int i = 0; i < b->nheld; ++i) b->held[i].a->held = false; /* (dropped: nothing waits for them) */
	b->nheld = 0;
	b->sc.sync_all();
	g_budget[b->sc.dev & 15].contexts(-1, --g_live_backends[b->sc.dev & 15]);
	const double t1 = wall_s();
	g_pool.put_stream(b->sc.dev, b->copy); /* (synchronises it: every staging copy is complete) */
	b->copy = nullptr;
	for (int i = 0; i < 128; ++i) stage_drop(b, i);
	for (auto &a : b->ar) {
		g_arenas.give(b->sc.dev, a); /* (every kernel reading it finished: sync_all above) */
		g_pool.put_event(b->sc.dev, false, a.consumed);
	}
	for (int i = 0; i < 128; ++i) {
		g_pool.put_event(b->sc.dev, false, b->slot_ev[i]);
		g_pool.put_event(b->sc.dev, true, b->d2h_ev[i][0]);
		g_pool.put_event(b->sc.dev, true, b->d2h_ev[i][1]);
	}
	for (auto &t : b->tr)
		for (auto &e : t.e) g_pool.put_event(b->sc.dev, true, e);
	const double t2 = wall_s();
	b->sc.destroy();
	if (dbg_knob("M2DEC_AMD_ASYNC_STATS"))
		fprintf(stderr, "be_destroy: sync %.2f ms, staging / arenas / events %.2f ms, scheduler %.2f ms\n",
		        1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (wall_s() - t2));
	delete b;
}

} // namespace

extern "C" int m2dec_amd_hip_pin(void *p, size_t n)
{
	if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) return -1;
	std::lock_guard<std::mutex> lk(g_pins.mu);
	g_pins.ranges.emplace_back((const uint8_t *)p, n);
	return 0;
}

extern "C" void m2dec_amd_hip_unpin(void *p)
{
	std::lock_guard<std::mutex> lk(g_pins.mu);
	for (size_t i = 0; i < g_pins.ranges.size(); ++i)
		if (g_pins.ranges[i].first == (const uint8_t *)p) {
			(void)hipHostUnregister(p);
			g_pins.ranges.erase(g_pins.ranges.begin() + (long)i);
			return;
		}
}

extern "C" int m2dec_amd_hip_available(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n > 0;
}

static int selftest_once(int device);

extern "C" int m2dec_amd_hip_backend_create(m2r_backend_t *out, int device)
{
	if (!out || !m2dec_amd_hip_available()) return -1;
	if (selftest_once(device) < 0) return -1; /* (the built-in known-answer test, once per process and device) */
	const double t0 = wall_s();
	HipBackend *b = new HipBackend();
	memset(b->stg, 0, sizeof(b->stg));
	memset(b->slot_pending, 0, sizeof(b->slot_pending));
	if (b->sc.init(device) < 0) {
		delete b;
		return -1;
	}
	for (int i = 0; i < 128; ++i) {
		CHECK(g_pool.event(device, false, &b->slot_ev[i]));
		CHECK(g_pool.event(device, true, &b->d2h_ev[i][0]));
		CHECK(g_pool.event(device, true, &b->d2h_ev[i][1]));
	}
	for (auto &t : b->tr)
		for (auto &e : t.e) CHECK(g_pool.event(device, true, &e));
	const char *tm = getenv("M2DEC_AMD_TIMING");
	b->timing = tm ? atoi(tm) != 0 : true;
	b->kcopy = kcopy_knob();
	b->kd2h = kcopy_d2h_knob();
	b->prestage = prestage_knob();
	out->self = b;
	out->set_frames = be_set_frames;
	out->acquire = be_acquire;
	out->submit = be_submit;
	out->sync_frame = be_sync;
	out->destroy = be_destroy;
	out->bind = be_bind;
	out->flush = be_flush;
	out->ready = be_ready;
	out->records_busy = be_records_busy;
	g_budget[device & 15].setup(device);
	g_budget[device & 15].contexts(+1, ++g_live_backends[device & 15]);
	if (const char *e = getenv("M2DEC_AMD_HOLD")) b->hold = atoi(e) != 0;
	if (const char *e = getenv("M2DEC_AMD_PICS_PER_LAUNCH")) /* tuning: 1 = one picture per launch */
		b->max_held = std::max(1, std::min(BMAX, atoi(e)));
	if (dbg_knob("M2DEC_AMD_ASYNC_STATS")) fprintf(stderr, "hip_backend_create: %.2f ms\n", 1e3 * (wall_s() - t0));
	return 0;
}

extern "C" int m2dec_amd_hip_backend_budget(const m2r_backend_t *be, m2dec_amd_hip_budget_t *out)
{
	if (!be || !be->self || !out) return -1;
	HipBackend *b = (HipBackend *)be->self;
	const Sched &sc = b->sc;
	SlotBudget &bg = g_budget[sc.dev & 15];
	memset(out, 0, sizeof(*out));
	out->resident_per_cu = sc.resident_per_cu;
	out->cap_workgroups = sc.cap_wg;
	out->wg_units = sc.wg_units;
	out->pics_fit = sc.pics_fit;
	out->launch_limit = b->limit;
	out->streams = nstreams();
	std::lock_guard<std::mutex> lk(bg.mu);
	out->cap_units = bg.cap_units;
	out->shared = bg.share != nullptr;
	out->max_procs = bg.max_procs;
	out->max_units = bg.max_total;
	return 0;
}

extern "C" void h264_async_pool_release(void);
extern "C" long long h264_async_pinned_bytes(long long *pooled);

/* Everything the process keeps pooled between decoder contexts: the parse pool's jobs with their
 * page-locked record arenas, the back ends' pinned record arenas and staging buffers, pooled device buffers.
 * Live contexts keep what they use. */
extern "C" void m2dec_amd_release_pools(void)
{
	h264_async_pool_release();
	{
		std::lock_guard<std::mutex> lk(g_arenas.mu);
		for (auto &bl : g_arenas.free_blocks) {
			(void)hipHostFree(bl.host);
			(void)hipFree(bl.dev_ptr);
		}
		g_arenas.free_blocks.clear();
		g_arenas.kept = 0;
	}
	{
		std::lock_guard<std::mutex> lk(g_stage.mu);
		for (auto &bl : g_stage.free_blocks) (void)hipHostFree(bl.first);
		g_stage.free_blocks.clear();
		g_stage.kept = 0;
	}
	{
		std::lock_guard<std::mutex> lk(g_dev.mu);
		for (auto &bl : g_dev.blocks) (void)hipFree(bl.p);
		g_dev.blocks.clear();
		g_dev.kept = 0;
	}
}

extern "C" long long m2dec_amd_pinned_bytes(long long *pooled)
{
	return h264_async_pinned_bytes(pooled);
}

extern "C" int m2dec_amd_configure_queues(int n)
{
	char v[16];
	snprintf(v, sizeof v, "%d", n < 1 ? 1 : n);
	setenv("GPU_MAX_HW_QUEUES", v, 0); /* (a value the caller set already wins) */
	return atoi(getenv("GPU_MAX_HW_QUEUES"));
}

extern "C" int m2dec_amd_hip_backend_timing(const m2r_backend_t *be, m2dec_amd_hip_timing_t *out)
{
	if (!be || !be->self || !out) return -1;
	HipBackend *b = (HipBackend *)be->self;
	for (auto &t : b->tr) flush_timing(b, t);
	*out = b->sc.tm;
	return 0;
}

/* ======================================================================== trace replay */
struct m2dec_amd_hip_replay {
	Sched sc;
	int npics = 0;
	int crop[4] = {0, 0, 0, 0};
	uint8_t *d_rec = nullptr;
	std::vector<m2dec_amd_trace_pic_t> pics; /* replay order (streams interleaved), slots / offsets rebased */
	std::vector<int> stream;                 /* the stream of each picture */
	std::vector<uint64_t> refs;
	std::vector<PicJob> jobs;
	/* timing: 2 events per launch (before / after its k_batch) */
	std::vector<hipEvent_t> tev;
	size_t tev_used = 0;
};

static void replay_free(m2dec_amd_hip_replay_t *r)
{
	r->sc.sync_all();
	for (hipEvent_t e : r->tev) (void)hipEventDestroy(e);
	if (r->d_rec) (void)hipFree(r->d_rec);
	r->sc.destroy();
	delete r;
}

extern "C" int m2dec_amd_hip_replay_create(const m2dec_amd_trace_t *t, int device, m2dec_amd_hip_replay_t **out)
{
	return m2dec_amd_hip_replay_create_multi(&t, 1, device, out);
}

/* Frame slots of one stream packed into k slots: a trace names the decoder's frame slots (the frame
 * LRU cycles through all of them), but only the pictures still read later are live.  Content c (the
 * picture written at decode index c) lives until its last reader; picture i takes the slot free the
 * longest among those whose content has no reader at or after i, and every reference in the inter
 * records is renamed to where its content went.  Returns the new slot per picture (and rewrites the
 * records), or an empty vector if k slots are not enough. */
static std::vector<int> pack_slots(uint8_t *rec, const m2dec_amd_trace_pic_t *pics, int np, int k)
{
	std::vector<int> writer(64, -1), last(np, -1), out(np, -1), holder(k, -1), freed(k, -1);
	std::vector<std::vector<int>> content(np); /* per picture: the writer index of each old slot it reads */
	for (int i = 0; i < np; ++i) {
		const uint64_t refs = refs_of((const m2r_inter_t *)(rec + pics[i].off_inter), pics[i].n_inter);
		for (int r = 0; r < 64; ++r)
			if (((refs >> r) & 1) && r != pics[i].slot) {
				if (writer[r] < 0) return {}; /* a reference no picture of the trace wrote */
				last[writer[r]] = i;
			}
		content[i].assign(writer.begin(), writer.end());
		writer[pics[i].slot & 63] = i;
	}
	std::vector<int> where(np, -1); /* new slot of each content */
	for (int i = 0; i < np; ++i) {
		int best = -1;
		for (int p = 0; p < k; ++p) {
			const int c = holder[p];
			if (c >= 0 && last[c] >= i) continue; /* still read by picture i or later */
			if (best < 0 || freed[p] < freed[best]) best = p;
		}
		if (best < 0) return {};
		m2r_inter_t *it = (m2r_inter_t *)(rec + pics[i].off_inter);
		for (int q = 0; q < pics[i].n_inter; ++q)
			for (int l = 0; l < 2; ++l)
				for (int b = 0; b < 4; ++b)
					if (it[q].slot[l][b] >= 0) it[q].slot[l][b] = (int8_t)where[content[i][it[q].slot[l][b] & 63]];
		if (holder[best] >= 0) freed[best] = i;
		holder[best] = i;
		where[i] = best;
		out[i] = best;
	}
	return out;
}

/* Host-only check of pack_slots on a trace (tests, no GPU): every reference of every picture must
 * name, after packing into k slots, the content (writer picture) it named before.  0: preserved,
 * -1: k slots are not enough, 1 + i: picture i reads other content. */
extern "C" int m2dec_amd_replay_pack_check(const m2dec_amd_trace_t *t, int k)
{
	int np, w, h, ns, nout;
	size_t len;
	if (!t || k <= 0 || k > 64 || m2dec_amd_trace_info(t, &np, &w, &h, &ns, &nout) < 0) return -1;
	const uint8_t *src = m2dec_amd_trace_records(t, &len);
	const m2dec_amd_trace_pic_t *pics = m2dec_amd_trace_pictures(t);
	std::vector<uint8_t> rec(src, src + len);
	const std::vector<int> ns_ = pack_slots(rec.data(), pics, np, k);
	if (ns_.empty()) return -1;
	int orig[64], packed[64];
	for (int i = 0; i < 64; ++i) orig[i] = packed[i] = -1;
	for (int i = 0; i < np; ++i) {
		const m2r_inter_t *a = (const m2r_inter_t *)(src + pics[i].off_inter);
		const m2r_inter_t *b = (const m2r_inter_t *)(rec.data() + pics[i].off_inter);
		for (int q = 0; q < pics[i].n_inter; ++q)
			for (int l = 0; l < 2; ++l)
				for (int s = 0; s < 4; ++s) {
					if ((a[q].slot[l][s] < 0) != (b[q].slot[l][s] < 0)) return 1 + i;
					if (a[q].slot[l][s] >= 0 && orig[a[q].slot[l][s] & 63] != packed[b[q].slot[l][s] & 63]) return 1 + i;
				}
		orig[pics[i].slot & 63] = i;
		packed[ns_[i]] = i;
	}
	return 0;
}

/* Several independent streams in one replay: their pictures interleaved one by one (stream 0's
 * first, stream 1's first, ...; each stream's pictures stay in decode order), every stream on its
 * own range of frame slots (packed, pack_slots), so one k_batch launch carries pictures of all of
 * them and the device orders only pictures of the same stream against each other (slot reuse,
 * reference rows). */
extern "C" int m2dec_amd_hip_replay_create_multi(const m2dec_amd_trace_t *const *ts, int n, int device,
                                                m2dec_amd_hip_replay_t **out)
{
	int W = 0, H = 0, nslots = 0, total = 0, most = 0;
	if (!ts || n <= 0 || !out || !m2dec_amd_hip_available()) return -1;
	std::vector<int> np(n), base(n);
	std::vector<std::vector<int>> newslot(n);
	std::vector<size_t> rbase(n);
	std::vector<uint8_t> rec;
	for (int s = 0; s < n; ++s) {
		int w, h, ns, nout;
		size_t len;
		if (!ts[s] || m2dec_amd_trace_info(ts[s], &np[s], &w, &h, &ns, &nout) < 0 || np[s] <= 0 || w <= 0 || h <= 0) return -1;
		if (s && (w != W || h != H)) return -1; /* one frame geometry per replay */
		W = w;
		H = h;
		base[s] = nslots;
		nslots += ns;
		total += np[s];
		most = std::max(most, np[s]);
		const m2dec_amd_trace_pic_t *pics = m2dec_amd_trace_pictures(ts[s]);
		for (int i = 0; i < np[s]; ++i)
			if (pics[i].slot < 0 || pics[i].slot >= ns || pics[i].width_mbs != W / 16 || pics[i].height_mbs != H / 16) return -1;
		const uint8_t *src = m2dec_amd_trace_records(ts[s], &len);
		rbase[s] = rec.size();
		rec.insert(rec.end(), src, src + len);
		rec.resize((rec.size() + 255) & ~(size_t)255); /* keep every record array as aligned as it was */
		if (n > 1) { /* pack the stream into its share of the 64 slots */
			const int k = 64 / n;
			newslot[s] = pack_slots(rec.data() + rbase[s], pics, np[s], k);
			if (newslot[s].empty()) return -1;
			nslots = base[s] + k;
		}
		/* the inter records name reference frame slots: move them into the stream's slot range */
		for (int i = 0; i < np[s]; ++i) {
			m2r_inter_t *it = (m2r_inter_t *)(rec.data() + rbase[s] + pics[i].off_inter);
			for (int k = 0; k < pics[i].n_inter; ++k)
				for (int l = 0; l < 2; ++l)
					for (int b = 0; b < 4; ++b)
						if (it[k].slot[l][b] >= 0) it[k].slot[l][b] = (int8_t)(it[k].slot[l][b] + base[s]);
		}
	}
	if (nslots > 64) return -1; /* slot bit masks (refs, SlotSeq) */
	m2dec_amd_hip_replay_t *r = new m2dec_amd_hip_replay_t();
	r->npics = total;
	m2dec_amd_trace_crop(ts[0], r->crop);
	for (int i = 0; i < most; ++i)
		for (int s = 0; s < n; ++s) {
			if (i >= np[s]) continue;
			m2dec_amd_trace_pic_t p = m2dec_amd_trace_pictures(ts[s])[i];
			p.slot = (n > 1 ? newslot[s][i] : p.slot) + base[s];
			p.off_mb += rbase[s];
			p.off_dbk += rbase[s];
			p.off_slice += rbase[s];
			p.off_inter += rbase[s];
			p.off_coef += rbase[s];
			r->pics.push_back(p);
			r->stream.push_back(s);
			r->refs.push_back(refs_of((const m2r_inter_t *)(rec.data() + p.off_inter), p.n_inter) & ~(1ull << p.slot));
		}
	const m2dec_amd_trace_pic_t *pics = r->pics.data();
	const int npics = total;
#define RCHECK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "m2dec_amd replay: %s failed\n", #x); replay_free(r); return -1; } } while (0)
	if (r->sc.init(device) < 0 || r->sc.configure(W, H, nslots) < 0) {
		replay_free(r);
		return -1;
	}
	RCHECK(hipMalloc(&r->d_rec, rec.size()));
	RCHECK(hipMemcpy(r->d_rec, rec.data(), rec.size(), hipMemcpyHostToDevice));
	for (int i = 0; i < npics; ++i) {
		const m2dec_amd_trace_pic_t &p = pics[i];
		PicJob j;
		j.r.mb = (const m2r_mb_t *)(r->d_rec + p.off_mb);
		j.r.dbk = (const m2r_deblock_t *)(r->d_rec + p.off_dbk);
		j.r.sl = (const m2r_slice_t *)(r->d_rec + p.off_slice);
		j.r.it = (const m2r_inter_t *)(r->d_rec + p.off_inter);
		j.r.coef = (const int16_t *)(r->d_rec + p.off_coef);
		j.slot = p.slot;
		j.n_inter = p.n_inter;
		j.n_intra = p.n_intra;
		j.deblock = p.deblock;
		j.refs = r->refs[i];
		r->jobs.push_back(j);
	}
	if (r->sc.batch_reserve(npics) < 0) {
		replay_free(r);
		return -1;
	}
#undef RCHECK
	*out = r;
	return 0;
}

static int replay_enqueue(m2dec_amd_hip_replay_t *r, int i, bool timed)
{
	const m2dec_amd_trace_pic_t &p = r->pics[i];
	Sched &sc = r->sc;
	PicJob j;
	j.r.mb = (const m2r_mb_t *)(r->d_rec + p.off_mb);
	j.r.dbk = (const m2r_deblock_t *)(r->d_rec + p.off_dbk);
	j.r.sl = (const m2r_slice_t *)(r->d_rec + p.off_slice);
	j.r.it = (const m2r_inter_t *)(r->d_rec + p.off_inter);
	j.r.coef = (const int16_t *)(r->d_rec + p.off_coef);
	j.slot = p.slot;
	j.n_inter = p.n_inter;
	j.n_intra = p.n_intra;
	j.deblock = p.deblock;
	j.refs = r->refs[i];
	const int k = sc.begin(j.slot, j.refs);
	if (k < 0) return -1;
	hipEvent_t *ev = nullptr;
	if (timed) {
		while (r->tev_used + 2 > r->tev.size()) {
			hipEvent_t e;
			CHECK(hipEventCreate(&e));
			r->tev.push_back(e);
		}
		ev = &r->tev[r->tev_used];
		r->tev_used += 2;
		CHECK(hipEventRecord(ev[0], sc.st[k]));
	}
	hipEvent_t inter_done;
	if (sc.launch(k, j, ev ? ev + 1 : nullptr, &inter_done) < 0) return -1;
	if (sc.end(k, j, inter_done) < 0) return -1;
	sc.tm.pictures++;
	sc.tm.record_bytes += p.record_bytes;
	sc.tm.ref_bytes += p.ref_bytes;
	sc.tm.frame_bytes += p.frame_bytes;
	return 0;
}

/* pictures [i0, i1) of the trace as batch launches on stream 0 (timed: events around each) */
static int replay_batches(m2dec_amd_hip_replay_t *r, int i0, int i1, bool timed, uint8_t *capture)
{
	Sched &sc = r->sc;
	for (int i = i0; i < i1;) {
		hipEvent_t *ev = nullptr;
		if (timed) {
			while (r->tev_used + 2 > r->tev.size()) {
				hipEvent_t e;
				CHECK(hipEventCreate(&e));
				r->tev.push_back(e);
			}
			ev = &r->tev[r->tev_used];
			r->tev_used += 2;
			CHECK(hipEventRecord(ev[0], sc.st[0]));
		}
		const int n = sc.launch_batch(&r->jobs[i], i1 - i, capture ? capture + (size_t)(i - i0) * sc.fsz : nullptr);
		if (n <= 0) return -1;
		if (ev) {
			CHECK(hipEventRecord(ev[1], sc.st[0]));
			sc.tm.kernel_launches++;
		}
		for (int k = i; k < i + n; ++k) {
			sc.tm.pictures++;
			sc.tm.record_bytes += r->pics[k].record_bytes;
			sc.tm.ref_bytes += r->pics[k].ref_bytes;
			sc.tm.frame_bytes += r->pics[k].frame_bytes;
		}
		i += n;
	}
	return 0;
}

extern "C" int m2dec_amd_hip_replay_run(m2dec_amd_hip_replay_t *r, int passes)
{
	if (!r) return -1;
	CHECK(hipSetDevice(r->sc.dev));
	const char *lim_env = getenv("M2DEC_AMD_REPLAY_LIMIT"); /* debug: first N pictures only */
	const int lim = lim_env && atoi(lim_env) > 0 ? std::min(atoi(lim_env), r->npics) : r->npics;
	const bool isolate = getenv("M2DEC_AMD_REPLAY_ISOLATE_LAST") != nullptr; /* debug: last picture alone */
	for (int k = 0; k < passes; ++k) {
		if (isolate && lim > 1) {
			if (replay_batches(r, 0, lim - 1, true, nullptr) < 0 || r->sc.sync_all() < 0) return -1;
			m2dec_amd_debug_stamps_clear();
			if (replay_batches(r, lim - 1, lim, true, nullptr) < 0) return -1;
		} else if (replay_batches(r, 0, lim, true, nullptr) < 0) {
			return -1;
		}
	}
	return 0;
}

extern "C" int m2dec_amd_hip_replay_sync(m2dec_amd_hip_replay_t *r)
{
	if (!r) return -1;
	if (r->sc.sync_all() < 0) return -1;
	return r->sc.check_err();
}

extern "C" int m2dec_amd_hip_replay_timing(m2dec_amd_hip_replay_t *r, m2dec_amd_hip_timing_t *out, int reset)
{
	if (!r || !out) return -1;
	CHECK(hipSetDevice(r->sc.dev));
	for (size_t i = 0; i + 2 <= r->tev_used; i += 2) {
		float ms;
		hipEvent_t *e = &r->tev[i];
		CHECK(hipEventSynchronize(e[1]));
		if (hipEventElapsedTime(&ms, e[0], e[1]) == hipSuccess) r->sc.tm.picture_us += ms * 1e3;
	}
	r->tev_used = 0;
	*out = r->sc.tm;
	if (reset) memset(&r->sc.tm, 0, sizeof(r->sc.tm));
	return 0;
}

/* MD5 of every picture in decode order.  per_picture false: ONE batch launch of the whole trace (k_batch),
 * exactly as replay_run runs it, each picture copied out by its last row workgroup before its slot is reused;
 * true: one k_picture launch per picture, synchronised (the decode path's kernel). */
static int replay_md5_impl(m2dec_amd_hip_replay_t *r, char *md5s, bool dbg)
{
	if (!r || !md5s) return -1;
	Sched &sc = r->sc;
	size_t ls = (size_t)sc.W * sc.H;
	std::vector<uint8_t> host(ls * 3 / 2);
	CHECK(hipSetDevice(sc.dev));
	if (sc.sync_all() < 0) return -1; /* no earlier work of either launch path may still run */
	uint8_t *cap = nullptr;
	if (!dbg) {
		CHECK(hipMalloc(&cap, sc.fsz * (size_t)r->npics));
		if (replay_batches(r, 0, r->npics, false, cap) < 0 || m2dec_amd_hip_replay_sync(r) < 0) {
			(void)hipFree(cap);
			return -1;
		}
	}
	for (int i = 0; i < r->npics; ++i) {
		if (dbg) {
			if (getenv("M2DEC_AMD_DEBUG"))
				fprintf(stderr, "replay_md5: picture %d slot %d n_inter %d n_intra %d\n", i, r->pics[i].slot, r->pics[i].n_inter, r->pics[i].n_intra);
			if (replay_enqueue(r, i, false) < 0 || m2dec_amd_hip_replay_sync(r) < 0) return -1;
			CHECK(hipMemcpy(host.data(), sc.frames + (size_t)r->pics[i].slot * sc.fsz, ls * 3 / 2, hipMemcpyDeviceToHost));
		} else if (hipMemcpy(host.data(), cap + (size_t)i * sc.fsz, ls * 3 / 2, hipMemcpyDeviceToHost) != hipSuccess) {
			(void)hipFree(cap);
			return -1;
		}
		m2d_frame_t f;
		memset(&f, 0, sizeof(f));
		f.luma = host.data();
		f.chroma = host.data() + ls;
		f.width = (int16_t)sc.W;
		f.height = (int16_t)sc.H;
		for (int k = 0; k < 4; ++k) f.crop[k] = (int16_t)r->crop[k];
		m2dec_amd_frame_md5(&f, md5s + 35 * (size_t)i);
	}
	if (cap) (void)hipFree(cap);
	return 0;
}

/* The raw NV12 pictures (W x H luma, then W x H / 2 interleaved chroma, uncropped) in decode order from ONE
 * batch launch of the whole trace, exactly as m2dec_amd_hip_replay_md5 runs it: a diagnostic for locating the
 * first wrong macroblock of a picture (tools/replay_diff.py).  out holds npics * W * H * 3 / 2 bytes. */
extern "C" int m2dec_amd_hip_replay_capture(m2dec_amd_hip_replay_t *r, uint8_t *out, size_t n)
{
	if (!r || !out) return -1;
	Sched &sc = r->sc;
	const size_t fb = (size_t)sc.W * sc.H * 3 / 2;
	if (n < fb * (size_t)r->npics) return -1;
	CHECK(hipSetDevice(sc.dev));
	if (sc.sync_all() < 0) return -1;
	uint8_t *cap = nullptr;
	CHECK(hipMalloc(&cap, sc.fsz * (size_t)r->npics));
	int rc = 0;
	if (replay_batches(r, 0, r->npics, false, cap) < 0 || m2dec_amd_hip_replay_sync(r) < 0) rc = -1;
	for (int i = 0; rc == 0 && i < r->npics; ++i)
		if (hipMemcpy(out + fb * (size_t)i, cap + (size_t)i * sc.fsz, fb, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
	(void)hipFree(cap);
	return rc;
}

/* Default: the batch path (k_batch); M2DEC_AMD_DEBUG=1: the decode path's kernel, one picture per launch */
extern "C" int m2dec_amd_hip_replay_md5(m2dec_amd_hip_replay_t *r, char *md5s)
{
	return replay_md5_impl(r, md5s, getenv("M2DEC_AMD_DEBUG") != nullptr);
}

/* ---- the built-in known-answer test.  Round 5 found that intra_row inlined into row_pair
 * reconstructed every I picture wrongly; round 6 showed the optimized LLVM IR of that build identical to one that
 * reconstructs bit-exactly and differing only in the register budget it is compiled for (waves-per-eu 4 = 128
 * VGPRs: wrong or faulting code; 3 = 168 VGPRs: exact; DESIGN.md §5 "Compiler hazards"): the AMDGPU back end
 * miscompiled that code.  A product library whose kernels were compiled wrongly must not decode anything, so
 * the first HIP back end of a process on a device reconstructs the known-answer streams of selftest_data.h
 * (tools/make_selftest.py: h264gen coverage streams, I P B B with PCM, constrained intra, deblocking idc 2,
 * explicit weights; MD5s from the CPU oracle) through both launch paths — k_batch and k_picture — and refuses
 * to start if any picture differs.  M2DEC_AMD_SELFTEST=0 skips it. */
#include "selftest_data.h"

extern "C" int m2dec_amd_hip_selftest(int device)
{
	int bad = 0;
	for (size_t k = 0; k < sizeof(k_selftest) / sizeof(k_selftest[0]) && !bad; ++k) {
		const SelftestStream &st = k_selftest[k];
		m2dec_amd_trace_t *t = nullptr;
		if (m2dec_amd_trace_capture(st.data, st.len, &t) != st.npics) {
			m2dec_amd_trace_free(t);
			return -1;
		}
		m2dec_amd_hip_replay_t *r = nullptr;
		if (m2dec_amd_hip_replay_create(t, device, &r) < 0) {
			m2dec_amd_trace_free(t);
			return -1;
		}
		std::vector<char> md5(35 * (size_t)st.npics + 1);
		for (int path = 0; path < 2 && !bad; ++path) {
			if (replay_md5_impl(r, md5.data(), path == 1) < 0) {
				bad = -1;
				break;
			}
			for (int i = 0; i < st.npics; ++i)
				if (memcmp(md5.data() + 35 * (size_t)i, st.md5[i], 32) != 0) {
					fprintf(stderr, "m2dec_amd: SELF-TEST FAILED on device %d: %s picture %d through %s reconstructs to %.32s, "
					        "expected %s — the gfx950 kernels of this build are wrong (compiler?); refusing to decode\n",
					        device, st.name, i, path ? "k_picture" : "k_batch", md5.data() + 35 * (size_t)i, st.md5[i]);
					bad = 1;
					break;
				}
		}
		m2dec_amd_hip_replay_destroy(r);
		m2dec_amd_trace_free(t);
	}
	return bad;
}

/* once per device and process: 0 passed (or skipped), otherwise the back end is not created */
static int selftest_once(int device)
{
	static std::mutex mu;
	static int state[16]; /* 0 not run, 1 passed, 2 failed */
	if (device < 0 || device >= 16) return -1;
	const char *e = getenv("M2DEC_AMD_SELFTEST");
	if (e && atoi(e) == 0) return 0;
	std::lock_guard<std::mutex> lk(mu);
	if (!state[device]) state[device] = m2dec_amd_hip_selftest(device) == 0 ? 1 : 2;
	return state[device] == 1 ? 0 : -1;
}

extern "C" int m2dec_amd_hip_replay_stream(const m2dec_amd_hip_replay_t *r, int i)
{
	if (!r || i < 0 || i >= r->npics) return -1;
	return r->stream[i];
}

extern "C" void m2dec_amd_hip_replay_destroy(m2dec_amd_hip_replay_t *r)
{
	if (r) replay_free(r);
}

/* Diagnostic: copy the per-stream scratch words and the error word while kernels may still run
 * (separate non-blocking stream). */
extern "C" int m2dec_amd_hip_replay_debug_scratch(m2dec_amd_hip_replay_t *r, int *out, int n)
{
	if (!r) return -1;
	Sched &sc = r->sc;
	int need = (int)sc.stream_words() * NSTREAMS + 1;
	if (n < need) return -1;
	hipStream_t s;
	CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	CHECK(hipMemcpyAsync(out, sc.prog, sizeof(int) * sc.stream_words() * NSTREAMS, hipMemcpyDeviceToHost, s));
	CHECK(hipMemcpyAsync(out + need - 1, sc.err, sizeof(int), hipMemcpyDeviceToHost, s));
	CHECK(hipStreamSynchronize(s));
	CHECK(hipStreamDestroy(s));
	return need;
}
