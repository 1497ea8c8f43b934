/*
 * m2dec_amd — extra C ABI of libm2dec_amd.so beyond the reference's m2d_func_table_t.
 *
 * Nothing here replaces a reference entry point; these are the hooks a maintainer needs to wire
 * the GPU back end into the reference's callers:
 *   - back-end selection (default: gfx950 HIP back end on `device`),
 *   - explicit release of GPU / heap resources (the reference's context is caller memory only),
 *   - a whole-stream driver equivalent to src/app/h264dec.cpp + m2decoder.h (used by bench/tests),
 *   - direct record-level access to the HIP reconstruction kernels (kernel parity tests).
 */
#ifndef M2DEC_AMD_H
#define M2DEC_AMD_H

#include <stddef.h>
#include <stdint.h>
#include "m2d.h"
#include "m2d_recon.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	int frames_out;
	int pictures;
	int last_error;
	int ahead; /* pictures submitted before the API context reached them (decode ahead, m2d_recon.h bind) */
	/* CLOCK_MONOTONIC seconds: the first decode_picture call, and the last frame delivered to the
	 * writer (on_frame returned; for the MD5 drivers: its MD5 line written) — the fps interval of
	 * SURVEY.md §8d.  setup_s: time inside the first set_frames (back-end creation, frame pinning). */
	double t_start, t_end, setup_s;
	/* the built-in HIP back end only (m2dec_amd_hip_timing_t of the decode): k_picture launches, their
	 * HIP-event time, and their algorithmic bytes (F_write + sum_PU 1.5 w h + R_pic) */
	double kernel_us;
	int64_t kernel_launches;
	int64_t alg_bytes;
	int64_t hold_waits; /* MD5 drivers: times the frame LRU waited for a frame the MD5 threads held */
	/* per-stage host view: record uploads and frame downloads (HIP-event time of the
	 * built-in back end's copies), and the CPU time of the slice-data parse on the parse-ahead workers */
	double h2d_us, d2h_us;
	double parse_cpu_s;
	/* pictures of several slices parsed slice-parallel, and those re-parsed sequentially after a try */
	int64_t slice_par_pictures, slice_par_fallbacks;
	/* the drivers: seconds spent releasing the decoder context after the last frame (outside t_end) */
	double teardown_s;
	/* the built-in HIP back end: frame bytes downloaded (d2h_us above is their copy time), and the host
	 * time of the staging -> caller-frame copies inside peek / get */
	int64_t d2h_bytes;
	double host_copy_us;
} m2dec_amd_stats_t;

/* ABI revision of the structs in this header and m2d_recon.h.  3: m2r_backend_t gained `bind` (decode
 * ahead) and m2dec_amd_stats_t grew to its current size; 4: m2r_backend_t gained `flush` (several
 * pictures per launch); 5: `ready`; 6: `records_busy` (M2R_PIC_EXTERNAL: uploads from the parser's own
 * pinned records).  A caller compiled against another revision
 * checks m2dec_amd_abi_version() before passing either struct; m2dec_amd_h264_set_backend2 accepts an
 * older (smaller) m2r_backend_t by size, and m2dec_amd_stats_size() is the size every stats pointer
 * must have room for. */
#define M2DEC_AMD_ABI_VERSION 6
int m2dec_amd_abi_version(void);
size_t m2dec_amd_stats_size(void);
/* 0 if the host CPU lacks the x86-64-v3 features the host library is built for (decoder inits then
 * fail with a message, cpucheck.c) */
int m2dec_amd_host_cpu_ok(void);

/* Use `be` instead of the default HIP back end for this decoder context (call after init).
 * The context takes ownership: be->destroy is called when the context is released or reclaimed.
 * be == NULL detaches the current back end without destroying it (a borrowed one). */
int m2dec_amd_h264_set_backend(void *ctx, const m2r_backend_t *be);
/* the same with the caller's sizeof(m2r_backend_t): members past be_size are taken as NULL */
int m2dec_amd_h264_set_backend2(void *ctx, const m2r_backend_t *be, size_t be_size);
/* GPU ordinal used by the default back end (call after init, before the first SPS). */
int m2dec_amd_h264_set_device(void *ctx, int device);
/* Slice data of up to `threads` pictures parsed ahead on worker threads (0: on the caller's thread).
 * Default with the built-in HIP back end: $M2DEC_AMD_PARSE_THREADS or 8; with a back end installed by
 * m2dec_amd_h264_set_backend: 0.  Call before the first set_frames. */
int m2dec_amd_h264_set_parse_threads(void *ctx, int threads);
/* Free the state behind a context at once (optional: as in the reference, a caller may also just
 * free the context memory; the library then reclaims the state itself — see h264_api.c). */
void m2dec_amd_h264_release(void *ctx);
/* Diagnostics: how often the H.264 parser took each reference-picture path (list modification idc 0 / 1 / 2,
 * MMCO 1..6, long-term picture in an active list, POC type 1 / 2, temporal direct onto a long-term picture,
 * IDR long_term_reference_flag, P list across the frame_num wrap), process-wide; reset clears them.
 * Returns the counters written. */
#define M2DEC_AMD_H264_HITS 16
int m2dec_amd_h264_parser_hits(long *out, int n, int reset);
/* Diagnostics: every P / B slice's active reference lists (POC, long-term flag per entry; the layout of
 * tools/h264gen --dump-refs) appended to `path` from now on; NULL stops.  0, or -1 if it cannot be opened. */
int m2dec_amd_h264_set_refdump(const char *path);

/* Decoder states alive in the process registry, and how many were reclaimed over the cap. */
int m2dec_amd_h264_registry(int *contexts, long *evicted);

/* Decode a whole Annex-B stream exactly like `h264dec` (m2decoder.h:132-157 output loop).
 * on_frame receives every output frame in output order.  backend may be NULL (a HIP back end is
 * created on `device` and destroyed at the end); a non-NULL backend is borrowed, not destroyed.
 * Returns the number of frames output, or -1 on error. */
int m2dec_amd_decode_stream(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device,
                            void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                            m2dec_amd_stats_t *stats);
/* Same with an explicit DPB size (h264d_func->init's dpb_max: -1 = from the level, 1 = bypass; the
 * reference's `h264dec -b / -d n`). */
int m2dec_amd_decode_stream2(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                             void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                             m2dec_amd_stats_t *stats);

/* HIP back end constructor (m2dec_amd/csrc/hip/recon_hip.hip). */
int m2dec_amd_hip_backend_create(m2r_backend_t *out, int device);
/* Non-zero if a gfx950 device is usable by this process. */
int m2dec_amd_hip_available(void);
/* page-lock host memory for the life of the process (or until unpin); HIP back ends then skip
 * registering caller frames that lie inside it */
int m2dec_amd_hip_pin(void *p, size_t n);
void m2dec_amd_hip_unpin(void *p);

/* Per-kernel timing of the HIP back end since creation (microseconds, HIP events). */
typedef struct {
	double picture_us;      /* kernel time: k_picture launches (decode path) / k_batch launches (replay) */
	double h2d_us, d2h_us;  /* decode path only: record upload, frame download (device -> staging) */
	int64_t pictures;       /* pictures reconstructed */
	int64_t inter_launches, intra_launches, deblock_launches; /* pictures with inter MBs / intra MBs / deblocked */
	int64_t record_bytes;   /* bytes of records uploaded (R_pic summed) */
	int64_t ref_bytes;      /* algorithmic reference bytes read by MC (sum over PUs and lists) */
	int64_t frame_bytes;    /* NV12 bytes written (1.5 W H per picture) */
	int64_t kernel_launches; /* k_picture / k_batch launches timed in picture_us */
	/* decode path: bytes copied device -> pinned staging (d2h_us is their HIP-event time on the copy
	 * stream), and the host time of staging -> caller frame copies inside sync_frame */
	int64_t d2h_bytes;
	double host_copy_us;
} m2dec_amd_hip_timing_t;
int m2dec_amd_hip_backend_timing(const m2r_backend_t *be, m2dec_amd_hip_timing_t *out);

/* The decode path's admission against the device-wide workgroup budget (DESIGN §5 "Forward-progress
 * invariant"): what this back end plans with at its current geometry, and what the device's budget saw. */
typedef struct {
	int resident_per_cu; /* k_picture workgroups resident per CU at this context's geometry */
	int cap_workgroups;  /* ... on the whole device */
	int wg_units;        /* budget units one of its workgroups costs */
	int cap_units;       /* the device's budget in units (all processes) */
	int pics_fit;        /* pictures per launch with which a launch per stream fits the capacity */
	int launch_limit;    /* pictures per launch this context uses (1 while other contexts decode on the device) */
	int streams;         /* launch streams of a decoder context */
	int shared;          /* 1: the budget is the device's cross-process segment (devshare.c) */
	int max_procs;       /* most processes seen holding budget units at once */
	int max_units;       /* most units seen in use at once */
} m2dec_amd_hip_budget_t;
int m2dec_amd_hip_backend_budget(const m2r_backend_t *be, m2dec_amd_hip_budget_t *out);

/* Hardware queues for the HIP runtime of this process: sets GPU_MAX_HW_QUEUES to n unless the caller's
 * environment has it already, and returns the value in effect.  The runtime reads it once, when it starts,
 * so call this before anything in the process uses HIP.  With 5 or more queues a decoder context uses 4
 * launch streams + a copy stream, else 3 (runtime.hip nstreams).  The library itself never changes the
 * caller's HIP configuration; the h264dec CLI and bench.py ask for 8. */
int m2dec_amd_configure_queues(int n);

/* Free what the process keeps pooled between decoder contexts: the parse pool's jobs with their page-locked
 * record arenas, the back ends' pinned record arenas and staging buffers, pooled device buffers (a service
 * that stops decoding for a while).  Live contexts are untouched.  m2dec_amd_pinned_bytes: page-locked bytes
 * of the parse jobs' record arenas (all; pooled in *pooled), bounded by M2DEC_AMD_POOL_PINNED_MB. */
void m2dec_amd_release_pools(void);
long long m2dec_amd_pinned_bytes(long long *pooled);

/* NUMA placement of the library's threads (numa.c): the CPUs chosen for a GPU given its PCI bus id, from
 * <sysfs_root>/sys/bus/pci/devices/<id>/numa_node and .../node<n>/cpulist intersected with the process's
 * affinity (sysfs_root "" = the real sysfs); returns the CPU count written to cpus (node: -1 unknown).
 * m2dec_amd_numa_node: the node the library's threads run on (-1: not placed; M2DEC_AMD_NUMA=0 disables). */
int m2dec_amd_numa_cpus(const char *sysfs_root, const char *pci_bus_id, int *cpus, int max, int *node);
int m2dec_amd_numa_node(void);

/* The host CPU share (cpushare.c): affinity ∩ cgroup CPU quota (v2 cpu.max up the hierarchy, v1 cfs quota)
 * ÷ the node's GPU ranks (ranks <= 0: LOCAL_WORLD_SIZE / M2DEC_AMD_LOCAL_RANKS) for a fake tree under
 * sysfs_root ("" = the real one) and an affinity of aff_cpus CPUs (<= 0: this process's).  *quota_milli: the
 * quota in milli-CPUs (-1 none).  m2dec_amd_cpu_gate: the share this process runs with, its busy-thread slots
 * (parse pool size; MD5 batches wait for a free one), the MD5 batches that waited so far, parse / MD5 work now. */
int m2dec_amd_cpu_share(const char *sysfs_root, int ranks, int aff_cpus, long *quota_milli, int *aff_out);
int m2dec_amd_cpu_gate(int *slots, unsigned long *waits, int *primary, int *busy);

/* The device-wide workgroup budget segment (devshare.c) under an arbitrary key, for tests and
 * diagnostics: open (creating it with cap_units), reserve (1 / 0), release, state, close. */
void *m2dec_amd_share_open(const char *key, int cap_units);
int m2dec_amd_share_try(void *s, int units);
void m2dec_amd_share_release(void *s, int units);
int m2dec_amd_share_state(void *s, int *cap, int *total, int *mine, int *procs, long *reclaimed);
void m2dec_amd_share_close(void *s);
int m2dec_amd_share_others_waiting(void *s);

/* NV12 output MD5 exactly as FileWriterMd5 (filewrite.h:11-29, 99-124): 32 hex chars + "\r\n". */
void m2dec_amd_frame_md5(const m2d_frame_t *f, char out[35]);
/* MD5 lines of n <= 16 frames at once (16-lane AVX-512 multi-buffer MD5 when the CPU has it and the
 * frames share one geometry without horizontal crop; else one by one); 0, or -1 for a bad n */
int m2dec_amd_frames_md5(const m2d_frame_t *f, int n, char (*out)[35]);

/* Throughput drivers over the same decode loop as m2dec_amd_decode_stream (h264dec -O): the HIP back
 * end on `device`, DPB size `dpb` (h264dec -d; -1 auto), one MD5 line (35 bytes) per output frame into
 * md5s (at most `max`), the MD5s on helper threads.  Returns the number of frames delivered or < 0. */
int m2dec_amd_decode_stream_md5(const uint8_t *data, size_t len, int device, int dpb, char *md5s, int max,
                                m2dec_amd_stats_t *stats);
/* the same driver over a borrowed back end (tests: the CPU oracle), with explicit parse / MD5 threads */
int m2dec_amd_decode_stream_md5_backend(const uint8_t *data, size_t len, const m2r_backend_t *backend, int parse_threads,
                                        int md5_threads, char *md5s, int max, m2dec_amd_stats_t *stats);
/* A back end that reconstructs nothing (acquire: one record arena; submit / sync: no-ops): decoding
 * through it times the host parse alone. */
int m2dec_amd_null_backend_create(m2r_backend_t *out);
/* the same with an explicit back end (NULL: HIP) and parse-ahead worker count (-1: default) */
int m2dec_amd_decode_stream3(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                             int parse_threads, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                             m2dec_amd_stats_t *stats);
/* n independent streams decoded concurrently on one device, one host thread and decoder context per
 * stream; frames[i] = frames delivered by stream i (or < 0).  Returns 0 if every stream succeeded. */
int m2dec_amd_decode_streams_md5(int n, const uint8_t *const *datas, const size_t *lens, int device,
                                 char *const *md5s, const int *max, int *frames);

/* M2Decoder (m2decoder.h:33-223) over any function table (h264d_func: h264 = 1, m2d_func: 0): the
 * header callback sizes a Frames pool, the output loop delivers every frame to on_frame in output
 * order; emptify = h264dec -e, skip = h264dec -f n.  Returns the last decode_picture result (-2: end
 * of the data; -1: error) also in *last_error. */
int m2dec_amd_decode_table(const m2d_func_table_t *func, int h264, const uint8_t *data, size_t len, int dpb,
                           int emptify, int skip, void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg,
                           int *last_error);
/* The same with an H.264 back end to borrow (NULL: the HIP back end) and parse-ahead workers (-1 default). */
int m2dec_amd_decode_table2(const m2d_func_table_t *func, int h264, const uint8_t *data, size_t len, int dpb,
                            int emptify, int skip, const m2r_backend_t *backend, int parse_threads,
                            void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error);

/* ---- MPEG-1/2 (m2d_func, m2dec_amd/csrc/host/mpeg2_dec.c) */
/* M2Decoder over m2d_func (as m2dec_amd_decode_table) with the pictures reconstructed on gfx950
 * device `device` (m2dec_amd_m2v_use_gpu), or on the host for device < 0.  Returns the last
 * decode_picture result, or -3 if the device is unusable (no host fallback). */
int m2dec_amd_decode_m2v(const uint8_t *data, size_t len, int device, int emptify,
                         void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error);
/* Free the heap an m2d_func context owns (its start-code unit buffer). */
void m2dec_amd_m2v_release(void *ctx);
/* CLIP255C arguments outside the reference table's domain [-256, 767] seen by a context. */
uint64_t m2dec_amd_m2v_clip_violations(const void *ctx);
/* Reconstruct this context's pictures on gfx950 device `device` (m2dec_amd/csrc/hip/m2v_hip.hip)
 * instead of the host: call after init, before set_frames.  Frames are written into the caller's
 * memory only inside peek / get.  -1 if no device (the context keeps the host reconstruction).
 * m2dec_amd_m2v_release frees the device state.  Host reconstruction only: motion-compensated reads
 * outside the reference frame seen (clamped; the reference reads out of bounds there), and the
 * CLIP255C count above. */
int m2dec_amd_m2v_use_gpu(void *ctx, int device);
uint64_t m2dec_amd_m2v_mc_out_of_frame(const void *ctx);
/* the two counters of the calling thread's last whole-stream m2d_func decode (decode_table* / decode_m2v) */
void m2dec_amd_m2v_last_checks(uint64_t *clip_violations, uint64_t *mc_out_of_frame);
/* GPU MPEG-2 back end, process-wide: HIP-event time of its k_m2v launches, the pictures, and their
 * SURVEY.md §8d algorithmic bytes (frame written + records read + one reference byte per predicted
 * sample per direction) since the last reset; pictures of a destroyed back end are all counted. */
int m2dec_amd_m2v_hip_timing(double *kernel_us, int64_t *pictures, int64_t *bytes, int reset);
/* VLC probes for the table tests: one codeword at the MSB end of bits32.  DCT (table 0 = B.14,
 * 1 = B.15): length incl. the sign bit, run (-1: EOB / escape), sign-folded level (2|l| + s).
 * Plain tables (0: macroblock_address_increment after its leading 0, 1 / 2: dct_dc_size luma /
 * chroma, 3: motion_code after its leading 0, signed): length and value.  0 = invalid code. */
int m2dec_amd_m2v_dct_code(int table, uint32_t bits32, int *run, int *level);
int m2dec_amd_m2v_vlc_code(int table, uint32_t bits32, int *value);
/* Block-level probes (fresh decoder state): the intra DC of component cc (0 luma) with predictor
 * `pred` -> *value (dequantised, << (3 - precision)); the AC coefficients of an intra block (DC in
 * coef[0]) dequantised with q_scale and qmat (NULL: flat 16), mismatch control / oddification
 * applied -> coef[64] raster.  Both return the bits consumed, or -1 on an undefined code. */
int m2dec_amd_m2v_intra_dc(const uint8_t *bits, size_t n, int cc, int dc_precision, int pred, int *value);
int m2dec_amd_m2v_intra_ac(const uint8_t *bits, size_t n, int mpeg2, int intra_vlc_format, int alternate_scan,
                           int q_scale, const uint8_t *qmat, int dc, int16_t coef[64]);

/* ---- H.265 (h265d_func, m2dec_amd/csrc/host/h265_dec.c) */
/* M2Decoder over h265d_func (m2decoder.h MODE_H265): every output frame to on_frame in output order;
 * `be` is a borrowed reconstruction back end (NULL: the gfx950 one on `device`, no host fallback).
 * Returns the last decode_picture result (-2: end of the data). */
int m2dec_amd_decode_h265(const uint8_t *data, size_t len, const h265r_backend_t *be, int device, int emptify,
                          void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, int *last_error);
/* The same loop with the `-O` MD5 line of every frame computed on the MD5 helper threads (16-lane batches,
 * as m2dec_amd_decode_stream_md5): each delivered frame is copied into one of the driver's buffers and
 * hashed there, since the H.265 frame LRU has no holds.  md5s: max x 35 bytes ("hex\r\n\0" each).
 * Returns the frames (>= 0) or -1; *last_error gets decode_picture's last return (-2 at the end). */
int m2dec_amd_decode_h265_md5(const uint8_t *data, size_t len, const h265r_backend_t *be, int device, char *md5s, int max,
                              int *last_error);
/* MPEG-1/2 the same way (m2dec_amd_decode_m2v; device < 0: host reconstruction); -1 also when the GPU
 * reconstruction was asked for and is unusable. */
int m2dec_amd_decode_m2v_md5(const uint8_t *data, size_t len, int device, char *md5s, int max, int *last_error);
/* Reconstruct an h265d_func context's pictures with `be` instead of the gfx950 back end (call after init,
 * before the first SPS; NULL detaches a borrowed one), or on GPU `device`. */
int m2dec_amd_h265_set_backend(void *ctx, const h265r_backend_t *be);
int m2dec_amd_h265_set_device(void *ctx, int device);
/* parse-ahead workers of an H.265 context (0: the whole decode on the caller's thread; default
 * M2DEC_AMD_H265_THREADS, 8); call before the first picture */
int m2dec_amd_h265_set_threads(void *ctx, int threads);
/* Free the heap and device state an h265d_func context owns. */
void m2dec_amd_h265_release(void *ctx);
/* Test hook: the parsed syntax (CU modes, residual levels) of later H.265 decodes into `path`, in
 * tools/h265gen --dump's format (NULL: stop). */
int m2dec_amd_h265_set_dump(const char *path);
/* test hook: coverage counters of the H.265 inter derivation (merge candidate kinds, AMVP predictor
 * sources, bi-prediction, low-delay slices, stale collocated index, motion-based deblocking strengths,
 * intra CUs of inter pictures), process-wide; returns the number of counters */
#define M2DEC_AMD_H265_HITS 16
int m2dec_amd_h265_parser_hits(long *out, int n, int reset);
/* CABAC bins decoded by a context (host-parse measurement). */
uint64_t m2dec_amd_h265_cabac_bins(const void *ctx);
/* The gfx950 H.265 reconstruction back end (m2dec_amd/csrc/hip/h265_hip.hip). */
int m2dec_amd_h265_hip_backend_create(h265r_backend_t *out, int device);
/* Its kernel time (HIP events over the intra / deblocking / SAO launches of a picture, all but the last
 * picture submitted), and the SURVEY.md §8d bytes of the pictures so far: R_pic (records uploaded) and
 * F_write (1.5 W H each).  reset restarts the counts. */
int m2dec_amd_h265_hip_timing(const h265r_backend_t *be, double *kernel_us, int64_t *timed_pictures,
                              int64_t *record_bytes, int64_t *frame_bytes, int reset);

/* ---- record traces (m2dec_amd/csrc/host/trace.c): a stream parsed once, records kept in memory */
typedef struct m2dec_amd_trace m2dec_amd_trace_t;
typedef struct {
	int32_t slot, width_mbs, height_mbs, n_inter, n_coef, n_slices, n_intra, deblock;
	uint64_t off_mb, off_dbk, off_slice, off_inter, off_coef; /* byte offsets into the record buffer */
	int64_t record_bytes;  /* R_pic */
	int64_t ref_bytes;     /* sum over PUs and lists of 1.5 w h */
	int64_t frame_bytes;   /* 1.5 W H */
} m2dec_amd_trace_pic_t;
/* Parse `data` (Annex B) with the host parser; returns the number of pictures or -1. */
int m2dec_amd_trace_capture(const uint8_t *data, size_t len, m2dec_amd_trace_t **out);
int m2dec_amd_trace_info(const m2dec_amd_trace_t *t, int *npics, int *width, int *height, int *nslots, int *nout);
const m2dec_amd_trace_pic_t *m2dec_amd_trace_pictures(const m2dec_amd_trace_t *t);
const uint8_t *m2dec_amd_trace_records(const m2dec_amd_trace_t *t, size_t *len);
const int *m2dec_amd_trace_output_order(const m2dec_amd_trace_t *t); /* picture index per output frame */
int m2dec_amd_trace_crop(const m2dec_amd_trace_t *t, int crop[4]);   /* output crop (m2d_frame_t.crop) */
void m2dec_amd_trace_free(m2dec_amd_trace_t *t);

/* ---- GPU replay of a trace with the records resident in HBM (recon_hip.hip) */
typedef struct m2dec_amd_hip_replay m2dec_amd_hip_replay_t;
int m2dec_amd_hip_replay_create(const m2dec_amd_trace_t *t, int device, m2dec_amd_hip_replay_t **out);
/* n independent streams (same frame size) in one replay: pictures interleaved one per stream in turn,
 * each stream on its own frame slots (at most 64 in all), so one k_batch launch carries all of them.
 * replay_md5 reports pictures in that interleaved order (m2dec_amd_hip_replay_stream gives each one's
 * stream; a stream's pictures keep their decoding order). */
int m2dec_amd_hip_replay_create_multi(const m2dec_amd_trace_t *const *ts, int n, int device, m2dec_amd_hip_replay_t **out);
int m2dec_amd_hip_replay_stream(const m2dec_amd_hip_replay_t *r, int i);
/* Host-only check of the multi-stream slot packing on one trace packed into k slots (tests): 0 when
 * every reference still names the picture it named before, -1 when k slots are too few, 1 + i when
 * picture i would read other content. */
int m2dec_amd_replay_pack_check(const m2dec_amd_trace_t *t, int k);
/* Enqueue `passes` reconstructions of every picture in decoding order (asynchronous). */
int m2dec_amd_hip_replay_run(m2dec_amd_hip_replay_t *r, int passes);
/* Wait for the enqueued work; returns -1 on a device error or wavefront hand-off timeout. */
int m2dec_amd_hip_replay_sync(m2dec_amd_hip_replay_t *r);
/* Per-kernel HIP-event times accumulated by runs since the last reset (call after sync). */
int m2dec_amd_hip_replay_timing(m2dec_amd_hip_replay_t *r, m2dec_amd_hip_timing_t *out, int reset);
/* One checked pass: after every picture, download it and write its MD5 line (35 bytes per picture,
 * decoding order) into md5s. */
int m2dec_amd_hip_replay_md5(m2dec_amd_hip_replay_t *r, char *md5s);
/* Diagnostic: the same checked pass, every picture's raw NV12 bytes (W x H x 3 / 2, uncropped, decoding
 * order) into out (n bytes, at least npics times that); tools/replay_diff.py locates wrong macroblocks. */
int m2dec_amd_hip_replay_capture(m2dec_amd_hip_replay_t *r, unsigned char *out, size_t n);
void m2dec_amd_hip_replay_destroy(m2dec_amd_hip_replay_t *r);
/* The HIP back end's built-in known-answer test (runtime.hip; data: tools/make_selftest.py): two small coverage
 * streams reconstructed through k_batch and k_picture against their oracle MD5s.  0 = every picture exact,
 * 1 = a picture differs (the kernels of this build are wrong: the back end refuses to start), -1 = no device.
 * m2dec_amd_hip_backend_create runs it once per process and device (M2DEC_AMD_SELFTEST=0 skips it). */
int m2dec_amd_hip_selftest(int device);

#ifdef __cplusplus
}
#endif
#endif
