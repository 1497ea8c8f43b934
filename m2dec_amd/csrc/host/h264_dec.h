/*
 * m2dec_amd host-side H.264 parser: internal state.
 *
 * The parser reproduces the reference's bitstream semantics (h264.cpp) and emits per-picture
 * reconstruction records (include/m2d_recon.h).  Reference anchors are cited per function.
 */
#ifndef M2DEC_AMD_H264_DEC_H
#define M2DEC_AMD_H264_DEC_H

#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include "m2d.h"
#include "m2d_recon.h"
#include "m2dec_amd.h"
#include "h264_spec_tables.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- bit reader (RBSP) */
typedef struct {
	const uint8_t *p;   /* next byte to load */
	const uint8_t *end;
	uint64_t cache;     /* MSB-aligned */
	int bits;           /* valid bits in cache */
} h264_bits_t;

static inline void hb_init(h264_bits_t *b, const uint8_t *p, size_t len)
{
	b->p = p;
	b->end = p + len;
	b->cache = 0;
	b->bits = 0;
}

static inline void hb_fill(h264_bits_t *b)
{
	while (b->bits <= 56) {
		uint64_t byte = (b->p < b->end) ? *b->p : 0;
		b->p++;
		b->cache |= byte << (56 - b->bits);
		b->bits += 8;
	}
}

static inline uint32_t hb_show(h264_bits_t *b, int n)
{
	if (b->bits < n) hb_fill(b);
	return n ? (uint32_t)(b->cache >> (64 - n)) : 0;
}

static inline void hb_skip(h264_bits_t *b, int n)
{
	if (b->bits < n) hb_fill(b);
	b->cache <<= n;
	b->bits -= n;
}

static inline uint32_t hb_get(h264_bits_t *b, int n)
{
	uint32_t v;
	if (n == 0) return 0;
	if (n > 32) n = 32;
	if (b->bits < n) hb_fill(b);
	v = (uint32_t)(b->cache >> (64 - n));
	b->cache <<= n;
	b->bits -= n;
	return v;
}

static inline uint32_t hb_get1(h264_bits_t *b)
{
	return hb_get(b, 1);
}

static inline uint32_t hb_ue(h264_bits_t *b)
{
	int lz;
	if (b->bits < 32) hb_fill(b);
	if (b->cache == 0) { hb_skip(b, 32); return 0xffffffffu; }
	lz = __builtin_clzll(b->cache);
	if (lz > 31) { hb_skip(b, 32); return 0xffffffffu; }
	hb_skip(b, lz);
	return hb_get(b, lz + 1) - 1;
}

static inline int32_t hb_se(h264_bits_t *b)
{
	uint32_t ue = hb_ue(b);
	int32_t t = (int32_t)((ue + 1) >> 1);
	return (ue & 1) ? t : -t;
}

/* bits consumed so far (position) */
static inline size_t hb_pos(const h264_bits_t *b, const uint8_t *start)
{
	return (size_t)(b->p - start) * 8 - (size_t)b->bits;
}

/* ---------------------------------------------------------------- CABAC engine */
typedef struct {
	uint64_t value;     /* codIOffset in the top, `bits` look-ahead bits below */
	uint32_t range;     /* codIRange, 9 bits */
	int bits;
	const uint8_t *p, *end;
} h264_cabac_eng_t;

typedef struct {
	h264_cabac_eng_t e;        /* kept apart from ctx so hot loops can hold it in registers */
	uint8_t ctx[H264_NUM_CTX]; /* (pStateIdx << 1) | valMPS */
} h264_cabac_t;

/* ---------------------------------------------------------------- parameter sets */
typedef struct {
	int valid;
	int profile_idc, level_idc, constraint_flags;
	int poc_type;
	int log2_max_frame_num;
	int log2_max_poc_lsb;
	int num_ref_frames;
	int delta_pic_order_always_zero_flag;
	int offset_for_non_ref_pic;
	int offset_for_top_to_bottom_field;
	int num_ref_frames_in_poc_cycle;
	int32_t offset_for_ref_frame[256]; /* cumulative, as the reference stores it (h264.cpp:291-299) */
	int gaps_allowed;
	int width, height; /* coded, samples */
	int max_dpb_in_mbs;
	int frame_mbs_only_flag;
	int direct_8x8_inference_flag;
	int crop[4];       /* left, right, top, bottom in samples (h264.cpp:351) */
} h264_sps_t;

typedef struct {
	int valid;
	int sps_id;
	int entropy_coding_mode_flag;
	int pic_order_present_flag;
	int num_ref_idx_active[2];
	int weighted_pred_flag;
	int weighted_bipred_idc;
	int pic_init_qp;
	int chroma_qp_index[2];
	int deblocking_filter_control_present_flag;
	int constrained_intra_pred_flag;
	int redundant_pic_cnt_present_flag;
	int transform_8x8_mode_flag;
} h264_pps_t;

/* ---------------------------------------------------------------- references / DPB (reference h264.h:236-320) */
enum { REF_UNUSED = 0, REF_SHORT = 1, REF_LONG = 2 };

typedef struct {
	int16_t in_use;
	int16_t frame_idx;
	uint32_t num;  /* frame_num (short) / long-term idx */
	int32_t poc;
	int16_t col;   /* index of the co-located motion store attached to this entry (list 1 only) */
} h264_ref_t;

typedef struct {
	int poc;
	int16_t frame_idx;
	int8_t is_idr;
	int8_t is_terminal;
} h264_dpb_elem_t;

typedef struct {
	int size, max, output, is_ready;
	h264_dpb_elem_t data[16];
} h264_dpb_t;

/* co-located motion store of one decoded picture (reference h264d_col_pic_t, h264.h:200-215) */
typedef struct {
	int8_t ref[4];          /* ref_idx per 8x8 (-1 intra) */
	int16_t mv[16][2];      /* raster 4x4 */
} h264_colmb_t;

typedef struct {
	int8_t map_col_frameidx[16];
	h264_colmb_t *mb;       /* [H264_COL_ENTRIES(n_mbs)] */
} h264_colpic_t;

/* A co-located store buffer holds one entry more than the picture has MBs: its first 4-aligned int is
 * the progress word of the parse writing the buffer (h264_col_progress; row pipelining, h264_async.c):
 * MBs stored so far, H264_COL_FINAL(n) once the picture parsed, -1 if its parse failed */
#define H264_COL_ENTRIES(n) ((size_t)(n) + 1)
#define H264_COL_FINAL(n) ((n) + 1)
static inline int *h264_col_progress(h264_colmb_t *mb, int n_mbs)
{
	return (int *)(((uintptr_t)(mb + n_mbs) + 3) & ~(uintptr_t)3);
}

/* ---------------------------------------------------------------- per-MB neighbour state */
enum {
	MBT_INxN = 0,       /* I4x4 / I8x8 */
	MBT_I16 = 1,        /* 1..24 */
	MBT_IPCM = 25,
	MBT_P16x16 = 26,
	MBT_P16x8 = 27,
	MBT_P8x16 = 28,
	MBT_P8x8 = 29,
	MBT_P8x8REF0 = 30,
	MBT_SKIP = 31,      /* P_Skip / B_Skip / B_Direct_16x16 (reference h264.h:77-80) */
	MBT_B_FIRST = 32,   /* B_L0_16x16 ... */
	MBT_B8x8 = 53
};

typedef struct {
	int8_t type;        /* unified type (reference adjust_mb_type, h264.cpp:9689) ; -1 = not decoded */
	uint8_t skip;
	uint8_t t8x8;
	uint8_t cbp;
	uint8_t cpm;        /* intra_chroma_pred_mode */
	uint8_t direct;     /* bit per 8x8 partition coded as direct (or skip / direct16x16: 0xf) */
	int16_t slice;      /* slice number in the picture */
	uint32_t cbf;       /* coded_block_flag: 0-15 luma blkIdx, 16 luma DC, 17-18 chroma DC, 19-26 chroma AC */
	uint8_t nnz[16];    /* TotalCoeff per luma 4x4 blkIdx (capped 15) */
	uint8_t nnzc[8];    /* chroma AC: Cb 0-3, Cr 0-3 */
	int8_t ipred[16];   /* Intra4x4PredMode per blkIdx (2 if not intra NxN) */
	int8_t ref[2][4];   /* ref_idx per 8x8 */
	int16_t fidx[2][4]; /* frame_idx of the reference per 8x8 (-1 unused) */
	int16_t mv[2][16][2];
	uint8_t mvd[2][16][2]; /* |mvd| clipped to 255 */
} h264_mbinfo_t;

/* ---------------------------------------------------------------- slice header */
typedef struct {
	int op;
	uint32_t arg1, arg2;
} h264_mmco_t;

typedef struct {
	int first_mb;
	int slice_type;     /* 0 P, 1 B, 2 I */
	int pps_id;
	uint32_t frame_num;
	uint32_t prev_frame_num;
	int idr;
	int nal_ref_idc;
	int nal_unit_type;
	int idr_pic_id;
	int poc;
	/* POC state carried across pictures (reference h264d_slice_header union) */
	uint32_t poc0_lsb, poc0_msb;
	int32_t delta_poc_bottom;
	uint32_t poc1_num_offset;
	int32_t delta_poc[2];
	uint32_t poc2_prev_frameoffset;
	int direct_spatial;
	int num_ref_idx_active[2];
	int cabac_init_idc;
	int qp;
	int disable_deblocking_filter_idc;
	int alpha_off, beta_off; /* *2 */
	/* marking */
	int no_output_of_prior_pics;
	int long_term_reference_flag;
	int adaptive_marking;
	int mmco5;
	h264_mmco_t mmco[16];
	/* weighted prediction */
	int wp_mode;
	int log2wd[2];
	int8_t w[2][32][3];
	int8_t o[2][32][3];
} h264_slice_t;

/* ---------------------------------------------------------------- decoder context */
typedef struct h264_dec h264_dec_t;

/* Frames the caller still reads after handing them back to the decoder (the MD5 threads of
 * m2dec_amd_decode_stream_md5 hash the caller's frame buffers in place): the frame LRU skips them
 * (find_empty_frame) and the driver frees frame memory only once none is held. */
typedef struct m2dec_hold {
	pthread_mutex_t mu;
	pthread_cond_t cv;
	const uint8_t *luma[64];
	int cnt[64];
	int n;
	long waits;   /* times the frame LRU waited for a release */
} m2dec_hold_t;
void m2dec_hold_init(m2dec_hold_t *h);
void m2dec_hold_destroy(m2dec_hold_t *h);
void m2dec_hold_add(m2dec_hold_t *h, const uint8_t *luma);
void m2dec_hold_release(m2dec_hold_t *h, const uint8_t *luma);
void m2dec_hold_wait_idle(m2dec_hold_t *h);
int m2dec_hold_busy(const m2dec_hold_t *h, const uint8_t *luma); /* h->mu held */

struct h264_dec {
	/* input */
	dec_bits stream_i;
	dec_bits *stream;
	int device;
	int (*header_callback)(void *, void *);
	void *header_callback_arg;
	uint8_t *nal;            /* current NAL as RBSP (emulation prevention removed) */
	size_t nal_len, nal_cap;
	int nal_pending;         /* a NAL was read but not consumed (new picture detected) */
	int nal_replay;          /* the current NAL is handed out again by the next h264_nal_next */
	int eos;                 /* the refill callback reported the end of the data in this decode_picture call */

	h264_sps_t sps[32];
	h264_pps_t pps[256];
	int active_sps;

	/* frames */
	int num_frames;
	m2d_frame_t frames[H264D_MAX_FRAME_NUM];
	int8_t lru[H264D_MAX_FRAME_NUM];
	int frames_ready;
	int curr_idx;            /* frame slot of the current picture */
	h264_ref_t refs[2][16];  /* the two reference arrays (reference h264d_frame_info_t.refs) */
	h264_dpb_t dpb;
	int dpb_max_arg;

	/* co-located stores: 16 attached to refs[1][i] + 1 current (reference init_mb_buffer) */
	h264_colpic_t colpic[17];
	int curr_col;            /* index into colpic of the current picture's store */

	/* picture geometry / state */
	int mb_w, mb_h, n_mbs;
	int mbs_decoded;
	int mbs_coded;          /* distinct MBs of the picture coded so far (mbs_decoded counts an MB of
	                           overlapping slices twice) */
	int slice_num;
	int in_picture;
	int last_firstline;      /* picture-final `firstline` (deblock idc 2 quirk) */
	h264_slice_t sh;
	h264_mbinfo_t *mbi;      /* [n_mbs] */
	size_t mbi_cap;

	/* per-slice derived */
	int8_t map_col_to_list0[16];
	int16_t dist_scale[16];

	/* records */
	m2r_backend_t backend;
	int have_backend;
	m2r_picture_t *pic;
	int slice_rec;           /* index of the current slice record */

	/* per-picture deblock parameters per slice number */
	int8_t slice_idc[1024];
	int8_t slice_alpha[1024], slice_beta[1024];

	/* CABAC / bit reader of the current slice */
	h264_bits_t bs;
	h264_cabac_t cabac;
	const uint8_t *slice_rbsp, *slice_rbsp_end, *cabac_start;
	size_t slice_rbsp_bits;     /* bit position of the rbsp_stop_one_bit */

	/* statistics */
	uint64_t pictures;

	/* parse-ahead pipeline (h264_async.c); NULL: slice data parsed on the caller's thread */
	struct h264_async *as;
	m2dec_hold_t *hold;      /* frames the caller holds (NULL: none) */
	int parse_threads;       /* requested workers (m2dec_amd_h264_set_parse_threads / env) */
	int par_first_mb;        /* slice-parallel parse: this slice's first MB; the MB-edge bS toward an MB
	                            before it (an earlier slice, parsed concurrently) is left to h264_fix_bs */
	/* row-pipelined co-located stores (h264_async.c "Co-located row pipelining"; worker contexts only):
	 * col_pub: progress word this picture's parse publishes into as its MBs' co-located motion is stored;
	 * col_sub: progress word of the picture whose store this B picture reads, still being parsed — direct
	 * prediction of MB addr waits until it passes addr (col_sub_ok: MBs known stored; col_sub_fail: that
	 * parse failed) */
	int *col_pub;
	const int *col_sub;
	int col_sub_ok, col_sub_fail;
	int col_pub_delay_us;    /* (tests: M2DEC_AMD_COL_PIPE_DELAY_US, a pause after each published MB row) */
	/* 1: this is the pipeline's lookahead context: it runs the header-level state machine ahead of
	 * the API-visible context, names pictures by virtual frame ids instead of frame slots (no DPB
	 * output, no caller frames, no header callback) and creates the slice-data jobs */
	int lookahead;
	long ahead_submits;       /* pictures submitted before this (API) context closed them (decode ahead) */
	int vid_next;            /* lookahead: round-robin cursor of the virtual frame id allocator */
	int stats;               /* M2DEC_AMD_ASYNC_STATS: time spent delivering frames */
	double t_drain, t_sync;

	/* process registry (h264_api.c): the caller's context memory holds only a handle naming this state */
	const void *owner;       /* the caller's context address this state was initialised on */
	uint64_t gen;            /* handle generation */
	struct h264_dec *reg_next;
	int in_call;             /* API calls in progress (registry mutex) */
	double last_call;        /* CLOCK_MONOTONIC seconds of the last API call */
	int finished;            /* the last decode_picture returned -2 (end of the data) */
	int drained;             /* ... and a peek / get since then found the DPB empty (registry: reclaimable) */
	int fault;               /* a frame could not be delivered: every later decode_picture returns -1 */
};

/* h264_syntax.c */
int h264_parse_sps(h264_dec_t *d, h264_bits_t *b);
int h264_parse_pps(h264_dec_t *d, h264_bits_t *b, size_t rbsp_len);
int h264_slice_header(h264_dec_t *d, h264_bits_t *b, int nal_unit_type, int nal_ref_idc);
int h264_picture_begin(h264_dec_t *d);
int h264_picture_finish(h264_dec_t *d);
void h264_picture_resolve_deblock(h264_dec_t *d);
void h264_fix_bs(h264_dec_t *d, int addr);
int h264_picture_mark(h264_dec_t *d);
void h264_dpb_init(h264_dpb_t *dpb, int maxsize);
int h264_dpb_peek(h264_dpb_t *dpb, int bypass);
int h264_dpb_pop(h264_dpb_t *dpb, int bypass);

/* h264_mb.c */
int h264_slice_data(h264_dec_t *d);
long long h264_col_spin_ns(void); /* time parse workers spent waiting for co-located rows (col_wait) */

/* h264_async.c */
/* h264_syntax.c: reference-picture path counters (m2dec_amd_h264_parser_hits) */
enum {
	H264_HIT_MOD0 = 0,   /* ref_pic_list_modification idc 0, 1, 2 (long-term) */
	H264_HIT_MMCO1 = 3,  /* MMCO 1 .. 6 */
	H264_HIT_LT_LIST = 9, /* a long-term picture in an active list */
	H264_HIT_POC1 = 10, H264_HIT_POC2 = 11,
	H264_HIT_TD_LT = 12, /* temporal direct onto a long-term L0 picture (zero vectors) */
	H264_HIT_LT_IDR = 13, /* IDR long_term_reference_flag */
	H264_HIT_FN_WRAP = 14 /* a P list across the frame_num wrap */
};
void h264_hit(int i);

/* timeline.c: M2DEC_AMD_TIMELINE diagnostics (no-op unless set) */
void m2d_tl(int kind, long a, long b);

int h264_async_start(h264_dec_t *d, int threads);
int h264_async_add_slice(h264_dec_t *d);
int h264_async_close(h264_dec_t *d);
int h264_async_drain(h264_dec_t *d, int slot);
int h264_async_pump_step(h264_dec_t *d);
int m2dec_parse_busy(void); /* parse-pool workers inside a job right now (all pipelines) */
/* parcopy.c: a large copy (up to 4 pieces) spread over a process-wide thread crew */
enum { M2DEC_CREW_SUBMIT, M2DEC_CREW_SYNC, M2DEC_CREWS };
void m2dec_par_memcpy(int crew, int n, void *const *dst, const void *const *src, const size_t *len);
void h264_async_stop(h264_dec_t *d);
void h264_async_records_wait(h264_dec_t *d);
/* pinned host memory from the device runtime (runtime.hip; NULL without a device) */
void *m2dec_amd_pinned_alloc(size_t n);
void m2dec_amd_pinned_free(void *p);
double h264_async_parse_seconds(h264_dec_t *d, long *par, long *par_fallback);
int h264_async_nal_next(h264_dec_t *d);
void h264_async_resume(h264_dec_t *d);
void h264_async_la_sps(h264_dec_t *la);
void h264_async_api_sps(h264_dec_t *d);
int h264_async_sps(h264_dec_t *d);
int h264_async_push_nal(h264_dec_t *la);
void h264_async_trim(h264_dec_t *d);
/* the process-wide job pool (h264_async.c): free every pooled job; page-locked bytes of job arenas (all, and
 * pooled) */
void h264_async_pool_release(void);
/* numa.c: the library's threads near the GPU of the process's first device back end (bus id from
 * hipDeviceGetPCIBusId); each library thread calls m2d_place_self before its work */
void m2d_place_device(const char *bus_id);
void m2d_place_self(void);
/* cpushare.c: this process's host CPU share (affinity ∩ cgroup quota ÷ the node's GPU ranks), and the gate that
 * keeps parse work (m2d_cpu_primary, counted) and MD5 batches (m2d_cpu_enter / leave, waiting) within
 * m2d_cpu_slots() busy threads */
int m2d_cpu_share(void);
int m2d_cpu_slots(void);
void m2d_cpu_primary(int delta);
void m2d_cpu_enter(void);
void m2d_cpu_leave(void);
int m2d_cpu_share_probe(const char *root, int ranks, int aff_cpus, long *quota_milli, int *aff_out);
long long h264_async_pinned_bytes(long long *pooled);

/* bitio.c */
int h264_nal_next(h264_dec_t *d);

/* h264_api.c: the NAL loop of decode_picture, shared by the API context and the lookahead context */
int h264_decode_loop(h264_dec_t *d);
/* the decoder state behind a caller context initialised by h264d_func->init (NULL: none / evicted) */
h264_dec_t *h264_state(void *ctx);
int h264_decode_stream_held(const uint8_t *data, size_t len, const m2r_backend_t *backend, int device, int dpb,
                            int parse_threads, int extra, m2dec_hold_t *hold,
                            void (*on_frame)(void *arg, const m2d_frame_t *f), void (*on_end)(void *arg), void *arg,
                            m2dec_amd_stats_t *stats);

#ifdef __cplusplus
}
#endif
#endif
