/*
 * H.265 / HEVC decoder behind the reference's m2d_func_table_t (h265d_func, h265.h:37, h265.cpp:5010-5025):
 * the host parses NAL units, parameter sets, slice headers and CABAC slice data into per-picture
 * reconstruction records (include/m2d_recon.h h265r_*); a back end reconstructs them (the gfx950 one,
 * m2dec_amd/csrc/hip/h265_hip.hip; tests: the CPU oracle, oracle/h265_oracle.c).
 *
 * Scope is the reference's own: Main profile, 8-bit 4:2:0, one slice per picture decoded per
 * decode_picture call (h265.cpp:4849-4866), NAL types TRAIL_N / TRAIL_R / IDR_W_RADL
 * (h265.cpp:4872-4877), no PCM, transquant bypass, cu_qp_delta, scaling lists, weighted prediction,
 * long-term references or list modification (all assert(0) in the reference: h265.cpp:333, 768, 782,
 * 832, 3008, 4024, 4092).  I slices are decoded; P / B slices are rejected (-1) until the inter
 * path exists.
 */
#ifndef M2DEC_H265_DEC_H
#define M2DEC_H265_DEC_H
#include <stdint.h>
#include <stddef.h>
#include "m2d.h"
#include "m2d_recon.h"

#ifdef __cplusplus
extern "C" {
#endif

/* context offsets: the syntax-element order of h265modules.h:303-331 (tools/gen_h265_tables.py) */
#define H265_CTX_SAO_MERGE 0
#define H265_CTX_SAO_TYPE 1
#define H265_CTX_SPLIT_CU 2
#define H265_CTX_TQ_BYPASS 5
#define H265_CTX_CU_SKIP 6
#define H265_CTX_PRED_MODE 9
#define H265_CTX_PART_MODE 10
#define H265_CTX_PREV_INTRA_LUMA 14
#define H265_CTX_INTRA_CHROMA 15
#define H265_CTX_RQT_ROOT_CBF 16
#define H265_CTX_MERGE_FLAG 17
#define H265_CTX_MERGE_IDX 18
#define H265_CTX_INTER_PRED_IDC 19
#define H265_CTX_REF_IDX 24
#define H265_CTX_MVP_FLAG 26
#define H265_CTX_SPLIT_TRANSFORM 27
#define H265_CTX_CBF_LUMA 30
#define H265_CTX_CBF_CHROMA 32
#define H265_CTX_ABS_MVD_GT 36
#define H265_CTX_CU_QP_DELTA 38
#define H265_CTX_TSKIP 40
#define H265_CTX_LAST_X 42
#define H265_CTX_LAST_Y 60
#define H265_CTX_CSBF 78
#define H265_CTX_SIG 82
#define H265_CTX_GT1 124
#define H265_CTX_GT2 148
#define H265_NUM_CTX 154

extern const int8_t h265_cabac_init_mn[3][H265_NUM_CTX][2];

/* NAL unit types decoded by the reference (h265modules.h:234-251) */
enum { H265_TRAIL_N = 0, H265_TRAIL_R = 1, H265_BLA_W_LP = 16, H265_BLA_N_LP = 18, H265_IDR_W_RADL = 19,
       H265_IDR_N_LP = 20, H265_RSV_IRAP_23 = 23, H265_VPS = 32, H265_SPS = 33, H265_PPS = 34, H265_AUD = 35 };

typedef struct {
	uint8_t num_pics[2];      /* negative, positive */
	uint16_t used[2];
	int16_t delta_poc[2][16];
	uint8_t total_curr;
} h265_st_rps_t;

typedef struct {
	int valid;
	int chroma_format_idc, separate_colour_plane;
	int pic_w, pic_h;
	int crop[4];              /* conformance window offsets as coded (units of 2 samples) */
	int bit_depth_luma_m8, bit_depth_chroma_m8;
	int log2_max_poc_lsb;
	int log2_min_cb, log2_ctb, log2_min_tb, log2_max_tb;
	int max_th_depth_inter, max_th_depth_intra;
	int scaling_list_enabled, amp, sao, pcm;
	int log2_min_pcm, log2_max_pcm;
	int num_st_rps;
	h265_st_rps_t st_rps[64];
	int long_term_present, num_lt_sps;
	int temporal_mvp, strong_intra_smoothing;
	/* derived (set_ctb_info, h265.cpp:536-550) */
	int ctb_cols, ctb_rows, stride, num_ctb_log2;
	int frame_num;            /* min(num_long_term_ref_pics_sps + num_short_term_ref_pic_sets, 8) */
} h265_sps_t;

typedef struct {
	int valid;
	int sps_id;
	int dependent_slices, output_flag_present, num_extra_bits;
	int sign_hiding, cabac_init_present;
	int num_ref_idx_default[2];
	int init_qp;
	int constrained_intra, transform_skip, cu_qp_delta, diff_cu_qp_delta_depth;
	int cb_qp_offset, cr_qp_offset, slice_chroma_qp_offsets_present;
	int weighted_pred, weighted_bipred, transquant_bypass, tiles, entropy_sync;
	int loop_filter_across_slices;
	int deblocking_control, deblocking_override_enabled, pps_deblocking_disabled;
	int pps_beta_offset_div2, pps_tc_offset_div2;
	int scaling_list_data, lists_modification, log2_parallel_merge_level, slice_header_extension;
} h265_pps_t;

typedef struct {
	int nal_type;
	int first_slice, no_output_of_prior_pics, pps_id;
	int dependent, address;
	int slice_type, pic_output;
	int poc_lsb, poc_msb, poc;          /* h265.cpp:736-750 (kept across slices) */
	h265_st_rps_t rps;
	int temporal_mvp;
	int sao_luma, sao_chroma;
	int num_ref_idx[2];
	int mvd_l1_zero, cabac_init_flag, col_from_l0, col_ref_idx, max_merge_cand;
	int ref_poc[2][16];                 /* the reference lists (init_ref_pic_list, h265.cpp:795-820) */
	int8_t ref_frame[2][16];
	int slice_qp, qpc_delta[2];
	int deblocking_disabled, deblocking_override;
	int beta_offset_div2, tc_offset_div2; /* set only by an override: kept from the previous slice otherwise (h265.cpp:894-901) */
	int loop_filter_across_slices;
} h265_slice_t;

typedef struct {
	int poc;
	int8_t frame_idx;
	uint8_t is_idr;
	long seq; /* parse ahead: the dispatched picture's sequence number (-1 on the sequential path) */
} h265_dpb_elem_t;

/* prediction info of a block (pred_info_t, h265modules.h:420-423): compared with memcmp by the merge list */
typedef struct {
	int16_t mv[2][2];
	int8_t ref[2];
} h265_pred_t;

/* what later blocks read of a 4x4 luma unit of the current picture (h265d_neighbour_t, h265modules.h:425-434) */
typedef struct {
	uint8_t pu_intra, pu_nz, tu_intra, tu_nz, skip, pad;
	h265_pred_t pred;
} h265_nb_t;

/* a 16x16 unit of a picture's motion field (colpics_t, h265modules.h:731-874) */
typedef struct {
	uint8_t intra, pad;
	h265_pred_t pred;
} h265_col_t;

/* the decoder state: the caller's context memory (m2d_func_table_t.context_size), plus heap arrays */
typedef struct h265_dec {
	dec_bits stream_i;
	int (*header_callback)(void *, void *);
	void *header_callback_arg;
	/* NAL unit bytes, emulation prevention removed */
	uint8_t *unit;
	size_t unit_len, unit_cap;
	int pending;
	h265_sps_t sps[16];
	h265_pps_t pps[64];
	h265_slice_t sh;
	/* frames and output (h265d_frame_info_t / h265d_dpb_t, h265modules.h:448-474) */
	int num_frames;
	m2d_frame_t frames[H265R_MAX_FRAMES];
	int8_t lru[H265R_MAX_FRAMES];
	int index;                /* frame of the picture being decoded */
	int dpb_size, dpb_max, dpb_output;
	h265_dpb_elem_t dpb[16];
	int frame_w, frame_h;     /* CTB-aligned geometry of the current frames */
	/* the picture's records and parse maps (heap) */
	h265r_picture_t pic;
	size_t cap_tu, cap_coef, cap_map, cap_bs, cap_sao, cap_units;
	uint8_t *cb_log2;         /* per luma 4x4 unit: log2 size of its CU (0: not decoded) */
	uint8_t *ipm;             /* per luma 4x4 unit: intra prediction mode */
	/* inter pictures */
	h265_nb_t *nb;            /* per luma 4x4 unit of the current picture */
	h265_col_t *col[H265R_MAX_FRAMES]; /* per frame: its motion field, 16x16 units (stride (pic_w + 15) / 16) */
	size_t cap_nb, cap_col, cap_pu;
	int8_t col_frame[H265R_MAX_FRAMES][2][16]; /* per frame: the frame slots of its reference lists (frameidx_record_t) */
	int frame_poc[H265R_MAX_FRAMES];   /* h265d_frame_info_t.poc */
	/* reconstruction back end */
	h265r_backend_t be;
	int have_be;
	int device;
	int pictures;
	uint64_t cabac_bins;
	/* parse-ahead pipeline (h265_dec.c "parse-ahead"): heap state, never caller memory; NULL = sequential */
	struct h265_pipe *pipe;
	int threads;              /* parse workers: -1 default (M2DEC_AMD_H265_THREADS, 8), 0 sequential */
	struct m2dec_hold *hold;  /* frames the caller reads after get (h264_dec.h m2dec_hold_t; NULL none): a
	                             sync_frame into such a frame waits for its release */
	uint8_t fresh[16];        /* frames given a new picture since their last sync_frame (only those are written) */
} h265_dec_t;

/* the caller's held frames (the MD5 driver hashing them in place; NULL: none) */
void h265_set_hold(void *ctx, struct m2dec_hold *hold);
/* driver.c: m2dec_amd_decode_h265 with held frames (driver_mt.c, the MD5 driver hashing in place) */
int m2dec_amd_decode_h265_held(const uint8_t *data, size_t len, const h265r_backend_t *be, int device,
                               void (*on_frame)(void *arg, const m2d_frame_t *f), void *arg, struct m2dec_hold *hold,
                               int *last_error);

/* default back end: the gfx950 reconstruction (m2dec_amd/csrc/hip/h265_hip.hip) */
int h265_hip_backend_create(h265r_backend_t *out, int device);

#ifdef __cplusplus
}
#endif
#endif
