/*
 * m2dec_amd MPEG-1/2 video decoder (CPU): BASELINE.json configs[0], "MPEG-2 MP@ML 720x480 I-frame-only
 * .m2v on reference CPU path (plumbing, no GPU)", behind the reference's m2d_func table
 * (mpeg2.cpp:1800-1811).  Intra pictures are decoded completely (intra DC / AC VLC, dequant,
 * mismatch control / MPEG-1 oddification, the reference's integer Chen-Wang IDCT, frame / field DCT
 * placement, concealment motion vectors parsed); P and B frame pictures with frame and field
 * prediction (motioncomp.cpp), reconstructed from per-MB records on the CPU or the GPU.
 */
#ifndef M2DEC_AMD_MPEG2_DEC_H
#define M2DEC_AMD_MPEG2_DEC_H

#include <stdint.h>
#include <stddef.h>
#include "m2d.h"
#include "m2d_recon.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	const char *code;
	int value;
} m2v_code_t;

typedef struct {
	const char *code;
	int run, level;
} m2v_dct_code_t;

extern const m2v_code_t m2v_mb_inc[], m2v_dc_luma[], m2v_dc_chroma[], m2v_motion_code[];
extern const m2v_code_t m2v_mb_type_p[], m2v_mb_type_b[], m2v_cbp[];
extern const m2v_dct_code_t m2v_dct0[], m2v_dct1[];
extern const int m2v_q_scale[2][32];
extern const uint8_t m2v_scan[2][64];
extern const uint8_t m2v_default_intra_qmat[64];

#define M2V_MAX_FRAMES 16 /* MAX_FRAME_NUM, mpeg2.h:113 */

enum { M2V_I = 1, M2V_P = 2, M2V_B = 3 };

typedef struct {
	/* input (reference m2d_context: stream_i, header_callback) */
	dec_bits stream_i;
	int (*header_callback)(void *, void *);
	void *header_callback_arg;
	uint8_t *unit;           /* payload of the current start-code unit */
	size_t unit_len, unit_cap;
	int pending;             /* the next unit's start code prefix was already consumed */
	/* sequence */
	int hsize, vsize, disp_w, disp_h;
	int mpeg2;
	uint8_t qmat_store[4][64];
	const uint8_t *qmat[2];  /* [0] intra, [1] non-intra (raster order) */
	/* picture */
	int temporal_reference, coding_type;
	int intra_dc_precision, picture_structure, frame_pred_frame_dct, concealment_mv, q_scale_type;
	int intra_vlc_format, alternate_scan;
	int r_size[2][2];
	/* macroblock state (reference m2d_mb_current) */
	int mbmax_x, mbmax_y, fw;
	int mb_x, mb_y;
	int frame_mode, dct_type;
	int dc_scale, dc_max;
	int16_t dc_pred[3];
	int16_t pmv[2][2][2];
	int q_scale;
	int prev_intra;
	const uint8_t *scan;
	int16_t coef[64];
	/* frames (reference m2d_frames) */
	int num;
	m2d_frame_t frames[M2V_MAX_FRAMES];
	int lru[M2V_MAX_FRAMES];
	int ref[2];
	int index;
	int out_state;
	int copy_src;            /* frame skipped / lost MBs are copied from (diff_to_ref[0]); -1: in place */
	/* P / B (reference m2d_mb_current: type, motion_type) */
	int prev_type;           /* macroblock_type flags of the last coded MB (M2V_MBF_*) */
	int mv_count, mv_field, mv_dmv; /* motion type of the current MB (m2d_motion_type) */
	/* the picture being parsed as records (m2d_recon.h), reconstructed when it is complete */
	m2v_picture_t pic;
	size_t coef_cap;
	int pic_open;
	/* reconstruction back end: NULL = this file's CPU reconstruction (the C1 path); else the GPU one
	 * (m2dec_amd_m2v_use_gpu) */
	void *gpu;
	int gpu_device;
	/* statistics / checks */
	uint64_t clip_out_of_domain; /* CLIP255C arguments outside [-256, 767] (reference UB) */
	uint64_t mc_out_of_frame;    /* prediction reads outside the frame (the reference reads outside its buffers) */
	uint64_t pictures;
} mpeg2_dec_t;

/* macroblock_type flags (the reference's MB_* values, mpeg2.h:175-182) */
enum { M2V_MBF_FWD = 1, M2V_MBF_BWD = 2, M2V_MBF_INTRA = 4, M2V_MBF_PATTERN = 8, M2V_MBF_QUANT = 16 };

/* CPU reconstruction of one picture's records into frames[] (mpeg2_dec.c); returns CLIP255C
 * out-of-domain arguments and prediction reads outside the frame via the counters */
void m2v_recon_picture_cpu(const m2v_picture_t *pic, const m2d_frame_t *frames, uint64_t *clip_bad, uint64_t *mc_bad);

/* GPU back end (m2dec_amd/csrc/hip/m2v_hip.hip) */
void *m2v_hip_create(int device);
int m2v_hip_set_frames(void *g, int n, const m2d_frame_t *frames, int width, int height);
int m2v_hip_submit(void *g, const m2v_picture_t *pic);
int m2v_hip_sync(void *g, int slot);
void m2v_hip_destroy(void *g);

#ifdef __cplusplus
}
#endif
#endif
