/* Synthetic H.264 stream generator — shared declarations.
 *
 * The generator is an open-loop syntax encoder: it chooses macroblock types, intra modes, motion,
 * coded block patterns and coefficient levels from a seeded RNG, under the constraints of
 * SURVEY.md Appendix A (the reference decoder's quirks), and writes a conforming Annex-B stream.
 * It never reconstructs pictures; the decoder under test does that.  It tracks exactly the
 * neighbour state that syntax needs (CABAC contexts, CAVLC nC, intra mode prediction) and keeps a
 * believed motion field so that motion vectors follow a target field rather than drifting.
 */
#ifndef H264GEN_GEN_H
#define H264GEN_GEN_H
#include <stdint.h>
#include <stdio.h>
#include "bitwriter.h"

typedef struct {
	int width, height;      /* coded size in samples (multiples of 16) */
	int crop_bottom;        /* output crop in samples (even) */
	int frames;
	int cabac;
	int bframes;            /* B pictures between anchors (0 = IPPP) */
	int t8x8;               /* transform_8x8_mode_flag (CABAC only) */
	int gop;                /* I picture period (display order); first is IDR */
	int idr_period;         /* 0: only the first picture is IDR */
	int slices;             /* slices per picture (row-aligned) */
	int profile, level;
	int wp_p;               /* weighted_pred_flag */
	int wp_b;               /* weighted_bipred_idc */
	int direct;             /* 0 temporal, 1 spatial, 2 random per slice */
	int qp_min, qp_max;
	int deblock;            /* 0: always idc 0 without offsets; 1: random idc 0/1 and offsets */
	int pcm_permille;
	int mv_px;              /* motion range in pixels */
	int num_ref_frames, l0_active, l1_active;
	int p_skip_pct, p_intra_pct;
	int i4_pct, i8_pct;     /* intra MB type mix (rest I16x16) */
	int sub8x8_pct;         /* share of 8x8 inter MBs */
	int coef_pct;           /* probability that a cbp bit is set */
	int planar;             /* allow plane prediction (off: Appendix A #2) */
	int cip;                /* constrained_intra_pred_flag (reference quirk A#8 reproduced by the decoder) */
	int idc2;               /* allow disable_deblocking_filter_idc 2 (reference quirk A#6) */
	int scaling;            /* SPS seq_scaling_matrix_present_flag with random lists (parsed, ignored: A#4) */
	int quirks;             /* reach the reference quirks the kernels reproduce: explicit weights up to 127
	                           (SSE2 int16 saturation, A#1), log2 denominator 7 with default weights (the
	                           int8 store of 128, A#16), DC-only 4x4 blocks with |adj| 200..255 (SWAR, A#17) */
	/* reference-picture machinery (h264.cpp:1417-1567 slice header, :1608-1653 list
	 * modification, :10665-11050 marking / DPB) */
	int poc_type;           /* 0, 1 (offsets of 1 per reference frame, deltas per slice) or 2 (IPPP only) */
	int log2_fn;            /* log2_max_frame_num (4: frame_num wraps every 16 pictures) */
	int reorder_pct;        /* P / B slices carrying ref_pic_list_modification */
	int mmco_pct;           /* reference pictures marked by adaptive MMCO ops 1 / 2 / 3 / 4 / 6 */
	int long_term;          /* allow long-term references (MMCO 3 / 4 / 6, IDR long_term_reference_flag) */
	int mmco5;              /* every mmco5-th anchor (display index) is a P picture with MMCO 5 (0: none) */
	int nonref_pct;         /* IPPP: P pictures coded as non-reference (nal_ref_idc 0) */
	uint64_t seed;
} params_t;

/* Per-macroblock dump of the generator's decisions (--dump), for parser cross-checks. */
typedef struct {
	int32_t pic;          /* coding-order picture index */
	int32_t mbaddr;
	uint8_t kind;         /* 0 I4x4, 1 I8x8, 2 I16x16, 3 PCM, 4 inter, 5 skip */
	uint8_t cbp;
	int8_t qp;
	uint8_t t8x8;
	uint8_t exact_mv;     /* ref[] / mv[] below equal the decoder's (direct blocks included) */
	uint8_t i16_pred, cmode;
	uint8_t dir8;         /* direct-predicted 8x8 blocks (B_Skip, B_Direct_16x16, direct sub-MBs) */
	int8_t ipm[16];       /* intra modes per blkIdx (I4x4) or per 8x8 (I8x8, first 4) */
	int8_t ref[2][4];     /* per 8x8 raster, -1 unused (direct: the derived refIdx) */
	int16_t mv[2][16][2]; /* per 4x4 raster */
	int16_t ldc[16];      /* luma DC levels, raster */
	int16_t luma[256];    /* 4x4: blkIdx*16 + raster; 8x8: b8*64 + raster */
	int16_t cdc[2][4];
	int16_t cac[2][4][16]; /* raster, [0] unused */
} gen_dump_t;

/* Per-slice reference lists of P / B slices (--dump-refs), compared with the decoder's (M2DEC_AMD_H264_REFDUMP,
 * tests/gen_check.py): the POC and long-term flag of every active entry of RefPicList0 / 1. */
typedef struct {
	int32_t pic;          /* coding-order picture index */
	int32_t first_mb;
	int32_t slice_type;   /* 0 P, 1 B, 2 I */
	int32_t poc;
	int32_t n[2];
	int32_t poc_l[2][16];
	int8_t lt[2][16];
} gen_refdump_t;

int gen_stream(const params_t *p, bw_t *out, FILE *dump, FILE *refdump);

#endif
