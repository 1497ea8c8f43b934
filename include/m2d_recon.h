/*
 * m2dec_amd — the parse -> reconstruction record ABI (plain C, no torch types).
 *
 * The reference fuses parse and reconstruction per macroblock (h264.cpp:2005-2022,
 * 3131-3143, 6438-6454, 7366-7371); this boundary does not exist there.  The host parser
 * (m2dec_amd/csrc/host) emits, per picture, one record arena; a reconstruction back end (the
 * gfx950 HIP back end in m2dec_amd/csrc/hip, or the CPU oracle in oracle/) turns it into NV12.
 * Record fields map 1:1 onto the arguments the reference's recon call sites receive:
 *   m2r_mb_t       : mb_code dispatch (h264.h:429-433), avail/avail_intra (h264.cpp:3271-3292),
 *                    qmat selection via qp (set_qp, h264.cpp:1092-1119)
 *   m2r_inter_t    : mb->inter_pred(mb, ref_idx[2], mv[2], size, ox, oy) (h264.h:396)
 *   m2r_slice_t    : pred_weight_table / implicit weights (h264.cpp:1686-1712, 7001-7025)
 *   m2r_deblock_t  : deblock_info_t (h264.h:344-348) with the raster carry of idc/slicehdr and the
 *                    picture-final firstline test of deblock_pb (h264.cpp:10553-10612) resolved.
 */
#ifndef M2DEC_AMD_M2D_RECON_H
#define M2DEC_AMD_M2D_RECON_H

#include <stdint.h>
#include "m2d.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
	M2R_MB_I4x4 = 0,
	M2R_MB_I8x8 = 1,
	M2R_MB_I16x16 = 2,
	M2R_MB_PCM = 3,
	M2R_MB_INTER = 4
};

/* nz bit layout of m2r_mb_t.nz (one bit per coefficient block present in the pool, in pool order) */
#define M2R_NZ_LUMA(blk) (1u << (blk))       /* blkIdx 0..15 (4x4) ; 8x8 block b uses bit 4*b */
#define M2R_NZ_LUMA_DC (1u << 16)            /* Intra16x16 DC block */
#define M2R_NZ_CDC(c) (1u << (17 + (c)))     /* chroma DC, c = 0 Cb / 1 Cr */
#define M2R_NZ_CAC(c, b) (1u << (19 + 4 * (c) + (b)))

#define M2R_FLAG_T8x8 1u

/* One macroblock, 32 bytes. */
typedef struct m2r_mb {
	uint8_t kind;         /* M2R_MB_* */
	uint8_t cbp;          /* bits 0-3 luma 8x8 coded, bits 4-5 chroma cbp (0, 1 = DC, 2 = DC+AC) */
	uint8_t avail_luma;   /* avail bits handed to the luma predictor (1 left, 2 top, 4 top-right, 8 top-left) */
	uint8_t avail_chroma; /* avail bits handed to the chroma predictor */
	int8_t qpy;
	int8_t qpc[2];
	uint8_t pred_mode;    /* I16x16: 0 V, 1 H, 2 DC, 3 plane */
	uint8_t chroma_mode;  /* 0 DC, 1 H, 2 V, 3 plane */
	uint8_t flags;        /* M2R_FLAG_T8x8 */
	uint16_t slice;       /* index into m2r_picture_t.slice */
	uint32_t ipred[2];    /* Intra4x4 (blkIdx order) / Intra8x8 (first 4) modes, 4 bits each */
	uint32_t coef;        /* offset in int16 units into the coefficient pool */
	uint32_t nz;          /* coded blocks present in the pool (M2R_NZ_*) */
	uint32_t inter;       /* index into m2r_picture_t.inter (kind == INTER) */
} m2r_mb_t;

/* Motion of one inter macroblock, 144 bytes. */
typedef struct m2r_inter {
	int16_t mv[2][16][2]; /* [list][4x4 raster idx = y*4 + x][x, y], quarter-pel */
	int8_t slot[2][4];    /* [list][8x8 raster idx] frame slot of the reference, -1 = list unused */
	int8_t refidx[2][4];  /* [list][8x8] ref_idx (weight table lookup) */
} m2r_inter_t;

enum { M2R_WP_DEFAULT = 0, M2R_WP_EXPLICIT = 1, M2R_WP_IMPLICIT = 2 };

/* Per-slice weighted-prediction state. */
typedef struct m2r_slice {
	uint8_t wp_mode;
	uint8_t log2wd[2];    /* explicit: luma / chroma log2 weight denominator */
	uint8_t pad[5];
	int8_t w[2][32][3];   /* explicit weight [list][ref_idx][Y, Cb, Cr] (int8 as stored by the reference) */
	int8_t o[2][32][3];   /* explicit offset */
	int8_t iw[32][32][2]; /* implicit (w0, w1) per (refIdxL0, refIdxL1), int8 wrap as the reference */
} m2r_slice_t;

#define M2R_DBK_LEFT 1u     /* filter the left MB edge */
#define M2R_DBK_TOP 2u      /* filter the top MB edge */
#define M2R_DBK_LEFT_BS4 4u /* left MB edge is bS 4 (strong) */
#define M2R_DBK_TOP_BS4 8u  /* top MB edge is bS 4 */
#define M2R_DBK_OFF 16u     /* disable_deblocking_filter_idc == 1: MB not filtered */

/* Deblocking input of one macroblock, 16 bytes. */
typedef struct m2r_deblock {
	/* bS 0..3 of the MB's edges, derived by the back end from the MB and motion records (the parser
	 * writes 0; recon_hip.hip bs_of, oracle/recon_oracle.c orc_bs): */
	uint32_t bs_v;        /* vertical edges x = 0,4,8,12: byte e = edge, 2 bits per 4-row segment (LSB = top) */
	uint32_t bs_h;        /* horizontal edges y = 0,4,8,12: byte e = edge, 2 bits per 4-column segment (LSB = left) */
	int8_t qpy;
	int8_t qpc[2];
	uint8_t flags;        /* M2R_DBK_* */
	int8_t alpha_off;     /* FilterOffsetA = slice_alpha_c0_offset_div2 * 2 */
	int8_t beta_off;      /* FilterOffsetB */
	uint8_t pad[2];
} m2r_deblock_t;

/* One picture's records.  Arrays live in one arena owned by the back end (pinned for the GPU). */
typedef struct m2r_picture {
	int32_t width_mbs, height_mbs;
	int32_t slot;          /* destination frame slot */
	int32_t n_inter;       /* used entries of inter[] */
	int32_t n_coef;        /* used int16 of coef[] */
	int32_t n_slices;      /* used entries of slice[] */
	int32_t n_intra;       /* number of intra (I4x4/I8x8/I16x16/PCM) macroblocks */
	int32_t deblock;       /* 0: no macroblock needs filtering */
	m2r_mb_t *mb;          /* [width_mbs * height_mbs] raster order */
	m2r_deblock_t *dbk;    /* [width_mbs * height_mbs] */
	m2r_slice_t *slice;    /* [cap_slices] */
	m2r_inter_t *inter;    /* [cap_inter] */
	int16_t *coef;         /* [cap_coef] */
	int32_t cap_slices, cap_inter, cap_coef;
	int32_t flags;         /* M2R_PIC_* */
	/* with M2R_PIC_REFS (ABI revision 6): a summary of inter[0, n_inter) the producer formed while the
	 * records were in its cache, so the back end does not scan them on the submission path */
	int32_t ref_blocks;    /* 8x8 (list, block) predictions: slot[l][b] >= 0 entries */
	uint64_t ref_slots;    /* bit s: some slot[l][b] == s */
} m2r_picture_t;

/* m2r_picture_t.flags: `slot` and every m2r_inter_t.slot are the back end's picture buffers (virtual
 * frame ids 0..63 of the parse-ahead pipeline), not caller frame slots; the picture reaches a caller
 * frame only through bind().  Set only for back ends that provide bind. */
#define M2R_PIC_VIRTUAL 1
/* m2r_picture_t.flags: the record arrays are not the acquired arena's but the parser's own, in host memory
 * the device runtime has pinned, laid out as m2r_arena_layout() from `mb` on (the back end uploads them
 * straight from there — no copy into its arena).  The parser keeps them unchanged until records_busy() says
 * the back end is done with them.  Set only for back ends that provide records_busy. */
#define M2R_PIC_EXTERNAL 2
/* m2r_picture_t.flags: ref_blocks / ref_slots hold the summary of inter[] */
#define M2R_PIC_REFS 4

/* Record arena layout shared by the parser's job arenas and the back ends' arenas (byte offsets from the
 * arena base, 256-byte aligned): mb | dbk | slice[M2R_ARENA_SLICES] | inter[n] | coef[n * 416].  The fixed
 * part (mb, dbk, slices) and each used prefix of inter / coef are contiguous, so an upload is two copies. */
#define M2R_ARENA_SLICES 256
#define M2R_COEF_PER_MB 416
typedef struct m2r_arena_layout {
	size_t mb, dbk, slice, inter, coef, size;
} m2r_arena_layout_t;

static inline m2r_arena_layout_t m2r_arena_layout(int n_mbs)
{
	m2r_arena_layout_t l;
	const size_t n = (size_t)n_mbs;
#define M2R_AL_(v) (((v) + 255) & ~(size_t)255)
	l.mb = 0;
	l.dbk = M2R_AL_(l.mb + n * sizeof(m2r_mb_t));
	l.slice = M2R_AL_(l.dbk + n * sizeof(m2r_deblock_t));
	l.inter = M2R_AL_(l.slice + M2R_ARENA_SLICES * sizeof(m2r_slice_t));
	l.coef = M2R_AL_(l.inter + n * sizeof(m2r_inter_t));
	l.size = M2R_AL_(l.coef + n * M2R_COEF_PER_MB * sizeof(int16_t));
#undef M2R_AL_
	return l;
}

/* A reconstruction back end.  The parser acquires an arena, fills it, and submits it; frames are
 * caller-owned NV12 buffers (set_frames), synchronised on demand (sync_frame) before the caller
 * reads them through peek/get_decoded_frame.
 *
 * bind (optional, NULL if absent): decode ahead of the caller.  Pictures are submitted with
 * M2R_PIC_VIRTUAL as soon as they are parsed, into the back end's own buffers named by virtual
 * frame ids, before the API context has given them a caller frame; bind(vid, slot) later says that
 * buffer `vid` holds the picture of caller frame `slot` (copied out by the time sync_frame(slot)
 * returns).  The caller guarantees: a virtual id is bound before any later picture that writes
 * the same id is submitted, and a picture is submitted before it is bound. */
typedef struct m2r_backend {
	void *self;
	int (*set_frames)(void *self, int n, const m2d_frame_t *frames, int width, int height);
	m2r_picture_t *(*acquire)(void *self, int width_mbs, int height_mbs);
	int (*submit)(void *self, m2r_picture_t *pic);
	int (*sync_frame)(void *self, int slot);
	void (*destroy)(void *self);
	int (*bind)(void *self, int vid, int slot);
	/* optional (ABI revision 4): submit may hold pictures back to launch several at once; flush launches
	 * the held ones (0), or keeps them while the device is busy (1: the decoder calls it again on its next
	 * step; bind launches a held picture anyway).  The decoder calls it after the last submit of a burst;
	 * bind, set_frames and acquire launch held pictures implicitly.  NULL: every submit is launched as it
	 * comes. */
	int (*flush)(void *self);
	/* optional (ABI revision 5): 1 when sync_frame(slot) would return without waiting (the frame's copy out
	 * of the device is complete), 0 otherwise; never blocks.  The decoder polls it while the caller waits
	 * in peek / get and keeps its lookahead parsing meanwhile.  NULL: sync_frame is called at once. */
	int (*ready)(void *self, int slot);
	/* optional (ABI revision 6): the back end takes M2R_PIC_EXTERNAL pictures.  1 while it may still read
	 * the external records starting at `records` (a submitted picture's `mb`), 0 once it never will again.
	 * wait = 0 never blocks (any thread, while the decoder's serial calls run); wait = 1 blocks until 0,
	 * launching a held picture first (only while no other call of this back end runs).  NULL: pictures are
	 * always copied into the acquired arena. */
	int (*records_busy)(void *self, const void *records, int wait);
} m2r_backend_t;

/* ---------------------------------------------------------------- MPEG-1/2 (m2d_func)
 * The MPEG-2 parser (m2dec_amd/csrc/host/mpeg2_dec.c) turns each picture into one record per macroblock
 * in raster order; a reconstruction back end (the CPU one in mpeg2_dec.c, the gfx950 one in
 * m2dec_amd/csrc/hip/m2v_hip.hip) builds the picture: the prediction of m2d_parse_inter_macroblock /
 * m2d_skip_mb_P / _B (mpeg2.cpp:715-810, 1355-1395, motioncomp.cpp), then the IDCT of each coded block
 * stored (intra) or added (inter) with CLIP255C (idct.cpp:286-422).  Nothing of a picture depends on
 * another macroblock of the same picture. */
#define M2V_REC_INTRA 1u      /* blocks are stored, not added */
#define M2V_REC_FWD 2u        /* prediction from the forward reference (fwd) */
#define M2V_REC_BWD 4u        /* prediction from the backward reference (bwd), averaged if FWD too */
#define M2V_REC_FIELD 8u      /* field prediction: vectors [dir][0] / [dir][1] for the top / bottom field lines */
#define M2V_REC_DCT_FIELD 16u /* field DCT: luma blocks 0/1 on even lines, 2/3 on odd lines */
#define M2V_REC_COPY 32u      /* skipped / lost MB: a copy of the `copy` picture (vector 0) */

/* One macroblock, 32 bytes. */
typedef struct m2v_mb {
	uint8_t flags;        /* M2V_REC_*; 0: the MB keeps what the frame holds */
	uint8_t cbp;          /* bit 5 - i: luma block i, bit 1 - i: chroma block i coded (64 coefficients each in the pool, in block order) */
	uint8_t field_sel;    /* field prediction: bit 2 * dir + i = the reference field (0 top, 1 bottom) of vector i */
	uint8_t pad0;
	uint16_t mbx, mby;
	int16_t mv[2][2][2];  /* [dir 0 fwd / 1 bwd][vector][x, y] in half samples (field lines for field vectors) */
	uint32_t coef;        /* offset in int16 units into the coefficient pool (dequantised, mismatch-controlled) */
	uint32_t pad1[2];
} m2v_mb_t;

/* One picture's records. */
typedef struct m2v_picture {
	int32_t width, height;   /* coded size (MB multiples); NV12, stride = width */
	int32_t cur, fwd, bwd, copy; /* frame slots: the picture, its forward / backward reference, the copy source (-1: none) */
	int32_t n_mbs;           /* records (width / 16 * height / 16) */
	int32_t n_coef;          /* int16 coefficients used in coef[] */
	m2v_mb_t *mb;
	int16_t *coef;
} m2v_picture_t;

/* ---------------------------------------------------------------- H.265 (h265d_func) records
 * The host parser (m2dec_amd/csrc/host/h265_dec.c) turns each picture into:
 *   - transform blocks in decoding order, each predicted (intra) then given its residual: the
 *     reference's transform_tree leaves (h265.cpp:3026-3075), luma and chroma (Cb + Cr together)
 *     as separate records;
 *   - a map from every 4x4 unit of each plane to the record that writes it (the GPU waits on the
 *     records that own a block's neighbour samples);
 *   - deblocking edge records (bS and edge QP per 4-sample segment on the 8x8 grid, h265modules.h
 *     h265d_deblocking_strength_t) and one SAO record per CTU (h265modules.h:338-351). */
#define H265R_MAX_FRAMES 8 /* H265D_MAX_FRAME_NUM (h265modules.h:40) */
enum { H265R_RES_NONE = 0, H265R_RES_DC = 1, H265R_RES_FULL = 2, H265R_RES_DST = 3, H265R_RES_SKIP = 4 };
#define H265R_TU_PRED 1u /* intra-predict the block before its residual (else: residual only) */

typedef struct {
	uint16_t x, y;        /* top-left sample in its plane (chroma: in chroma samples) */
	uint8_t log2;         /* 2..5 */
	uint8_t plane;        /* 0 luma, 1 chroma (Cb and Cr, interleaved NV12) */
	uint8_t mode;         /* intra prediction mode 0..34 */
	uint8_t flags;        /* H265R_TU_PRED */
	int16_t avail_top;    /* samples of the row above available from x on (top + top-right), -1: none */
	int16_t avail_left;   /* samples of the column left available from y on (left + bottom-left), -1: none */
	uint8_t res[2];       /* residual kind H265R_RES_*: luma [0]; chroma Cb [0], Cr [1] */
	uint8_t strong;       /* luma: strong intra smoothing enabled (sps) */
	uint8_t pad;
	uint32_t coef[2];     /* coefficient-pool offsets (dequantised int16, (1 << log2)^2 raster) */
} h265r_tu_t;

/* One inter prediction block (P / B pictures): motion compensation of the luma and chroma samples of the
 * rectangle from one or two reference frames (inter_pred_onedir / merge_pred, h265.cpp:3552-3595, 3868-3903):
 * 8-tap luma / 4-tap chroma interpolation with the reference's rounding, bi-prediction averaged.  Written
 * before any transform block of the picture (every PU reads only reference frames). */
typedef struct {
	uint16_t x, y;        /* top-left luma sample */
	uint8_t w, h;         /* luma size, 4..64 */
	int8_t ref[2];        /* frame slot of the L0 / L1 reference (-1: list unused) */
	int16_t mv[2][2];     /* quarter-sample luma vectors (chroma: the same, eighth-sample) */
} h265r_pu_t;

typedef struct {
	uint8_t type[3];      /* per component: 0 off, 1 band offset, 2 edge offset */
	uint8_t band[3];      /* band position */
	uint8_t eo[3];        /* edge class 0..3 (Cr shares Cb's) */
	uint8_t pad[3];
	int8_t off[3][4];     /* offsets, signs applied (edge: categories 1, 2 >= 0; 3, 4 <= 0) */
} h265r_sao_t;

#define H265R_PIC_DEBLOCK 1
#define H265R_PIC_SAO_LUMA 2
#define H265R_PIC_SAO_CHROMA 4

typedef struct {
	int32_t width, height;       /* frame: CTB-aligned, luma stride = width */
	int32_t pic_w, pic_h;        /* pic_width / height_in_luma_samples */
	int32_t ctb_log2, slot;      /* CTB size, caller frame written */
	int32_t n_tu, n_coef;
	int32_t flags;               /* H265R_PIC_* */
	int32_t beta_offset, tc_offset;    /* slice_beta_offset_div2 * 2, slice_tc_offset_div2 * 2 */
	int32_t cb_qp_offset, cr_qp_offset; /* pps_cb / cr_qp_offset (chroma deblocking) */
	h265r_tu_t *tu;
	int16_t *coef;
	int32_t *map;                /* luma (width/4 x height/4) then chroma (width/8 x height/8) 4x4 units: record index */
	uint8_t *bs_v;               /* vertical edges [height/4][width/8]: (qp << 2) | bS, edge x = 8 i, rows 4 j.. */
	uint8_t *bs_h;               /* horizontal edges [height/8][width/4]: edge y = 8 j, columns 4 i.. */
	h265r_sao_t *sao;            /* per CTU, raster */
	int32_t n_pu;                /* inter prediction blocks (P / B pictures; 0 in I pictures) */
	h265r_pu_t *pu;
} h265r_picture_t;

/* An H.265 reconstruction back end (default: the gfx950 one, m2dec_amd/csrc/hip/h265_hip.hip). */
typedef struct h265r_backend {
	void *self;
	int (*set_frames)(void *self, int n, const m2d_frame_t *frames, int width, int height);
	int (*submit)(void *self, const h265r_picture_t *pic);
	int (*sync_frame)(void *self, int slot); /* the picture last submitted into `slot` is in the caller's frame */
	void (*destroy)(void *self);
	/* optional (H.265 ABI revision 2): a parse worker hands a parsed picture to the back end before its submit,
	 * from any thread and concurrently with the other calls, so that copies of its records are off the serial
	 * submission path; the same `pic` (its record buffers unchanged) is then submitted, or handed again with
	 * discard = 1 when it never will be.  NULL: submit takes every picture as it is. */
	int (*stage)(void *self, const h265r_picture_t *pic, int discard);
} h265r_backend_t;

#ifdef __cplusplus
}
#endif
#endif
