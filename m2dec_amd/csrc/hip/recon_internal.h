/*
 * Internal interface between the gfx950 reconstruction kernels (recon_hip.hip) and the host
 * runtime that schedules them (runtime.hip).  Not part of the public C ABI.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "m2d_recon.h"

#define HBI_BYTES 48 /* I-picture intra hand-off per MB: bottom luma row (16 B) + bottom chroma row (16 B) in six
                        * u64 words of 6 bytes + a 16-bit picture tag each */
#define HBD_BYTES 96 /* deblock hand-off per MB: luma rows 12..15 (4 x 16 B) + chroma rows 6..7 (2 x 16 B) */
#define DBK_WAVES 4  /* deblocking workgroup: loader, filter A, storer, filter B waves */
#ifndef DBK_RING
#define DBK_RING 16  /* deblocking: MB slots of the LDS ring (power of two) */
#endif
#ifndef DBK_SG
#define DBK_SG 4     /* deblocking storer: frame stores in groups of DBK_SG MBs (power of two, <= DBK_RING / 2) */
#endif
#define DBK_RW (DBK_RING * 16) /* ring line width in bytes */

/* row progress word: picture seq's MB row has its first `cols` MB columns final (all 16 luma / 8 chroma
 * sample rows).  An entry (seq % ROWFLAG_N) only ever grows, also across pictures: a reader of picture
 * q may see picture q + ROWFLAG_N's value, so ROWFLAG_N must exceed the decode-order distance between
 * a picture and its last reader plus the pictures in flight (interleaved multi-stream batches: the
 * streams multiply that distance). */
#define ROWFLAG_N 256
#define ROWFLAG(seq, cols) ((((unsigned long long)(seq) + 1) << 16) | (unsigned long long)(cols))

#define WAR_MAX 16 /* readers of one slot's content a batch picture can wait for */

/* seq + 1 of the picture currently held by each frame slot (0: none) */
struct SlotSeq {
	int s[64];
};

/* per-launch scratch words (zeroed before every launch): intra luma / chroma progress, deblock
 * progress, inter segment counters, hand-off-ready flags ([Hmb] each), then the work-queue head */
#define SCR_IPROG(Hmb) 0
#define SCR_IPROGC(Hmb) (Hmb)
#define SCR_DPROG(Hmb) (2 * (Hmb))
#define SCR_INTER(Hmb) (3 * (Hmb))
#define SCR_HBIRDY(Hmb) (4 * (Hmb))
#define SCR_QUEUE(Hmb) (5 * (Hmb))
/* then one done flag per inter work item (MB row y, 8-MB segment s) at SCR_SEG + y * nseg + s */
#define SCR_SEG(Hmb) (5 * (Hmb) + 4)
#define NSEG(Wmb) (((Wmb) + 7) >> 3)
#define SCR_WORDS(Hmb, Wmb) ((5 * (Hmb) + 4 + (Hmb) * NSEG(Wmb) + 3) & ~3)
/* P/B pictures: neighbour records of the MBs an intra MB reads (written by the inter workers):
 * bottom luma row, bottom chroma row (CbCr), right luma column, right chroma column (CbCr pairs);
 * row stride NSEG * 8 MBs so that no 128-byte line holds records of two work items */
#define HBP_BYTES 64
/* inter worker: LDS row stride of a work item's staged output (8 MBs x 16 bytes) */
#define SEG_ROW 128

struct PictureArgs {
	const m2r_mb_t *mbs;
	const m2r_inter_t *inters;
	const m2r_slice_t *slices;
	const int16_t *pool;
	const m2r_deblock_t *dbk;
	uint8_t *frames;
	size_t fsz;
	int W, H, Wmb, Hmb;
	int slot, seq, n_inter, n_intra;
	int inter_workers;
	int row_wgs;      /* P / B pictures: row-pair workgroups (taking pairs from a queue) */
	int *scratch;     /* SCR_* words of this launch */
	uint8_t *hbi, *hbd; /* hand-off records of this launch's stream */
	uint8_t *hbp;       /* [Hmb][NSEG * 8] HBP_BYTES neighbour records (P/B pictures) */
	unsigned long long *rowflag; /* [64][Hmb] column progress of picture rows: ROWFLAG(seq, c) once MB
	                               columns 0 .. c-1 of the row are final (entry seq & 63) */
	int *err;
	SlotSeq ss;
	/* batch launches (k_batch) only: the slot's write-after-read / write-after-write on the device */
	int *fin;         /* [2 * batch] zeroed per launch: [2p] inter workers done, [2p + 1] row workgroups done; null: single launch */
	int pidx;         /* dispatch position of this picture in the batch */
	int didx;         /* decode-order index in the batch (diagnostics) */
	int n_war;        /* earlier pictures of the batch that read the slot's previous content ... */
	int war[WAR_MAX]; /* ... (their inter workers must be done) */
	int war_writer;   /* the batch picture that wrote the previous content (its rows must be done), or -1 */
	uint8_t *capture; /* verification only: the finished frame is copied here before the slot is released */
	/* decode-path launches (k_picture): the picture's workgroups [blk0, blk0 + nblk) of the launch — a
	 * picture without inter MBs has no inter workers, a P / B picture only its row_wgs row workgroups */
	int blk0, nblk;
};

/* a batch of pictures in decode order, picture p owning blocks [p * bpp, (p + 1) * bpp) */
__global__ void k_batch(const PictureArgs *pics, int bpp);
__global__ void k_picture(const PictureArgs *pics, int n);

/* workgroups of one picture in a k_batch launch: persistent inter workers + one per pair of MB rows */
static inline int picture_blocks(int inter_workers, int Hmb) { return inter_workers + (Hmb + 1) / 2; }
/* workgroups of one picture in a k_picture launch: only those with work (an I picture: its row pairs; a P / B
 * picture: its inter workers and row_wgs row workgroups) */
static inline int picture_blocks_dp(int inter_workers, int row_wgs, int Hmb, bool has_inter)
{
	const int pairs = (Hmb + 1) / 2;
	return has_inter ? inter_workers + (row_wgs < pairs ? row_wgs : pairs) : pairs;
}

/* dynamic LDS bytes of one k_deblock workgroup for a W-sample-wide picture */
size_t m2r_deblock_lds_bytes(int W, int Wmb);
extern "C" int m2dec_amd_debug_stamps_clear(void); /* no-op unless built with M2DEC_STAMPS */
/* polls after which a hand-off wait is reported in err[1] (and goes on) on the current device; abort: ~2^26 polls */
extern "C" int m2dec_amd_hip_set_spin_report(unsigned polls);
