/*
 * Internal interface between the gfx950 reconstruction kernels (recon_hip.hip) and the host
 * runtime that schedules them (runtime.hip).  Not part of the public C ABI.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "m2d_recon.h"

#define HBI_BYTES 32 /* intra hand-off per MB: bottom luma row (16 B) + bottom chroma row (16 B) */
#define HBD_BYTES 96 /* deblock hand-off per MB: luma rows 12..15 (4 x 16 B) + chroma rows 6..7 (2 x 16 B) */
#define DBK_WAVES 3  /* k_deblock workgroup: loader, filter, storer waves */
#define DBK_PAD 16   /* k_deblock LDS pad each side of a line (keeps 16-B rows aligned) */

__global__ void k_inter(const m2r_mb_t *__restrict__ mbs, const m2r_inter_t *__restrict__ inters,
                        const m2r_slice_t *__restrict__ slices, const int16_t *__restrict__ pool, uint8_t *frames,
                        size_t fsz, int W, int H, int Wmb, int slot);
__global__ void k_intra(const m2r_mb_t *__restrict__ mbs, const int16_t *__restrict__ pool, uint8_t *cur, int W, int H,
                        int Wmb, uint8_t *hbi, int *progress, int *err);
__global__ void k_deblock(const m2r_deblock_t *__restrict__ dbk, uint8_t *cur, int W, int H, int Wmb, int Hmb,
                          uint8_t *hbd, int *progress, int *err);

/* dynamic LDS bytes of one k_deblock workgroup for a W-sample-wide picture */
size_t m2r_deblock_lds_bytes(int W, int Wmb);
