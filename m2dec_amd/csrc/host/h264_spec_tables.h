/* ITU-T H.264 constant tables (generated into h264_spec_tables.c by tools/gen_spec_tables.py). */
#ifndef M2DEC_AMD_H264_SPEC_TABLES_H
#define M2DEC_AMD_H264_SPEC_TABLES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H264_NUM_CTX 460

typedef struct {
	int16_t value; /* -1 terminates a table */
	uint8_t len;
	uint32_t code;
} h264_vlc_code_t;

extern const int8_t h264_cabac_init_mn[4][H264_NUM_CTX][2];
extern const uint8_t h264_range_lps[64][4];
extern const uint8_t h264_trans_idx_lps[64];
extern const uint8_t h264_sig8x8_frame[63];
extern const uint8_t h264_last8x8[63];
extern const uint8_t h264_me_cbp[2][48];

/* coeff_token value = (TrailingOnes << 5) | TotalCoeff; index 0..3 = nC ranges 0-1, 2-3, 4-7, >=8; 4 = chroma DC */
extern const h264_vlc_code_t * const h264_coeff_token_tab[5];
extern const h264_vlc_code_t * const h264_total_zeros_tab[16]; /* [TotalCoeff] (4x4 blocks) */
extern const h264_vlc_code_t * const h264_run_before_tab[8];   /* [min(zerosLeft, 7)] */

#ifdef __cplusplus
}
#endif
#endif
