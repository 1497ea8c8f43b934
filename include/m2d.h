/*
 * m2dec_amd — public decode API (drop-in for the reference's m2d.h / bitio.h / h264.h surface).
 *
 * Mirrors the reference interface the callers (M2Decoder, h264dec, thrplay) bind:
 *   m2d_frame_t       /root/reference/src/lib/m2d.h:35-42
 *   m2d_info_t        /root/reference/src/lib/m2d.h:58-65
 *   m2d_func_table_t  /root/reference/src/lib/m2d.h:66-75
 *   h264d_func        /root/reference/src/lib/h264.h:457, h264.cpp:12057-12068
 *   h265d_func        /root/reference/src/lib/h265.h:37, h265.cpp:5010-5025
 *   bitio API         /root/reference/src/lib/bitio.h:57-75 (+ m2d_next_start_code, m2d.h:77-80)
 * Same names, argument meaning and return conventions (decode_picture: 1 picture done,
 * -1 syntax error, -2 end of data; peek/get: 1 frame, 0 none, -1 bad args).
 *
 * The decoded NV12 planes (luma stride = coded width, interleaved CbCr, half height) are written
 * into the caller-owned frames exactly as the reference does; reconstruction runs on a gfx950 GPU.
 */
#ifndef M2DEC_AMD_M2D_H
#define M2DEC_AMD_M2D_H

#include <stddef.h>
#include <stdint.h>
#include <setjmp.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned char byte_t;

typedef struct {
	uint8_t *luma;
	uint8_t *chroma;
	void *id;
	int32_t cnt;          /* picture order count */
	int16_t width, height; /* coded (MB-aligned) size; luma stride = width */
	int16_t crop[4];       /* left, right, top, bottom in samples */
} m2d_frame_t;

typedef struct {
	int16_t src_width, src_height;
	int16_t disp_width, disp_height;
	int16_t frame_num;
	int16_t crop[4];
	int additional_size;
} m2d_info_t;

/* Bit-stream feeder.  The decoder pulls data through this object; when it runs dry it calls
 * error_func(error_arg), which is expected to call dec_bits_set_data() with the next chunk and
 * return 0, or return <0 at end of stream (reference bitio.c:112-126 protocol). */
typedef uintptr_t cache_t;
/* Field order and types follow the reference's struct dec_bits_t (bitio.h:39-50) so that code
 * compiled against the reference's bitio.h (inline readers) sees the same layout. */
typedef struct dec_bits_t {
	cache_t cache_;
	int cache_len_;
	int8_t prev_[2];
	const byte_t *buf_;
	void (*load_bytes)(struct dec_bits_t *, int bytes);
	const byte_t *buf_tail_;
	const byte_t *buf_head_;
	int (*error_func_)(void *);
	void *error_arg_;
	void *id;
	jmp_buf jmp;
} dec_bits;

typedef struct {
	size_t context_size;
	int (*init)(void *, int, int (*)(void *, void *), void *);
	dec_bits *(*stream_pos)(void *);
	int (*get_info)(void *, m2d_info_t *);
	int (*set_frames)(void *, int, m2d_frame_t *, uint8_t *, int);
	int (*decode_picture)(void *);
	int (*peek_decoded_frame)(void *, m2d_frame_t *, int);
	int (*get_decoded_frame)(void *, m2d_frame_t *, int);
} m2d_func_table_t;

/* bitio (reference bitio.h:57-75) */
int dec_bits_open(dec_bits *ths, void (*loadbytes_func)(dec_bits *, int bytes));
void dec_bits_close(dec_bits *ths);
void dec_bits_set_callback(dec_bits *ths, int (*error_func)(void *), void *error_arg);
int dec_bits_set_data(dec_bits *ths, const byte_t *buf, size_t buf_len, void *id);
uint32_t show_bits(dec_bits *ths, int bit_len);
uint32_t show_onebit(dec_bits *ths);
uint32_t get_bits(dec_bits *ths, int bit_len);
uint32_t get_onebit(dec_bits *ths);
void skip_bits(dec_bits *ths, int bit_len);
int not_aligned_bits(dec_bits *ths);
void byte_align(dec_bits *ths);
void skip_bytes(dec_bits *ths, int byte_len);
const byte_t *dec_bits_current(dec_bits *ths);
const byte_t *dec_bits_tail(dec_bits *ths);
void m2d_load_bytes_skip03(dec_bits *ths, int read_bytes);
/* reference m2d.h:77-80: byte offset just past the next 00 00 01, or -1 */
int m2d_next_start_code(const byte_t *org_src, int byte_len);

/* H.264 NAL / slice constants the applications use (reference h264.h:49-83) */
enum {
	SLICE_NONIDR_NAL = 1,
	SLICE_IDR_NAL = 5,
	SEI_NAL = 6,
	SPS_NAL = 7,
	PPS_NAL = 8,
	H264D_MAX_FRAME_NUM = 64
};

/* The H.264 decoder: GPU reconstruction behind the reference's function table. */
extern const m2d_func_table_t * const h264d_func;
/* The MPEG-1/2 video decoder (mpeg2.cpp:1800-1811; mpeg2.h): I, P and B frame pictures, reconstructed on the
 * CPU (BASELINE.json configs[0], the reference's own configuration) or on gfx950 (m2dec_amd_m2v_use_gpu). */
extern const m2d_func_table_t * const m2d_func;
/* h265.h:37, h265.cpp:5010-5025 (m2dec_amd/csrc/host/h265_dec.c) */
extern const m2d_func_table_t * const h265d_func;

#ifdef __cplusplus
}
#endif
#endif
