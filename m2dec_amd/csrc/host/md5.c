/*
 * RFC 1321 MD5 and the FileWriterMd5 line format of the reference application
 * (src/app/filewrite.h:11-29 cropped NV12 rows, :99-105 "%02x" x16 + "\r\n").
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "m2dec_amd.h"

typedef struct {
	uint32_t h[4];
	uint64_t len;
	uint8_t buf[64];
	size_t fill;
} md5_t;

#define ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))

/* unrolled rounds (the register roles rotate instead of moving values: a <- d, d <- c, c <- b) */
#define F(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define G(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define H(x, y, z) ((x) ^ (y) ^ (z))
#define I(x, y, z) ((y) ^ ((x) | ~(z)))
#define STEP(f, a, b, c, d, x, k, s) \
	do { \
		a += f(b, c, d) + (x) + (k); \
		a = ROTL(a, s) + b; \
	} while (0)

static void md5_block(md5_t *m, const uint8_t *p)
{
	uint32_t w[16], a = m->h[0], b = m->h[1], c = m->h[2], d = m->h[3];
	memcpy(w, p, 64); /* little-endian host (x86-64) */
	STEP(F, a, b, c, d, w[0], 0xd76aa478u, 7);
	STEP(F, d, a, b, c, w[1], 0xe8c7b756u, 12);
	STEP(F, c, d, a, b, w[2], 0x242070dbu, 17);
	STEP(F, b, c, d, a, w[3], 0xc1bdceeeu, 22);
	STEP(F, a, b, c, d, w[4], 0xf57c0fafu, 7);
	STEP(F, d, a, b, c, w[5], 0x4787c62au, 12);
	STEP(F, c, d, a, b, w[6], 0xa8304613u, 17);
	STEP(F, b, c, d, a, w[7], 0xfd469501u, 22);
	STEP(F, a, b, c, d, w[8], 0x698098d8u, 7);
	STEP(F, d, a, b, c, w[9], 0x8b44f7afu, 12);
	STEP(F, c, d, a, b, w[10], 0xffff5bb1u, 17);
	STEP(F, b, c, d, a, w[11], 0x895cd7beu, 22);
	STEP(F, a, b, c, d, w[12], 0x6b901122u, 7);
	STEP(F, d, a, b, c, w[13], 0xfd987193u, 12);
	STEP(F, c, d, a, b, w[14], 0xa679438eu, 17);
	STEP(F, b, c, d, a, w[15], 0x49b40821u, 22);
	STEP(G, a, b, c, d, w[1], 0xf61e2562u, 5);
	STEP(G, d, a, b, c, w[6], 0xc040b340u, 9);
	STEP(G, c, d, a, b, w[11], 0x265e5a51u, 14);
	STEP(G, b, c, d, a, w[0], 0xe9b6c7aau, 20);
	STEP(G, a, b, c, d, w[5], 0xd62f105du, 5);
	STEP(G, d, a, b, c, w[10], 0x02441453u, 9);
	STEP(G, c, d, a, b, w[15], 0xd8a1e681u, 14);
	STEP(G, b, c, d, a, w[4], 0xe7d3fbc8u, 20);
	STEP(G, a, b, c, d, w[9], 0x21e1cde6u, 5);
	STEP(G, d, a, b, c, w[14], 0xc33707d6u, 9);
	STEP(G, c, d, a, b, w[3], 0xf4d50d87u, 14);
	STEP(G, b, c, d, a, w[8], 0x455a14edu, 20);
	STEP(G, a, b, c, d, w[13], 0xa9e3e905u, 5);
	STEP(G, d, a, b, c, w[2], 0xfcefa3f8u, 9);
	STEP(G, c, d, a, b, w[7], 0x676f02d9u, 14);
	STEP(G, b, c, d, a, w[12], 0x8d2a4c8au, 20);
	STEP(H, a, b, c, d, w[5], 0xfffa3942u, 4);
	STEP(H, d, a, b, c, w[8], 0x8771f681u, 11);
	STEP(H, c, d, a, b, w[11], 0x6d9d6122u, 16);
	STEP(H, b, c, d, a, w[14], 0xfde5380cu, 23);
	STEP(H, a, b, c, d, w[1], 0xa4beea44u, 4);
	STEP(H, d, a, b, c, w[4], 0x4bdecfa9u, 11);
	STEP(H, c, d, a, b, w[7], 0xf6bb4b60u, 16);
	STEP(H, b, c, d, a, w[10], 0xbebfbc70u, 23);
	STEP(H, a, b, c, d, w[13], 0x289b7ec6u, 4);
	STEP(H, d, a, b, c, w[0], 0xeaa127fau, 11);
	STEP(H, c, d, a, b, w[3], 0xd4ef3085u, 16);
	STEP(H, b, c, d, a, w[6], 0x04881d05u, 23);
	STEP(H, a, b, c, d, w[9], 0xd9d4d039u, 4);
	STEP(H, d, a, b, c, w[12], 0xe6db99e5u, 11);
	STEP(H, c, d, a, b, w[15], 0x1fa27cf8u, 16);
	STEP(H, b, c, d, a, w[2], 0xc4ac5665u, 23);
	STEP(I, a, b, c, d, w[0], 0xf4292244u, 6);
	STEP(I, d, a, b, c, w[7], 0x432aff97u, 10);
	STEP(I, c, d, a, b, w[14], 0xab9423a7u, 15);
	STEP(I, b, c, d, a, w[5], 0xfc93a039u, 21);
	STEP(I, a, b, c, d, w[12], 0x655b59c3u, 6);
	STEP(I, d, a, b, c, w[3], 0x8f0ccc92u, 10);
	STEP(I, c, d, a, b, w[10], 0xffeff47du, 15);
	STEP(I, b, c, d, a, w[1], 0x85845dd1u, 21);
	STEP(I, a, b, c, d, w[8], 0x6fa87e4fu, 6);
	STEP(I, d, a, b, c, w[15], 0xfe2ce6e0u, 10);
	STEP(I, c, d, a, b, w[6], 0xa3014314u, 15);
	STEP(I, b, c, d, a, w[13], 0x4e0811a1u, 21);
	STEP(I, a, b, c, d, w[4], 0xf7537e82u, 6);
	STEP(I, d, a, b, c, w[11], 0xbd3af235u, 10);
	STEP(I, c, d, a, b, w[2], 0x2ad7d2bbu, 15);
	STEP(I, b, c, d, a, w[9], 0xeb86d391u, 21);
	m->h[0] += a;
	m->h[1] += b;
	m->h[2] += c;
	m->h[3] += d;
}

static void md5_init(md5_t *m)
{
	m->h[0] = 0x67452301;
	m->h[1] = 0xefcdab89;
	m->h[2] = 0x98badcfe;
	m->h[3] = 0x10325476;
	m->len = 0;
	m->fill = 0;
}

static void md5_update(md5_t *m, const uint8_t *p, size_t n)
{
	m->len += n;
	if (m->fill) {
		size_t k = 64 - m->fill;
		if (k > n) k = n;
		memcpy(m->buf + m->fill, p, k);
		m->fill += k;
		p += k;
		n -= k;
		if (m->fill == 64) {
			md5_block(m, m->buf);
			m->fill = 0;
		}
	}
	while (n >= 64) {
		md5_block(m, p);
		p += 64;
		n -= 64;
	}
	if (n) {
		memcpy(m->buf, p, n);
		m->fill = n;
	}
}

static void md5_final(md5_t *m, uint8_t out[16])
{
	uint64_t bits = m->len * 8;
	uint8_t pad = 0x80;
	uint8_t zero = 0;
	md5_update(m, &pad, 1);
	while (m->fill != 56) md5_update(m, &zero, 1);
	for (int i = 0; i < 8; ++i) {
		uint8_t c = (uint8_t)(bits >> (8 * i));
		md5_update(m, &c, 1);
	}
	for (int i = 0; i < 4; ++i) {
		out[i * 4] = (uint8_t)m->h[i];
		out[i * 4 + 1] = (uint8_t)(m->h[i] >> 8);
		out[i * 4 + 2] = (uint8_t)(m->h[i] >> 16);
		out[i * 4 + 3] = (uint8_t)(m->h[i] >> 24);
	}
}

static void md5_line(const uint8_t dg[16], char out[35])
{
	static const char hex[] = "0123456789abcdef";
	for (int i = 0; i < 16; ++i) {
		out[i * 2] = hex[dg[i] >> 4];
		out[i * 2 + 1] = hex[dg[i] & 15];
	}
	out[32] = '\r';
	out[33] = '\n';
	out[34] = 0;
}

void m2dec_amd_frame_md5(const m2d_frame_t *f, char out[35])
{
	md5_t m;
	uint8_t dg[16];
	int stride = f->width;
	int height = f->height - f->crop[2] - f->crop[3];
	int width = stride - f->crop[0] - f->crop[1];
	const uint8_t *src = f->luma + stride * f->crop[2] + f->crop[0];
	md5_init(&m);
	for (int y = 0; y < height; ++y) {
		md5_update(&m, src, (size_t)width);
		src += stride;
	}
	src = f->chroma + stride * (f->crop[2] >> 1) + f->crop[0];
	height >>= 1;
	for (int y = 0; y < height; ++y) {
		md5_update(&m, src, (size_t)width);
		src += stride;
	}
	md5_final(&m, dg);
	md5_line(dg, out);
}

/* ---------------------------------------------------------------- 2-3 frames on one core, scalar
 * The scalar chain is latency-bound (~5 dependent ALU operations per step) and leaves most of the
 * core's integer ports idle: two or three frames' chains stepped side by side run at about the latency
 * of one (the 16-lane AVX-512 kernel below takes twice that for any batch of 2-16).  The tail of a
 * stream (frames hashed as they leave the decoder, one thread each) is where this pays: two frames per
 * core instead of one. */
#define SSTEP(f, a, b, c, d, wi, k, s) \
	do { \
		for (int j = 0; j < NCH; ++j) { \
			uint32_t x_; \
			memcpy(&x_, lp[j] + 64 * n + 4 * (wi), 4); \
			a[j] += f(b[j], c[j], d[j]) + x_ + (k); \
			a[j] = ROTL(a[j], s) + b[j]; \
		} \
	} while (0)
#define MD5XN_BLOCKS(name, NCH_) \
	static void name(uint32_t st[][4], const uint8_t *const lp[], size_t nblocks) \
	{ \
		enum { NCH = NCH_ }; \
		for (size_t n = 0; n < nblocks; ++n) { \
			uint32_t a[NCH], b[NCH], c[NCH], d[NCH]; \
			for (int j = 0; j < NCH; ++j) { \
				a[j] = st[j][0]; \
				b[j] = st[j][1]; \
				c[j] = st[j][2]; \
				d[j] = st[j][3]; \
			} \
			MD5XN_STEPS \
			for (int j = 0; j < NCH; ++j) { \
				st[j][0] += a[j]; \
				st[j][1] += b[j]; \
				st[j][2] += c[j]; \
				st[j][3] += d[j]; \
			} \
		} \
	}
#define MD5XN_STEPS \
SSTEP(F, a, b, c, d, 0, 0xd76aa478u, 7); \
SSTEP(F, d, a, b, c, 1, 0xe8c7b756u, 12); \
SSTEP(F, c, d, a, b, 2, 0x242070dbu, 17); \
SSTEP(F, b, c, d, a, 3, 0xc1bdceeeu, 22); \
SSTEP(F, a, b, c, d, 4, 0xf57c0fafu, 7); \
SSTEP(F, d, a, b, c, 5, 0x4787c62au, 12); \
SSTEP(F, c, d, a, b, 6, 0xa8304613u, 17); \
SSTEP(F, b, c, d, a, 7, 0xfd469501u, 22); \
SSTEP(F, a, b, c, d, 8, 0x698098d8u, 7); \
SSTEP(F, d, a, b, c, 9, 0x8b44f7afu, 12); \
SSTEP(F, c, d, a, b, 10, 0xffff5bb1u, 17); \
SSTEP(F, b, c, d, a, 11, 0x895cd7beu, 22); \
SSTEP(F, a, b, c, d, 12, 0x6b901122u, 7); \
SSTEP(F, d, a, b, c, 13, 0xfd987193u, 12); \
SSTEP(F, c, d, a, b, 14, 0xa679438eu, 17); \
SSTEP(F, b, c, d, a, 15, 0x49b40821u, 22); \
SSTEP(G, a, b, c, d, 1, 0xf61e2562u, 5); \
SSTEP(G, d, a, b, c, 6, 0xc040b340u, 9); \
SSTEP(G, c, d, a, b, 11, 0x265e5a51u, 14); \
SSTEP(G, b, c, d, a, 0, 0xe9b6c7aau, 20); \
SSTEP(G, a, b, c, d, 5, 0xd62f105du, 5); \
SSTEP(G, d, a, b, c, 10, 0x02441453u, 9); \
SSTEP(G, c, d, a, b, 15, 0xd8a1e681u, 14); \
SSTEP(G, b, c, d, a, 4, 0xe7d3fbc8u, 20); \
SSTEP(G, a, b, c, d, 9, 0x21e1cde6u, 5); \
SSTEP(G, d, a, b, c, 14, 0xc33707d6u, 9); \
SSTEP(G, c, d, a, b, 3, 0xf4d50d87u, 14); \
SSTEP(G, b, c, d, a, 8, 0x455a14edu, 20); \
SSTEP(G, a, b, c, d, 13, 0xa9e3e905u, 5); \
SSTEP(G, d, a, b, c, 2, 0xfcefa3f8u, 9); \
SSTEP(G, c, d, a, b, 7, 0x676f02d9u, 14); \
SSTEP(G, b, c, d, a, 12, 0x8d2a4c8au, 20); \
SSTEP(H, a, b, c, d, 5, 0xfffa3942u, 4); \
SSTEP(H, d, a, b, c, 8, 0x8771f681u, 11); \
SSTEP(H, c, d, a, b, 11, 0x6d9d6122u, 16); \
SSTEP(H, b, c, d, a, 14, 0xfde5380cu, 23); \
SSTEP(H, a, b, c, d, 1, 0xa4beea44u, 4); \
SSTEP(H, d, a, b, c, 4, 0x4bdecfa9u, 11); \
SSTEP(H, c, d, a, b, 7, 0xf6bb4b60u, 16); \
SSTEP(H, b, c, d, a, 10, 0xbebfbc70u, 23); \
SSTEP(H, a, b, c, d, 13, 0x289b7ec6u, 4); \
SSTEP(H, d, a, b, c, 0, 0xeaa127fau, 11); \
SSTEP(H, c, d, a, b, 3, 0xd4ef3085u, 16); \
SSTEP(H, b, c, d, a, 6, 0x04881d05u, 23); \
SSTEP(H, a, b, c, d, 9, 0xd9d4d039u, 4); \
SSTEP(H, d, a, b, c, 12, 0xe6db99e5u, 11); \
SSTEP(H, c, d, a, b, 15, 0x1fa27cf8u, 16); \
SSTEP(H, b, c, d, a, 2, 0xc4ac5665u, 23); \
SSTEP(I, a, b, c, d, 0, 0xf4292244u, 6); \
SSTEP(I, d, a, b, c, 7, 0x432aff97u, 10); \
SSTEP(I, c, d, a, b, 14, 0xab9423a7u, 15); \
SSTEP(I, b, c, d, a, 5, 0xfc93a039u, 21); \
SSTEP(I, a, b, c, d, 12, 0x655b59c3u, 6); \
SSTEP(I, d, a, b, c, 3, 0x8f0ccc92u, 10); \
SSTEP(I, c, d, a, b, 10, 0xffeff47du, 15); \
SSTEP(I, b, c, d, a, 1, 0x85845dd1u, 21); \
SSTEP(I, a, b, c, d, 8, 0x6fa87e4fu, 6); \
SSTEP(I, d, a, b, c, 15, 0xfe2ce6e0u, 10); \
SSTEP(I, c, d, a, b, 6, 0xa3014314u, 15); \
SSTEP(I, b, c, d, a, 13, 0x4e0811a1u, 21); \
SSTEP(I, a, b, c, d, 4, 0xf7537e82u, 6); \
SSTEP(I, d, a, b, c, 11, 0xbd3af235u, 10); \
SSTEP(I, c, d, a, b, 2, 0x2ad7d2bbu, 15); \
SSTEP(I, b, c, d, a, 9, 0xeb86d391u, 21);
MD5XN_BLOCKS(md5x2_blocks, 2)
MD5XN_BLOCKS(md5x3_blocks, 3)

/* ---------------------------------------------------------------- 16 frames at once (AVX-512F)
 * Multi-buffer MD5: lane l of every 512-bit register carries frame l's chain, so one core runs 16
 * independent MD5s at about the latency of one (the per-frame MD5 of FileWriterMd5 is a sequential
 * chain; frames are what can go side by side).  A frame's message is its cropped luma rows then its
 * cropped chroma rows; without horizontal crop each is one contiguous run, and every full 64-byte
 * block of a run is hashed in the lanes; the last partial block and the padding go through the
 * scalar code from the lane's chaining value. */
#if defined(__x86_64__)
#include <immintrin.h>

/* a + M + K does not depend on the previous step: the chain through b is F, add, rotate, add */
#define VSTEP(imm, a, b, c, d, wi, k, s) \
	do { \
		a = _mm512_add_epi32(a, _mm512_add_epi32(w[wi], _mm512_set1_epi32((int)(k)))); \
		a = _mm512_add_epi32(a, _mm512_ternarylogic_epi32(b, c, d, imm)); \
		a = _mm512_add_epi32(_mm512_rol_epi32(a, s), b); \
	} while (0)
/* ternary-logic truth tables over (b, c, d): F = b ? c : d, G = d ? b : c, H = b ^ c ^ d, I = c ^ (b | ~d) */
#define TF 0xca
#define TG 0xe4
#define TH 0x96
#define TI 0x39

/* 16 rows of 16 dwords -> 16 columns (r[i] lane l = row l word i) */
__attribute__((target("avx512f"))) static inline void transpose16(__m512i r[16])
{
	__m512i t[16];
	for (int i = 0; i < 8; ++i) {
		t[2 * i] = _mm512_unpacklo_epi32(r[2 * i], r[2 * i + 1]);
		t[2 * i + 1] = _mm512_unpackhi_epi32(r[2 * i], r[2 * i + 1]);
	}
	for (int i = 0; i < 4; ++i) {
		r[4 * i + 0] = _mm512_unpacklo_epi64(t[4 * i], t[4 * i + 2]);
		r[4 * i + 1] = _mm512_unpackhi_epi64(t[4 * i], t[4 * i + 2]);
		r[4 * i + 2] = _mm512_unpacklo_epi64(t[4 * i + 1], t[4 * i + 3]);
		r[4 * i + 3] = _mm512_unpackhi_epi64(t[4 * i + 1], t[4 * i + 3]);
	}
	for (int h = 0; h < 2; ++h)
		for (int i = 0; i < 4; ++i) {
			t[8 * h + i] = _mm512_shuffle_i32x4(r[8 * h + i], r[8 * h + 4 + i], 0x88);
			t[8 * h + 4 + i] = _mm512_shuffle_i32x4(r[8 * h + i], r[8 * h + 4 + i], 0xdd);
		}
	for (int i = 0; i < 8; ++i) {
		r[i] = _mm512_shuffle_i32x4(t[i], t[8 + i], 0x88);
		r[8 + i] = _mm512_shuffle_i32x4(t[i], t[8 + i], 0xdd);
	}
}

/* lane l hashes nblocks 64-byte blocks at base + off[l]: each block step loads one 64-byte block per
 * lane and transposes them (gathers measured 2.5x slower on the EPYC host) */
__attribute__((target("avx512f"))) static void md5x16_blocks(uint32_t st[4][16], const uint8_t *const lp[16],
                                                              size_t nblocks)
{
	__m512i va = _mm512_loadu_si512(st[0]), vb = _mm512_loadu_si512(st[1]);
	__m512i vc = _mm512_loadu_si512(st[2]), vd = _mm512_loadu_si512(st[3]);
	for (size_t n = 0; n < nblocks; ++n) {
		__m512i w[16];
		__m512i a = va, b = vb, c = vc, d = vd;
		for (int l = 0; l < 16; ++l) w[l] = _mm512_loadu_si512(lp[l] + 64 * n);
		transpose16(w);
		VSTEP(TF, a, b, c, d, 0, 0xd76aa478u, 7);
		VSTEP(TF, d, a, b, c, 1, 0xe8c7b756u, 12);
		VSTEP(TF, c, d, a, b, 2, 0x242070dbu, 17);
		VSTEP(TF, b, c, d, a, 3, 0xc1bdceeeu, 22);
		VSTEP(TF, a, b, c, d, 4, 0xf57c0fafu, 7);
		VSTEP(TF, d, a, b, c, 5, 0x4787c62au, 12);
		VSTEP(TF, c, d, a, b, 6, 0xa8304613u, 17);
		VSTEP(TF, b, c, d, a, 7, 0xfd469501u, 22);
		VSTEP(TF, a, b, c, d, 8, 0x698098d8u, 7);
		VSTEP(TF, d, a, b, c, 9, 0x8b44f7afu, 12);
		VSTEP(TF, c, d, a, b, 10, 0xffff5bb1u, 17);
		VSTEP(TF, b, c, d, a, 11, 0x895cd7beu, 22);
		VSTEP(TF, a, b, c, d, 12, 0x6b901122u, 7);
		VSTEP(TF, d, a, b, c, 13, 0xfd987193u, 12);
		VSTEP(TF, c, d, a, b, 14, 0xa679438eu, 17);
		VSTEP(TF, b, c, d, a, 15, 0x49b40821u, 22);
		VSTEP(TG, a, b, c, d, 1, 0xf61e2562u, 5);
		VSTEP(TG, d, a, b, c, 6, 0xc040b340u, 9);
		VSTEP(TG, c, d, a, b, 11, 0x265e5a51u, 14);
		VSTEP(TG, b, c, d, a, 0, 0xe9b6c7aau, 20);
		VSTEP(TG, a, b, c, d, 5, 0xd62f105du, 5);
		VSTEP(TG, d, a, b, c, 10, 0x02441453u, 9);
		VSTEP(TG, c, d, a, b, 15, 0xd8a1e681u, 14);
		VSTEP(TG, b, c, d, a, 4, 0xe7d3fbc8u, 20);
		VSTEP(TG, a, b, c, d, 9, 0x21e1cde6u, 5);
		VSTEP(TG, d, a, b, c, 14, 0xc33707d6u, 9);
		VSTEP(TG, c, d, a, b, 3, 0xf4d50d87u, 14);
		VSTEP(TG, b, c, d, a, 8, 0x455a14edu, 20);
		VSTEP(TG, a, b, c, d, 13, 0xa9e3e905u, 5);
		VSTEP(TG, d, a, b, c, 2, 0xfcefa3f8u, 9);
		VSTEP(TG, c, d, a, b, 7, 0x676f02d9u, 14);
		VSTEP(TG, b, c, d, a, 12, 0x8d2a4c8au, 20);
		VSTEP(TH, a, b, c, d, 5, 0xfffa3942u, 4);
		VSTEP(TH, d, a, b, c, 8, 0x8771f681u, 11);
		VSTEP(TH, c, d, a, b, 11, 0x6d9d6122u, 16);
		VSTEP(TH, b, c, d, a, 14, 0xfde5380cu, 23);
		VSTEP(TH, a, b, c, d, 1, 0xa4beea44u, 4);
		VSTEP(TH, d, a, b, c, 4, 0x4bdecfa9u, 11);
		VSTEP(TH, c, d, a, b, 7, 0xf6bb4b60u, 16);
		VSTEP(TH, b, c, d, a, 10, 0xbebfbc70u, 23);
		VSTEP(TH, a, b, c, d, 13, 0x289b7ec6u, 4);
		VSTEP(TH, d, a, b, c, 0, 0xeaa127fau, 11);
		VSTEP(TH, c, d, a, b, 3, 0xd4ef3085u, 16);
		VSTEP(TH, b, c, d, a, 6, 0x04881d05u, 23);
		VSTEP(TH, a, b, c, d, 9, 0xd9d4d039u, 4);
		VSTEP(TH, d, a, b, c, 12, 0xe6db99e5u, 11);
		VSTEP(TH, c, d, a, b, 15, 0x1fa27cf8u, 16);
		VSTEP(TH, b, c, d, a, 2, 0xc4ac5665u, 23);
		VSTEP(TI, a, b, c, d, 0, 0xf4292244u, 6);
		VSTEP(TI, d, a, b, c, 7, 0x432aff97u, 10);
		VSTEP(TI, c, d, a, b, 14, 0xab9423a7u, 15);
		VSTEP(TI, b, c, d, a, 5, 0xfc93a039u, 21);
		VSTEP(TI, a, b, c, d, 12, 0x655b59c3u, 6);
		VSTEP(TI, d, a, b, c, 3, 0x8f0ccc92u, 10);
		VSTEP(TI, c, d, a, b, 10, 0xffeff47du, 15);
		VSTEP(TI, b, c, d, a, 1, 0x85845dd1u, 21);
		VSTEP(TI, a, b, c, d, 8, 0x6fa87e4fu, 6);
		VSTEP(TI, d, a, b, c, 15, 0xfe2ce6e0u, 10);
		VSTEP(TI, c, d, a, b, 6, 0xa3014314u, 15);
		VSTEP(TI, b, c, d, a, 13, 0x4e0811a1u, 21);
		VSTEP(TI, a, b, c, d, 4, 0xf7537e82u, 6);
		VSTEP(TI, d, a, b, c, 11, 0xbd3af235u, 10);
		VSTEP(TI, c, d, a, b, 2, 0x2ad7d2bbu, 15);
		VSTEP(TI, b, c, d, a, 9, 0xeb86d391u, 21);
		va = _mm512_add_epi32(va, a);
		vb = _mm512_add_epi32(vb, b);
		vc = _mm512_add_epi32(vc, c);
		vd = _mm512_add_epi32(vd, d);
	}
	_mm512_storeu_si512(st[0], va);
	_mm512_storeu_si512(st[1], vb);
	_mm512_storeu_si512(st[2], vc);
	_mm512_storeu_si512(st[3], vd);
}

static int have_avx512(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("M2DEC_AMD_MD5_SCALAR"); /* (tests: force the scalar path) */
		__builtin_cpu_init();
		v = __builtin_cpu_supports("avx512f") && !(e && atoi(e));
	}
	return v;
}
#endif

/* one geometry, rows contiguous (no horizontal crop): each frame's message is a luma run then a chroma run */
static int same_runs(const m2d_frame_t *f, int n)
{
	for (int i = 0; i < n; ++i) {
		const m2d_frame_t *g = &f[i];
		if (g->width != f[0].width || g->height != f[0].height || g->crop[2] != f[0].crop[2] ||
		    g->crop[3] != f[0].crop[3] || g->crop[0] || g->crop[1])
			return 0;
	}
	return f[0].height - f[0].crop[2] - f[0].crop[3] > 0;
}

/* the scalar tail of lane l after its full blocks: the last partial block, the padding, the line */
static void lane_finish(const uint32_t h[4], const uint8_t *pa, const uint8_t *pb, size_t la, size_t lb, size_t na,
                        size_t nb, char out[35])
{
	md5_t m;
	uint8_t dg[16];
	for (int k = 0; k < 4; ++k) m.h[k] = h[k];
	m.len = (uint64_t)(na + nb) * 64;
	m.fill = 0;
	if (nb) {
		md5_update(&m, pb + nb * 64, lb - nb * 64);
	} else {
		md5_update(&m, pa + na * 64, la - na * 64);
		md5_update(&m, pb, lb);
	}
	md5_final(&m, dg);
	md5_line(dg, out);
}

static const uint32_t md5_iv[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};

static int stitch_on(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("M2DEC_AMD_MD5_STITCH"); /* (A/B: 0 = batches of 2-3 on the 16-lane kernel) */
		v = !(e && atoi(e) == 0);
	}
	return v;
}

int m2dec_amd_frames_md5(const m2d_frame_t *f, int n, char (*out)[35])
{
	if (n <= 0 || n > 16) return -1;
	const int runs = n >= 2 && same_runs(f, n);
	const int stride = f[0].width, h = f[0].height - f[0].crop[2] - f[0].crop[3];
	const size_t la = (size_t)stride * (size_t)(h > 0 ? h : 0), lb = (size_t)stride * (size_t)(h > 0 ? h >> 1 : 0);
	const size_t na = la / 64, nb = (la % 64) ? 0 : lb / 64;
	if (runs && n <= 3 && stitch_on()) {
		uint32_t st[3][4];
		const uint8_t *pa[3], *pb[3];
		for (int l = 0; l < n; ++l) {
			pa[l] = f[l].luma + (size_t)stride * f[0].crop[2];
			pb[l] = f[l].chroma + (size_t)stride * (f[0].crop[2] >> 1);
			memcpy(st[l], md5_iv, sizeof(md5_iv));
		}
		if (n == 2) {
			md5x2_blocks(st, pa, na);
			md5x2_blocks(st, pb, nb);
		} else {
			md5x3_blocks(st, pa, na);
			md5x3_blocks(st, pb, nb);
		}
		for (int l = 0; l < n; ++l) lane_finish(st[l], pa[l], pb[l], la, lb, na, nb, out[l]);
		return 0;
	}
#if defined(__x86_64__)
	if (runs && have_avx512()) {
		uint32_t st[4][16];
		const uint8_t *pa[16], *pb[16];
		for (int l = 0; l < 16; ++l) {
			const m2d_frame_t *g = &f[l < n ? l : 0]; /* idle lanes repeat lane 0 */
			pa[l] = g->luma + (size_t)stride * f[0].crop[2];
			pb[l] = g->chroma + (size_t)stride * (f[0].crop[2] >> 1);
			for (int k = 0; k < 4; ++k) st[k][l] = md5_iv[k];
		}
		md5x16_blocks(st, pa, na);
		md5x16_blocks(st, pb, nb);
		for (int l = 0; l < n; ++l) {
			const uint32_t hl[4] = {st[0][l], st[1][l], st[2][l], st[3][l]};
			lane_finish(hl, pa[l], pb[l], la, lb, na, nb, out[l]);
		}
		return 0;
	}
#endif
	for (int i = 0; i < n; ++i) m2dec_amd_frame_md5(&f[i], out[i]);
	return 0;
}
