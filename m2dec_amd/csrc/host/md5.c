/*
 * RFC 1321 MD5 and the FileWriterMd5 line format of the reference application
 * (src/app/filewrite.h:11-29 cropped NV12 rows, :99-105 "%02x" x16 + "\r\n").
 */
#include <stdint.h>
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

void m2dec_amd_frame_md5(const m2d_frame_t *f, char out[35])
{
	static const char hex[] = "0123456789abcdef";
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
	for (int i = 0; i < 16; ++i) {
		out[i * 2] = hex[dg[i] >> 4];
		out[i * 2 + 1] = hex[dg[i] & 15];
	}
	out[32] = '\r';
	out[33] = '\n';
	out[34] = 0;
}
