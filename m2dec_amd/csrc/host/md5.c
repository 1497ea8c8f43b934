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

static const uint32_t K[64] = {
	0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
	0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
	0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
	0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
	0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
	0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
	0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
	0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t R[64] = {
	7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
	5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20,
	4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
	6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_block(md5_t *m, const uint8_t *p)
{
	uint32_t w[16], a = m->h[0], b = m->h[1], c = m->h[2], d = m->h[3];
	for (int i = 0; i < 16; ++i)
		w[i] = (uint32_t)p[i * 4] | ((uint32_t)p[i * 4 + 1] << 8) | ((uint32_t)p[i * 4 + 2] << 16) | ((uint32_t)p[i * 4 + 3] << 24);
	for (int i = 0; i < 64; ++i) {
		uint32_t f;
		int g;
		if (i < 16) { f = (b & c) | (~b & d); g = i; }
		else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
		else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
		else { f = c ^ (b | ~d); g = (7 * i) & 15; }
		f = f + a + K[i] + w[g];
		a = d;
		d = c;
		c = b;
		b = b + ROTL(f, R[i]);
	}
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
