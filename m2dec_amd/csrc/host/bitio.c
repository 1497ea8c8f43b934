/*
 * dec_bits — the reference's stream-feeding protocol (bitio.h:57-75, bitio.c:56-126): the caller
 * hands buffers with dec_bits_set_data(); when the decoder runs dry it calls error_func(arg),
 * which either supplies the next buffer (returns 0) or signals end of stream (returns < 0).
 *
 * The H.264 parser consumes the feeder through h264_nal_next(), which extracts one NAL unit at a
 * time into an RBSP buffer (start-code scan + emulation-prevention removal), across buffer
 * boundaries.  The plain bit-reading entry points are provided for API completeness.
 */
#include <stdlib.h>
#include <string.h>
#include "h264_dec.h"

int dec_bits_open(dec_bits *ths, void (*loadbytes_func)(dec_bits *, int bytes))
{
	if (!ths) return -1;
	memset(ths, 0, sizeof(*ths));
	ths->load_bytes = loadbytes_func;
	return 0;
}

void dec_bits_close(dec_bits *ths)
{
	(void)ths;
}

void dec_bits_set_callback(dec_bits *ths, int (*error_func)(void *), void *error_arg)
{
	ths->error_func_ = error_func;
	ths->error_arg_ = error_arg;
}

int dec_bits_set_data(dec_bits *ths, const byte_t *buf, size_t buf_len, void *id)
{
	if (!ths || !buf) return -1;
	ths->buf_head_ = buf;
	ths->buf_ = buf;
	ths->buf_tail_ = buf + buf_len;
	ths->id = id;
	ths->cache_ = 0;
	ths->cache_len_ = 0;
	return 0;
}

static int refill(dec_bits *ths)
{
	if (!ths->error_func_) return -1;
	return ths->error_func_(ths->error_arg_);
}

static int next_byte(dec_bits *ths)
{
	while (ths->buf_ >= ths->buf_tail_) {
		if (refill(ths) < 0) return -1;
	}
	return *ths->buf_++;
}

/* the byte-level feeder for the start-code scanners of the codecs (H.264 NALs, MPEG-2 units) */
int m2d_stream_next_byte(dec_bits *ths)
{
	return next_byte(ths);
}

uint32_t show_bits(dec_bits *ths, int bit_len)
{
	while (ths->cache_len_ < bit_len) {
		int b = next_byte(ths);
		if (b < 0) b = 0;
		ths->cache_ |= (uint64_t)b << (56 - ths->cache_len_);
		ths->cache_len_ += 8;
	}
	return bit_len ? (uint32_t)(ths->cache_ >> (64 - bit_len)) : 0;
}

uint32_t get_bits(dec_bits *ths, int bit_len)
{
	uint32_t v = show_bits(ths, bit_len);
	ths->cache_ <<= bit_len;
	ths->cache_len_ -= bit_len;
	return v;
}

uint32_t show_onebit(dec_bits *ths) { return show_bits(ths, 1); }
uint32_t get_onebit(dec_bits *ths) { return get_bits(ths, 1); }
void skip_bits(dec_bits *ths, int bit_len) { get_bits(ths, bit_len); }
int not_aligned_bits(dec_bits *ths) { return ths->cache_len_ & 7; }
void byte_align(dec_bits *ths) { get_bits(ths, ths->cache_len_ & 7); }
void skip_bytes(dec_bits *ths, int byte_len) { while (byte_len-- > 0) get_bits(ths, 8); }
const byte_t *dec_bits_current(dec_bits *ths) { return ths->buf_ - (ths->cache_len_ >> 3); }
const byte_t *dec_bits_tail(dec_bits *ths) { return ths->buf_tail_; }

void m2d_load_bytes_skip03(dec_bits *ths, int read_bytes)
{
	(void)ths;
	(void)read_bytes;
}

/* m2d.cpp:130-155: byte count up to and including the next 00 00 01, or -1 */
int m2d_next_start_code(const byte_t *org_src, int byte_len)
{
	int zeros = 0;
	for (int i = 0; i < byte_len; ++i) {
		byte_t c = org_src[i];
		if (c == 0) {
			zeros++;
		} else {
			if (c == 1 && zeros >= 2) return i + 1;
			zeros = 0;
		}
	}
	return -1;
}

/* ------------------------------------------------------------------ NAL extraction */
/* room for n more bytes (and the 16 bytes of zero padding) */
static int nal_reserve(h264_dec_t *d, size_t n)
{
	if (d->nal_len + n + 16 >= d->nal_cap) {
		size_t cap = d->nal_cap ? d->nal_cap * 2 : (1u << 20);
		while (d->nal_len + n + 16 >= cap) cap *= 2;
		uint8_t *p = (uint8_t *)realloc(d->nal, cap);
		if (!p) return -1;
		d->nal = p;
		d->nal_cap = cap;
	}
	return 0;
}

static int nal_push(h264_dec_t *d, uint8_t c)
{
	if (nal_reserve(d, 1) < 0) return -1;
	d->nal[d->nal_len++] = c;
	return 0;
}

/* Read the next NAL unit (header byte + RBSP) into d->nal. Returns 0, or -1 at end of stream. */
int h264_nal_next(h264_dec_t *d)
{
	dec_bits *st = d->stream;
	int zeros = 0, c;
	if (d->nal_replay) { /* the parse-ahead pipeline closed a picture on this NAL: hand it out again */
		d->nal_replay = 0;
		return 0;
	}
	/* the refill callback reported the end of the data: like the reference's error exit (longjmp out of
	 * decode_picture, bitio.c / h264.cpp:673-685), nothing more is read in this decode_picture call;
	 * the next call asks the callback again (h264dec -f feeds the stream after its header replay) */
	if (d->eos) return -1;
	/* find a start code */
	if (!d->nal_pending) {
		for (;;) {
			c = next_byte(st);
			if (c < 0) {
				d->eos = 1;
				return -1;
			}
			if (c == 0) {
				zeros++;
			} else {
				if (c == 1 && zeros >= 2) break;
				zeros = 0;
			}
		}
	}
	d->nal_pending = 0;
	d->nal_len = 0;
	zeros = 0;
	for (;;) {
		/* a run without zero bytes is payload as it is: copied in bulk up to the next zero (the
		 * lookahead extracts every NAL of the stream on the API thread; byte by byte it took ~0.1 ms
		 * per 1080p picture, the pace at which the parse pool got work) */
		if (zeros == 0 && st->buf_ < st->buf_tail_) {
			const uint8_t *p = st->buf_;
			const uint8_t *z = (const uint8_t *)memchr(p, 0, (size_t)(st->buf_tail_ - p));
			const size_t n = (size_t)((z ? z : st->buf_tail_) - p);
			if (n) {
				if (nal_reserve(d, n) < 0) return -1;
				memcpy(d->nal + d->nal_len, p, n);
				d->nal_len += n;
				st->buf_ = p + n;
			}
		}
		c = next_byte(st);
		if (c < 0) {
			d->eos = 1;
			break;
		}
		if (zeros >= 2 && c == 1) {
			/* next start code: drop the zero bytes that belong to it */
			d->nal_len -= (size_t)((zeros > 3) ? 3 : zeros);
			d->nal_pending = 1;
			break;
		}
		if (zeros == 2 && c == 3) {
			/* emulation prevention byte */
			zeros = 0;
			continue;
		}
		if (nal_push(d, (uint8_t)c) < 0) return -1;
		zeros = (c == 0) ? zeros + 1 : 0;
	}
	/* trailing_zero_8bits */
	while (d->nal_len > 0 && d->nal[d->nal_len - 1] == 0) d->nal_len--;
	memset(d->nal + d->nal_len, 0, 16);
	return d->nal_len ? 0 : (c < 0 ? -1 : 0);
}
