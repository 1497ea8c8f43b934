/*
 * Test harness: drives libm2dec_amd's h264d_func exactly the way the reference's application layer
 * does (src/app/m2decoder.h, src/app/frames.h), written independently for the boundary tests:
 *
 *   - the context is `new uint8_t[context_size]`, init(ctx, -1, header_callback, this), the reread
 *     callback set on stream_pos(ctx)                               (M2Decoder::set_codec, :167-193)
 *   - the header callback sizes a Frames pool; when it is not sufficient it DELETES the old frames
 *     and allocates new ones (luma / chroma separately, 16-byte aligned), then set_frames
 *                                                                    (M2Decoder::SetFrames, :54-80)
 *   - decode / decode_residual output loop                           (m2decoder.h:132-157)
 *   - the destructor deletes the frames, then `delete[]` the context — no release call of any kind
 *                                                                    (M2Decoder::~M2Decoder, :39-46)
 *
 * Usage: m2decoder_like [-o liboracle.so] [-t threads] [-n iterations] [-m max_frames] [-k] stream.264...
 *   Every stream is decoded by a fresh decoder, once per iteration; one MD5 line per output frame
 *   (FileWriterMd5 format, via m2dec_amd_frame_md5) goes to stdout, then "#iter i threads T rss_kb R
 *   contexts C evicted E" once per iteration.  -o: reconstruct with the CPU oracle (test-only
 *   checker) instead of the GPU; -m: drop the decoder after that many frames (mid-stream); -k: never
 *   free a context's memory (leaked instead of delete[]), so that no context reuses a dropped one's
 *   address and the library cannot tell a dropped context from a live one but by its calls.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

extern "C" {
#include "m2dec_amd.h"
}

static int (*g_oracle_create)(m2r_backend_t *);
static int g_threads = -1;
static int g_keep = 0;
static int g_pause = 0; /* -p: all streams to their end, then drain (tests/test_boundary_cpu.py) */

class Frames {
	size_t luma_len_;
	std::vector<m2d_frame_t> raw_, aligned_;
	std::vector<uint8_t> second_;
	static uint8_t *align16(uint8_t *p) { return (uint8_t *)(((uintptr_t)p + 15) & ~(uintptr_t)15); }

public:
	Frames(int width, int height, int n, int second_len, void *id)
	    : luma_len_((size_t)((width + 15) & ~15) * (size_t)((height + 15) & ~15)), raw_(n), aligned_(n),
	      second_(second_len ? second_len : 1)
	{
		for (int i = 0; i < n; ++i) {
			memset(&raw_[i], 0, sizeof(raw_[i]));
			raw_[i].luma = new uint8_t[luma_len_ + 15];
			raw_[i].chroma = new uint8_t[(luma_len_ >> 1) + 15];
			aligned_[i] = raw_[i];
			aligned_[i].luma = align16(raw_[i].luma);
			aligned_[i].chroma = align16(raw_[i].chroma);
			aligned_[i].id = id;
		}
	}
	~Frames()
	{
		for (auto &f : raw_) {
			delete[] f.luma;
			delete[] f.chroma;
		}
	}
	m2d_frame_t *aligned() { return &aligned_[0]; }
	uint8_t *second() { return &second_[0]; }
	bool sufficient(size_t n, size_t luma_len, size_t add) const
	{
		return n <= aligned_.size() && luma_len <= luma_len_ && add <= second_.size();
	}
	void set_id(void *id)
	{
		for (auto &f : aligned_) f.id = id;
	}
};

class Decoder {
	Frames *frames_ = nullptr;
	uint8_t *context_ = nullptr;
	const m2d_func_table_t *func_ = h264d_func;
	const uint8_t *data_;
	size_t len_, pos_ = 0;

	static int reread(void *arg)
	{
		Decoder *d = (Decoder *)arg;
		if (d->pos_ >= d->len_) return -1;
		dec_bits_set_data(d->func_->stream_pos(d->context_), d->data_ + d->pos_, d->len_ - d->pos_, 0);
		d->pos_ = d->len_;
		return 0;
	}
	static int header_callback(void *arg, void *id)
	{
		((Decoder *)arg)->set_frames(id);
		return 0;
	}
	void set_frames(void *id)
	{
		m2d_info_t info;
		func_->get_info(context_, &info);
		const int w = (info.src_width + 15) & ~15, h = (info.src_height + 15) & ~15;
		int n = info.frame_num + 16;
		if (n > 64) n = 64;
		if (frames_) {
			if (frames_->sufficient((size_t)n, (size_t)w * h, (size_t)info.additional_size)) {
				frames_->set_id(id);
				return;
			}
			delete frames_; /* while the decoder may still be working: it must not touch them again */
			fputs("#realloc\n", stdout); /* frames still in the DPB now point at the new, unwritten memory */
		}
		fprintf(stderr, "%d x %d x %d\n", info.src_width - info.crop[0] - info.crop[1],
		        info.src_height - info.crop[2] - info.crop[3], info.frame_num);
		frames_ = new Frames(w, h, n, info.additional_size, id);
		if (func_->set_frames(context_, n, frames_->aligned(), frames_->second(), info.additional_size) < 0) {
			fprintf(stderr, "set_frames failed\n");
			exit(3);
		}
	}

public:
	Decoder(const uint8_t *data, size_t len) : data_(data), len_(len)
	{
		context_ = new uint8_t[func_->context_size];
		func_->init(context_, -1, header_callback, this);
		if (g_oracle_create) { /* test-only: the CPU checker as the reconstruction back end */
			m2r_backend_t be = {};
			if (g_oracle_create(&be) < 0 || m2dec_amd_h264_set_backend(context_, &be) < 0) exit(4);
		}
		if (g_threads >= 0) m2dec_amd_h264_set_parse_threads(context_, g_threads);
		dec_bits_set_callback(func_->stream_pos(context_), reread, this);
	}
	~Decoder()
	{
		fwrite(out.data(), 1, out.size(), stdout);
		delete frames_;
		if (!g_keep) delete[] context_; /* no release: the reference API has none */
	}
	/* -p: the frames of this decoder go to `out` (printed when it is deleted), and run() returns at the
	 * end of the data without draining the DPB: drain() does that later, after other contexts were made */
	std::string out;
	bool paused = false;
	int drain()
	{
		m2d_frame_t frm;
		int n = 0;
		while (func_->peek_decoded_frame(context_, &frm, 1)) {
			emit(frm);
			n++;
			func_->get_decoded_frame(context_, &frm, 1);
		}
		return n;
	}
	/* M2Decoder::decode / decode_residual; returns frames written, stops after max (>= 0) */
	int run(int max, bool stop_at_end = false)
	{
		m2d_frame_t frm;
		int n = 0;
		for (;;) {
			while (func_->peek_decoded_frame(context_, &frm, 0) <= 0) {
				const int err = func_->decode_picture(context_);
				if (err < 0) {
					if (stop_at_end) {
						paused = true;
						return n;
					}
					/* m2decoder.h:138 tests peek's result for truth, so -1 would loop here as it does there */
					while (func_->peek_decoded_frame(context_, &frm, 1)) {
						if (max >= 0 && n >= max) return n;
						emit(frm);
						n++;
						func_->get_decoded_frame(context_, &frm, 1);
					}
					return n;
				}
			}
			if (max >= 0 && n >= max) return n;
			func_->get_decoded_frame(context_, &frm, 0);
			emit(frm);
			n++;
			if (func_->decode_picture(context_) < 0) {
				if (stop_at_end) {
					paused = true;
					return n;
				}
				while (func_->peek_decoded_frame(context_, &frm, 1) > 0) {
					if (max >= 0 && n >= max) return n;
					emit(frm);
					n++;
					func_->get_decoded_frame(context_, &frm, 1);
				}
				return n;
			}
		}
	}
	void emit(const m2d_frame_t &f)
	{
		char line[35];
		m2dec_amd_frame_md5(&f, line);
		if (g_pause) out.append(line, 34);
		else fwrite(line, 1, 34, stdout);
	}
};

static long proc_status(const char *key)
{
	FILE *f = fopen("/proc/self/status", "r");
	char buf[256];
	long v = -1;
	if (!f) return -1;
	while (fgets(buf, sizeof(buf), f))
		if (!strncmp(buf, key, strlen(key))) v = atol(buf + strlen(key));
	fclose(f);
	return v;
}

int main(int argc, char **argv)
{
	int iters = 1, max = -1, i = 1;
	for (; i < argc && argv[i][0] == '-'; ++i) {
		if (!strcmp(argv[i], "-o") && i + 1 < argc) {
			void *h = dlopen(argv[++i], RTLD_NOW);
			if (!h || !(g_oracle_create = (int (*)(m2r_backend_t *))dlsym(h, "oracle_backend_create"))) {
				fprintf(stderr, "cannot load the oracle: %s\n", dlerror());
				return 2;
			}
		} else if (!strcmp(argv[i], "-t") && i + 1 < argc) {
			g_threads = atoi(argv[++i]);
		} else if (!strcmp(argv[i], "-n") && i + 1 < argc) {
			iters = atoi(argv[++i]);
		} else if (!strcmp(argv[i], "-m") && i + 1 < argc) {
			max = atoi(argv[++i]);
		} else if (!strcmp(argv[i], "-k")) {
			g_keep = 1;
		} else if (!strcmp(argv[i], "-p")) {
			g_pause = 1;
		} else {
			fprintf(stderr, "usage: %s [-o liboracle.so] [-t threads] [-n iters] [-m max] [-k] [-p] stream...\n", argv[0]);
			return 2;
		}
	}
	std::vector<std::string> data;
	for (; i < argc; ++i) {
		FILE *f = fopen(argv[i], "rb");
		if (!f) return 2;
		std::string s;
		char buf[65536];
		size_t r;
		while ((r = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, r);
		fclose(f);
		data.push_back(s);
	}
	for (int it = 0; it < iters; ++it) {
		if (g_pause) {
			/* every stream decoded to its end (decode_picture -2) with its DPB not drained yet, all
			 * contexts alive at once; then each is drained the way M2Decoder::decode does */
			std::vector<Decoder *> ds;
			for (auto &s : data) {
				ds.push_back(new Decoder((const uint8_t *)s.data(), s.size()));
				ds.back()->run(max, true);
			}
			int ctxs = 0;
			long ev = 0;
			m2dec_amd_h264_registry(&ctxs, &ev);
			printf("#paused contexts %d evicted %ld\n", ctxs, ev);
			for (Decoder *d : ds) {
				d->drain();
				delete d;
			}
		}
		for (auto &s : data) {
			if (g_pause) break;
			Decoder *d = new Decoder((const uint8_t *)s.data(), s.size());
			d->run(max);
			delete d;
		}
		int ctxs = 0;
		long ev = 0;
		m2dec_amd_h264_registry(&ctxs, &ev);
		printf("#iter %d threads %ld rss_kb %ld contexts %d evicted %ld\n", it, proc_status("Threads:"),
		       proc_status("VmRSS:"), ctxs, ev);
		fflush(stdout);
	}
	return 0;
}
