/*
 * h264dec — command-line decoder with the reference's interface (src/app/h264dec.cpp:89-160),
 * reconstructing on the gfx950 GPU through libm2dec_amd.so, so that test.sh-style checks
 * (`h264dec -O stream.264` then `cmp stream.md5 stream.out`) run unchanged.
 *
 *   -O  MD5 output: one "32 hex + CRLF" line per frame (FileWriterMd5, filewrite.h:89-124)
 *   -o  RAW output: cropped NV12, Y rows then CbCr rows (FileWriter::write_cropping, filewrite.h:11-29)
 *   -b / -d <n>  DPB size (reference semantics: -b = 1, -d n <= 32)
 * The output file is the input's base name with the extension replaced by "out", in the current
 * directory (filewrite.h:42-63).  MPEG-2 (-m / -s) is not part of this back end.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include "m2dec_amd.h"

typedef struct {
	FILE *fo;
	int md5;
	long frames;
} writer_t;

static void on_frame(void *arg, const m2d_frame_t *f)
{
	writer_t *w = (writer_t *)arg;
	w->frames++;
	if (!w->fo) return;
	if (w->md5) {
		char line[35];
		m2dec_amd_frame_md5(f, line);
		fwrite(line, 1, 34, w->fo);
		fflush(w->fo);
	} else {
		int stride = f->width;
		int height = f->height - f->crop[2] - f->crop[3];
		int width = stride - f->crop[0] - f->crop[1];
		const uint8_t *src = f->luma + stride * f->crop[2] + f->crop[0];
		for (int y = 0; y < height; ++y, src += stride) fwrite(src, 1, (size_t)width, w->fo);
		src = f->chroma + stride * (f->crop[2] >> 1) + f->crop[0];
		for (int y = 0; y < (height >> 1); ++y, src += stride) fwrite(src, 1, (size_t)width, w->fo);
	}
}

static void usage(void)
{
	fprintf(stderr, "Usage: h264dec [-b] [-d <dpb_size>] [-o | -O] <input.264>\n"
	                "\t\t-b: bypass DPB (dpb size 1)\n\t\t-d <n>: DPB size (<= 32)\n"
	                "\t\t-o: RAW output\n\t\t-O: MD5 output\n");
	exit(1);
}

int main(int argc, char **argv)
{
	int opt, mode = 0, dpb = -1;
	writer_t w = {0, 0, 0};
	while ((opt = getopt(argc, argv, "bd:ef:moOsx")) != -1) {
		switch (opt) {
		case 'b': dpb = 1; break;
		case 'd':
			dpb = (int)strtol(optarg, 0, 0);
			if ((unsigned)dpb > 32) usage();
			break;
		case 'O': mode = 1; break;
		case 'o': mode = 2; break;
		case 'e': case 'f': case 'x': break;
		case 'm': case 's':
			fprintf(stderr, "h264dec: MPEG-2 input is not handled by the m2dec_amd back end\n");
			return 1;
		default: usage();
		}
	}
	if (optind >= argc) usage();
	FILE *fi = fopen(argv[optind], "rb");
	if (!fi) usage();
	fseek(fi, 0, SEEK_END);
	long len = ftell(fi);
	fseek(fi, 0, SEEK_SET);
	uint8_t *data = (uint8_t *)malloc((size_t)len + 1);
	if (!data || fread(data, 1, (size_t)len, fi) != (size_t)len) return 1;
	fclose(fi);
	if (mode) {
		char dst[4096];
		const char *base = strrchr(argv[optind], '/');
		base = base ? base + 1 : argv[optind];
		const char *ext = strrchr(base, '.');
		size_t n = ext ? (size_t)(ext - base) : strlen(base);
		if (n + 5 >= sizeof(dst)) return 1;
		memcpy(dst, base, n);
		strcpy(dst + n, ".out");
		w.fo = fopen(dst, "wb");
		if (!w.fo) return 1;
		w.md5 = (mode == 1);
	}
	m2dec_amd_stats_t st;
	int r = m2dec_amd_decode_stream2(data, (size_t)len, NULL, 0, dpb, on_frame, &w, &st);
	if (w.fo) fclose(w.fo);
	free(data);
	if (r < 0) {
		fprintf(stderr, "h264dec: decode failed after %ld frames (error %d)\n", w.frames, st.last_error);
		return 1;
	}
	return 0;
}
