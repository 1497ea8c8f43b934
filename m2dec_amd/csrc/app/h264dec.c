/*
 * h264dec — the reference's command-line decoder (src/app/h264dec.cpp) over libm2dec_amd.so, so that
 * test.sh-style checks (`h264dec -O stream.264`, then `cmp stream.md5 stream.out`) run unchanged.
 * H.264 reconstructs on the gfx950 GPU (h264d_func); MPEG-1/2 intra pictures decode on the CPU
 * (m2d_func, BASELINE.json configs[0]).
 *
 *   -b            bypass the DPB (dpb size 1)
 *   -d <n>        DPB size, n <= 32 (-1 auto)
 *   -e            emptify the DPB before the next frames (M2Decoder::decode, m2decoder.h:147-149)
 *   -f <n>        skip to the key frame before frame n, replaying the SPS / PPS seen on the way
 *                 (M2Decoder::skip_frames, m2decoder.h:96-131)
 *   -m            MPEG-2 elementary stream input (otherwise chosen by extension, m2decoder.h:236-260:
 *                 .m2v MPEG-2, .264 / .jsv H.264, .vob MPEG-2 PS, .265 H.265, anything else MPEG-2)
 *   -o / -O       RAW (cropped NV12, filewrite.h:11-29, 72-86) / MD5 (filewrite.h:89-124) output
 *                 into <basename>.out in the current directory
 *   -s            MPEG-2 program stream input (not supported: no demuxer in this library)
 *   -x            trap SIGABRT / SIGSEGV ("trap <no>", exit 0) and exit 0 (h264dec.cpp:217-249)
 * Exit status as the reference: 0 when decoding ended with "end of data" (-2), else the error code;
 * 0 with -x.
 */
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <unistd.h>
#include "m2dec_amd.h"

enum { MODE_MPEG2, MODE_MPEG2PS, MODE_H264, MODE_H265, MODE_NONE };

typedef struct {
	FILE *fo;
	int md5;
} writer_t;

static void write_frame(void *arg, const m2d_frame_t *f)
{
	writer_t *w = (writer_t *)arg;
	if (!w->fo) return;
	if (w->md5) {
		char line[35];
		m2dec_amd_frame_md5(f, line);
		fwrite(line, 1, 34, w->fo);
	} else {
		const int stride = f->width;
		const int height = f->height - f->crop[2] - f->crop[3];
		const int width = stride - f->crop[0] - f->crop[1];
		const uint8_t *src = f->luma + stride * f->crop[2] + f->crop[0];
		for (int y = 0; y < height; ++y, src += stride) fwrite(src, 1, (size_t)width, w->fo);
		src = f->chroma + stride * (f->crop[2] >> 1) + f->crop[0];
		for (int y = 0; y < (height >> 1); ++y, src += stride) fwrite(src, 1, (size_t)width, w->fo);
	}
	fflush(w->fo);
}

static void blame_user(void)
{
	fprintf(stderr, "Usage:\n"
	                "\th264dec [-b] [-d <dpb_size>] [-o|O ] <infile>\n"
	                "\t\t-b: Bypass DPB\n"
	                "\t\t-d <dpb_size>: Specify number of DPB frames -1, 1..16 (default: -1(auto))\n"
	                "\t\t-e: emptifiy DPB before next frames\n"
	                "\t\t-f <skip_num>: Specify number of frames to be skipped\n"
	                "\t\t-m: MPEG2 elementary input\n"
	                "\t\t-o: RAW output\n"
	                "\t\t-O: MD5 output\n"
	                "\t\t-s: MPEG2 PS input\n"
	                "\t\t-x: Mask SIGABRT on error.");
	exit(1);
}

/* detect_file, m2decoder.h:236-260 */
static int detect_file(const char *name)
{
	static const struct {
		int mode;
		const char *ext;
	} map[] = {{MODE_MPEG2, "m2v"}, {MODE_MPEG2PS, "vob"}, {MODE_H264, "264"}, {MODE_H264, "jsv"}, {MODE_H265, "265"}};
	const char *e = strrchr(name, '.');
	if (e++)
		for (size_t i = 0; i < sizeof(map) / sizeof(map[0]); ++i)
			if (!strcasecmp(map[i].ext, e)) return map[i].mode;
	return MODE_MPEG2;
}

static void trap(int no)
{
	fprintf(stderr, "trap %d\n", no);
	exit(0);
}

int main(int argc, char **argv)
{
	int opt, wmode = 0, dpb = -1, codec = MODE_NONE, emptify = 0, force_exec = 0, skip = 0, err = -1;
	writer_t w = {0, 0};
	/* this process's HIP runtime: 8 hardware queues (4 launch streams + the copy stream per decoder), asked for
	 * before anything uses HIP; the library leaves a caller's setting alone */
	m2dec_amd_configure_queues(8);
	while ((opt = getopt(argc, argv, "bd:ef:moOsx")) != -1) {
		switch (opt) {
		case 'b': dpb = 1; break;
		case 'd':
			dpb = (int)strtol(optarg, 0, 0);
			if (32 < (unsigned)dpb) blame_user();
			break;
		case 'e': emptify = 1; break;
		case 'f': skip = (int)strtol(optarg, 0, 0); break;
		case 'm': codec = MODE_MPEG2; break;
		case 'O': wmode = 1; break;
		case 'o': wmode = 2; break;
		case 's': codec = MODE_MPEG2PS; break;
		case 'x': force_exec = 1; break;
		default: blame_user();
		}
	}
	FILE *fi = optind < argc ? fopen(argv[optind], "rb") : NULL;
	if (!fi) blame_user();
	if (codec == MODE_NONE) codec = detect_file(argv[optind]);
	if (wmode) { /* <basename without extension>.out in the current directory (h264dec.cpp:31-47) */
		char dst[256];
		const char *base = strrchr(argv[optind], '/');
		base = base ? base + 1 : argv[optind];
		const char *ext = strrchr(base, '.');
		const size_t n = ext ? (size_t)(ext - base) : strlen(base);
		if (n + 5 <= sizeof(dst)) {
			memcpy(dst, base, n);
			strcpy(dst + n, ".out");
			w.fo = fopen(dst, "wb");
		}
		w.md5 = (wmode == 1);
	}
	fseek(fi, 0, SEEK_END);
	const long len = ftell(fi);
	fseek(fi, 0, SEEK_SET);
	uint8_t *data = (uint8_t *)malloc((size_t)len + 1);
	if (!data || fread(data, 1, (size_t)len, fi) != (size_t)len) return 1;
	fclose(fi);
	if (len <= 0) return -1;
	if (force_exec) {
		struct sigaction sa;
		memset(&sa, 0, sizeof(sa));
		sa.sa_handler = trap;
		sigaction(SIGABRT, &sa, 0);
		sigaction(SIGSEGV, &sa, 0);
	}
	switch (codec) {
	case MODE_H264:
		m2dec_amd_decode_table(h264d_func, 1, data, (size_t)len, dpb, emptify, skip, write_frame, &w, &err);
		break;
	case MODE_MPEG2:
		m2dec_amd_decode_table(m2d_func, 0, data, (size_t)len, dpb, emptify, skip, write_frame, &w, &err);
		break;
	case MODE_H265: /* M2Decoder MODE_H265 (m2decoder.h:180-182): reconstructed on GPU 0 */
		m2dec_amd_decode_h265(data, (size_t)len, NULL, 0, emptify, write_frame, &w, &err);
		break;
	default:
		fprintf(stderr, "h264dec: MPEG-2 program stream input is not supported by this library\n");
		err = -1;
		break;
	}
	if (w.fo) fclose(w.fo);
	free(data);
	return force_exec ? 0 : ((err == -2) ? 0 : err);
}
