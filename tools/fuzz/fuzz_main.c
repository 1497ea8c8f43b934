/* AddressSanitizer harness over the host parsers and the CPU oracles (tools/fuzz/run_asan.sh): decodes
 * every file given after the codec name (264 / 265 / m2v) with the oracle back ends, no GPU. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "m2dec_amd.h"
#include "m2d_recon.h"
int oracle_backend_create(m2r_backend_t *out);
int h265_oracle_backend_create(h265r_backend_t *out);
static void on_frame(void *arg, const m2d_frame_t *f) { (void)arg; (void)f; }
int main(int argc, char **argv)
{
	const int h265 = !strcmp(argv[1], "265");
	for (int a = 2; a < argc; ++a) {
		FILE *f = fopen(argv[a], "rb"); static uint8_t buf[16 << 20]; size_t n = fread(buf, 1, sizeof buf, f); fclose(f);
		int err = 0;
		if (!strcmp(argv[1], "m2v")) {
			m2dec_amd_decode_m2v(buf, n, -1, 0, on_frame, NULL, &err);
		} else if (h265) {
			h265r_backend_t be; h265_oracle_backend_create(&be);
			m2dec_amd_decode_h265(buf, n, &be, 0, 0, on_frame, NULL, &err);
			be.destroy(be.self);
		} else {
			m2r_backend_t be; memset(&be, 0, sizeof be); oracle_backend_create(&be);
			m2dec_amd_decode_stream3(buf, n, &be, 0, -1, 2, on_frame, NULL, NULL);
			be.destroy(be.self);
		}
	}
	printf("done %d\n", argc - 2);
	return 0;
}
