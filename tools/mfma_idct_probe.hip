/* Probe: the int8-MFMA inverse DCT (m2dec_amd/csrc/hip/h265_mfma.h) against the reference's integer two-pass
 * transform on the CPU, for N = 16 and 32, over random blocks (sparse and dense, int16 extremes included).
 *   hipcc --offload-arch=gfx950 -O3 -Im2dec_amd/csrc/hip tools/mfma_idct_probe.hip -o tools/_build/mfma_idct_probe
 *   tools/_build/mfma_idct_probe [blocks]    -> "N=32: 0 of B blocks differ" ... */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "h265_mfma.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

template <int N>
__global__ __launch_bounds__(64) void k_probe(const int16_t *coef, int *out)
{
	__shared__ h265mfma::Tabs tb;
	__shared__ int16_t c[N * N];
	const int lane = threadIdx.x;
	h265mfma::tabs_init(tb, lane, 64);
	for (int i = lane; i < N * N; i += 64) c[i] = coef[(size_t)blockIdx.x * N * N + i];
	__syncthreads();
	int r[h265mfma::per_lane<N>()];
	h265mfma::idct<N>(c, tb, lane, r);
	for (int i = 0; i < h265mfma::per_lane<N>(); ++i)
		out[(size_t)blockIdx.x * N * N + h265mfma::acc_row<N>(i, lane) * N + h265mfma::acc_col<N>(lane)] = r[i];
}

static int sat16h(long v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : (int)v); }

template <int N>
static void ref(const int16_t *c, int *r)
{
	int g[N * N];
	for (int y = 0; y < N; ++y)
		for (int x = 0; x < N; ++x) {
			long e = 0;
			for (int k = 0; k < N; ++k) e += (long)h265mfma::t32(k * 32 / N, y) * c[k * N + x];
			g[y * N + x] = sat16h((e + 64) >> 7);
		}
	for (int y = 0; y < N; ++y)
		for (int x = 0; x < N; ++x) {
			long e = 0;
			for (int k = 0; k < N; ++k) e += (long)h265mfma::t32(k * 32 / N, x) * g[y * N + k];
			r[y * N + x] = sat16h((e + 2048) >> 12);
		}
}

template <int N>
static int run(int nb)
{
	std::vector<int16_t> c((size_t)nb * N * N);
	srand(1234 + N);
	for (int b = 0; b < nb; ++b) {
		int16_t *p = &c[(size_t)b * N * N];
		const int kind = b % 5;
		for (int i = 0; i < N * N; ++i) {
			int v = 0;
			if (kind == 0) v = (rand() % 8 == 0) ? rand() % 512 - 256 : 0;               /* sparse, small */
			else if (kind == 1) v = (rand() & 0xffff) - 32768;                           /* dense, full int16 */
			else if (kind == 2) v = (rand() % 3 == 0) ? ((rand() & 1) ? 32767 : -32768) : 0; /* extremes */
			else if (kind == 3) v = i < 3 ? rand() % 4096 - 2048 : 0;                    /* low frequencies */
			else v = rand() % 65 - 32;
			p[i] = (int16_t)v;
		}
	}
	int16_t *dc;
	int *dr;
	CK(hipMalloc(&dc, c.size() * 2));
	CK(hipMalloc(&dr, c.size() * 4));
	CK(hipMemcpy(dc, c.data(), c.size() * 2, hipMemcpyHostToDevice));
	hipLaunchKernelGGL(k_probe<N>, dim3(nb), dim3(64), 0, 0, dc, dr);
	CK(hipGetLastError());
	std::vector<int> out(c.size());
	CK(hipMemcpy(out.data(), dr, out.size() * 4, hipMemcpyDeviceToHost));
	int bad = 0;
	for (int b = 0; b < nb; ++b) {
		int r[N * N];
		ref<N>(&c[(size_t)b * N * N], r);
		int diff = 0, first = -1;
		for (int i = 0; i < N * N; ++i)
			if (r[i] != out[(size_t)b * N * N + i]) {
				if (first < 0) first = i;
				++diff;
			}
		if (diff) {
			if (bad < 4)
				fprintf(stderr, "N=%d block %d (kind %d): %d samples differ, first (%d,%d) ref %d got %d\n", N, b, b % 5, diff,
				        first % N, first / N, r[first], out[(size_t)b * N * N + first]);
			++bad;
		}
	}
	printf("N=%d: %d of %d blocks differ\n", N, bad, nb);
	CK(hipFree(dc));
	CK(hipFree(dr));
	return bad;
}

int main(int argc, char **argv)
{
	const int nb = argc > 1 ? atoi(argv[1]) : 500;
	const int bad = run<16>(nb) + run<32>(nb);
	return bad ? 1 : 0;
}
