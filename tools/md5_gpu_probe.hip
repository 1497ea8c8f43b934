// How long one FileWriterMd5 chain (RFC 1321 over a frame's cropped rows, reference src/app/filewrite.h:99-124)
// takes on gfx950: the measurement behind DESIGN §1 row (f)3.  A frame's MD5 is one sequential chain of
// compression steps; the GPU can only run it on one wave (wave-uniform chain, SALU/VALU) or one lane, and many
// frames side by side.  Variants:
//   wave: one workgroup of 64 lanes per frame, the chain wave-uniform (the loads are uniform);
//   lane: one lane per frame (frames side by side in a wave).
// Chaining values after the full blocks are checked against a host restatement.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/md5_gpu_probe tools/md5_gpu_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) \
	do { \
		hipError_t e_ = (x); \
		if (e_ != hipSuccess) { \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
			exit(1); \
		} \
	} while (0)

static uint32_t hK[64], hS[64], hG[64];

static void tables()
{
	static const uint32_t s4[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
	for (int i = 0; i < 64; ++i) {
		hK[i] = (uint32_t)(uint64_t)(fabs(sin((double)(i + 1))) * 4294967296.0);
		hS[i] = s4[i / 16][i % 4];
		hG[i] = i < 16 ? i : i < 32 ? (5 * i + 1) % 16 : i < 48 ? (3 * i + 5) % 16 : (7 * i) % 16;
	}
}

__host__ __device__ static inline uint32_t rotl(uint32_t x, uint32_t s) { return (x << s) | (x >> (32 - s)); }

template <bool DEV>
__host__ __device__ static inline void block(uint32_t h[4], const uint32_t *w, const uint32_t *K, const uint32_t *S,
                                             const uint32_t *G)
{
	uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#pragma unroll
	for (int i = 0; i < 64; ++i) {
		uint32_t f;
		if (i < 16) f = d ^ (b & (c ^ d));
		else if (i < 32) f = c ^ (d & (b ^ c));
		else if (i < 48) f = b ^ c ^ d;
		else f = c ^ (b | ~d);
		const uint32_t t = d;
		d = c;
		c = b;
		b = b + rotl(a + f + K[i] + w[G[i]], S[i]);
		a = t;
	}
	h[0] += a;
	h[1] += b;
	h[2] += c;
	h[3] += d;
}

// the round constants as literals: the device loop is fully unrolled, so K/S/G fold to immediates
__device__ static inline void dblock(uint32_t h[4], const uint32_t *w)
{
	static constexpr uint32_t K[64] = {
	    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
	    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
	    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
	    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
	    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
	    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
	    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
	    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
	static constexpr uint32_t S[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
	uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#pragma unroll
	for (int i = 0; i < 64; ++i) {
		uint32_t f;
		int g;
		if (i < 16) f = d ^ (b & (c ^ d)), g = i;
		else if (i < 32) f = c ^ (d & (b ^ c)), g = (5 * i + 1) % 16;
		else if (i < 48) f = b ^ c ^ d, g = (3 * i + 5) % 16;
		else f = c ^ (b | ~d), g = (7 * i) % 16;
		const uint32_t t = d;
		d = c;
		c = b;
		b = b + rotl(a + f + K[i] + w[g], S[i / 16][i % 4]);
		a = t;
	}
	h[0] += a;
	h[1] += b;
	h[2] += c;
	h[3] += d;
}

// one workgroup (one wave) per frame: every lane runs the same chain on the same words (wave-uniform)
__global__ __launch_bounds__(64) void k_md5_wave(const uint8_t *__restrict__ frames, size_t fbytes, size_t nblocks,
                                                  uint32_t *__restrict__ out)
{
	const uint32_t *p = (const uint32_t *)(frames + (size_t)blockIdx.x * fbytes);
	uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
	for (size_t n = 0; n < nblocks; ++n) {
		uint32_t w[16];
#pragma unroll
		for (int i = 0; i < 16; ++i) w[i] = __builtin_nontemporal_load(p + 16 * n + i);
		dblock(h, w);
	}
	// (lane-dependent address: a vector store)
	out[((size_t)blockIdx.x * 64 + threadIdx.x) * 4 + 0] = h[0];
	out[((size_t)blockIdx.x * 64 + threadIdx.x) * 4 + 1] = h[1];
	out[((size_t)blockIdx.x * 64 + threadIdx.x) * 4 + 2] = h[2];
	out[((size_t)blockIdx.x * 64 + threadIdx.x) * 4 + 3] = h[3];
}

// one lane per frame
__global__ __launch_bounds__(64) void k_md5_lane(const uint8_t *__restrict__ frames, size_t fbytes, size_t nblocks,
                                                  int nframes, uint32_t *__restrict__ out)
{
	const int f = blockIdx.x * 64 + threadIdx.x;
	if (f >= nframes) return;
	const uint4 *p = (const uint4 *)(frames + (size_t)f * fbytes);
	uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
	for (size_t n = 0; n < nblocks; ++n) {
		uint32_t w[16];
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint4 v = p[4 * n + i];
			w[4 * i] = v.x;
			w[4 * i + 1] = v.y;
			w[4 * i + 2] = v.z;
			w[4 * i + 3] = v.w;
		}
		dblock(h, w);
	}
	out[(size_t)f * 4 + 0] = h[0];
	out[(size_t)f * 4 + 1] = h[1];
	out[(size_t)f * 4 + 2] = h[2];
	out[(size_t)f * 4 + 3] = h[3];
}

int main(int argc, char **argv)
{
	const int W = 1920, H = 1080;
	const size_t fbytes = (size_t)W * H * 3 / 2, nblocks = fbytes / 64;
	const int nf = argc > 1 ? atoi(argv[1]) : 64;
	tables();
	std::vector<uint8_t> host(fbytes * nf);
	uint32_t x = 12345;
	for (auto &v : host) v = (uint8_t)((x = x * 1664525u + 1013904223u) >> 24);
	uint8_t *d;
	uint32_t *o;
	CK(hipMalloc(&d, host.size()));
	CK(hipMalloc(&o, (size_t)nf * 64 * 16));
	CK(hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice));
	// host check values for the first two frames
	uint32_t want[2][4];
	for (int f = 0; f < 2 && f < nf; ++f) {
		uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
		for (size_t n = 0; n < nblocks; ++n) {
			uint32_t w[16];
			memcpy(w, host.data() + f * fbytes + 64 * n, 64);
			block<false>(h, w, hK, hS, hG);
		}
		memcpy(want[f], h, 16);
	}
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	std::vector<uint32_t> got((size_t)nf * 64 * 4);
	for (int v = 0; v < 2; ++v)
		for (int frames : {1, nf}) {
			for (int rep = 0; rep < 2; ++rep) {
				CK(hipEventRecord(e0, 0));
				if (v == 0) hipLaunchKernelGGL(k_md5_wave, dim3(frames), dim3(64), 0, 0, d, fbytes, nblocks, o);
				else hipLaunchKernelGGL(k_md5_lane, dim3((frames + 63) / 64), dim3(64), 0, 0, d, fbytes, nblocks, frames, o);
				CK(hipGetLastError());
				CK(hipEventRecord(e1, 0));
				CK(hipEventSynchronize(e1));
				float ms = 0;
				CK(hipEventElapsedTime(&ms, e0, e1));
				CK(hipMemcpy(got.data(), o, got.size() * 4, hipMemcpyDeviceToHost));
				int ok = 1;
				for (int f = 0; f < 2 && f < frames; ++f) {
					const uint32_t *g = v == 0 ? &got[(size_t)f * 64 * 4] : &got[(size_t)f * 4];
					ok &= !memcmp(g, want[f], 16);
				}
				if (rep) printf("%s-per-frame  frames %3d  %8.2f ms  (%.2f ms per frame-chain, %.3f GB/s aggregate)  %s\n",
				                v == 0 ? "wave" : "lane", frames, ms, ms, (double)fbytes * frames / (ms * 1e6),
				                ok ? "chaining values match the host" : "MISMATCH");
			}
		}
	CK(hipFree(d));
	CK(hipFree(o));
	return 0;
}
