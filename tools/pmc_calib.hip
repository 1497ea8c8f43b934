// FETCH_SIZE calibration for the access widths the reconstruction kernels use (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel reads a 1 GiB buffer (4x the 256 MiB Infinity Cache, so re-reads cannot hide on-die) once:
//   k_wide16    16 B per lane, coalesced (the guide's calibrated case: FETCH_SIZE = 1/2 of the bytes)
//   k_dword     4 B per lane, coalesced (whole 256-B wave footprints)
//   k_win12     the inter workers' reference-window pattern: per lane three dwords (12 bytes) of one row,
//               lanes 16 rows apart (recon_hip.hip luma_mc_win), every byte of the buffer read once
//   k_byte      1 B per lane, coalesced
// and writes nothing.  Run under rocprofv3 --pmc FETCH_SIZE (tools/gpu_pmc_calib.sh): FETCH_SIZE x 1024 /
// 2^30 per dispatch is the factor for that width.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N_BYTES (1ull << 30)

__global__ void k_wide16(const uint4 *p, uint32_t *sink)
{
	const size_t n = N_BYTES / 16;
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const uint4 v = p[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_dword(const uint32_t *p, uint32_t *sink)
{
	const size_t n = N_BYTES / 4;
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i];
	if (acc == 0x12345678u) sink[0] = acc;
}

// rows of 192 bytes (16 lanes x 12 bytes): lane l of a 16-lane group reads dwords 3l..3l+2 of its row, so a
// group covers one 192-byte row; the 4 groups of a wave take 4 rows 1 KiB apart (windows of different blocks)
__global__ void k_win12(const uint32_t *p, uint32_t *sink)
{
	const size_t rows = N_BYTES / 192;
	const int lane = threadIdx.x & 63, g = lane >> 4, l = lane & 15;
	uint32_t acc = 0;
	const size_t waves = (size_t)gridDim.x * (blockDim.x / 64), w = blockIdx.x * (size_t)(blockDim.x / 64) + (threadIdx.x >> 6);
	for (size_t r = w * 4 + g; r < rows; r += waves * 4) {
		const uint32_t *q = p + r * 48 + 3 * l;
		acc ^= q[0] ^ q[1] ^ q[2];
	}
	if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_byte(const uint8_t *p, uint32_t *sink)
{
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N_BYTES; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i];
	if (acc == 0x12345678u) sink[0] = acc;
}

int main()
{
	uint8_t *buf = nullptr;
	uint32_t *sink = nullptr;
	if (hipMalloc(&buf, N_BYTES) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
	if (hipMemset(buf, 1, N_BYTES) != hipSuccess) return 1;
	const int grid = 256 * 8, block = 256;
	for (int rep = 0; rep < 2; ++rep) {
		hipLaunchKernelGGL(k_wide16, dim3(grid), dim3(block), 0, 0, (const uint4 *)buf, sink);
		hipLaunchKernelGGL(k_dword, dim3(grid), dim3(block), 0, 0, (const uint32_t *)buf, sink);
		hipLaunchKernelGGL(k_win12, dim3(grid), dim3(block), 0, 0, (const uint32_t *)buf, sink);
		hipLaunchKernelGGL(k_byte, dim3(grid), dim3(block), 0, 0, buf, sink);
	}
	if (hipDeviceSynchronize() != hipSuccess) return 1;
	printf("ok %llu bytes per kernel\n", (unsigned long long)N_BYTES);
	return 0;
}
