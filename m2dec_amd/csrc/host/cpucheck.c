/*
 * Host CPU guard.  The host library is built for x86-64-v3 (AVX2 / BMI1 / BMI2 / LZCNT / MOVBE / FMA,
 * Makefile HOST_ARCH); this file alone is compiled for baseline x86-64, so the check runs before any
 * v3 instruction can.  On a CPU without those features every decoder init (h264d_func / m2d_func)
 * fails with a message instead of the process dying of SIGILL inside the parser.
 */
#include <stdio.h>
#include <stdlib.h>

int m2dec_host_cpu_ok = 1;

__attribute__((constructor)) static void m2dec_host_cpu_check(void)
{
	__builtin_cpu_init();
	if (!(__builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi") && __builtin_cpu_supports("bmi2") &&
	      __builtin_cpu_supports("fma") && __builtin_cpu_supports("popcnt"))) {
		m2dec_host_cpu_ok = 0;
		fprintf(stderr, "libm2dec_amd: this host CPU lacks x86-64-v3 (AVX2/BMI2/FMA); the library was built with "
		                "HOST_ARCH=-march=x86-64-v3 — rebuild with HOST_ARCH= for a baseline build\n");
	}
}

int m2dec_amd_host_cpu_ok(void) { return m2dec_host_cpu_ok; }
