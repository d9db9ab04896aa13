// Development microbenchmark (round 6): how long a chain of dependent packed-u16 VALU ops
// takes per wave, alone and with other waves, and whether the waves of one workgroup run
// concurrently.  Each wave runs N iterations of a 4-op dependent chain (psubs, pmax, pmax,
// perm -- the DP fill's loop-carried path) plus K independent ops per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint32_t psubs(uint32_t a, uint32_t b) {
	typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b) {
	typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}

template<int K>
__global__ void chain(uint32_t* out, int n, uint32_t s0, uint32_t s1) {
	uint32_t h = threadIdx.x, e = threadIdx.x * 3u, f = 7u;
	uint32_t x[8];
	for(int k = 0; k < 8; k++) x[k] = threadIdx.x + k;
	for(int i = 0; i < n; i++) {
#pragma unroll
		for(int r = 0; r < 8; r++) {
			const uint32_t hl = __builtin_amdgcn_perm(h, e, s0);
			const uint32_t ho = psubs(hl, s1);
			e = pmax(ho, e);
			h = pmax(pmax(h, e), f);
#pragma unroll
			for(int k = 0; k < K; k++) x[k & 7] = pmax(psubs(x[k & 7], s1), x[(k + 1) & 7]);
		}
	}
	uint32_t acc = h ^ e;
	for(int k = 0; k < 8; k++) acc ^= x[k];
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template<int K>
float run(int blocks, int threads, int n, uint32_t* d) {
	hipEvent_t a, b;
	hipEventCreate(&a); hipEventCreate(&b);
	hipLaunchKernelGGL(chain<K>, dim3(blocks), dim3(threads), 0, 0, d, n, 0x05040100u, 0x00030003u);
	hipEventRecord(a);
	hipLaunchKernelGGL(chain<K>, dim3(blocks), dim3(threads), 0, 0, d, n, 0x05040100u, 0x00030003u);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms = 0;
	hipEventElapsedTime(&ms, a, b);
	return ms;
}

int main() {
	uint32_t* d;
	hipMalloc(&d, 64 << 20);
	const int n = 20000;
	// per wave: n * 8 * (4 + 2K) VALU
	struct Cfg { int blocks, threads; const char* what; } cfgs[] = {
		{256, 64, "1 wave / CU"}, {1024, 64, "1 wave / SIMD (64-thread groups)"},
		{512, 128, "2-wave groups, 1024 waves"}, {256, 256, "4-wave groups, 1024 waves"},
		{2048, 64, "2 waves / SIMD (64-thread groups)"}, {1024, 128, "2-wave groups, 2048 waves"},
		{4096, 64, "4 waves / SIMD"}, {8192, 64, "8 waves / SIMD"}};
	for(const Cfg& c : cfgs) {
		const float m0 = run<0>(c.blocks, c.threads, n, d);
		const float m8 = run<8>(c.blocks, c.threads, n, d);
		const double per0 = (double)n * 8 * 4, per8 = (double)n * 8 * 20;
		std::printf("%-36s K=0: %7.3f ms (%.2f ns/dep-op)   K=8: %7.3f ms (%.3f ns/op per wave)\n", c.what,
		            m0, m0 * 1e6 / per0, m8, m8 * 1e6 / per8);
	}
	return 0;
}
