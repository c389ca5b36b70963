// Microbenchmark: ds_read_b32 at random byte addresses that are dword aligned
// vs not (low two bits random), 128 KiB of LDS, 1024 threads per block, as the
// counting kernel's filter reads.  Checks every lane's xor of the values read
// against a host recomputation (is an unaligned read the 4 bytes at that byte
// address, little-endian?) and reports cycles per read.
//   hipcc --offload-arch=gfx950 -O3 -o lds_unaligned tools/lds_unaligned.hip && ./lds_unaligned
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int LDS_BYTES = 128 * 1024;
constexpr int ITERS = 256;

__host__ __device__ inline uint32_t fill_byte(uint32_t i) { return (i * 2654435761u >> 13) & 0xFFu; }
__host__ __device__ inline uint32_t step(uint32_t s) { return s * 1664525u + 1013904223u; }

template <bool ALIGNED>
__global__ __launch_bounds__(1024) void kern(uint32_t *out, uint32_t seed)
{
	extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
	for (uint32_t i = threadIdx.x; i < LDS_BYTES + 16; i += blockDim.x) sm[i] = (unsigned char)fill_byte(i);
	__syncthreads();
	uint32_t s[16];
	for (int j = 0; j < 16; ++j) s[j] = (blockIdx.x * 1024u + threadIdx.x) * 16u + j + seed;
	uint32_t acc = 0;
	for (int it = 0; it < ITERS; ++it) {
#pragma unroll
		for (int j = 0; j < 16; ++j) {
			s[j] = step(s[j]);
			uint32_t a = (s[j] >> 15) & (LDS_BYTES - 1);
			if (ALIGNED) a &= ~3u;
			const uint32_t v = *reinterpret_cast<const uint32_t *>(sm + a);
			acc = (acc ^ v) * 3u + (v >> 7);
		}
	}
	out[blockIdx.x * 1024u + threadIdx.x] = acc;
}

static uint32_t host_lane(uint32_t gid, uint32_t seed, bool aligned)
{
	uint32_t s[16];
	for (int j = 0; j < 16; ++j) s[j] = gid * 16u + j + seed;
	uint32_t acc = 0;
	for (int it = 0; it < ITERS; ++it)
		for (int j = 0; j < 16; ++j) {
			s[j] = step(s[j]);
			uint32_t a = (s[j] >> 15) & (LDS_BYTES - 1);
			if (aligned) a &= ~3u;
			uint32_t v = 0;
			for (int b = 0; b < 4; ++b) v |= fill_byte(a + b) << (8 * b);
			acc = (acc ^ v) * 3u + (v >> 7);
		}
	return acc;
}

int main()
{
	hipDeviceProp_t p;
	CK(hipGetDeviceProperties(&p, 0));
	const int blocks = p.multiProcessorCount * 8;
	const size_t n = (size_t)blocks * 1024;
	uint32_t *d;
	CK(hipMalloc(&d, n * 4));
	const size_t lds = LDS_BYTES + 16;
	CK(hipFuncSetAttribute((const void *)kern<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
	CK(hipFuncSetAttribute((const void *)kern<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	std::vector<uint32_t> h(n);
	for (int aligned = 1; aligned >= 0; --aligned) {
		float best = 1e30f;
		for (int rep = 0; rep < 5; ++rep) {
			CK(hipEventRecord(e0));
			if (aligned) hipLaunchKernelGGL(kern<true>, dim3(blocks), dim3(1024), lds, 0, d, 7u);
			else hipLaunchKernelGGL(kern<false>, dim3(blocks), dim3(1024), lds, 0, d, 7u);
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			if (ms < best) best = ms;
		}
		CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
		int bad = 0;
		for (size_t i = 0; i < n; i += 997)
			if (h[i] != host_lane((uint32_t)i, 7u, aligned)) ++bad;
		// wave-reads per CU: blocks/CU * 16 waves * ITERS * 16
		const double wave_reads_per_cu = 8.0 * 16 * ITERS * 16;
		const double cyc = best * 1e-3 * 2.4e9 / wave_reads_per_cu;
		printf("%s: %.3f ms, %.2f CU cycles per wave ds_read_b32, lanes checked %zu, mismatches %d\n",
		       aligned ? "aligned  " : "unaligned", best, cyc, (n + 996) / 997, bad);
	}
	CK(hipFree(d));
	return 0;
}
