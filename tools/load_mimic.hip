// load_mimic.hip -- the counting kernel's global-load pattern with no other
// work (tools only): one lane per 150-byte read, the read's dwords fetched as
// in scan_span_quad (one dword + four dwordx4 per trip of 64 bytes), XORed,
// one dword stored per lane.  Same grid (one 1024-thread block per CU, grid-
// striding over groups of 1024 reads).  If this runs at the HBM rate, its
// time gives the bytes the pattern really moves, whatever the EA request
// counters say.  Also a plain streaming pass over the same buffer.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/load_mimic tools/load_mimic.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

__global__ void __launch_bounds__(1024) mimic(const uint32_t *s32, uint64_t n_reads, uint32_t L, uint64_t wmax,
                                              uint32_t *out)
{
	uint32_t acc = 0;
	for (uint64_t g = blockIdx.x; g * 1024 < n_reads; g += gridDim.x) {
		const uint64_t r = g * 1024 + threadIdx.x;
		if (r >= n_reads) break;
		const uint64_t wi = (r * L) >> 2;
		const int nq = (int)((L + 15) / 16) + 3;     // quads the scan requests (nit + 3, PEEL + 4-chunk trips)
		acc ^= s32[wi];
		for (int q = 0; q < nq; ++q) {
			uint64_t i = wi + 1 + 4 * (uint64_t)q;
			if (i + 3 > wmax) i = wmax - 3;
			const u32x4a4 v = *reinterpret_cast<const u32x4a4 *>(s32 + i);
			acc ^= v.x ^ v.y ^ v.z ^ v.w;
		}
	}
	out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

__global__ void stream(const uint4 *p, uint64_t n16, uint32_t *out)
{
	uint32_t acc = 0;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint4 v = p[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
	const uint64_t R = 100000000ull, L = 150, bytes = R * L;
	uint8_t *d;
	uint32_t *out;
	CK(hipMalloc(&d, bytes + 64));
	CK(hipMalloc(&out, 1024 * 1024 * 4));
	CK(hipMemset(d, 0x41, bytes + 64));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	int ncu = 0;
	CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	for (int rep = 0; rep < 5; ++rep) {
		float ms1, ms2;
		CK(hipEventRecord(a));
		hipLaunchKernelGGL(mimic, dim3(ncu), dim3(1024), 0, 0, (const uint32_t *)d, R, (uint32_t)L, bytes / 4 - 1, out);
		CK(hipEventRecord(b));
		CK(hipEventSynchronize(b));
		CK(hipEventElapsedTime(&ms1, a, b));
		CK(hipEventRecord(a));
		hipLaunchKernelGGL(stream, dim3(ncu * 8), dim3(256), 0, 0, (const uint4 *)d, bytes / 16, out);
		CK(hipEventRecord(b));
		CK(hipEventSynchronize(b));
		CK(hipEventElapsedTime(&ms2, a, b));
		printf("mimic %.3f ms (%.0f GB/s of read bytes)   stream %.3f ms (%.0f GB/s)\n", ms1, bytes / (ms1 * 1e6), ms2,
		       bytes / (ms2 * 1e6));
	}
	return 0;
}
