// atomic_locality.hip -- does bucketing by table region pay for the kc-c4
// table (tools only)?  N relaxed 64-bit atomicAdds into a
// table of S 16-byte slots (the kc slot layout), at indices drawn uniformly:
//   random  -- in random order (what kc_count_kernel does today),
//   bucket  -- the same indices grouped into B table regions, region by region
//              (the order a partition pass would produce), regions of S/B slots.
//   hipcc --offload-arch=gfx950 -O3 -o tools/atomic_locality tools/atomic_locality.hip && tools/atomic_locality
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t mix(uint64_t x)
{
	x ^= x >> 33;
	x *= 0xff51afd7ed558ccdull;
	x ^= x >> 33;
	x *= 0xc4ceb9fe1a85ec53ull;
	x ^= x >> 33;
	return x;
}

// index i of the stream: random slot
__global__ void k_random(unsigned long long *t, uint64_t n, uint32_t sbits)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t s = mix(i) >> (64 - sbits);
		atomicAdd(&t[2 * s + 1], 1ull);
	}
}

// stream position i -> bucket (i / per), random slot inside that bucket's region
__global__ void k_bucket(unsigned long long *t, uint64_t n, uint32_t sbits, uint32_t bbits)
{
	const uint64_t per = n >> bbits;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t b = i / per;
		const uint64_t s = (b << (sbits - bbits)) | (mix(i) >> (64 - (sbits - bbits)));
		atomicAdd(&t[2 * s + 1], 1ull);
	}
}

// 32-bit counters, random order (same slot layout, low word of the count)
__global__ void k_random32(unsigned int *t, uint64_t n, uint32_t sbits)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t s = mix(i) >> (64 - sbits);
		atomicAdd(&t[4 * s + 2], 1u);
	}
}

int main()
{
	const uint32_t sbits = 29;                 // 2^29 slots x 16 B = 8.6 GB (kc_bench's table)
	const uint64_t n = 1160000000ull;          // k-mers of kc_bench's step
	unsigned long long *t;
	if (hipMalloc(&t, ((size_t)16) << sbits) != hipSuccess) return 1;
	hipMemset(t, 0, ((size_t)16) << sbits);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	const int grid = 256 * 16, block = 256;
	for (int rep = 0; rep < 2; ++rep) {
		float ms;
		hipEventRecord(e0);
		hipLaunchKernelGGL(k_random, dim3(grid), dim3(block), 0, 0, t, n, sbits);
		hipEventRecord(e1);
		hipEventSynchronize(e1);
		hipEventElapsedTime(&ms, e0, e1);
		printf("random order            %8.2f ms  %.2f G atomics/s\n", ms, n / ms / 1e6);
		hipEventRecord(e0);
		hipLaunchKernelGGL(k_random32, dim3(grid), dim3(block), 0, 0, (unsigned int *)t, n, sbits);
		hipEventRecord(e1);
		hipEventSynchronize(e1);
		hipEventElapsedTime(&ms, e0, e1);
		printf("random order, 32-bit    %8.2f ms  %.2f G atomics/s\n", ms, n / ms / 1e6);
		for (uint32_t bb : {4u, 6u, 8u, 10u}) {
			hipEventRecord(e0);
			hipLaunchKernelGGL(k_bucket, dim3(grid), dim3(block), 0, 0, t, n, sbits, bb);
			hipEventRecord(e1);
			hipEventSynchronize(e1);
			hipEventElapsedTime(&ms, e0, e1);
			printf("%4u regions of %5.0f MB %8.2f ms  %.2f G atomics/s\n", 1u << bb,
			       (double)(((size_t)16) << (sbits - bb)) / 1e6, ms, n / ms / 1e6);
		}
	}
	hipFree(t);
	return 0;
}
