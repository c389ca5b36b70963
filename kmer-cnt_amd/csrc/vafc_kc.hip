// vafc_kc.hip -- kc-c4 on the GPU: the number of
// occurrences of every distinct canonical k-mer of the reads, then the
// histogram of those numbers (kc-c4.c:85-101 count_seq_buf, :117-128
// worker_for, :196-223 print_hist).
//
// The reference splits k-mers over 2^p khashl sub-tables by the low p bits
// of hash64(canonical) (kc-c4.c:34-44, 68-83) with 10-bit saturating counts
// in the low key bits.  Its output depends only on how often each distinct
// canonical k-mer occurs (hash64 is invertible on 2k bits; min(count, 255)
// is what the histogram keeps, below the 1023 saturation), so the device
// table is laid out for HBM instead:
//
//   * one open-addressing table of 16-byte slots {u64 key, u64 count} in HBM,
//     linear probing, key = hash64(canonical) + 1 (0 = empty, so a memset
//     clears the table); one slot is one 16-byte piece of a cache line: the
//     probe load brings the line into L2 and the count's atomic add finds it
//     there;
//   * an optional partition of the hash64 range (n_parts slices) so a k-mer
//     set larger than the table is counted in several passes over the input,
//     or on several GPUs at once;
//   * reads up to KC_LONG bases: one lane each, rolling 2-bit state; longer
//     reads (FASTA records) go to a list and are cut into KC_SEG-base segments
//     plus a (k-1)-base halo, one lane per segment.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vafc_kc.h"

namespace {

// kc-c4.c:21-38 seq_nt4_table: bytes 0..3 are codes themselves, A/C/G/T and
// a/c/g/t (and U/u) map to 0..3, everything else to 4
__device__ __forceinline__ uint32_t nt4(uint32_t b)
{
	if (b < 4) return b;
	const uint32_t u = b & 0xDF;   // upper case
	if (u == 'A') return 0;
	if (u == 'C') return 1;
	if (u == 'G') return 2;
	if (u == 'T' || u == 'U') return 3;
	return 4;
}

// kc-c4.c:34-44 hash64 (invertible on the bits of mask)
__device__ __forceinline__ uint64_t kc_hash64(uint64_t key, uint64_t mask)
{
	key = (~key + (key << 21)) & mask;
	key = key ^ key >> 24;
	key = ((key + (key << 3)) + (key << 8)) & mask;
	key = key ^ key >> 14;
	key = ((key + (key << 2)) + (key << 4)) & mask;
	key = key ^ key >> 28;
	key = (key + (key << 31)) & mask;
	return key;
}

struct Local {
	uint64_t kmers = 0, fresh = 0;
	bool overflow = false;
};

__device__ __forceinline__ void kc_insert(const KcArgs &A, uint64_t y, Local &L)
{
	const uint64_t h = kc_hash64(y, A.kmask);
	if (A.n_parts > 1 && (uint32_t)(((h & 0xFFFFFFFFull) * A.n_parts) >> 32) != A.part) return;
	const unsigned long long key = h + 1;
	uint64_t i = (h * 0x9E3779B97F4A7C15ull) >> (64 - A.tbits);
	unsigned long long *T = A.table;
	for (uint32_t probe = 0; probe < KC_MAX_PROBE; ++probe) {
		unsigned long long cur = __hip_atomic_load(&T[2 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (cur == 0) {
			cur = atomicCAS(&T[2 * i], 0ull, key);
			if (cur == 0) {
				++L.fresh;
				atomicAdd(&T[2 * i + 1], 1ull);
				return;
			}
		}
		if (cur == key) {
			atomicAdd(&T[2 * i + 1], 1ull);
			return;
		}
		i = (i + 1) & A.tmask;
	}
	L.overflow = true;
	__hip_atomic_store(&A.stats[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every canonical k-mer of bases [a, b) of a read whose windows end at or
// after `emit_from` (kc-c4.c:85-101: an invalid base restarts the k-mer)
__device__ __forceinline__ void kc_scan(const KcArgs &A, const uint8_t *s, uint32_t a, uint32_t b, uint32_t emit_from,
                                        Local &L)
{
	const int k = A.k;
	const uint32_t shift = 2 * (k - 1);
	uint64_t x0 = 0, x1 = 0;
	int l = 0;
	for (uint32_t j = a; j < b; ++j) {
		const uint32_t c = nt4(s[j]);
		if (c < 4) {
			x0 = (x0 << 2 | c) & A.kmask;
			x1 = x1 >> 2 | (uint64_t)(3 - c) << shift;
			if (++l >= k && j >= emit_from) {
				++L.kmers;
				if (!L.overflow) kc_insert(A, x0 < x1 ? x0 : x1, L);
			}
		} else {
			l = 0;
			x0 = x1 = 0;
		}
	}
}

__device__ void kc_flush(const KcArgs &A, const Local &L)
{
	__shared__ unsigned long long s_kmers, s_fresh;
	__shared__ int s_over;
	if (threadIdx.x == 0) {
		s_kmers = s_fresh = 0;
		s_over = 0;
	}
	__syncthreads();
	if (L.kmers) atomicAdd(&s_kmers, (unsigned long long)L.kmers);
	if (L.fresh) atomicAdd(&s_fresh, (unsigned long long)L.fresh);
	if (L.overflow) s_over = 1;
	__syncthreads();
	if (threadIdx.x == 0) {
		if (s_kmers) atomicAdd(&A.stats[0], s_kmers);
		if (s_fresh) atomicAdd(&A.stats[1], s_fresh);
		if (s_over) atomicOr(&A.stats[2], 1ull);
	}
}

__global__ __launch_bounds__(KC_THREADS) void kc_count_kernel(KcArgs A)
{
	Local L;
	for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < A.n_reads;
	     r += (uint64_t)gridDim.x * blockDim.x) {
		const uint32_t len = A.lens[r];
		if (len > KC_LONG) {
			const uint32_t slot = atomicAdd(A.nlong, 1u);
			if (slot < A.long_cap) A.longlist[slot] = (uint32_t)r;
			continue;
		}
		if (!L.overflow && __hip_atomic_load(&A.stats[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
			L.overflow = true;   // the table is full: only the k-mers are tallied from here on
		kc_scan(A, A.seq + A.offs[r], 0, len, 0, L);
	}
	kc_flush(A, L);
}

// Long reads: segment t of the list's reads, in list order; segstart[i] is
// the first global segment of list entry i (exclusive scan, kc_long_scan).
__global__ void kc_long_scan(KcArgs A)
{
	// one block: sequential prefix over the (short) long-read list
	if (threadIdx.x != 0 || blockIdx.x != 0) return;
	const uint32_t n = *A.nlong < A.long_cap ? *A.nlong : A.long_cap;
	uint64_t acc = 0;
	for (uint32_t i = 0; i < n; ++i) {
		A.segstart[i] = acc;
		acc += (A.lens[A.longlist[i]] + KC_SEG - 1) / KC_SEG;
	}
	A.segstart[n] = acc;
}

__global__ __launch_bounds__(KC_THREADS) void kc_long_kernel(KcArgs A)
{
	Local L;
	const uint32_t n = *A.nlong < A.long_cap ? *A.nlong : A.long_cap;
	const uint64_t total = n ? A.segstart[n] : 0;
	for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
	     g += (uint64_t)gridDim.x * blockDim.x) {
		uint32_t lo = 0, hi = n;   // last entry with segstart <= g
		while (hi - lo > 1) {
			const uint32_t mid = (lo + hi) / 2;
			if (A.segstart[mid] <= g) lo = mid;
			else hi = mid;
		}
		const uint64_t r = A.longlist[lo];
		const uint32_t len = A.lens[r];
		const uint32_t seg = (uint32_t)(g - A.segstart[lo]);
		const uint32_t s0 = seg * KC_SEG, s1 = s0 + KC_SEG < len ? s0 + KC_SEG : len;
		const uint32_t from = s0 >= (uint32_t)(A.k - 1) ? s0 - (uint32_t)(A.k - 1) : 0;
		if (!L.overflow && __hip_atomic_load(&A.stats[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
			L.overflow = true;
		kc_scan(A, A.seq + A.offs[r], from, s1, s0, L);
	}
	kc_flush(A, L);
}

// min(count, 255) of every occupied slot (kc-c4.c:196-223)
__global__ __launch_bounds__(256) void kc_hist_kernel(const unsigned long long *table, uint64_t slots,
                                                      unsigned long long *hist)
{
	__shared__ uint32_t h[256];
	h[threadIdx.x] = 0;
	__syncthreads();
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * blockDim.x) {
		if (table[2 * i] == 0) continue;
		const unsigned long long c = table[2 * i + 1];
		atomicAdd(&h[c < 255 ? c : 255], 1u);
	}
	__syncthreads();
	if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

} // namespace

extern "C" hipError_t vc_launch_kc(const KcArgs *A, int grid, hipStream_t st)
{
	const hipError_t e = hipMemsetAsync(A->nlong, 0, sizeof(uint32_t), st);
	if (e != hipSuccess) return e;
	hipLaunchKernelGGL(kc_count_kernel, dim3(grid), dim3(KC_THREADS), 0, st, *A);
	hipLaunchKernelGGL(kc_long_scan, dim3(1), dim3(64), 0, st, *A);
	hipLaunchKernelGGL(kc_long_kernel, dim3(grid), dim3(KC_THREADS), 0, st, *A);
	return hipGetLastError();
}

extern "C" hipError_t vc_launch_kc_hist(const unsigned long long *table, uint64_t slots, unsigned long long *hist,
                                        int grid, hipStream_t st)
{
	hipLaunchKernelGGL(kc_hist_kernel, dim3(grid), dim3(256), 0, st, table, slots, hist);
	return hipGetLastError();
}
