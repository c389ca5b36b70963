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

__device__ __forceinline__ void kc_insert(const KcArgs &A, uint64_t y, uint64_t stamp, Local &L)
{
	const uint64_t h = kc_hash64(y, A.kmask);
	// partitions follow the low 10 bits: whole kc-c4 / yak sub-tables (p >= 10)
	if (A.n_parts > 1 && (uint32_t)(((h & 1023) * A.n_parts) >> 10) != A.part) return;
	const unsigned long long key = h + 1;
	uint64_t i = (h * 0x9E3779B97F4A7C15ull) >> (64 - A.tbits);
	unsigned long long *T = A.table;
	for (uint32_t probe = 0; probe < KC_MAX_PROBE; ++probe) {
		unsigned long long cur = __hip_atomic_load(&T[2 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (A.lookup_only) {   // yak pass 2 (yak-count.c:171-175): existing keys only
			if (cur == 0) return;
			if (cur == key) {
				if (__hip_atomic_load(&T[2 * i + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != KC_DROPPED)
					atomicAdd(&T[2 * i + 1], 1ull);
				return;
			}
			i = (i + 1) & A.tmask;
			continue;
		}
		if (cur == 0) {
			cur = atomicCAS(&T[2 * i], 0ull, key);
			if (cur == 0) {
				++L.fresh;
				atomicAdd(&T[2 * i + 1], 1ull);
				if (A.first) atomicMin(&A.first[i], stamp);
				return;
			}
		}
		if (cur == key) {
			atomicAdd(&T[2 * i + 1], 1ull);
			if (A.first) atomicMin(&A.first[i], stamp);
			return;
		}
		i = (i + 1) & A.tmask;
	}
	if (A.lookup_only) return;
	L.overflow = true;
	__hip_atomic_store(&A.stats[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every canonical k-mer of bases [a, b) of a read whose windows end at or
// after `emit_from` (kc-c4.c:85-101: an invalid base restarts the k-mer)
__device__ __forceinline__ void kc_scan(const KcArgs &A, const uint8_t *s, uint32_t a, uint32_t b, uint32_t emit_from,
                                        uint64_t read, Local &L)
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
				if (!L.overflow) kc_insert(A, x0 < x1 ? x0 : x1, (A.read_base + read) << 32 | j, L);
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
		kc_scan(A, A.seq + A.offs[r], 0, len, 0, r, L);
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
		kc_scan(A, A.seq + A.offs[r], from, s1, s0, r, L);
	}
	kc_flush(A, L);
}

// hist[min(count, n_bins - 1)] over the occupied slots with count >= min_count
// (kc-c4.c:206-223: 256 bins; yak-count.c:209-240 + the shrink to [2, 1023]
// of :268-288: 1024 bins); dropped keys are skipped.  hist[n_bins] gets the
// number of slots counted.
__global__ __launch_bounds__(256) void kc_hist_kernel(const unsigned long long *table, uint64_t slots,
                                                      unsigned long long *hist, uint32_t n_bins, uint64_t min_count)
{
	__shared__ uint32_t h[1024];
	__shared__ uint32_t tot;
	for (uint32_t b = threadIdx.x; b < n_bins; b += blockDim.x) h[b] = 0;
	if (threadIdx.x == 0) tot = 0;
	__syncthreads();
	uint32_t mine = 0;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * blockDim.x) {
		if (table[2 * i] == 0) continue;
		const unsigned long long c = table[2 * i + 1];
		if (c == KC_DROPPED || c < min_count) continue;
		atomicAdd(&h[c < n_bins - 1 ? c : n_bins - 1], 1u);
		++mine;
	}
	if (mine) atomicAdd(&tot, mine);
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < n_bins; b += blockDim.x)
		if (h[b]) atomicAdd(&hist[b], (unsigned long long)h[b]);
	if (threadIdx.x == 0 && tot) atomicAdd(&hist[n_bins], (unsigned long long)tot);
}

// ---- yak-count's Bloom filter, replayed (yak-count.c:91-108, 150-176) ----
//
// Pass 1 of yak-count -b puts a k-mer into its sub-table only when all n_hash
// bits of its hash in that sub-table's blocked Bloom filter were set before
// (by earlier k-mers of the stream; every k-mer sets its bits).  A k-mer seen
// twice is therefore always kept; one seen once is kept iff each of its bits
// was set by a k-mer occurring earlier, i.e. iff for each bit the smallest
// first-occurrence stamp among the k-mers using that bit is below its own.
// Only the bits of singletons matter, so they go into a scratch hash table
// (wtab) whose values are those minimum stamps.

// the n_hash bit ids of hash h: sub-table s = h & (2^pre - 1), x = h >> pre,
// block x & (2^(ns-9) - 1), bits h1 + i*h2 mod 512 (h2 bumped off multiples
// of 32); id = s << ns | block << 9 | bit
struct YakBits {
	uint64_t base;
	uint32_t z, h2;
};
__device__ __forceinline__ YakBits yak_bits(uint64_t h, uint32_t pre, uint32_t ns)
{
	const uint64_t s = h & (((uint64_t)1 << pre) - 1), x = h >> pre;
	const uint32_t xs = ns - 9;
	YakBits b;
	b.base = s << ns | (x & (((uint64_t)1 << xs) - 1)) << 9;
	b.z = (uint32_t)(x >> xs) & 511;
	b.h2 = (uint32_t)(x >> ns) & 511;
	if ((b.h2 & 31) == 0) b.h2 = (b.h2 + 1) & 511;
	return b;
}

__device__ __forceinline__ uint64_t yak_wslot(uint64_t id, uint32_t wbits)
{
	return (id * 0xD6E8FEB86659FD93ull) >> (64 - wbits);
}

// 1: the bit ids of every singleton into wtab (value: +inf)
__global__ __launch_bounds__(256) void yak_wanted_kernel(YakBloom B)
{
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.slots; i += (uint64_t)gridDim.x * blockDim.x) {
		const unsigned long long key = B.table[2 * i];
		if (key == 0 || B.table[2 * i + 1] != 1) continue;
		YakBits b = yak_bits(key - 1, B.pre, B.ns);
		uint32_t z = b.z;
		for (uint32_t n = 0; n < B.n_hash; ++n, z = (z + b.h2) & 511) {
			const unsigned long long id = (b.base | z) + 1;
			uint64_t w = yak_wslot(id, B.wbits);
			for (uint64_t probe = 0;; ++probe) {
				if (probe == B.wslots) {
					atomicOr(B.overflow, 1ull);
					return;
				}
				const unsigned long long cur = atomicCAS(&B.wtab[2 * w], 0ull, id);
				if (cur == 0) {   // new bit: no stamp yet (+inf)
					B.wtab[2 * w + 1] = KC_DROPPED;
					break;
				}
				if (cur == id) break;
				w = (w + 1) & (B.wslots - 1);
			}
		}
	}
}

// 2: for every key and each of its bits present in wtab: min(first stamp)
__global__ __launch_bounds__(256) void yak_mintime_kernel(YakBloom B)
{
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.slots; i += (uint64_t)gridDim.x * blockDim.x) {
		const unsigned long long key = B.table[2 * i];
		if (key == 0) continue;
		const unsigned long long t = B.first[i];
		YakBits b = yak_bits(key - 1, B.pre, B.ns);
		uint32_t z = b.z;
		for (uint32_t n = 0; n < B.n_hash; ++n, z = (z + b.h2) & 511) {
			const unsigned long long id = (b.base | z) + 1;
			uint64_t w = yak_wslot(id, B.wbits);
			for (uint64_t probe = 0; probe < B.wslots; ++probe) {
				const unsigned long long cur = B.wtab[2 * w];
				if (cur == 0) break;
				if (cur == id) {
					atomicMin(&B.wtab[2 * w + 1], t);
					break;
				}
				w = (w + 1) & (B.wslots - 1);
			}
		}
	}
}

// 3: keep = seen twice, or a singleton whose bits were all set before it;
// kept keys restart at count 0 (yak_ch_clear, yak-count.c:191-207), the rest
// are dropped
__global__ __launch_bounds__(256) void yak_select_kernel(YakBloom B)
{
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.slots; i += (uint64_t)gridDim.x * blockDim.x) {
		const unsigned long long key = B.table[2 * i];
		if (key == 0) continue;
		const unsigned long long c = B.table[2 * i + 1];
		bool keep = c >= 2 || B.n_hash == 0;   // n_hash 0: no filter, every key stays
		if (!keep && c == 1) {
			const unsigned long long t = B.first[i];
			YakBits b = yak_bits(key - 1, B.pre, B.ns);
			uint32_t z = b.z;
			keep = true;
			for (uint32_t n = 0; n < B.n_hash && keep; ++n, z = (z + b.h2) & 511) {
				const unsigned long long id = (b.base | z) + 1;
				uint64_t w = yak_wslot(id, B.wbits);
				unsigned long long m = KC_DROPPED;
				for (uint64_t probe = 0; probe < B.wslots; ++probe) {
					const unsigned long long cur = B.wtab[2 * w];
					if (cur == 0) break;
					if (cur == id) {
						m = B.wtab[2 * w + 1];
						break;
					}
					w = (w + 1) & (B.wslots - 1);
				}
				keep = m < t;
			}
		}
		B.counts_out[2 * i + 1] = keep ? 0ull : KC_DROPPED;
	}
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
                                        uint32_t n_bins, uint64_t min_count, int grid, hipStream_t st)
{
	if (n_bins < 2 || n_bins > 1024) return hipErrorInvalidValue;
	hipLaunchKernelGGL(kc_hist_kernel, dim3(grid), dim3(256), 0, st, table, slots, hist, n_bins, min_count);
	return hipGetLastError();
}

extern "C" hipError_t vc_launch_yak_select(const YakBloom *B, int grid, hipStream_t st)
{
	hipLaunchKernelGGL(yak_wanted_kernel, dim3(grid), dim3(256), 0, st, *B);
	hipLaunchKernelGGL(yak_mintime_kernel, dim3(grid), dim3(256), 0, st, *B);
	hipLaunchKernelGGL(yak_select_kernel, dim3(grid), dim3(256), 0, st, *B);
	return hipGetLastError();
}
