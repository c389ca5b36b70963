// vafc_kc.h -- argument block and launchers of the kc-c4 kernels
// (vafc_kc.hip), shared with the host library.  Not part of the C ABI.
#ifndef VAFC_KC_H
#define VAFC_KC_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define KC_THREADS 256
#define KC_LONG 4096          // reads longer than this are cut into segments
#define KC_SEG 1024           // bases per long-read segment (plus a k-1 halo)
#define KC_MAX_PROBE 1024     // a longer probe sequence marks the table full
#define KC_DROPPED (~0ull)    // count of a key yak's Bloom filter kept out of the table

struct KcArgs {
	const uint8_t *seq;
	const uint64_t *offs;
	const uint32_t *lens;
	uint64_t n_reads;
	unsigned long long *table;   // 2 * slots: key (hash64 + 1, 0 = empty), count
	uint64_t tmask;
	uint32_t tbits;
	uint32_t n_parts, part;      // count k-mers with ((hash64 & 1023) * n_parts) >> 10 == part
	uint64_t *first;             // yak two-file Bloom mode: first-occurrence stamp per slot, or null
	uint64_t read_base;          // stamp = (read_base + read index) << 32 | end position in the read
	int lookup_only;             // yak pass 2: count only keys already present and not dropped
	int k;
	uint64_t kmask;
	unsigned long long *stats;   // [0] k-mers seen, [1] distinct inserted, [2] overflow
	uint32_t *nlong;
	uint32_t *longlist;
	uint32_t long_cap;
	uint64_t *segstart;          // long_cap + 1
};

#ifdef __cplusplus
extern "C" {
#endif
hipError_t vc_launch_kc(const KcArgs *A, int grid, hipStream_t st);
hipError_t vc_launch_kc_hist(const unsigned long long *table, uint64_t slots, unsigned long long *hist,
                             uint32_t n_bins, uint64_t min_count, int grid, hipStream_t st);

// yak-count's Bloom filter (yak-count.c:71-108) replayed on the pass-1 table:
// geometry of the filter and the scratch table of the bits singletons use
struct YakBloom {
	const unsigned long long *table;   // 2 * slots
	unsigned long long *counts_out;    // = table: counts rewritten in place
	const uint64_t *first;
	uint64_t slots;
	uint32_t pre, ns, n_hash;          // ns = bf_shift - pre (bits per sub-table filter, log2)
	unsigned long long *wtab;          // 2 * wslots: bit id + 1, min first stamp
	uint64_t wslots;
	uint32_t wbits;
	unsigned long long *overflow;
};
hipError_t vc_launch_yak_select(const YakBloom *B, int grid, hipStream_t st);
#ifdef __cplusplus
}
#endif

#endif
