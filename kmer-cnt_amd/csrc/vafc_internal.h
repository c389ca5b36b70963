// vafc_internal.h -- kernel argument block and launchers shared by the host
// library (vafc_host.cpp) and the kernels (vafc_kernels.hip).  Not part of
// the public C ABI (include/vafc.h).
#ifndef VAFC_INTERNAL_H
#define VAFC_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "vafc_common.h"

#ifndef VC_BLOCK
#define VC_BLOCK 1024        // threads per block: 16 waves, one block per CU (-DVC_BLOCK=768 etc.: A/B)
#endif
#define VC_KV_FLANK 128      // kernel variant: flank-bitmap prefilter (vc_flank_*, k >= VC_FLANK_MIN_K)
#define VC_KV_BIG 512        // kernel variant: large-panel Bloom filter (vc_big_word, k >= VC_FLANK_MIN_K)
#define VC_QCAP 240          // per-wave LDS queue entries (u64): 16 waves x 1920 B + 128 KiB filter fit in 160 KiB

struct VcKernelArgs {
	const uint8_t *seq;          // 4-byte aligned base of the read bytes
	uint64_t seq_words;          // readable dwords from seq
	uint64_t off_adj;            // added to every offset (seq realignment)
	const uint64_t *offs;
	const uint32_t *lens;
	uint64_t n_reads;
	const vc_slot_t *table;      // exact table, 2^tbits slots, key VC_EMPTY_KEY = empty
	uint32_t tbits, tmask;
	const uint32_t *filter;      // 2^wbits 32-bit words
	uint32_t wbits;
	uint32_t fsh;                // filter word shift (vc_filter_shift)
	uint32_t flank;              // 1: the filter is the flank bitmap (vc_flank_*), not the Bloom filter
	uint32_t big;                // 1: the large-panel Bloom filter (vc_big_word, fwords words)
	uint32_t fwords;             // LDS filter words (2^wbits, or VC_BIG_FILTER_WORDS)
	uint32_t qcap;               // LDS queue entries per wave (VC_QCAP, or VC_BIG_QCAP)
	const uint32_t *l2f;         // second-level filter (vc_l2f_*), NULL = off
	uint32_t l2bits;
	int ablate;                  // ablation builds only (VAFC_ABLATE), 0 otherwise
	uint32_t variant;            // A/B experiment knobs (VAFC_VARIANT), 0 = the default kernel
	uint32_t nt4;                // 1: seq_nt4_table decode everywhere (snp-pattern-gen), 0: vaf-counter
	int k;
	uint64_t kmask;              // (1 << 2k) - 1
	uint32_t *counts;            // [2 * n_patterns]
	unsigned long long *tally;   // valid k-mers extracted
	uint32_t *nlong;             // long-read list fill (zeroed per launch)
	uint32_t *longlist;
	uint32_t long_cap;
	uint32_t *flags;             // bit 0: more long reads than long_cap (sticky until vc_reset)
};

// LDS: prefilter words + 4 zero words (16-byte aligned), then the per-wave queues.
__host__ __device__ static inline uint32_t vc_filter_lds_words(uint32_t fwords) { return fwords + 4u; }
static inline size_t vc_lds_bytes(uint32_t fwords, uint32_t qcap)
{
	return (size_t)4 * vc_filter_lds_words(fwords) + (size_t)(VC_BLOCK / 64) * qcap * 8;
}

#ifdef __cplusplus
extern "C" {
#endif
hipError_t vc_kernel_setup(void);
hipError_t vc_launch_count(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st);
hipError_t vc_launch_decode(const uint8_t *seq, uint64_t seq_bytes, const uint64_t *offs,
                            const uint32_t *lens, uint64_t n_reads, uint8_t *codes, hipStream_t st);
hipError_t vc_launch_synth(uint8_t *seq, uint64_t *offs, uint32_t *lens, uint64_t first,
                           uint64_t n_reads, uint32_t L, uint64_t seed, uint64_t thr,
                           const uint8_t *win, const uint8_t *dosage, uint32_t n_snp, hipStream_t st);
hipError_t vc_launch_shard_add(uint32_t *dst, uint32_t *src, uint64_t n, unsigned long long *dst_tally,
                               unsigned long long *src_tally, hipStream_t st);
#ifdef __cplusplus
}
#endif

#endif
