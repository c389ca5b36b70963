/*
 * vafc_common.h -- definitions shared by the host table builder and the
 * device kernels.  The device never reproduces khashl's hash or bucket layout
 * (khashl.h:98,137-150, vaf-counter.c:56-67): only the key -> value mapping
 * must match, so the table and its prefilter use their own layout here.
 */
#ifndef VAFC_COMMON_H
#define VAFC_COMMON_H

#include <stdint.h>

#if defined(__HIPCC__)
#define VC_HD __host__ __device__ __forceinline__
#else
#define VC_HD static inline
#endif

/* An empty slot of the device key table.  Valid keys are < 4^31 < 2^62. */
#define VC_EMPTY_KEY 0xFFFFFFFFFFFFFFFFull

/* Reads longer than this go to the segmented long-read kernel. */
#define VC_LONG_READ 16384
/* Positions per segment of a long read (multiple of 16). */
#define VC_LONG_SEG 256

/* Largest LDS prefilter: 2^15 words = 128 KiB. */
#define VC_MAX_FILTER_WBITS 15

/* 32-bit mix of a canonical k-mer; all table and filter indices derive from
 * it.  Two multiplies on 32-bit halves (v_mul_lo_u32 on gfx950). */
VC_HD uint32_t vc_hash(uint64_t key)
{
	uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
	uint32_t x = lo ^ (hi * 0x9E3779B1u);
	x ^= x >> 16;
	return x * 0x85EBCA77u;
}

/* Reverse complement of a right-aligned 2-bit k-mer (vaf-counter.c:130-139). */
VC_HD uint64_t vc_revcomp(uint64_t x, int k)
{
	uint64_t r = 0;
	for (int i = 0; i < k; ++i, x >>= 2) r = (r << 2) | (3u - (x & 3u));
	return r;
}

/* Blocked Bloom prefilter in LDS: 2^wbits 32-bit words (wbits <= 15), two
 * bits per key inside one word.  Its hash runs once per k-mer, so it is one
 * add: fx = lo32(fwd) + lo32(revcomp), symmetric in the two strands and hence
 * a function of the canonical k-mer without computing min(fwd, rc) (the low
 * 32 bits of the two strands together cover every base of a k <= 32 k-mer).
 * Bits 0..4 pick the first bit, bits 5..19 the word, bits 20..24 the second. */
VC_HD uint32_t vc_filter_hash(uint64_t key, int k)
{
	return (uint32_t)key + (uint32_t)vc_revcomp(key, k);
}
/* Second symmetric hash (XOR instead of ADD) for extra filter bits. */
VC_HD uint32_t vc_filter_hash2(uint64_t key, int k)
{
	return (uint32_t)key ^ (uint32_t)vc_revcomp(key, k);
}
VC_HD uint32_t vc_filter_word(uint32_t fx, uint32_t wbits) { return (fx >> 5) & ((1u << wbits) - 1u); }
/* 32-bit-word filter: two bits. */
VC_HD uint32_t vc_filter_mask(uint32_t fx) { return (1u << (fx & 31u)) | (1u << ((fx >> 20) & 31u)); }
/* 64-bit-word filter (wbits <= 14): two bits in each half of the word. */
VC_HD uint32_t vc_filter_mask_lo(uint32_t fx) { return (1u << (fx & 31u)) | (1u << ((fx >> 19) & 31u)); }
VC_HD uint32_t vc_filter_mask_hi(uint32_t fx, uint32_t fy) { return (1u << ((fx >> 24) & 31u)) | (1u << (fy >> 27)); }

/* Filter layouts (vc_ctx chooses one). */
#define VC_FILTER_W32 32
#define VC_FILTER_W64 64

/* Device key table slot: 16 bytes, one load per probe step. */
typedef struct {
	uint64_t key;
	uint32_t val;
	uint32_t pad;
} vc_slot_t;

/* Home slot of a key in a table of 2^tbits slots (tbits in 1..32). */
VC_HD uint32_t vc_table_slot(uint32_t h, uint32_t tbits)
{
	return tbits >= 32u ? h : (h >> (32u - tbits));
}

#endif
