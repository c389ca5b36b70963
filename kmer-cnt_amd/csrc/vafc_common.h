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

/* Blocked Bloom prefilter with 2^wbits 32-bit words: the word is chosen by
 * the top wbits of the hash, two bits inside it by the next two 5-bit
 * fields.  wbits must be in 1..22. */
VC_HD uint32_t vc_filter_word(uint32_t h, uint32_t wbits) { return h >> (32u - wbits); }
VC_HD uint32_t vc_filter_mask(uint32_t h, uint32_t wbits)
{
	return (1u << ((h >> (27u - wbits)) & 31u)) | (1u << ((h >> (22u - wbits)) & 31u));
}

/* Home slot of a key in a table of 2^tbits slots (tbits in 1..32). */
VC_HD uint32_t vc_table_slot(uint32_t h, uint32_t tbits)
{
	return tbits >= 32u ? h : (h >> (32u - tbits));
}

#endif
