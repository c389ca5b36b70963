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
 * bits per key inside one word.  It runs once per k-mer, on the low 32 bits
 * of the two strands, flo = lo32(fwd) and rlo = lo32(revcomp), and uses only
 * functions symmetric in them, so it is a function of the canonical k-mer
 * without computing min(fwd, rc):
 *   word = bits [fsh, fsh + wbits) of lo24(flo) * lo24(rlo)   (v_mul_u32_u24)
 *   bits = 1 << (flo & 31), 1 << (rlo & 31)                   (v_lshlrev)
 * The bit positions are the newest and the (complemented) oldest bases of the
 * window.  The word comes from a product because any bitwise symmetric
 * combination (sum, xor, ...) of the two strands is constant at the bits of a
 * self-paired base (the centre of an odd k), which left a quarter of the
 * words empty; the product's middle bits mix all 48 input bits. */
VC_HD uint32_t vc_filter_shift(int k, uint32_t wbits)
{
	/* SNP panels hold ref/alt k-mer pairs that differ only in the centre base
	 * (bits k-1, k of flo and of rlo): keep it out of the word and the pair
	 * sets the same two bits, halving the filter's load.  The product's bits
	 * [lo, lo+wbits) depend on operand bits [0, lo+wbits) only; lo >= 5 keeps
	 * the word independent of the bit positions (operand bits 0..4). */
	if (k - 1 >= 24) return 32u - wbits;                     /* centre outside lo24 */
	if (k - 1 - (int)wbits >= 5) return 5u;                  /* centre above the word */
	/* otherwise: the top wbits of the product's 4k significant bits, skipping its skewed top 4 */
	const int top = 4 * k - 4 < 32 ? 4 * k - 4 : 32;
	return top > (int)wbits ? (uint32_t)(top - (int)wbits) : 0u;
}
VC_HD uint32_t vc_filter_mix(uint32_t flo, uint32_t rlo) { return (flo & 0xFFFFFFu) * (rlo & 0xFFFFFFu); }
VC_HD uint32_t vc_filter_word(uint32_t flo, uint32_t rlo, uint32_t fsh, uint32_t wbits)
{
	return (vc_filter_mix(flo, rlo) >> fsh) & ((1u << wbits) - 1u);
}
VC_HD uint32_t vc_filter_mask(uint32_t flo, uint32_t rlo) { return (1u << (flo & 31u)) | (1u << (rlo & 31u)); }

/* Flank bitmap (k >= 21, small panels): an exact 2^20-bit set S of 10-mers,
 * 128 KiB of LDS, holding four 10-mers of every key and of its reverse
 * complement: the ones ending at distances VC_FLANK_DIST(k, t), t = 0..3,
 * before the key's last base (t = 0: its last ten bases, t = 3: its first
 * ten, t = 1, 2: evenly between).  S is closed under reverse complement
 * (the distances are symmetric: d(t) + d(3 - t) = k - 10), so a window that
 * is a key in either orientation has all four of its forward 10-mers in S.
 * The kernel looks up the forward 10-mer ending at every base once and ANDs
 * the four bits of each window -- a necessary condition, 4 VALU per base
 * plus about 4 per 16 windows.  For k >= 21 the first and last 10-mers
 * exclude the centre base (the middle two do not; a SNP's ref and alt
 * k-mers then add separate middle entries).  A random window passes with
 * about the fourth power of S's density: on the GRCh38 panel (k = 21) 21 %
 * of S is set and 0.22 % of the benchmark's windows pass (1.6 % of which
 * are true hits), against 7.7 % and 0.59 % with the first and last 10-mers
 * alone (tools/flank_fp.py).
 * 10-mer v (20 bits, first base high, the k-mer encoding): byte v >> 3,
 * bit v & 7 (= word v >> 5, bit v & 31 on a little-endian word array). */
#define VC_FLANK_BASES 10
#define VC_FLANK_MIN_K 21
#define VC_FLANK_WBITS (2 * VC_FLANK_BASES - 5)  /* 2^15 words */
#define VC_FLANK_TESTS 4
#define VC_FLANK_DIST(k, t) (((t) * ((k) - VC_FLANK_BASES) + 1) / 3)
VC_HD void vc_flank_mark(uint32_t *bm, uint64_t kmer, int k)
{
	const uint32_t m = (1u << (2 * VC_FLANK_BASES)) - 1u;
	for (int t = 0; t < VC_FLANK_TESTS; ++t) {
		const uint32_t v = (uint32_t)(kmer >> (2 * VC_FLANK_DIST(k, t))) & m;
		bm[v >> 5] |= 1u << (v & 31u);
	}
}

/* Second-level filter for large key sets (> 2^16 keys, where the LDS
 * prefilter saturates): 2^l2bits 32-bit words in HBM, small enough to stay
 * L2/MALL-resident, three bits per key.  The queue drain checks it before
 * probing the exact table, whose random 16-byte slots would otherwise come
 * from HBM for every LDS false positive.  Word from vc_hash's top bits, bits
 * from an independent second hash of the canonical key. */
#define VC_L2F_MIN_KEYS 65536u
#define VC_L2F_MAX_BITS 19          /* 2 MiB */
VC_HD uint32_t vc_hash2(uint64_t key)
{
	return ((uint32_t)(key >> 17) ^ (uint32_t)key) * 0x9E3779B1u;
}
VC_HD uint32_t vc_l2f_mask(uint32_t h2)
{
	return (1u << (h2 & 31u)) | (1u << ((h2 >> 5) & 31u)) | (1u << ((h2 >> 10) & 31u));
}

/* The same filter keyed by the two strands' low 32 bits instead of the
 * canonical k-mer (the large-panel kernels, VC_KV_BIG; -DVC_BIG_RAWQ restores
 * the round-4 form for A/B): the queue holds (rlo << 32) | flo, which the drain
 * tests with two multiplies and no reverse complement; only survivors rebuild
 * the canonical k-mer (vc_canon_from_strands).  Symmetric in (flo, rlo), so it is a
 * function of the canonical k-mer.  Word from the top bits of one mix, bits
 * from a second one. */
#define VC_L2S_M 0x9E3779B1u
/* the two mixes of the strands' products u = flo * M, v = rlo * M */
VC_HD uint32_t vc_l2s_mix1(uint32_t u, uint32_t v)
{
	uint32_t x = u + v;
	x ^= x >> 15;
	return x * 0x85EBCA77u;
}
VC_HD uint32_t vc_l2s_mix2(uint32_t u, uint32_t v)
{
	uint32_t y = u ^ v;
	y ^= y >> 13;
	return y * 0xC2B2AE3Du;
}
VC_HD uint32_t vc_l2s_hash(uint32_t flo, uint32_t rlo) { return vc_l2s_mix1(flo * VC_L2S_M, rlo * VC_L2S_M); }
VC_HD uint32_t vc_l2s_hash2(uint32_t flo, uint32_t rlo) { return vc_l2s_mix2(flo * VC_L2S_M, rlo * VC_L2S_M); }

/* Large panels (a second-level filter in use) and k >= 21: a larger LDS
 * Bloom filter, VC_BIG_FILTER_WORDS 32-bit words (144 KiB: the queues shrink
 * to VC_BIG_QCAP entries per wave to make room), not a power of two.  Word
 * from the low 32 bits of the 40-bit product of the two strands' low 20 bits
 * (the last ten bases of the window and of its reverse complement: for
 * k >= 21 they exclude the centre base, so a SNP's ref and alt k-mers share
 * the word) scaled to the word count by a multiply-high; the same two bits as
 * the 32-bit-word filter.  On the 200k-SNP C5 panel the false-positive rate
 * drops from 11.4 % (128 KiB) to 9.3 % (tools/c5_filter_fp.py). */
#define VC_BIG_FILTER_WORDS 36860u
#define VC_BIG_QCAP 128u
VC_HD uint32_t vc_big_word(uint32_t flo, uint32_t rlo, uint32_t nwords)
{
	const uint32_t p = (flo & 0xFFFFFu) * (rlo & 0xFFFFFu);
	return (uint32_t)(((uint64_t)p * nwords) >> 32);
}

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
