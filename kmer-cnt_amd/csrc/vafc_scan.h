// vafc_scan.h -- the counting kernels of the vaf-counter hot path, templated
// on the k-mer length K (K = 0: run-time k).  Each K in 16..31 is instantiated
// in one of the vafc_kernels_kNN.hip translation units (built in parallel);
// vafc_kernels.hip dispatches on k.  See the comment below for the design.
#ifndef VAFC_SCAN_H
#define VAFC_SCAN_H
// HIP kernels of the vaf-counter hot path for gfx950 (CDNA4).
//
// Replaces steps 1+2 of the reference pipeline: the SSSE3 2-bit encode
// (vaf-counter.c:261-291), the rolling canonical k-mer extraction
// (vaf-counter.c:349-427) and the khashl lookup + relaxed atomic increment
// (vaf-counter.c:449-479, khashl.h:137-150).  Integer work only, no MFMA.
//
// Design (DESIGN.md has the full story):
//  * One lane per read, one wave = 64 reads, 1024-thread persistent blocks
//    (one per CU, 16 waves/CU) grid-striding over groups of 1024 reads.
//  * Read bytes are fetched as dwords from the read's 4-byte-aligned start and
//    realigned with v_alignbyte; 16 bases (one "chunk") per loop trip, with
//    the next chunk's dwords in flight during the current one.
//  * Decode is SWAR on 4 bytes at a time with v_perm_b32 as a 8-entry LUT --
//    the same nibble table as the reference's PSHUFB; the reference decodes
//    the last len%16 bytes of a read with seq_nt4_table instead, so the lane
//    switches to an exact SWAR seq_nt4_table for that tail chunk.
//  * Rolling forward / reverse-complement k-mers in 64-bit registers; validity
//    from a 32-bit shift register of invalid-base flags (a window is valid iff
//    its last k flags are zero) -- equivalent to the reference's reset-on-N.
//  * Every valid canonical k-mer probes a blocked Bloom filter held in LDS
//    (2 bits in one 32-bit word, up to 128 KiB).  Filter hits are compacted
//    per wave into an LDS queue (ballot + mbcnt); a full queue is drained by
//    all 64 lanes probing the exact HBM/L2-resident table at once, and hits do
//    atomicAdd on uint32 counts[(pattern<<1)|is_alt].
//  * Reads longer than VC_LONG_READ are appended to a list and counted by a
//    second kernel in which every lane of the grid takes a VC_LONG_SEG-base
//    segment (plus a k-1 halo) of the read.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "vafc_common.h"
#include "vafc_internal.h"

#define WAVE 64

// Build-time A/B knobs (make XFLAGS=...; tools/ab_libs.sh): the round-2 forms
// of two parts of the flank kernels, kept for comparison.
#ifdef VC_FLANK_WORD
#define VC_FLANK_U8 0          // flank lookups: 32-bit words, per-base extraction
#else
#define VC_FLANK_U8 1          // flank lookups: bytes, two v_bfe_u32 of one register
#endif
#ifdef VC_DEFER_BIG
#define VC_KV_BIG_DEFER VC_KV_BIG   // large-panel kernels: one hit loop per chunk pair
#else
#define VC_KV_BIG_DEFER 0
#endif
#ifdef VC_SCAN_BWD
#define VC_SCAN_FB 1           // odd lanes scan backwards (scan_span_quad_fb; measured slower)
#else
#define VC_SCAN_FB 0           // every lane scans forwards (the quad loop)
#endif

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------

// Wave maximum of a small non-negative value (< 2048) from 11 ballots: no
// cross-lane data movement, so no LDS round trips.
__device__ __forceinline__ int wave_max_i32(int v)
{
	int m = 0;
#pragma unroll
	for (int b = 10; b >= 0; --b) {
		const int t = m | (1 << b);
		if (__ballot(v >= t)) m = t;
	}
	return m;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
	return v;
}

// Nibble LUT of the reference's PSHUFB decode (vaf-counter.c:272-275) for
// low nibbles 0..7, {4,0,4,1,3,3,4,2}; nibbles 8..15 are all 4 (invalid).
// v_perm_b32 selector bytes 0..3 pick bytes of the 2nd operand, 4..7 of the 1st.
#define NIB_LO 0x01040004u
#define NIB_HI 0x02040303u
// Expected high nibble (with the lower-case bit cleared) of an ACGTU letter
// for each low nibble 0..7; 0xFF never matches.
#define LET_LO 0x04FF04FFu
#define LET_HI 0x04FF0505u

// Head decode of 4 bytes: code byte = LUT[b & 15]; bit 2 set <=> invalid.
__device__ __forceinline__ uint32_t dec_head(uint32_t b)
{
	uint32_t t = __builtin_amdgcn_perm(NIB_HI, NIB_LO, b & 0x07070707u);
	return t | ((b >> 1) & 0x04040404u);
}

// The same without the byte-bit-3 term: codes, and bit 2 for the nibbles the
// LUT marks invalid.  The packed scan tests bit 3 of the raw bytes once per
// chunk instead of once per dword (dec_bit3) and folds it in only on the rare
// invalid-base path.
__device__ __forceinline__ uint32_t dec_code(uint32_t b)
{
	return __builtin_amdgcn_perm(NIB_HI, NIB_LO, b & 0x07070707u);
}
__device__ __forceinline__ uint32_t dec_bit3(uint32_t b) { return (b >> 1) & 0x04040404u; }

// Tail decode = seq_nt4_table (vaf-counter.c:73-90) on 4 bytes: ACGTU/acgtu
// keep their nibble code, bytes 0..3 map to themselves, all else invalid.
__device__ __forceinline__ uint32_t dec_tail(uint32_t b)
{
	uint32_t t = dec_head(b);
	uint32_t e = __builtin_amdgcn_perm(LET_HI, LET_LO, b & 0x07070707u);
	uint32_t m = ((b >> 4) & 0x0D0D0D0Du) ^ e;
	uint32_t nz = (((m & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | m) & 0x80808080u;  // byte != 0
	t |= nz >> 5;
	uint32_t y = b & 0xFCFCFCFCu;
	uint32_t small = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u; // byte < 4
	uint32_t sel = (small >> 7) * 0xFFu;
	return (t & ~sel) | (b & sel);
}

// Tail decode of 4 bytes from their head codes t = dec_code(b): the same
// result as dec_tail in 10 VALU instead of 17.  A byte is a valid letter iff
// (b & 0xDF) equals the upper-case ACGTU letter expected for its low three
// bits (EXP_*; 0xFF never matches, and a set bit 3 or bit 7 never matches);
// its code is then the head code.  Bytes 0..3 map to themselves (a rare
// branch).  tests/test_gpu_parity.py::test_tail_bytes_vs_oracle.
#define EXP_LO 0x43FF41FFu   // low bits 0..3: -, 'A', -, 'C'
#define EXP_HI 0x47FF5554u   // low bits 4..7: 'T', 'U', -, 'G'
__device__ __forceinline__ uint32_t dec_tail_from(uint32_t b, uint32_t t)
{
	const uint32_t e = __builtin_amdgcn_perm(EXP_HI, EXP_LO, b & 0x07070707u);
	const uint32_t d = (b & 0xDFDFDFDFu) ^ e;
	const uint32_t bad = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;   // byte is no letter
	t |= bad >> 5;
	const uint32_t big = (((b & 0x7C7C7C7Cu) + 0x7F7F7F7Fu) | b) & 0x80808080u;   // byte >= 4
	if (__ballot(big != 0x80808080u)) {
		if (big != 0x80808080u) {
			const uint32_t sel = ((~big & 0x80808080u) >> 7) * 0xFFu;
			t = (t & ~sel) | (b & sel);
		}
	}
	return t;
}

// The tail chunk of a read (cm == tail_c; tail_r = len & 15 bytes of it are
// the read's): t_m = dec_code(b_m) on entry, tail semantics for the dwords
// that hold tail bytes of some lane of the wave.  Dwords past every tail
// lane's last byte keep their head codes: they decode bytes past the read's
// end, whose windows are outside the read (masked by V) and whose invalid
// flags only move U for chunks that do not exist.
__device__ __forceinline__ void dec_tail_chunk(bool tl, int tail_r, uint32_t b0, uint32_t b1, uint32_t b2,
                                               uint32_t b3, uint32_t &t0, uint32_t &t1, uint32_t &t2, uint32_t &t3)
{
	if (__ballot(tl)) {
		if (tl) t0 = dec_tail_from(b0, t0);
		if (__ballot(tl && tail_r > 4)) {
			if (tl) t1 = dec_tail_from(b1, t1);
			if (__ballot(tl && tail_r > 8)) {
				if (tl) t2 = dec_tail_from(b2, t2);
				if (__ballot(tl && tail_r > 12)) {
					if (tl) t3 = dec_tail_from(b3, t3);
				}
			}
		}
	}
}

// Invalid-flag mask for the bytes of a word whose first position is P, given
// the valid position range [lo, hi): bytes outside get bit 2 set.
__device__ __forceinline__ uint32_t range_mask_hi(int rel_hi)
{
	// bytes i >= rel_hi are outside
	return rel_hi >= 4 ? 0u : (rel_hi <= 0 ? 0x04040404u : (0x04040404u << (8 * rel_hi)));
}
__device__ __forceinline__ uint32_t range_mask_lo(int rel_lo)
{
	// bytes i < rel_lo are outside
	return rel_lo <= 0 ? 0u : (rel_lo >= 4 ? 0x04040404u : (0x04040404u & ((1u << (8 * rel_lo)) - 1u)));
}

__device__ __forceinline__ uint32_t ldw(const uint32_t *__restrict__ s32, uint64_t i, uint64_t wmax)
{
	return s32[i < wmax ? i : wmax];
}

// Four consecutive dwords from a 4-byte-aligned index: one global_load_dwordx4
// when all four are inside the buffer, else four clamped dword loads (the
// last reads of a batch).  Loaded bytes past a read's end are masked later.
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
// The read stream's 16-byte loads.  -DVC_NT_READS (A/B): non-temporal loads,
// meant to keep the streamed reads from pushing the second-level filter out of
// the L2 -- but a lane's consecutive chunk loads share cache lines, which the
// non-temporal loads lose: C5 10.58 -> 12.19 ms, C2 4.91 -> 7.70 ms
// (profiles/r05v_ab.log, r05w_ab.log).
__device__ __forceinline__ u32x4a4 ld16(const uint32_t *__restrict__ p)
{
#ifdef VC_NT_READS
	return __builtin_nontemporal_load(reinterpret_cast<const u32x4a4 *>(p));
#else
	return *reinterpret_cast<const u32x4a4 *>(p);
#endif
}
__device__ __forceinline__ void ld4(const uint32_t *__restrict__ s32, uint64_t i, uint64_t wmax,
                                    uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	if (i + 3 <= wmax) {
		const u32x4a4 v = ld16(s32 + i);
		a = v.x; b = v.y; c = v.z; d = v.w;
	} else {
		a = ldw(s32, i, wmax); b = ldw(s32, i + 1, wmax); c = ldw(s32, i + 2, wmax); d = ldw(s32, i + 3, wmax);
	}
}

// LDS word at byte offset (x & m) from an LDS base whose low bits are clear:
// one v_and_or_b32 forms the address (base | offset), which the compiler
// would otherwise add with a separate v_add (the base is a link-time symbol).
typedef const uint32_t __attribute__((address_space(3))) lds_u32_t;
__device__ __forceinline__ uint32_t lds_base(const uint32_t *p)
{
	return (uint32_t)(uintptr_t)(lds_u32_t *)p;
}
__device__ __forceinline__ uint32_t lds_word(uint32_t base, uint32_t x, uint32_t m)
{
	return *(lds_u32_t *)(uintptr_t)((x & m) | base);
}

// ---------------------------------------------------------------------------
// exact table probe (drain side)
// ---------------------------------------------------------------------------

// Reverse complement of a right-aligned k-mer with bit tricks (drain side only).
__device__ __forceinline__ uint64_t revcomp_dev(uint64_t x, int k)
{
	const uint32_t lo = __builtin_bitreverse32((uint32_t)x), hi = __builtin_bitreverse32((uint32_t)(x >> 32));
	uint64_t r = ((uint64_t)lo << 32) | hi;                                  // bit-reversed
	r = ((r >> 1) & 0x5555555555555555ull) | ((r & 0x5555555555555555ull) << 1); // restore 2-bit order
	return (~r) >> (64 - 2 * k);
}

// Ablation bits of the drain (VC_ABLATION builds only, with ABL 1/2/4 above;
// results are wrong by design): 1024 = queued entries are dropped, never
// drained; 2048 = the drain computes every entry's second-level word and
// mask but issues no gather and probes nothing; 4096 = the second-level
// gather runs, survivors are not probed in the exact table.
#define VC_ABL_NODRAIN 1024
#define VC_ABL_NOGATHER 2048
#define VC_ABL_NOPROBE 4096

// key: the raw forward k-mer (bits above 2k may hold older bases).
__device__ __forceinline__ void probe_and_count(const VcKernelArgs &A, uint64_t fwd_raw)
{
	const uint64_t f = fwd_raw & A.kmask;
	const uint64_t r = revcomp_dev(f, A.k);
	const uint64_t key = f < r ? f : r;
	uint32_t s = vc_table_slot(vc_hash(key), A.tbits);
	for (;;) {
		const uint4 e = *reinterpret_cast<const uint4 *>(&A.table[s]);
		const uint64_t k2 = ((uint64_t)e.y << 32) | e.x;
		if (k2 == key) {
			atomicAdd(&A.counts[e.z], 1u);
			break;
		}
		if (k2 == VC_EMPTY_KEY) break;
		s = (s + 1u) & A.tmask;
	}
}

struct WaveQueue {
	uint64_t *q;     // LDS, A.qcap entries
	uint32_t n;      // wave-uniform fill
	// drain_pipe (large-panel kernels): the previous near-full drain's
	// entries, one per lane, whose second-level words are still in flight
	uint64_t pe[2];     // the entries (VC_PIPE_ROUNDS of them per lane)
	uint32_t pm[2], pw[2];  // their filter masks and filter words (empty: pm = 1, pw = 0)
	bool pend;          // wave-uniform: pe / pm / pw hold a drain
};

// Probe the exact table for queue entries [lo, hi) (up to 4 per lane); the
// first table load of every entry is issued before any is resolved, so one
// memory latency covers the whole drain.
// Large key sets: every entry is first checked against the second-level
// filter (one L2-resident dword), and only survivors probe the exact table.
template <int ABL>
__device__ __forceinline__ void probe_key(const VcKernelArgs &A, uint64_t key, uint32_t h)
{
	if constexpr ((ABL & VC_ABL_NOPROBE) != 0) {
		asm volatile("" :: "v"(h), "v"(key));
		return;
	}
	uint32_t t = vc_table_slot(h, A.tbits);
	for (;;) {
		const uint4 e = *reinterpret_cast<const uint4 *>(&A.table[t]);
		const uint64_t k2 = ((uint64_t)e.y << 32) | e.x;
		if (k2 == key) {
			atomicAdd(&A.counts[e.z], 1u);
			break;
		}
		if (k2 == VC_EMPTY_KEY) break;
		t = (t + 1u) & A.tmask;
	}
}

template <int ABL>
__device__ __forceinline__ void drain_range_l2f(const VcKernelArgs &A, const uint64_t *q, uint32_t lo,
                                             uint32_t hi, int lane)
{
	uint64_t key[4];
	uint32_t h[4], w[4], m[4];
	const uint32_t l2sh = 32u - A.l2bits;
#pragma unroll
	for (int r = 0; r < 4; ++r) {
		const uint32_t i = lo + (uint32_t)(r * WAVE + lane);
		key[r] = VC_EMPTY_KEY;
		h[r] = 0;
		w[r] = 0;
		m[r] = 1;
		if (i < hi) {
			const uint64_t f = q[i] & A.kmask;
			const uint64_t rc = revcomp_dev(f, A.k);
			key[r] = f < rc ? f : rc;
			h[r] = vc_hash(key[r]);
			m[r] = vc_l2f_mask(vc_hash2(key[r]));
			if constexpr ((ABL & VC_ABL_NOGATHER) != 0) asm volatile("" :: "v"(h[r] >> l2sh), "v"(m[r]));
			else w[r] = A.l2f[h[r] >> l2sh];
		}
	}
	if constexpr ((ABL & VC_ABL_NOGATHER) != 0) return;
#pragma unroll
	for (int r = 0; r < 4; ++r) {
		if ((w[r] & m[r]) != m[r]) continue;      // also skips empty entries (w = 0, m = 1)
		probe_key<ABL>(A, key[r], h[r]);
	}
}

// Canonical k-mer of a window from its two strands' low 32 bits (K >= 16:
// the first sixteen bases, complemented, are rlo; the last sixteen are flo):
// forward = rc16(rlo) << 2(K - 16) | flo, reverse = rc16(flo) << 2(K - 16) | rlo.
__device__ __forceinline__ uint32_t rc16(uint32_t x)
{
	x = __builtin_bitreverse32(x);
	// swap the bits of each pair and complement: ~(M ? x >> 1 : x << 1),
	// M = 0x55555555, in one v_bitop3 (table 0x1B); the compiler's own form
	// spent a v_and on x << 1 first
	return __builtin_amdgcn_bitop3_b32(x >> 1, x << 1, 0x55555555u, 0x1B);
}
__device__ __forceinline__ uint64_t vc_canon_from_strands(uint32_t flo, uint32_t rlo, int k)
{
	const uint32_t sh = 2u * (uint32_t)(k - 16);
	const uint64_t f = ((uint64_t)rc16(rlo) << sh) | flo;
	const uint64_t r = ((uint64_t)rc16(flo) << sh) | rlo;
	return f < r ? f : r;
}

#ifdef VC_BIG_RAWQ   // A/B: the large-panel kernels queue forward k-mers like the others (round 4)
#define VC_SYMQ(ABL) false
#else
#define VC_SYMQ(ABL) (((ABL) & VC_KV_BIG) != 0)
#endif
// The hit loops queue the forward k-mer's high word unmasked (bits above 2k
// hold older bases): every drain masks the entry with A.kmask, and the
// large-panel drain reads only bits below 2k (the low word and bits
// 2(k - 16) .. 2k of the entry).  -DVC_HIT_MASK (A/B) masks it in the loop.
#ifdef VC_HIT_MASK
#define VC_HIT_HIM HIM
#else
#define VC_HIT_HIM (HIM | ~0u)
#endif
#ifdef VC_BIG_DRAIN_ALL
#define VC_DRAIN_ALL 1
#else
#define VC_DRAIN_ALL 0
#endif
#ifdef VC_NO_DEFER_PROBE   // A/B: near-full drains probe their survivors at once (round 4)
#define VC_DEFER_PROBE 0
#else
#define VC_DEFER_PROBE 1
#endif

// Large-panel kernels (VC_SYMQ): the second-level filter is keyed by the two
// strands' low words (vc_l2s_*).  The queue holds the forward k-mer as every
// kernel queues it; the drain takes flo = its low word and rlo = the reverse
// complement of its first sixteen bases (one v_alignbit at a run-time shift
// and a 16-base reverse complement), with no 64-bit reverse complement,
// canonical minimum or 64-bit hash; only survivors rebuild the canonical
// k-mer (vc_canon_from_strands) and hash it for the exact table.
// A near-full drain (KEEP) does not probe its survivors: it writes them back
// at the bottom of the drained range and returns how many, so that they wait
// in the queue for the read group's final drain, where one probe latency
// covers them all, instead of costing this drain a dependent table load.
// When more survive than `room` entries (a read set dense in keys), they are
// probed at once.  The final drain (KEEP = false) probes every survivor.
template <int ABL, bool KEEP>
__device__ __forceinline__ uint32_t drain_range_sym(const VcKernelArgs &A, uint64_t *q, uint32_t lo,
                                                    uint32_t hi, int lane, uint32_t room)
{
	// rounds of WAVE entries: a near-full drain takes exactly the queue's top
	// WAVE entries (queue_append), the final drain at most VC_BIG_QCAP (the
	// large-panel queues), so no round is spent on lanes known to be empty
	constexpr int NR = (KEEP && !VC_DRAIN_ALL) ? 1 : (int)(VC_BIG_QCAP / WAVE);
	constexpr bool FULL = KEEP && !VC_DRAIN_ALL;   // every lane holds an entry
	static_assert(NR >= 1 && NR <= 4, "drain rounds");
	uint32_t fl[4], rl[4], w[4], m[4];
	uint64_t e64[4];
	const uint32_t l2sh = 32u - A.l2bits;
	const uint32_t fsh16 = 2u * (uint32_t)(A.k - 16);   // the window's first sixteen bases
#pragma unroll
	for (int r = 0; r < NR; ++r) {
		const uint32_t i = lo + (uint32_t)(r * WAVE + lane);
		fl[r] = rl[r] = 0;
		w[r] = 0;
		m[r] = 1;
		if (FULL || i < hi) {
			const uint64_t e = q[i];
			e64[r] = e;
			fl[r] = (uint32_t)e;
			rl[r] = rc16(__builtin_amdgcn_alignbit((uint32_t)(e >> 32), (uint32_t)e, fsh16));
			// vc_l2s_hash / vc_l2s_hash2 sharing the strands' two products
			// (the empty asm keeps the compiler from rewriting u + v as
			// (flo + rlo) * M and multiplying again for u ^ v)
			uint32_t u = fl[r] * VC_L2S_M, v = rl[r] * VC_L2S_M;
			asm("" : "+v"(u), "+v"(v));
			const uint32_t hw = vc_l2s_mix1(u, v);
			m[r] = vc_l2f_mask(vc_l2s_mix2(u, v));
			if constexpr ((ABL & VC_ABL_NOGATHER) != 0) asm volatile("" :: "v"(hw >> l2sh), "v"(m[r]));
			else w[r] = A.l2f[hw >> l2sh];
		}
	}
	if constexpr ((ABL & VC_ABL_NOGATHER) != 0) return 0;
	bool surv[4];
#pragma unroll
	for (int r = 0; r < NR; ++r) surv[r] = (w[r] & m[r]) == m[r];   // false for empty entries (w = 0, m = 1)
	if constexpr (KEEP && VC_DEFER_PROBE) {
		uint64_t bal[4];
		uint32_t n = 0;
#pragma unroll
		for (int r = 0; r < NR; ++r) {
			bal[r] = __ballot(surv[r]);
			n += (uint32_t)__popcll(bal[r]);
		}
		if (n == 0) return 0;
		if (n <= room) {
			uint32_t at = lo;
#pragma unroll
			for (int r = 0; r < NR; ++r) {
				const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32),
				                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0u));
				if (surv[r]) q[at + pre] = e64[r];
				at += (uint32_t)__popcll(bal[r]);
			}
			return n;
		}
	}
#pragma unroll
	for (int r = 0; r < NR; ++r) {
		if (!surv[r]) continue;
		const uint64_t key = vc_canon_from_strands(fl[r], rl[r], A.k);
		probe_key<ABL>(A, key, vc_hash(key));
	}
	return 0;
}

// Drain queue entries [lo, hi).  KEEP (near-full drains of the large-panel
// kernels): survivors of the second-level filter may be kept at q[lo ..
// lo + returned) for a later drain, at most `room` of them; otherwise every
// entry is resolved and 0 is returned.
template <int ABL, bool KEEP = false>
__device__ __forceinline__ uint32_t drain_range(const VcKernelArgs &A, uint64_t *q, uint32_t lo,
                                                uint32_t hi, int lane, uint32_t room = 0)
{
	__builtin_amdgcn_wave_barrier();
	if constexpr ((ABL & VC_ABL_NODRAIN) != 0) {
		asm volatile("" :: "v"(q[lo + (uint32_t)lane]));
		return 0;
	}
	if constexpr (VC_SYMQ(ABL)) {
		return drain_range_sym<ABL, KEEP>(A, q, lo, hi, lane, room);
	}
	if (A.l2bits) {
		drain_range_l2f<ABL>(A, q, lo, hi, lane);
		return 0;
	}
	uint64_t key[4];
	uint32_t s[4];
	uint4 e[4];
#pragma unroll
	for (int r = 0; r < 4; ++r) {
		const uint32_t i = lo + (uint32_t)(r * WAVE + lane);
		key[r] = VC_EMPTY_KEY;
		s[r] = 0;
		if (i < hi) {
			const uint64_t f = q[i] & A.kmask;
			const uint64_t rc = revcomp_dev(f, A.k);
			key[r] = f < rc ? f : rc;
			s[r] = vc_table_slot(vc_hash(key[r]), A.tbits);
			e[r] = *reinterpret_cast<const uint4 *>(&A.table[s[r]]);
		}
	}
#pragma unroll
	for (int r = 0; r < 4; ++r) {
		if (key[r] == VC_EMPTY_KEY) continue;
		uint4 x = e[r];
		uint32_t t = s[r];
		for (;;) {
			const uint64_t k2 = ((uint64_t)x.y << 32) | x.x;
			if (k2 == key[r]) {
				atomicAdd(&A.counts[x.z], 1u);
				break;
			}
			if (k2 == VC_EMPTY_KEY) break;
			t = (t + 1u) & A.tmask;
			x = *reinterpret_cast<const uint4 *>(&A.table[t]);
		}
	}
	return 0;
}

// Large-panel kernels: a near-full drain takes the queue's top WAVE entries
// into registers (one per lane), hashes them and issues their second-level
// gathers, but tests them only at the NEXT near-full drain (or the final
// one), so the gathers' latency runs under the scan instead of stalling the
// wave.  The previous drain's survivors go back into the queue where room
// allows (as KEEP does), else they are probed at once.  Returns the new
// fill.  C5 10.43-10.45 -> 10.35-10.37 ms (profiles/r05pp_ab.log);
// -DVC_NO_PIPE_DRAIN restores drain_range<KEEP> for them.
#ifndef VC_NO_PIPE_DRAIN
#define VC_PIPE(ABL) (VC_SYMQ(ABL) && !VC_DRAIN_ALL && ((ABL) & (VC_ABL_NODRAIN | VC_ABL_NOGATHER)) == 0)
#else
#define VC_PIPE(ABL) false
#endif
template <int ABL>
__device__ __forceinline__ void pipe_probe(const VcKernelArgs &A, uint64_t e)
{
	const uint32_t fl = (uint32_t)e;
	const uint32_t rl = rc16(__builtin_amdgcn_alignbit((uint32_t)(e >> 32), fl, 2u * (uint32_t)(A.k - 16)));
	const uint64_t key = vc_canon_from_strands(fl, rl, A.k);
	probe_key<ABL>(A, key, vc_hash(key));
}
// VC_PIPE_ROUNDS = 2 (A/B): the drain takes the whole queue (65..128
// entries, two per lane) instead of its top 64: 10.72 against 10.35 ms
// (profiles/r05p2_ab.log), not the default.
#ifndef VC_PIPE_ROUNDS
#define VC_PIPE_ROUNDS 1
#endif
template <int ABL>
__device__ __forceinline__ uint32_t drain_pipe(const VcKernelArgs &A, WaveQueue &Q, int lane)
{
	constexpr int PR = VC_PIPE_ROUNDS;
	static_assert(PR == 1 || PR == 2, "pipe rounds");
	__builtin_amdgcn_wave_barrier();
	const uint32_t lo = PR == 1 ? Q.n - WAVE : 0u;   // PR = 2: Q.n > WAVE, so round 0 is full
	uint64_t e[PR];
	uint32_t m[PR], w[PR];
#pragma unroll
	for (int r = 0; r < PR; ++r) {
		const uint32_t i = lo + (uint32_t)(r * WAVE + lane);
		e[r] = 0;
		m[r] = 1;
		w[r] = 0;
		if (r == 0 || i < Q.n) {
			e[r] = Q.q[i];
			const uint32_t fl = (uint32_t)e[r];
			const uint32_t rl = rc16(__builtin_amdgcn_alignbit((uint32_t)(e[r] >> 32), fl, 2u * (uint32_t)(A.k - 16)));
			uint32_t u = fl * VC_L2S_M, v = rl * VC_L2S_M;
			asm("" : "+v"(u), "+v"(v));
			m[r] = vc_l2f_mask(vc_l2s_mix2(u, v));
			w[r] = A.l2f[vc_l2s_mix1(u, v) >> (32u - A.l2bits)];   // not awaited here
		}
	}
	uint32_t n = 0;
	if (Q.pend) {
		bool surv[PR];
		uint64_t bal[PR];
#pragma unroll
		for (int r = 0; r < PR; ++r) {
			surv[r] = (Q.pw[r] & Q.pm[r]) == Q.pm[r];   // false for empty slots (pw = 0, pm = 1)
			bal[r] = __ballot(surv[r]);
			n += (uint32_t)__popcll(bal[r]);
		}
		if (n) {
			if (n <= A.qcap - WAVE - lo) {
				uint32_t at = lo;
#pragma unroll
				for (int r = 0; r < PR; ++r) {
					const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32),
					                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0u));
					if (surv[r]) Q.q[at + pre] = Q.pe[r];
					at += (uint32_t)__popcll(bal[r]);
				}
			} else {
#pragma unroll
				for (int r = 0; r < PR; ++r)
					if (surv[r]) pipe_probe<ABL>(A, Q.pe[r]);
				n = 0;
			}
		}
	}
#pragma unroll
	for (int r = 0; r < PR; ++r) {
		Q.pe[r] = e[r];
		Q.pm[r] = m[r];
		Q.pw[r] = w[r];
	}
	Q.pend = true;
	return lo + n;
}

// Lanes with `hit` append `key` (bal = ballot(hit) != 0).  The queue is
// normally drained once per read group (queue_flush); only a nearly full
// queue is drained here, 64 entries from its top.
template <int ABL>
__device__ __forceinline__ void queue_append(const VcKernelArgs &A, WaveQueue &Q, uint64_t bal,
                                             bool hit, uint64_t key, int lane)
{
	const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
	                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
	if (hit) Q.q[Q.n + pre] = key;
	Q.n = __builtin_amdgcn_readfirstlane(Q.n + (uint32_t)__popcll(bal));
	if (Q.n > A.qcap - WAVE) {        // A.qcap >= 2 WAVE
		if constexpr (VC_PIPE(ABL)) {
			Q.n = drain_pipe<ABL>(A, Q, lane);
		} else {
			// kept survivors must leave room for one more full append (<= WAVE);
			// VC_BIG_DRAIN_ALL (A/B): the large-panel kernels drain the whole queue
			const uint32_t lo = (VC_SYMQ(ABL) && VC_DRAIN_ALL) ? 0u : Q.n - WAVE;
			Q.n = lo + drain_range<ABL, true>(A, Q.q, lo, Q.n, lane, A.qcap - WAVE - lo);
			// leave nothing in flight on this (rare) path, so that the compiler
			// can keep counting the scan's prefetches across it
			__builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
		}
	}
}

template <int ABL>
__device__ __forceinline__ void queue_flush(const VcKernelArgs &A, WaveQueue &Q, int lane)
{
	if constexpr (VC_PIPE(ABL)) {
		// the pending drain's survivors join the final drain where they fit
		if (Q.pend) {
#pragma unroll
			for (int r = 0; r < VC_PIPE_ROUNDS; ++r) {
				const bool surv = (Q.pw[r] & Q.pm[r]) == Q.pm[r];
				const uint64_t bal = __ballot(surv);
				if (bal) {
					const uint32_t n = (uint32_t)__popcll(bal);
					if (Q.n + n <= A.qcap) {
						const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
						                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
						if (surv) Q.q[Q.n + pre] = Q.pe[r];
						Q.n += n;
					} else if (surv) {
						pipe_probe<ABL>(A, Q.pe[r]);
					}
				}
			}
			Q.pend = false;
		}
	}
	if (Q.n) drain_range<ABL>(A, Q.q, 0, Q.n, lane);
	Q.n = 0;
}

// ---------------------------------------------------------------------------
// rolling forward / reverse-complement k-mers (vaf-counter.c:368-394)
// ---------------------------------------------------------------------------
//
// K > 0: compile-time k, k-mers held as 32-bit halves and rolled with
// v_alignbit / v_lshl_or; K == 0: run-time k on 64-bit values.  Instead of
// resetting on an invalid base (the reference's `l = 0; x = 0`), a 32-bit
// register of invalid flags is shifted right with v_alignbit (newest flag in
// bit 31): the window is valid iff its top k bits are zero, i.e. the register
// is below 2^(32-k).  fwd/rev hold exactly the last k codes once it is.
template <int K>
struct Roller {
	uint32_t flo, fhi, rlo, rhi, inv;
	uint32_t vthr;        // valid <=> inv < vthr
	uint64_t kmask;
	uint32_t rsh;

	__device__ __forceinline__ void init(const VcKernelArgs &A)
	{
		flo = fhi = rlo = rhi = 0;
		inv = 0xFFFFFFFFu;
		const int k = K ? K : A.k;
		vthr = 1u << (32 - k);
		kmask = A.kmask;
		rsh = 2u * (uint32_t)(k - 1);
	}
	// c: 2-bit code, bad: bit 0 = invalid flag (higher bits ignored)
	__device__ __forceinline__ void push(uint32_t c, uint32_t bad)
	{
		const uint32_t cc = c ^ 3u;
		if constexpr (K >= 17) {
			constexpr uint32_t HIM = (1u << (2 * K - 32)) - 1u;
			fhi = __builtin_amdgcn_alignbit(fhi, flo, 30) & HIM;
			flo = (flo << 2) | c;
			rlo = __builtin_amdgcn_alignbit(rhi, rlo, 2);
			rhi = (rhi >> 2) | (cc << (2 * K - 34));
		} else if constexpr (K > 0) {
			constexpr uint32_t M = K == 16 ? 0xFFFFFFFFu : ((1u << (2 * K)) - 1u);
			flo = ((flo << 2) | c) & M;
			rlo = (rlo >> 2) | (cc << (2 * K - 2));
		} else {
			uint64_t f = ((((uint64_t)fhi << 32) | flo) << 2 | c) & kmask;
			uint64_t r = ((((uint64_t)rhi << 32) | rlo) >> 2) | ((uint64_t)cc << rsh);
			flo = (uint32_t)f; fhi = (uint32_t)(f >> 32);
			rlo = (uint32_t)r; rhi = (uint32_t)(r >> 32);
		}
		inv = __builtin_amdgcn_alignbit(bad, inv, 1);
	}
	__device__ __forceinline__ bool valid() const { return inv < vthr; }
};

__device__ __forceinline__ uint64_t canonical_of(uint32_t flo, uint32_t fhi, uint32_t rlo, uint32_t rhi)
{
	const uint64_t f = ((uint64_t)fhi << 32) | flo, r = ((uint64_t)rhi << 32) | rlo;
	return f < r ? f : r;
}

// ---------------------------------------------------------------------------
// scan one span of one read per lane, wave-uniform trip count
// ---------------------------------------------------------------------------
//
// Lane processes chunks [c_lo, c_hi) of its read (chunk c = read positions
// 16c..16c+15), emitting the canonical k-mers whose whole window lies in the
// valid position range [vlo, vhi) (vlo = 0, vhi = len for a whole read).
// The lane's count of valid k-mers accumulates in `tl`.
// ABL (ablation builds only, -DVC_ABLATION; results are wrong by design):
//   1 = no LDS filter reads, 2 = no global read-byte loads, 4 = no queue appends
template <int K, bool HAS_LO, int ABL = 0>
__device__ __forceinline__ void scan_span(const VcKernelArgs &A, const uint32_t *__restrict__ s32,
                                          uint64_t wmax, uint64_t off, int len, int c_lo, int c_hi,
                                          int vlo, int vhi, int nit, const uint32_t *__restrict__ filt,
                                          WaveQueue &Q, uint32_t &tl, int lane)
{
	const uint32_t fsh = A.fsh;
	const uint32_t zero_word = A.fwords;        // an all-zero LDS word past the filter
	// the read's tail chunk decodes with seq_nt4_table (vaf-counter.c:261-291);
	// in seq_nt4 mode (snp-pattern-gen) every chunk does: tail_c = -1 and the
	// test (c | -1) == -1 always holds (the OR is scalar in the reads kernel)
	const int tail_c = A.nt4 ? -1 : ((len & 15) ? (len >> 4) : -1);
	const int nt4m = -(int)A.nt4;   // 0 or -1 (the host stores 0 / 1); kept arithmetic so
	                                  // the test stays one compare, not (c == tail_c) || nt4

	uint64_t addr = off + 16ull * (uint64_t)c_lo;
	uint64_t wi = addr >> 2;
	const uint32_t sh = (uint32_t)(addr & 3u);
	uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0;
	uint32_t x1 = 0, x2 = 0, x3 = 0, x4 = 0;
	if (c_lo < c_hi) {
		ld4(s32, wi, wmax, w0, w1, w2, w3);
		w4 = ldw(s32, wi + 4, wmax);
	}
	if (c_lo + 1 < c_hi) ld4(s32, wi + 5, wmax, x1, x2, x3, x4);
	Roller<K> R;
	R.init(A);

	for (int it = 0; it < nit; ++it) {
		const int c = c_lo + it;
		// the dwords of the next two chunks are in flight while this one is processed
		uint32_t y1 = 0, y2 = 0, y3 = 0, y4 = 0;
		if (c + 2 < c_hi) {
			if constexpr ((ABL & 2) != 0) {
				y1 = (uint32_t)wi * 0x9E3779B1u; y2 = y1 ^ 0x41434754u; y3 = y1 + 0x54474341u; y4 = y1 * 5u;
			} else {
				ld4(s32, wi + 9, wmax, y1, y2, y3, y4);
			}
		}
		const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
		const uint32_t b1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
		const uint32_t b2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
		const uint32_t b3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
		uint32_t t0 = dec_head(b0), t1 = dec_head(b1), t2 = dec_head(b2), t3 = dec_head(b3);
		const int cm = c | nt4m;
		if (__ballot(cm == tail_c)) {
			if (cm == tail_c) { t0 = dec_tail(b0); t1 = dec_tail(b1); t2 = dec_tail(b2); t3 = dec_tail(b3); }
		}
		const int P = 16 * c;
		if (__ballot(P + 16 > vhi)) {   // past the span end (and inactive lanes: P >= vhi)
			t0 |= range_mask_hi(vhi - P);
			t1 |= range_mask_hi(vhi - P - 4);
			t2 |= range_mask_hi(vhi - P - 8);
			t3 |= range_mask_hi(vhi - P - 12);
		}
		if (HAS_LO) {
			if (__ballot(P < vlo)) {
				t0 |= range_mask_lo(vlo - P);
				t1 |= range_mask_lo(vlo - P - 4);
				t2 |= range_mask_lo(vlo - P - 8);
				t3 |= range_mask_lo(vlo - P - 12);
			}
		}

#pragma unroll
		for (int half = 0; half < 2; ++half) {
			const uint32_t ta = half ? t2 : t0, tb = half ? t3 : t1;
			uint32_t fl[8], fh[8], fw[8], fm[8];
#pragma unroll
			for (int j = 0; j < 8; ++j) {
				const uint32_t tw = j < 4 ? ta : tb;
				const uint32_t x = tw >> (8 * (j & 3));
				R.push(x & 3u, x >> 2);
				const bool valid = R.valid();
				tl += valid ? 1u : 0u;
				const uint32_t widx = valid ? vc_filter_word(R.flo, R.rlo, fsh, A.wbits) : zero_word;
				if constexpr ((ABL & 1) != 0) { asm volatile("" :: "v"(widx)); fw[j] = 0u; }
				else fw[j] = filt[widx];
				fm[j] = vc_filter_mask(R.flo, R.rlo);
				fl[j] = R.flo; fh[j] = R.fhi;
			}
#pragma unroll
			for (int j = 0; j < 8; ++j) {
				const bool hit = (fw[j] & fm[j]) == fm[j];
				const uint64_t bal = __ballot(hit);
				if constexpr ((ABL & 4) != 0) { asm volatile("" :: "s"(bal)); }
				else if (bal) queue_append<ABL>(A, Q, bal, hit, ((uint64_t)fh[j] << 32) | fl[j], lane);
			}
		}
		w0 = w4; w1 = x1; w2 = x2; w3 = x3; w4 = x4;
		x1 = y1; x2 = y2; x3 = y3; x4 = y4;
		wi += 4;
	}
}

// ---------------------------------------------------------------------------
// packed-stream scan for compile-time k in 16..31 (the hot path)
// ---------------------------------------------------------------------------
//
// Each 16-base chunk is packed once into 2-bit streams:
//   L  little-endian codes, base j at bits 2j           (complemented: C = ~L)
//   B  big-endian codes,    base j at bits 2(15-j)      (pair-reversed L)
// The forward k-mer's low 32 bits at base j are one v_alignbit of (B[c-1]:B[c])
// and the reverse complement's low 32 bits one v_alignbit of the C stream, with
// compile-time shifts; the prefilter needs nothing else.  Filter passes set
// bits of a per-lane 16-bit mask hm (bit 15-j <-> window ending at base j).
//
// Window validity is not tracked per base: per chunk, V (same bit order as
// hm) holds the windows that lie inside [vlo, vhi) and contain no invalid
// base; hm &= V.  Windows ending at base j are valid iff j >= L + K - 16c
// (L = last invalid position before the chunk, vlo - 1 at the start) and
// 16c + j < vhi; U = 16 - (L + K - 16c) and Qe = 16 - (vhi - 16c) are carried
// per lane.  A chunk with an invalid base of its own (an N; rare) also
// invalidates its windows from the first such base on and moves L to the last.
// Only at the end of a chunk, and only if some lane of the wave has a hit,
// are the full forward k-mers of the hit positions extracted (variable
// shift) and queued.

// 4x4 transpose of 2-bit fields: (byte r, field c) <-> (byte c, field r).
__device__ __forceinline__ uint32_t transpose2x4x4(uint32_t a)
{
	uint32_t t = ((a >> 6) ^ a) & 0x00CC00CCu;
	a ^= t ^ (t << 6);
	t = ((a >> 12) ^ a) & 0x0000F0F0u;
	a ^= t ^ (t << 12);
	return a;
}

// Reverse the order of the 16 2-bit fields of a word.
__device__ __forceinline__ uint32_t pairrev(uint32_t x)
{
	x = __builtin_bitreverse32(x);
	return ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
}

// The 2-bit codes of a chunk's 16 bases from its four decoded dwords, base j
// at bits 2j.  One multiply gathers a dword's four codes (bits 0-1 of each
// byte) into its top byte: code r times 2^(6m), m = 1..4, lands at bit
// 8r + 6m, the top byte takes m = 4 - r, and the other products sit in
// disjoint 2-bit fields below bit 24 (no carries).  Two v_perm_b32 and an OR
// join the four top bytes.
__device__ __forceinline__ uint32_t pack_codes(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3)
{
	const uint32_t g0 = (t0 & 0x03030303u) * 0x01041040u;
	const uint32_t g1 = (t1 & 0x03030303u) * 0x01041040u;
	const uint32_t g2 = (t2 & 0x03030303u) * 0x01041040u;
	const uint32_t g3 = (t3 & 0x03030303u) * 0x01041040u;
	const uint32_t lo = __builtin_amdgcn_perm(g1, g0, 0x0C0C0703u);   // bytes 0, 1: g0, g1 top bytes
	const uint32_t hi = __builtin_amdgcn_perm(g3, g2, 0x07030C0Cu);   // bytes 2, 3: g2, g3 top bytes
	return lo | hi;
}

// The big-endian stream pairrev(pack_codes(...)) directly (flank kernels,
// which need no little-endian stream): multiplying by 2^30 + 2^20 + 2^10 + 1
// puts code r of a dword at bit 30 - 2r of its top byte (the partial products
// land in disjoint 2-bit fields: 8r + {0, 10, 20, 30}), i.e. the byte holds
// its four codes reversed, and the perms place dword m's byte at byte 3 - m.
// Saves the 4-VALU pair reversal per chunk.
__device__ __forceinline__ uint32_t pack_codes_rev(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3)
{
	const uint32_t g0 = (t0 & 0x03030303u) * 0x40100401u;
	const uint32_t g1 = (t1 & 0x03030303u) * 0x40100401u;
	const uint32_t g2 = (t2 & 0x03030303u) * 0x40100401u;
	const uint32_t g3 = (t3 & 0x03030303u) * 0x40100401u;
	const uint32_t lo = __builtin_amdgcn_perm(g2, g3, 0x0C0C0703u);   // bytes 0, 1: g3, g2 top bytes
	const uint32_t hi = __builtin_amdgcn_perm(g0, g1, 0x07030C0Cu);   // bytes 2, 3: g1, g0 top bytes
	return lo | hi;
}

// Invalid-base flags of a chunk, base j at bit 2j (the layout of pack_codes):
// byte r of dword m is invalid if its LUT code has bit 2 set or its raw byte
// has bit 3 set.  One multiply gathers a dword's four flags (bit 2 of each
// byte, at 8r + 2) into its top byte: the terms 2^4, 2^10, 2^16, 2^22 put flag
// r at 24 + 2r and every other partial product at a distinct position below
// bit 24, so nothing carries; pack_codes' perms join the four top bytes.  15
// VALU against 23 for a mask-and-shift gather plus a 4x4 2-bit transpose; it
// runs on the invalid-base path, which a wave takes for 64 % of its chunks at
// 0.1 % N (one N among 1,024 bases).
__device__ __forceinline__ uint32_t invalid_flags(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t b0,
                                                  uint32_t b1, uint32_t b2, uint32_t b3)
{
	const uint32_t g0 = ((t0 | (b0 >> 1)) & 0x04040404u) * 0x00410410u;
	const uint32_t g1 = ((t1 | (b1 >> 1)) & 0x04040404u) * 0x00410410u;
	const uint32_t g2 = ((t2 | (b2 >> 1)) & 0x04040404u) * 0x00410410u;
	const uint32_t g3 = ((t3 | (b3 >> 1)) & 0x04040404u) * 0x00410410u;
	const uint32_t lo = __builtin_amdgcn_perm(g1, g0, 0x0C0C0703u);
	const uint32_t hi = __builtin_amdgcn_perm(g3, g2, 0x07030C0Cu);
	return lo | hi;
}

__device__ __forceinline__ int clamp16(int v) { return v < 0 ? 0 : (v > 16 ? 16 : v); }

// Flank-bitmap lookups of one chunk (VC_KV_FLANK): R with bit 15 - j set iff
// the 10-mer ending at base j (the low 20 bits of the forward stream there) is
// in the bitmap -- word bits 5..19, bit bits 0..4 (v_bfe_u32 uses the low 5
// bits of its offset).  5 VALU per base: extraction, shift, mask, test, merge.
// Bases j < J0 or j >= J1 are not looked up (their bits stay 0).
//
// Byte form (the default; -DVC_FLANK_WORD = the word form below): the bitmap
// is the same bytes read one byte at a time, byte v >> 3, bit v & 7.  The
// byte address (bits 3..19 of the 10-mer) and the bit index (bits 0..2) are
// two v_bfe_u32 of ONE register that holds the whole 10-mer: Bc for bases
// 9..15, B7 = bases -7..8 for bases 7 and 8, B9 = bases -9..6 for bases 0..6
// (two v_alignbit per chunk).  4 VALU per base plus 2 per chunk, against 5
// per base: no per-base extraction, and no mask (the byte address needs none;
// the 32-bit word address needed shift + mask).
template <int J0, int J1, int ABL = 0>
__device__ __forceinline__ uint32_t flank_bits_u8(uint32_t Bm1, uint32_t Bc)
{
	typedef const uint8_t __attribute__((address_space(3))) lds_u8_t;
	const uint32_t B9 = J0 <= 6 ? __builtin_amdgcn_alignbit(Bm1, Bc, 18u) : 0u;              // bases -9 .. 6
	const uint32_t B7 = J0 <= 8 && J1 > 7 ? __builtin_amdgcn_alignbit(Bm1, Bc, 14u) : 0u;   // bases -7 .. 8
	uint32_t fb[16], fi[16];
#pragma unroll
	for (int j = J0; j < J1; ++j) {
		const uint32_t src = j >= 9 ? Bc : (j >= 7 ? B7 : B9);
		const uint32_t s = j >= 9 ? 2u * (15 - j) : (j >= 7 ? 2u * (8 - j) : 2u * (6 - j));
		const uint32_t a = __builtin_amdgcn_ubfe(src, s + 3u, 2 * VC_FLANK_BASES - 3);
		fi[j] = __builtin_amdgcn_ubfe(src, s, 3u);
		if constexpr ((ABL & 1) != 0) { asm volatile("" :: "v"(a)); fb[j] = a; }
		else fb[j] = *(lds_u8_t *)(uintptr_t)a;   // the filter sits at LDS address 0
	}
	uint32_t R0 = 0, R1 = 0;
#pragma unroll
	for (int j = J0; j < J1; ++j) {
		const uint32_t t = __builtin_amdgcn_ubfe(fb[j], fi[j], 1u);
		uint32_t &R = (j & 1) ? R1 : R0;
		asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(R) : "v"(t), "i"(15 - j), "v"(R));
	}
	return R0 | R1;
}

template <int J0, int J1, int ABL = 0>
__device__ __forceinline__ uint32_t flank_bits(uint32_t fbase, uint32_t Bm1, uint32_t Bc)
{
	uint32_t fw[16], fx[16];
#pragma unroll
	for (int j = J0; j < J1; ++j) {
		const uint32_t x = __builtin_amdgcn_alignbit(Bm1, Bc, (uint32_t)(2 * (15 - j)));
		const uint32_t a = x >> 3;
		if constexpr ((ABL & 1) != 0) { asm volatile("" :: "v"(a)); fw[j] = a; }
		else fw[j] = lds_word(fbase, a, ((1u << (2 * VC_FLANK_BASES - 5)) - 1u) << 2);
		fx[j] = x;
	}
	// merged with one v_lshl_or_b32 per base into two chains (the compiler's
	// own shift + or3 tree costs 1.5 VALU per base)
	uint32_t R0 = 0, R1 = 0;
#pragma unroll
	for (int j = J0; j < J1; ++j) {
		const uint32_t t = __builtin_amdgcn_ubfe(fw[j], fx[j], 1u);
		uint32_t &R = (j & 1) ? R1 : R0;
		asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(R) : "v"(t), "i"(15 - j), "v"(R));
	}
	return R0 | R1;
}

// The flank test of a chunk's 16 windows (vafc_common.h): window j passes iff
// the 10-mers ending at j - d, d = VC_FLANK_DIST(K, 0..3), are all in the
// bitmap.  hm = R of chunk c (bit 15 - j for base j), P = R of chunks c-1 | c,
// H >> 16 = R of chunk c-2; the bit of base j - d sits d bits above base j's.
// The two middle distances are below 16 (P alone), the first ten's (K - 10
// <= 21) may reach chunk c-2.  Two shifts and a three-input AND more than the
// two-test form, for a quarter of its passes on the benchmark panel.
template <int K>
__device__ __forceinline__ uint32_t flank_windows(uint32_t hm, uint32_t H, uint32_t P)
{
	constexpr int D1 = VC_FLANK_DIST(K, 1), D2 = VC_FLANK_DIST(K, 2), D3 = VC_FLANK_DIST(K, 3);
	static_assert(VC_FLANK_TESTS == 4 && D1 < D2 && D2 <= 16 && D3 == K - VC_FLANK_BASES && D3 <= 32, "flank tests");
	const uint32_t first = __builtin_amdgcn_alignbit(H >> 16, P, (uint32_t)D3);
	return hm & (P >> D1) & (P >> D2) & first;
}

// Large-panel Bloom filter (VC_KV_BIG, vc_big_word): per window the strands'
// low 20 bits, each ONE v_bfe_u32 of a register that holds the whole field --
// the forward stream's 10-mer ending at base j (Bc, or one of two registers
// over (B[c-1]:B[c]) starting at bases -9 and -7), and the complement
// stream's ten bases from the window's first (C[c-2], C[c-1], C[c], or up to
// two more registers placed by BigPlan) -- then the 40-bit product's low word,
// a multiply-high by the word count and the same two-bit test as the
// 32-bit-word filter.  9 VALU per window plus about 4 per chunk, as for the
// power-of-two filter (2 v_alignbit, multiply, shift, and-or).
template <int K> struct BigPlan {
	int co[16];      // start (chunk-relative base) of the C-stream register for window j
	constexpr BigPlan() : co{}
	{
		bool cov[16] = {};
		const int free_o[3] = {0, -16, -32};
		for (int j = 0; j < 16; ++j) {
			const int q0 = j - K + 1;
			for (int f = 0; f < 3; ++f)
				if (!cov[j] && free_o[f] <= q0 && q0 <= free_o[f] + 6) {
					co[j] = free_o[f];
					cov[j] = true;
				}
		}
		for (int j = 0; j < 16; ++j)
			if (!cov[j]) {
				const int o = j - K + 1;
				for (int jj = j; jj < 16; ++jj)
					if (!cov[jj] && jj - K + 1 <= o + 6) {
						co[jj] = o;
						cov[jj] = true;
					}
			}
	}
};

// The C-stream register (base p of chunks c-2, c-1, c at bit 2(p + 32) of
// Cc:Cm1:Cm2) that starts at base o, o in [-32, 0] (a constant after unrolling).
__device__ __forceinline__ uint32_t c_reg(int o, uint32_t Cm2, uint32_t Cm1, uint32_t Cc)
{
	if (o == -32) return Cm2;
	if (o == -16) return Cm1;
	if (o == 0) return Cc;
	if (o < -16) return __builtin_amdgcn_alignbit(Cm1, Cm2, (uint32_t)(2 * (o + 32)));
	return __builtin_amdgcn_alignbit(Cc, Cm1, (uint32_t)(2 * (o + 16)));
}

template <int K, int J0, int J1, int ABL>
__device__ __forceinline__ uint32_t bloom_bits_big(const VcKernelArgs &A, uint32_t fbase, uint32_t Bm1, uint32_t Bc,
                                                  uint32_t Cm2, uint32_t Cm1, uint32_t Cc)
{
	constexpr BigPlan<K> plan{};
	const uint32_t nw4 = A.fwords << 2;
	const uint32_t B9 = __builtin_amdgcn_alignbit(Bm1, Bc, 18u);    // bases -9 .. 6
	const uint32_t B7 = __builtin_amdgcn_alignbit(Bm1, Bc, 14u);    // bases -7 .. 8
	uint32_t fw[16], fl[16], rl[16];
#pragma unroll
	for (int j = J0; j < J1; ++j) {
		const int bo = j >= 9 ? 0 : (j <= 6 ? -9 : -7);             // B register holding the 10-mer ending at j
		const uint32_t bsrc = bo == 0 ? Bc : (bo == -9 ? B9 : B7);
		const uint32_t f20 = __builtin_amdgcn_ubfe(bsrc, (uint32_t)(2 * (bo + 15 - j)), 20u);
		const int co = plan.co[j];
		const uint32_t r20 = __builtin_amdgcn_ubfe(c_reg(co, Cm2, Cm1, Cc), (uint32_t)(2 * (j - K + 1 - co)), 20u);
		// the filter sits at LDS address 0 (checked at kernel entry): a plain
		// v_and_b32 makes the word address, not a v_and_or_b32 with fbase
		const uint32_t a = __umulhi(f20 * r20, nw4) & ~3u;
		if constexpr ((ABL & 1) != 0) { asm volatile("" :: "v"(a)); fw[j] = a; }
		else fw[j] = *(lds_u32_t *)(uintptr_t)a;
		fl[j] = f20;
		rl[j] = r20;
	}
	uint32_t hm = 0;
#pragma unroll
	for (int j = J0; j < J1; ++j) hm = (hm << 1) | ((fw[j] >> (fl[j] & 31u)) & (fw[j] >> (rl[j] & 31u)) & 1u);
	if constexpr (J1 < 16) hm <<= 16 - J1;
	return hm;
}

// A chunk's filter lookups issued VC_BIG_GROUP / VC_FLANK_GROUP windows at a
// time, each group's bits tested before the next group's lookups issue (an
// empty asm with a memory clobber keeps the compiler from hoisting them): the
// live ranges of the looked-up words and their operands shrink (C5 kernel 124
// -> 112 VGPRs), and the compiler no longer re-derives the bit positions it
// could not keep in registers.  The lookup latency is covered by the other
// three waves of the SIMD.  C5 10.69-10.73 -> 10.58-10.62 ms with the plain
// address mask above (profiles/r05o_ab.log, r05p_ab.log; groups of 4 the same);
// the flank kernel's lookups in groups of 8 or 4 were not faster (r05q_ab.log).
#ifndef VC_BIG_GROUP
#define VC_BIG_GROUP 8
#endif
#ifndef VC_FLANK_GROUP
#define VC_FLANK_GROUP 16
#endif
template <int K, int J0, int J1, int ABL>
__device__ __forceinline__ uint32_t bloom_bits_big_grouped(const VcKernelArgs &A, uint32_t fbase, uint32_t Bm1, uint32_t Bc,
                                                          uint32_t Cm2, uint32_t Cm1, uint32_t Cc)
{
	if constexpr (J1 - J0 <= VC_BIG_GROUP) {
		return bloom_bits_big<K, J0, J1, ABL>(A, fbase, Bm1, Bc, Cm2, Cm1, Cc);
	} else {
		constexpr int JM = J0 + VC_BIG_GROUP;
		uint32_t h = bloom_bits_big<K, J0, JM, ABL>(A, fbase, Bm1, Bc, Cm2, Cm1, Cc);
		asm volatile("" : "+v"(h) :: "memory");
		return h | bloom_bits_big_grouped<K, JM, J1, ABL>(A, fbase, Bm1, Bc, Cm2, Cm1, Cc);
	}
}
template <int J0, int J1, int ABL>
__device__ __forceinline__ uint32_t flank_bits_u8_grouped(uint32_t Bm1, uint32_t Bc)
{
	if constexpr (J1 - J0 <= VC_FLANK_GROUP) {
		return flank_bits_u8<J0, J1, ABL>(Bm1, Bc);
	} else {
		constexpr int JM = J0 + VC_FLANK_GROUP;
		uint32_t h = flank_bits_u8<J0, JM, ABL>(Bm1, Bc);
		asm volatile("" : "+v"(h) :: "memory");
		return h | flank_bits_u8_grouped<JM, J1, ABL>(Bm1, Bc);
	}
}

// One 16-base chunk c of the packed scan from its five dwords (w0: the dword
// holding the chunk's first byte, realigned by sh); (B1, C1) / (B2, C2) are
// the streams of chunks c-1 / c-2 and move on to c / c-1.
template <int K, int ABL, int J0 = 0, int J1 = 16, bool DEFER = false>
__device__ __forceinline__ uint32_t packed_chunk(const VcKernelArgs &A, int c, int tail_c, int tail_r, int nt4m, uint32_t sh,
                                             uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
                                             uint32_t &Bm1, uint32_t &Bm2, uint32_t &Cm1, uint32_t &Cm2,
                                             int &U, int &Qe, uint32_t &H, const uint32_t *__restrict__ filt,
                                             WaveQueue &Q, uint32_t &tl, int lane)
{
	constexpr uint32_t HIM = (1u << (2 * K - 32)) - 1u;
	const uint32_t fsh = A.fsh;
	const uint32_t wmask4 = ((1u << A.wbits) - 1u) << 2;
	const uint32_t fbase = lds_base(filt);       // the filter sits at a 16-byte aligned LDS base
	const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
	const uint32_t b1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
	const uint32_t b2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
	const uint32_t b3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
	uint32_t t0 = dec_code(b0), t1 = dec_code(b1), t2 = dec_code(b2), t3 = dec_code(b3);
	dec_tail_chunk((c | nt4m) == tail_c, tail_r, b0, b1, b2, b3, t0, t1, t2, t3);
	U += 16;
	Qe += 16;
	constexpr bool FL = (ABL & VC_KV_FLANK) != 0;
	const uint32_t L = FL ? 0u : pack_codes(t0, t1, t2, t3);  // base j at bits 2j
	const uint32_t Cc = ~L;                          // complement codes, little-endian (unused by FL)
	const uint32_t Bc = FL ? pack_codes_rev(t0, t1, t2, t3) : pairrev(L);   // big-endian codes

	uint32_t hm = 0;                                 // filter pass, bit 15 - j for base j
	if constexpr ((ABL & VC_KV_FLANK) != 0) {
		// flank bitmap (vc_flank_*): one lookup per base, of the 10-mer ending
		// there; window j passes iff the 10-mers ending at j (its last ten
		// bases) and at j - (K - 10) (its first ten) are both in the set
		(void)fsh; (void)wmask4; (void)Cm2;
		if constexpr (VC_FLANK_U8) hm = flank_bits_u8_grouped<J0, J1, ABL>(Bm1, Bc);
		else hm = flank_bits<J0, J1, ABL>(fbase, Bm1, Bc);
		const uint32_t P = (H << 16) | hm;           // R of chunks c-1 | c, c-2 in H >> 16
		hm = flank_windows<K>(hm, H, P);
		H = P;
	} else if constexpr ((ABL & VC_KV_BIG) != 0) {
		(void)fsh; (void)wmask4;
		hm = bloom_bits_big_grouped<K, J0, J1, ABL>(A, fbase, Bm1, Bc, Cm2, Cm1, Cc);
	} else {
	// pass <=> bits (flo & 31) and (rlo & 31) of the filter word are set:
	// hm = (hm << 1) | ((w >> flo) & (w >> rlo) & 1), 4 VALU per window
	// windows j < J0 or j >= J1 are known invalid (see scan_span_packed) and
	// not looked up
	uint32_t fw[16], fl[16], rl[16];
#pragma unroll
	for (int j = J0; j < J1; ++j) {
		const uint32_t flo = __builtin_amdgcn_alignbit(Bm1, Bc, (uint32_t)(2 * (15 - j)));
		const int s2 = j - K + 1 + 32;               // window start relative to chunk c-2
		uint32_t rlo;
		if (s2 == 32) rlo = Cc;                      // k = 16, j = 15: the window is chunk c
		else if (s2 >= 16) rlo = __builtin_amdgcn_alignbit(Cc, Cm1, (uint32_t)(2 * (s2 - 16)));
		else rlo = __builtin_amdgcn_alignbit(Cm1, Cm2, (uint32_t)(2 * s2));
		// byte address of word (mix >> fsh) & (2^wbits - 1): fsh >= 5 for k >= 16
		const uint32_t wsh = vc_filter_mix(flo, rlo) >> (fsh - 2u);
		if constexpr ((ABL & 1) != 0) { asm volatile("" :: "v"(wsh)); fw[j] = wsh; }
		else fw[j] = lds_word(fbase, wsh, wmask4);
		fl[j] = flo;
		rl[j] = rlo;
	}
#pragma unroll
	for (int j = J0; j < J1; ++j)
		hm = (hm << 1) | ((fw[j] >> (fl[j] & 31u)) & (fw[j] >> (rl[j] & 31u)) & 1u);
	if constexpr (J1 < 16) hm <<= 16 - J1;          // window j at bit 15 - j
	}
	// windows of this chunk inside [vlo, vhi) with no earlier invalid base
	uint32_t V = ((1u << clamp16(U)) - 1u) & ~((1u << clamp16(Qe)) - 1u);
	const uint32_t anyinv = ((t0 | t1 | t2 | t3) & 0x04040404u) | ((b0 | b1 | b2 | b3) & 0x08080808u);
	if (__ballot(anyinv != 0u)) {
		if (anyinv != 0u) {
			// invalid flags packed like the codes: base j at bit 2j of F
			const uint32_t F = invalid_flags(t0, t1, t2, t3, b0, b1, b2, b3);
			const int j0 = (int)((uint32_t)__builtin_ctz(F) >> 1);          // first invalid base
			const int j1 = (int)((31u - (uint32_t)__builtin_clz(F)) >> 1);  // last invalid base
			V &= ~((2u << (15 - j0)) - 1u);          // windows ending at j >= j0
			const int u1 = 16 - j1 - K;
			U = U < u1 ? U : u1;
		}
	}
	hm &= V;
	tl += (uint32_t)__builtin_popcount(V);
	// queue the hit positions' forward k-mers (bit b <-> base j = 15 - b);
	// DEFER: the caller runs one hit loop for two chunks (hit_loop2)
	if constexpr (DEFER) {
		Bm2 = Bm1; Bm1 = Bc;
		Cm2 = Cm1; Cm1 = Cc;
		return hm;
	} else if constexpr ((ABL & 4) != 0) {
		asm volatile("" :: "v"(hm));
	} else if (__ballot(hm != 0u)) {
		for (;;) {
			const bool has = hm != 0u;
			const uint64_t bal = __ballot(has);
			if (!bal) break;
			// lowest pass first; lanes without one compute a garbage key they do not append
			const uint32_t b = (uint32_t)__builtin_ctz(hm | 0x80000000u);   // hm < 2^16
			const uint32_t flo = __builtin_amdgcn_alignbit(Bm1, Bc, 2u * b);
			const uint32_t fhi = __builtin_amdgcn_alignbit(Bm2, Bm1, 2u * b) & VC_HIT_HIM;
			queue_append<ABL>(A, Q, bal, has, ((uint64_t)fhi << 32) | flo, lane);
			hm &= hm - 1u;
		}
	}
	Bm2 = Bm1; Bm1 = Bc;
	Cm2 = Cm1; Cm1 = Cc;
	return 0u;
}

// One hit loop for two consecutive chunks a, a + 1 (packed_chunk<DEFER>):
// hm = (hm_a << 16) | hm_a+1, streams B[a-2] .. B[a+1].  A trip takes every
// lane's lowest pass; a lane's passes in 32 windows need fewer trips than in
// two separate 16-window loops (about 1.7 against 2.5 per chunk pair at the
// benchmark panel's pass rate), at 4 VALU per trip to pick the chunk's
// streams.  v_alignbit uses the low 5 bits of its shift, so 2b serves both
// halves.
template <int K, int ABL>
__device__ __forceinline__ void hit_loop2(const VcKernelArgs &A, WaveQueue &Q, uint32_t hm, uint32_t Bam2,
                                          uint32_t Bam1, uint32_t Ba, uint32_t Bb, int lane)
{
	constexpr uint32_t HIM = (1u << (2 * K - 32)) - 1u;
	if constexpr ((ABL & 4) != 0) {
		asm volatile("" :: "v"(hm));
	} else if (__ballot(hm != 0u)) {
		for (;;) {
			const bool has = hm != 0u;
			const uint64_t bal = __ballot(has);
			if (!bal) break;
			uint32_t b;   // lowest pass; lanes without one get ~0 and append nothing
			asm("v_ffbl_b32 %0, %1" : "=v"(b) : "v"(hm));
			const bool ina = b >= 16u;
			const uint32_t lo = ina ? Ba : Bb, hi = ina ? Bam1 : Ba, hi2 = ina ? Bam2 : Bam1;
			const uint32_t flo = __builtin_amdgcn_alignbit(hi, lo, 2u * b);
			const uint32_t fhi = __builtin_amdgcn_alignbit(hi2, hi, 2u * b) & VC_HIT_HIM;
			queue_append<ABL>(A, Q, bal, has, ((uint64_t)fhi << 32) | flo, lane);
			hm &= hm - 1u;
		}
	}
}

// Chunk c's streams only, for a chunk in which no window can be valid (chunk
// 0 of a whole read when K >= 17: its windows end at positions 0..15 < K - 1):
// decode, pack, the invalid-base bookkeeping (an N here still invalidates
// the windows that span it) and the stream rotation of packed_chunk, without
// its 16 filter lookups, validity mask, tally or hit loop.
template <int K, int ABL>
__device__ __forceinline__ void packed_streams(const VcKernelArgs &A, int c, int tail_c, int tail_r, int nt4m, uint32_t sh, uint32_t w0, uint32_t w1,
                                               uint32_t w2, uint32_t w3, uint32_t w4, uint32_t &Bm1, uint32_t &Bm2,
                                               uint32_t &Cm1, uint32_t &Cm2, int &U, int &Qe, uint32_t &H,
                                               const uint32_t *__restrict__ filt)
{
	const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
	const uint32_t b1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
	const uint32_t b2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
	const uint32_t b3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
	uint32_t t0 = dec_code(b0), t1 = dec_code(b1), t2 = dec_code(b2), t3 = dec_code(b3);
	dec_tail_chunk((c | nt4m) == tail_c, tail_r, b0, b1, b2, b3, t0, t1, t2, t3);
	U += 16;
	Qe += 16;
	constexpr bool FL = (ABL & VC_KV_FLANK) != 0;
	const uint32_t L = FL ? 0u : pack_codes(t0, t1, t2, t3);
	const uint32_t anyinv = ((t0 | t1 | t2 | t3) & 0x04040404u) | ((b0 | b1 | b2 | b3) & 0x08080808u);
	if (__ballot(anyinv != 0u)) {
		if (anyinv != 0u) {   // as in packed_chunk: U moves to the last invalid base
			const uint32_t F = invalid_flags(t0, t1, t2, t3, b0, b1, b2, b3);
			const int j1 = (int)((31u - (uint32_t)__builtin_clz(F)) >> 1);
			const int u1 = 16 - j1 - K;
			U = U < u1 ? U : u1;
		}
	}
	const uint32_t Bc = FL ? pack_codes_rev(t0, t1, t2, t3) : pairrev(L);
	if constexpr ((ABL & VC_KV_FLANK) != 0) {
		// the first window (ending at K - 1) starts with the 10-mer ending at
		// base 9: chunk 0's bases 9..15 are looked up for the later windows
		static_assert(K - VC_FLANK_BASES >= 9, "flank mode needs the first window's head in chunk 0");
		if constexpr (VC_FLANK_U8) H = flank_bits_u8_grouped<VC_FLANK_BASES - 1, 16, ABL>(Bm1, Bc);
		else H = flank_bits<VC_FLANK_BASES - 1, 16, ABL>(lds_base(filt), Bm1, Bc);
	}
	Bm2 = Bm1; Bm1 = Bc;
	Cm2 = Cm1; Cm1 = ~L;
}

// One global_load_dwordx4 of dwords [q, q+4), always exactly one load
// instruction, so that the compiler can count loads in flight and wait only
// for the quad a chunk is about to use.  A quad that would pass the end of
// the buffer is loaded from its last four dwords instead (the host guarantees
// at least four) and the return value says how far it was moved back; the
// user shifts the dwords into place (quad_fix).  Dwords past the end of the
// buffer are never part of a read.
__device__ __forceinline__ uint32_t ldq(const uint32_t *__restrict__ s32, uint64_t q, uint64_t wmax,
                                        uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	const uint64_t lim = wmax - 3u;
	const bool clamp = q > lim;
	const u32x4a4 v = ld16(s32 + (clamp ? lim : q));
	a = v.x; b = v.y; c = v.z; d = v.w;
	return clamp ? (q - lim > 3u ? 3u : (uint32_t)(q - lim)) : 0u;
}

// Unclamped load for read groups whose every load is known to lie inside
// the buffer (checked once per group, see vc_count_reads_kernel).
template <bool SAFE>
__device__ __forceinline__ uint32_t ldq_s(const uint32_t *__restrict__ s32, uint64_t q, uint64_t wmax,
                                          uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	if constexpr (SAFE) {
		const u32x4a4 v = ld16(s32 + q);
		a = v.x; b = v.y; c = v.z; d = v.w;
		return 0u;
	} else {
		return ldq(s32, q, wmax, a, b, c, d);
	}
}

__device__ __forceinline__ void quad_fix(uint32_t sft, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	if (__ballot(sft != 0u)) {       // only the last reads of a buffer
		asm volatile("");            // keep this rare branch a branch
		if (sft != 0u) {
			a = sft == 1u ? b : (sft == 2u ? c : d);
			b = sft == 1u ? c : d;
			c = d;
		}
	}
}

template <int J> struct J0Tag { static constexpr int value = J; };

// Chunks are processed in pairs.  The 8 dwords of the next pair are requested
// (two dwordx4 from the same lines, back to back) while the current pair is
// scanned, so each load has two chunks of work to hide behind.  The steady
// loop issues the same loads on every trip (lanes past their span re-read
// harmless bytes), the last pair is peeled: the compiler then waits for a
// pair's data only when the pair starts.
template <int K, bool HAS_LO, int ABL = 0, bool SAFE = false>
__device__ __forceinline__ void scan_span_packed(const VcKernelArgs &A, const uint32_t *__restrict__ s32,
                                                 uint64_t wmax, uint64_t off, int len, int c_lo, int c_hi,
                                                 int vlo, int vhi, int nit,
                                                 const uint32_t *__restrict__ filt, WaveQueue &Q,
                                                 uint32_t &tl, int lane)
{
	static_assert(K >= 16 && K <= 31, "packed scan needs 16 <= k <= 31");
	// the read's tail chunk decodes with seq_nt4_table (vaf-counter.c:261-291);
	// in seq_nt4 mode (snp-pattern-gen) every chunk does: tail_c = -1 and the
	// test (c | -1) == -1 always holds (the OR is scalar in the reads kernel)
	const int tail_c = A.nt4 ? -1 : ((len & 15) ? (len >> 4) : -1);
	// seq_nt4 mode decodes all 16 bytes of every chunk with the table: every
	// dword of the chunk holds "tail" bytes (dec_tail_chunk tests tail_r)
	const int tail_r = A.nt4 ? 16 : (len & 15);
	const int nt4m = -(int)A.nt4;   // 0 or -1 (the host stores 0 / 1); kept arithmetic so
	                                  // the test stays one compare, not (c == tail_c) || nt4

	uint64_t addr = off + 16ull * (uint64_t)c_lo;
	uint64_t wi = addr >> 2;
	const uint32_t sh = (uint32_t)(addr & 3u);
	uint32_t w0, w1, w2, w3, w4, w5, w6, w7, w8;
	w0 = SAFE ? s32[wi] : ldw(s32, wi, wmax);
	uint32_t d1 = ldq_s<SAFE>(s32, wi + 1, wmax, w1, w2, w3, w4);
	uint32_t d5 = ldq_s<SAFE>(s32, wi + 5, wmax, w5, w6, w7, w8);
	// whole reads, K >= 17: chunk 0 only builds streams (below), so chunk 2's
	// dwords are needed one chunk after chunk 1's and are requested up front
	constexpr bool PEEL = !HAS_LO && K >= 17 && (ABL & 32) == 0;
	[[maybe_unused]] uint32_t x5 = 0, x6 = 0, x7 = 0, x8 = 0, d9 = 0;
	if constexpr (PEEL) d9 = ldq_s<SAFE>(s32, wi + 9, wmax, x5, x6, x7, x8);

	uint32_t Bm1 = 0, Bm2 = 0, Cm1 = 0, Cm2 = 0;   // streams of the two previous chunks
	uint32_t H = 0;                                  // flank mode: 10-mer hits of chunks c-2 | c-1
	int U = 1 - K - vlo + 16 * c_lo;                 // +16 at the top of every chunk
	int Qe = -vhi + 16 * c_lo;

	[[maybe_unused]] uint32_t abl_sink = 0;
	int it = 0;
	// Whole reads, K >= 17: no window ends in chunk 0 (positions 0..15 < K - 1),
	// so chunk 0 only builds the streams (about 16 % fewer VALU for 150 bp
	// reads); the pair loop then starts at chunk 1.  The dwords of chunk 1 are
	// w4..w8 already, chunk 2's were requested with them (x5..x8: requested
	// here, the large-panel config waited a whole memory latency at chunk 2,
	// +4.5 %), and everything after moves on by 16 bytes -- the loads stay
	// within the group's clear range (8 ceil(nit / 2) + 13 dwords from the
	// first).  A.variant bit 0 turns this off at run time (A/B).
	if constexpr (PEEL) {
		if (nit > 0 && (A.variant & 1u) == 0) {
			quad_fix(d1, w1, w2, w3, w4);
			packed_streams<K, ABL>(A, c_lo, tail_c, tail_r, nt4m, sh, w0, w1, w2, w3, w4, Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt);
			w0 = w4; w1 = w5; w2 = w6; w3 = w7; w4 = w8; d1 = d5;
			w5 = x5; w6 = x6; w7 = x7; w8 = x8; d5 = d9;
			wi += 4;
			it = 1;
		}
	}
	auto trip = [&](auto j0tag) {
		constexpr int J0 = decltype(j0tag)::value;
		const int c = c_lo + it;
		uint32_t n0, n1, n2, n3, n4, n5, n6, n7, dn0, dn4;
		if constexpr ((ABL & 2) != 0) {
			n0 = (uint32_t)wi * 0x9E3779B1u; n1 = n0 ^ 0x41434754u; n2 = n0 + 0x54474341u; n3 = n0 * 5u;
			n4 = n0 ^ 0x5A5A5A5Au; n5 = n1 + 7u; n6 = n2 ^ n3; n7 = n4 * 3u;
			dn0 = dn4 = 0;
		} else if constexpr ((ABL & 16) != 0) {
			// timing experiment: issue the real loads but consume them only
			// after the scan (isolates the cost of waiting from issuing)
			uint32_t t0_, t1_, t2_, t3_, t4_, t5_, t6_, t7_;
			ldq(s32, wi + 9, wmax, t0_, t1_, t2_, t3_);
			ldq(s32, wi + 13, wmax, t4_, t5_, t6_, t7_);
			abl_sink ^= t0_ ^ t1_ ^ t2_ ^ t3_ ^ t4_ ^ t5_ ^ t6_ ^ t7_;
			n0 = (uint32_t)wi * 0x9E3779B1u; n1 = n0 ^ 0x41434754u; n2 = n0 + 0x54474341u; n3 = n0 * 5u;
			n4 = n0 ^ 0x5A5A5A5Au; n5 = n1 + 7u; n6 = n2 ^ n3; n7 = n4 * 3u;
			dn0 = dn4 = 0;
		} else if constexpr ((ABL & 8) != 0) {
			// timing experiment: the memory pattern of a wave-tiled layout
			// (chunk c of lane l at 16 * (64 c + l) from a wave base)
			const uint64_t tb = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(off >> 4)) << 2) +
			                    (uint64_t)(64 * (it + 2) + lane) * 4u;
			dn0 = ldq(s32, tb, wmax, n0, n1, n2, n3);
			dn4 = ldq(s32, tb + 256, wmax, n4, n5, n6, n7);
		} else {
			dn0 = ldq_s<SAFE>(s32, wi + 9, wmax, n0, n1, n2, n3);
			dn4 = ldq_s<SAFE>(s32, wi + 13, wmax, n4, n5, n6, n7);
		}
		quad_fix(d1, w1, w2, w3, w4);
		quad_fix(d5, w5, w6, w7, w8);
		packed_chunk<K, ABL, J0>(A, c, tail_c, tail_r, nt4m, sh, w0, w1, w2, w3, w4, Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q, tl, lane);
		packed_chunk<K, ABL>(A, c + 1, tail_c, tail_r, nt4m, sh, w4, w5, w6, w7, w8, Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q, tl, lane);
		w0 = w8;
		w1 = n0; w2 = n1; w3 = n2; w4 = n3; d1 = dn0;
		w5 = n4; w6 = n5; w7 = n6; w8 = n7; d5 = dn4;
		wi += 8;
	};
	// chunk 1 of a whole read: its windows end at 16..31, those before K - 1
	// are invalid, so its first K - 17 filter lookups are skipped
	// (flank mode looks up every base: chunk 1's are the heads of later windows)
	if constexpr (!HAS_LO && K >= 18 && (ABL & 32) == 0 && (ABL & VC_KV_FLANK) == 0) {
		if (it == 1 && it + 2 < nit && (A.variant & 2u) == 0) {
			trip(J0Tag<K - 17>{});
			it += 2;
		}
	}
	for (; it + 2 < nit; it += 2) trip(J0Tag<0>{});
	if constexpr ((ABL & 16) != 0) tl += abl_sink & 1u;
	if (it < nit) {
		quad_fix(d1, w1, w2, w3, w4);
		quad_fix(d5, w5, w6, w7, w8);
		const bool pair = it + 1 < nit;
		if (pair)
			packed_chunk<K, ABL>(A, c_lo + it, tail_c, tail_r, nt4m, sh, w0, w1, w2, w3, w4, Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q,
			                     tl, lane);
		// the wave's last chunk: windows j end at 16 cl + j and are valid only
		// below vhi, so when no lane has more than 8 of them (150-bp reads: 6)
		// the upper 8 windows are not looked up (A.variant bit 2: always all)
		const int cl = c_lo + nit - 1;
		const uint32_t x0 = pair ? w4 : w0, x1 = pair ? w5 : w1, x2 = pair ? w6 : w2, x3 = pair ? w7 : w3,
		               x4 = pair ? w8 : w4;
		if ((A.variant & 4u) == 0 && __ballot(vhi - 16 * cl > 8) == 0)
			packed_chunk<K, ABL, 0, 8>(A, cl, tail_c, tail_r, nt4m, sh, x0, x1, x2, x3, x4, Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q, tl,
			                           lane);
		else
			packed_chunk<K, ABL>(A, cl, tail_c, tail_r, nt4m, sh, x0, x1, x2, x3, x4, Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q, tl,
			                     lane);
	}
}

// The same scan with chunks in quads: each lane requests the next 64 bytes of
// its read (four dwordx4 from one or two lines, back to back) while the
// current four chunks are scanned.  Every lane of a wave reads a different
// read, so every request misses the 32 KiB L1 (16 waves x 64 lanes keep
// 128 KiB of lines live); the L1's outstanding misses, not instruction issue,
// bound the pair loop once the flank prefilter cut the VALU per base
// (TCP_PENDING_STALL_CYCLES 70 % of the kernel).  Four requests to one line
// back to back cost it one miss instead of two.  A.variant bit 3 selects the
// pair loop (A/B).
template <int K, bool HAS_LO, int ABL = 0, bool SAFE = false>
__device__ __forceinline__ void scan_span_quad(const VcKernelArgs &A, const uint32_t *__restrict__ s32,
                                               uint64_t wmax, uint64_t off, int len, int c_lo, int vlo, int vhi,
                                               int nit, const uint32_t *__restrict__ filt, WaveQueue &Q,
                                               uint32_t &tl, int lane)
{
	if (nit == 0) return;            // wave-uniform; the loads below assume a chunk
	const int tail_c = A.nt4 ? -1 : ((len & 15) ? (len >> 4) : -1);
	// seq_nt4 mode decodes all 16 bytes of every chunk with the table: every
	// dword of the chunk holds "tail" bytes (dec_tail_chunk tests tail_r)
	const int tail_r = A.nt4 ? 16 : (len & 15);
	const int nt4m = -(int)A.nt4;
	const uint64_t addr = off + 16ull * (uint64_t)c_lo;
	uint64_t wi = addr >> 2;
	const uint32_t sh = (uint32_t)(addr & 3u);
	uint32_t w[17], d[4];
	w[0] = SAFE ? s32[wi] : ldw(s32, wi, wmax);
#pragma unroll
	for (int q = 0; q < 4; ++q) d[q] = ldq_s<SAFE>(s32, wi + 1 + 4 * q, wmax, w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], w[4 * q + 4]);
	constexpr bool PEEL = !HAS_LO && K >= 17 && (ABL & 32) == 0;
	[[maybe_unused]] uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0, dx = 0;
	if constexpr (PEEL) dx = ldq_s<SAFE>(s32, wi + 17, wmax, x0, x1, x2, x3);

	uint32_t Bm1 = 0, Bm2 = 0, Cm1 = 0, Cm2 = 0, H = 0;
	int U = 1 - K - vlo + 16 * c_lo;
	int Qe = -vhi + 16 * c_lo;
	int it = 0;
	// chunk 0 of a whole read builds only the streams (see scan_span_packed);
	// the quads then start at chunk 1, chunk 4's dwords requested up front
	if constexpr (PEEL) {
		if ((A.variant & 1u) == 0) {
			quad_fix(d[0], w[1], w[2], w[3], w[4]);
			packed_streams<K, ABL>(A, c_lo, tail_c, tail_r, nt4m, sh, w[0], w[1], w[2], w[3], w[4], Bm1, Bm2, Cm1, Cm2, U, Qe, H,
			                       filt);
#pragma unroll
			for (int i = 0; i < 13; ++i) w[i] = w[i + 4];
			w[13] = x0; w[14] = x1; w[15] = x2; w[16] = x3;
			d[0] = d[1]; d[1] = d[2]; d[2] = d[3]; d[3] = dx;
			wi += 4;
			it = 1;
		}
		// a wave whose reads all fit in one chunk (<= 16 bases) is done: the
		// tail below assumes at least one chunk left (wave-uniform)
		if (it == nit) return;
	}
	auto chunk = [&](auto j0tag, auto j1tag, int c, int b) {
		packed_chunk<K, ABL, decltype(j0tag)::value, decltype(j1tag)::value>(
			A, c, tail_c, tail_r, nt4m, sh, w[b], w[b + 1], w[b + 2], w[b + 3], w[b + 4], Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q,
			tl, lane);
	};
	auto dchunk = [&](auto j0tag, int c, int b) -> uint32_t {
		return packed_chunk<K, ABL, decltype(j0tag)::value, 16, true>(
			A, c, tail_c, tail_r, nt4m, sh, w[b], w[b + 1], w[b + 2], w[b + 3], w[b + 4], Bm1, Bm2, Cm1, Cm2, U, Qe, H, filt, Q,
			tl, lane);
	};
	auto trip = [&](auto j0tag) {
		const int c = c_lo + it;
		uint32_t n[16], dn[4];
#pragma unroll
		for (int q = 0; q < 4; ++q)
			dn[q] = ldq_s<SAFE>(s32, wi + 17 + 4 * q, wmax, n[4 * q], n[4 * q + 1], n[4 * q + 2], n[4 * q + 3]);
#pragma unroll
		for (int q = 0; q < 4; ++q) quad_fix(d[q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], w[4 * q + 4]);
		// flank mode: one hit loop per chunk pair (the Bloom-filter kernels are
		// at the 128-VGPR limit and would spill; ablation builds: A.variant
		// bit 6 = per chunk)
		// (the large-panel Bloom kernels too: VC_DEFER_BIG, A/B)
		bool defer = (ABL & (VC_KV_FLANK | VC_KV_BIG_DEFER)) != 0;
#ifdef VC_ABLATION
		defer = defer && (A.variant & 64u) == 0;
#endif
		if constexpr ((ABL & (VC_KV_FLANK | VC_KV_BIG_DEFER)) == 0) defer = false;
		if (defer) {
#pragma unroll
			for (int p = 0; p < 2; ++p) {
				const uint32_t s2 = Bm2, s1 = Bm1;
				uint32_t h = p == 0 ? dchunk(j0tag, c, 0) : dchunk(J0Tag<0>{}, c + 2, 8);
				h = (h << 16) | dchunk(J0Tag<0>{}, c + 2 * p + 1, 8 * p + 4);
				hit_loop2<K, ABL>(A, Q, h, s2, s1, Bm2, Bm1, lane);
			}
		} else {
			chunk(j0tag, J0Tag<16>{}, c, 0);
			chunk(J0Tag<0>{}, J0Tag<16>{}, c + 1, 4);
			chunk(J0Tag<0>{}, J0Tag<16>{}, c + 2, 8);
			chunk(J0Tag<0>{}, J0Tag<16>{}, c + 3, 12);
		}
		w[0] = w[16];
#pragma unroll
		for (int i = 0; i < 16; ++i) w[i + 1] = n[i];
#pragma unroll
		for (int q = 0; q < 4; ++q) d[q] = dn[q];
		wi += 16;
	};
	if constexpr (!HAS_LO && K >= 18 && (ABL & 32) == 0 && (ABL & VC_KV_FLANK) == 0) {
		if (it == 1 && it + 4 < nit && (A.variant & 2u) == 0) {
			trip(J0Tag<K - 17>{});
			it += 4;
		}
	}
	for (; it + 4 < nit; it += 4) trip(J0Tag<0>{});
	// the last 1..4 chunks, all in w already (wave-uniform count)
#pragma unroll
	for (int q = 0; q < 4; ++q) quad_fix(d[q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], w[4 * q + 4]);
	const int r = nit - it;
	if (r >= 2) chunk(J0Tag<0>{}, J0Tag<16>{}, c_lo + it, 0);
	if (r >= 3) chunk(J0Tag<0>{}, J0Tag<16>{}, c_lo + it + 1, 4);
	if (r >= 4) chunk(J0Tag<0>{}, J0Tag<16>{}, c_lo + it + 2, 8);
	// the wave's last chunk: only its lower 8 windows when no lane has more
	// valid ones (see scan_span_packed)
	const int b = 4 * (r - 1);
	if (b != 0) {
		w[0] = b == 4 ? w[4] : (b == 8 ? w[8] : w[12]);
		w[1] = b == 4 ? w[5] : (b == 8 ? w[9] : w[13]);
		w[2] = b == 4 ? w[6] : (b == 8 ? w[10] : w[14]);
		w[3] = b == 4 ? w[7] : (b == 8 ? w[11] : w[15]);
		w[4] = b == 4 ? w[8] : (b == 8 ? w[12] : w[16]);
	}
	const int cl = c_lo + nit - 1;
	if ((A.variant & 4u) == 0 && __ballot(vhi - 16 * cl > 8) == 0)
		chunk(J0Tag<0>{}, J0Tag<8>{}, cl, 0);
	else
		chunk(J0Tag<0>{}, J0Tag<16>{}, cl, 0);
}

// ---------------------------------------------------------------------------
// flank kernels, whole reads: odd lanes scan their read backwards
// ---------------------------------------------------------------------------
//
// Lane r reads read r, and read r's last bytes share a 128-byte line with
// read r + 1's first bytes.  Scanned forwards by both lanes, that line is
// fetched by lane r + 1 at its first trip and by lane r at its last, about
// 15 us apart, and the L2 has usually dropped it in between (HBM traffic
// 1.6x the read bytes).  Here odd lanes scan the reverse complement of their
// read, last chunk first: lane 2i + 1 starts at the line it shares with lane
// 2i + 2 and ends at the one it shares with lane 2i, so each shared line is
// requested by both lanes in the same load instruction.
//
// A backward lane's chunk c' is read bytes [len - 16c' - 16, len - 16c') of
// its read, complemented and reversed.  The canonical k-mers, the window
// validity (in reverse-complement coordinates [0, len)), the tally and the
// flank test (the bitmap is closed under reverse complement) are unchanged;
// the queued k-mers are the reverse complements, canonicalised by the drain.
//
// Registers: quad q of a window holds the chunk's first four dwords in
// address order for both directions, w[0] the fifth dword of the window's
// first chunk (forwards: the dword after, backwards: the dword after, too --
// which for a backward lane is the first dword of the chunk scanned before).
// The four realigned dwords in quad order are q0..q3; forwards they are the
// chunk's bytes 0..15, backwards bytes 12..15, 0..3, 4..7, 8..11 (q1..q3 are
// the same v_alignbyte for both).  Packing then differs only in per-lane
// constants: the multiplier (codes reversed inside a byte, or not), one perm
// selector and the complement (Dir).  Cost: 2 v_cndmask per chunk.

struct Dir {
	bool bwd;
	uint32_t mul;     // 0x40100401: a byte's codes reversed (forwards); 0x01041040: in order (backwards)
	uint32_t sel13;   // perm selector placing dwords q1 and q3
	uint32_t inv;     // 0 forwards, ~0 backwards (the complement)
};

// Byte mask of the bytes i >= e of a dword (e <= 0: all, e >= 4: none).
__device__ __forceinline__ uint32_t bytes_from(int e)
{
	return e <= 0 ? 0xFFFFFFFFu : (e >= 4 ? 0u : (0xFFFFFFFFu << (8 * e)));
}

// Decode of a chunk's four realigned dwords (quad order) with the read's
// tail rule (vaf-counter.c:261-291): forwards the tail chunk decodes with
// seq_nt4_table throughout; backwards chunk 0 holds the read's last 16
// bytes, of which the last len % 16 (its first bytes in scan order:
// tail_e = 16 - len % 16 in read order) are the tail.
__device__ __forceinline__ void dec_chunk_fb(const Dir &D, int c, int tail_c, int nt4m, int tail_e, uint32_t q0,
                                             uint32_t q1, uint32_t q2, uint32_t q3, uint32_t &t0, uint32_t &t1,
                                             uint32_t &t2, uint32_t &t3)
{
	t0 = dec_code(q0); t1 = dec_code(q1); t2 = dec_code(q2); t3 = dec_code(q3);
	const int cm = c | nt4m;
	if (__ballot(cm == tail_c)) {
		if (cm == tail_c) {
			// read-order dword of q_m: forwards m, backwards (m + 3) & 3
			const int e = D.bwd ? tail_e : -64;
			uint32_t mk = bytes_from(e - 12);
			t0 = (dec_tail(q0) & mk) | (t0 & ~mk);
			mk = bytes_from(e);
			t1 = (dec_tail(q1) & mk) | (t1 & ~mk);
			mk = bytes_from(e - 4);
			t2 = (dec_tail(q2) & mk) | (t2 & ~mk);
			mk = bytes_from(e - 8);
			t3 = (dec_tail(q3) & mk) | (t3 & ~mk);
		}
	}
}

// The chunk's big-endian stream in scan order (see Dir).
__device__ __forceinline__ uint32_t pack_fb(const Dir &D, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3)
{
	const uint32_t g0 = (t0 & 0x03030303u) * D.mul;
	const uint32_t g1 = (t1 & 0x03030303u) * D.mul;
	const uint32_t g2 = (t2 & 0x03030303u) * D.mul;
	const uint32_t g3 = (t3 & 0x03030303u) * D.mul;
	const uint32_t p13 = __builtin_amdgcn_perm(g1, g3, D.sel13);
	const uint32_t p02 = __builtin_amdgcn_perm(g0, g2, 0x070C030Cu);   // byte 1: q2, byte 3: q0
	return (p13 | p02) ^ D.inv;
}

// Invalid bases of the chunk, base j (scan order) at bit 2j; slow path.
__device__ __forceinline__ uint32_t invalid_bits_fb(const Dir &D, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                                    uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3)
{
	const uint32_t F = invalid_flags(t0, t1, t2, t3, q0, q1, q2, q3);   // quad-order byte p at bit 2p
	// backwards: quad order -> read order (rotate by one dword), then reverse
	return D.bwd ? pairrev(__builtin_amdgcn_alignbit(F, F, 8u)) : F;
}

template <int K, int ABL, int J0 = 0, int J1 = 16, bool DEFER = false>
__device__ __forceinline__ uint32_t packed_chunk_fb(const VcKernelArgs &A, const Dir &D, int c, int tail_c, int nt4m,
                                                    int tail_e, uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3,
                                                    uint32_t &Bm1, uint32_t &Bm2, int &U, int &Qe, uint32_t &H,
                                                    const uint32_t *__restrict__ filt, WaveQueue &Q, uint32_t &tl,
                                                    int lane)
{
	constexpr uint32_t HIM = (1u << (2 * K - 32)) - 1u;
	uint32_t t0, t1, t2, t3;
	dec_chunk_fb(D, c, tail_c, nt4m, tail_e, q0, q1, q2, q3, t0, t1, t2, t3);
	U += 16;
	Qe += 16;
	const uint32_t Bc = pack_fb(D, t0, t1, t2, t3);
	uint32_t hm;
	if constexpr (VC_FLANK_U8) hm = flank_bits_u8_grouped<J0, J1, ABL>(Bm1, Bc);
	else hm = flank_bits<J0, J1, ABL>(lds_base(filt), Bm1, Bc);
	const uint32_t P = (H << 16) | hm;
	hm = flank_windows<K>(hm, H, P);
	H = P;
	uint32_t V = ((1u << clamp16(U)) - 1u) & ~((1u << clamp16(Qe)) - 1u);
	const uint32_t anyinv = ((t0 | t1 | t2 | t3) & 0x04040404u) | ((q0 | q1 | q2 | q3) & 0x08080808u);
	if (__ballot(anyinv != 0u)) {
		if (anyinv != 0u) {
			const uint32_t F = invalid_bits_fb(D, t0, t1, t2, t3, q0, q1, q2, q3);
			const int j0 = (int)((uint32_t)__builtin_ctz(F) >> 1);
			const int j1 = (int)((31u - (uint32_t)__builtin_clz(F)) >> 1);
			V &= ~((2u << (15 - j0)) - 1u);
			const int u1 = 16 - j1 - K;
			U = U < u1 ? U : u1;
		}
	}
	hm &= V;
	tl += (uint32_t)__builtin_popcount(V);
	if constexpr (DEFER) {
		Bm2 = Bm1; Bm1 = Bc;
		return hm;
	} else if constexpr ((ABL & 4) != 0) {
		asm volatile("" :: "v"(hm));
	} else if (__ballot(hm != 0u)) {
		for (;;) {
			const bool has = hm != 0u;
			const uint64_t bal = __ballot(has);
			if (!bal) break;
			const uint32_t b = (uint32_t)__builtin_ctz(hm | 0x80000000u);
			const uint32_t flo = __builtin_amdgcn_alignbit(Bm1, Bc, 2u * b);
			const uint32_t fhi = __builtin_amdgcn_alignbit(Bm2, Bm1, 2u * b) & VC_HIT_HIM;
			queue_append<ABL>(A, Q, bal, has, ((uint64_t)fhi << 32) | flo, lane);
			hm &= hm - 1u;
		}
	}
	Bm2 = Bm1; Bm1 = Bc;
	return 0u;
}

// Chunk 0 of a whole read (no window can end in it, K >= 17): streams only.
template <int K, int ABL>
__device__ __forceinline__ void packed_streams_fb(const VcKernelArgs &A, const Dir &D, int c, int tail_c, int nt4m,
                                                  int tail_e, uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3,
                                                  uint32_t &Bm1, uint32_t &Bm2, int &U, int &Qe, uint32_t &H)
{
	uint32_t t0, t1, t2, t3;
	dec_chunk_fb(D, c, tail_c, nt4m, tail_e, q0, q1, q2, q3, t0, t1, t2, t3);
	U += 16;
	Qe += 16;
	const uint32_t anyinv = ((t0 | t1 | t2 | t3) & 0x04040404u) | ((q0 | q1 | q2 | q3) & 0x08080808u);
	if (__ballot(anyinv != 0u)) {
		if (anyinv != 0u) {
			const uint32_t F = invalid_bits_fb(D, t0, t1, t2, t3, q0, q1, q2, q3);
			const int j1 = (int)((31u - (uint32_t)__builtin_clz(F)) >> 1);
			const int u1 = 16 - j1 - K;
			U = U < u1 ? U : u1;
		}
	}
	const uint32_t Bc = pack_fb(D, t0, t1, t2, t3);
	static_assert(K - VC_FLANK_BASES >= 9, "flank mode needs the first window's head in chunk 0");
	if constexpr (VC_FLANK_U8) H = flank_bits_u8_grouped<VC_FLANK_BASES - 1, 16, ABL>(Bm1, Bc);
	else H = flank_bits<VC_FLANK_BASES - 1, 16, ABL>(0u, Bm1, Bc);
	Bm2 = Bm1; Bm1 = Bc;
}

// A quad of dwords [q, q + 4) loaded from inside [0, wmax]: a quad that would
// leave the buffer is loaded from its nearest end and the return value says
// how far it was moved (positive: back from the end, negative: up from the
// start); quad_fix_fb shifts the dwords into place.  Dwords outside the
// buffer are never part of a read.
__device__ __forceinline__ int ldq_fb(const uint32_t *__restrict__ s32, int64_t q, uint64_t wmax,
                                      uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	const int64_t lim = (int64_t)wmax - 3;
	const int64_t cq = q < 0 ? 0 : (q > lim ? lim : q);
	const u32x4a4 v = ld16(s32 + cq);
	a = v.x; b = v.y; c = v.z; d = v.w;
	const int64_t sft = q - cq;
	return sft > 3 ? 3 : (sft < -3 ? -3 : (int)sft);
}

template <bool SAFE>
__device__ __forceinline__ int ldq_fb_s(const uint32_t *__restrict__ s32, int64_t q, uint64_t wmax,
                                        uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	if constexpr (SAFE) {
		const u32x4a4 v = ld16(s32 + q);
		a = v.x; b = v.y; c = v.z; d = v.w;
		return 0;
	} else {
		return ldq_fb(s32, q, wmax, a, b, c, d);
	}
}

__device__ __forceinline__ void quad_fix_fb(int sft, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
	if (__ballot(sft != 0)) {        // only the reads at either end of the buffer
		asm volatile("");
		// new[s] = old[s + sft] where 0 <= s + sft <= 3 (the rest is outside the buffer)
		const uint32_t a0 = a, b0 = b, c0 = c, d0 = d;
		a = sft == 1 ? b0 : (sft == 2 ? c0 : (sft == 3 ? d0 : a0));
		b = sft == 1 ? c0 : (sft >= 2 ? d0 : (sft == -1 ? a0 : b0));
		c = sft == 1 ? d0 : (sft == -1 ? b0 : (sft <= -2 ? a0 : c0));
		d = sft == -1 ? c0 : (sft == -2 ? b0 : (sft == -3 ? a0 : d0));
	}
}

template <int K, int ABL = 0, bool SAFE = false>
__device__ __forceinline__ void scan_span_quad_fb(const VcKernelArgs &A, const uint32_t *__restrict__ s32,
                                                  uint64_t wmax, uint64_t off, int len, int nit,
                                                  const uint32_t *__restrict__ filt, WaveQueue &Q, uint32_t &tl,
                                                  int lane)
{
	static_assert(K >= VC_FLANK_MIN_K, "flank kernels only");
	if (nit == 0) return;
	Dir D;
	D.bwd = (lane & 1) != 0 && (A.variant & 256u) == 0;   // A.variant bit 8: all lanes forwards (A/B)
	D.mul = D.bwd ? 0x01041040u : 0x40100401u;
	D.sel13 = D.bwd ? 0x0C030C07u : 0x0C070C03u;
	D.inv = D.bwd ? 0xFFFFFFFFu : 0u;
	const int nt4m = -(int)A.nt4;
	const int tail_c = A.nt4 ? -1 : ((len & 15) ? (D.bwd ? 0 : (len >> 4)) : -1);
	const int tail_e = 16 - (len & 15);
	// forwards: chunk c at read bytes 16c..; backwards at len - 16c - 16..
	const int64_t a0 = D.bwd ? (int64_t)off + len - 16 : (int64_t)off;
	const int64_t x0 = a0 >> 2;                                      // floor, also below 0
	const uint32_t sh = (uint32_t)(a0 & 3);
	const int64_t qs = D.bwd ? -4 : 4;                               // dwords per chunk, signed
	int64_t qb = D.bwd ? x0 : x0 + 1;                                // quad of the window's first chunk
	uint32_t w[17];
	int d[4];
	{
		const int64_t w0i = D.bwd ? x0 + 4 : x0;
		const int64_t w0c = w0i < 0 ? 0 : ((uint64_t)w0i > wmax ? (int64_t)wmax : w0i);
		w[0] = s32[SAFE ? w0i : w0c];
	}
#pragma unroll
	for (int q = 0; q < 4; ++q)
		d[q] = ldq_fb_s<SAFE>(s32, qb + q * qs, wmax, w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], w[4 * q + 4]);
	uint32_t x0_ = 0, x1 = 0, x2 = 0, x3 = 0;
	int dx = ldq_fb_s<SAFE>(s32, qb + 4 * qs, wmax, x0_, x1, x2, x3);

	uint32_t Bm1 = 0, Bm2 = 0, H = 0;
	int U = 1 - K;
	int Qe = -len;
	// realigned dwords of window chunk i (quad order)
	auto quads = [&](int i, uint32_t &q0, uint32_t &q1, uint32_t &q2, uint32_t &q3) {
		const uint32_t G = D.bwd ? (i == 0 ? w[0] : w[4 * i - 3]) : w[4 * i + 1];
		const uint32_t Hh = D.bwd ? w[4 * i + 4] : w[4 * i];
		q0 = __builtin_amdgcn_alignbyte(G, Hh, sh);
		q1 = __builtin_amdgcn_alignbyte(w[4 * i + 2], w[4 * i + 1], sh);
		q2 = __builtin_amdgcn_alignbyte(w[4 * i + 3], w[4 * i + 2], sh);
		q3 = __builtin_amdgcn_alignbyte(w[4 * i + 4], w[4 * i + 3], sh);
	};
	// chunk 0 builds only the streams
	{
		quad_fix_fb(d[0], w[1], w[2], w[3], w[4]);
		uint32_t q0, q1, q2, q3;
		quads(0, q0, q1, q2, q3);
		packed_streams_fb<K, ABL>(A, D, 0, tail_c, nt4m, tail_e, q0, q1, q2, q3, Bm1, Bm2, U, Qe, H);
		const uint32_t e1 = D.bwd ? w[1] : w[4];                    // the fifth dword of chunk 1
#pragma unroll
		for (int i = 1; i < 13; ++i) w[i] = w[i + 4];
		w[0] = e1;
		w[13] = x0_; w[14] = x1; w[15] = x2; w[16] = x3;
		d[0] = d[1]; d[1] = d[2]; d[2] = d[3]; d[3] = dx;
		qb += qs;
	}
	if (nit == 1) return;            // wave-uniform
	int it = 1;
	auto chunk = [&](auto j1tag, int c, int i) {
		uint32_t q0, q1, q2, q3;
		quads(i, q0, q1, q2, q3);
		packed_chunk_fb<K, ABL, 0, decltype(j1tag)::value>(A, D, c, tail_c, nt4m, tail_e, q0, q1, q2, q3, Bm1, Bm2,
		                                                    U, Qe, H, filt, Q, tl, lane);
	};
	auto dchunk = [&](int c, int i) -> uint32_t {
		uint32_t q0, q1, q2, q3;
		quads(i, q0, q1, q2, q3);
		return packed_chunk_fb<K, ABL, 0, 16, true>(A, D, c, tail_c, nt4m, tail_e, q0, q1, q2, q3, Bm1, Bm2, U, Qe,
		                                            H, filt, Q, tl, lane);
	};
	for (; it + 4 < nit; it += 4) {
		uint32_t n[16];
		int dn[4];
#pragma unroll
		for (int q = 0; q < 4; ++q)
			dn[q] = ldq_fb_s<SAFE>(s32, qb + (4 + q) * qs, wmax, n[4 * q], n[4 * q + 1], n[4 * q + 2], n[4 * q + 3]);
#pragma unroll
		for (int q = 0; q < 4; ++q) quad_fix_fb(d[q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], w[4 * q + 4]);
#pragma unroll
		for (int p = 0; p < 2; ++p) {
			const uint32_t s2 = Bm2, s1 = Bm1;
			uint32_t h = dchunk(it + 2 * p, 2 * p);
			h = (h << 16) | dchunk(it + 2 * p + 1, 2 * p + 1);
			hit_loop2<K, ABL>(A, Q, h, s2, s1, Bm2, Bm1, lane);
		}
		w[0] = D.bwd ? w[13] : w[16];
#pragma unroll
		for (int i = 0; i < 16; ++i) w[i + 1] = n[i];
#pragma unroll
		for (int q = 0; q < 4; ++q) d[q] = dn[q];
		qb += 4 * qs;
	}
	// the last 1..4 chunks, all in w already (wave-uniform count)
#pragma unroll
	for (int q = 0; q < 4; ++q) quad_fix_fb(d[q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], w[4 * q + 4]);
	const int r = nit - it;
	if (r >= 2) chunk(J0Tag<16>{}, it, 0);
	if (r >= 3) chunk(J0Tag<16>{}, it + 1, 1);
	if (r >= 4) chunk(J0Tag<16>{}, it + 2, 2);
	// the wave's last chunk (window chunk r - 1): only its lower 8 windows when
	// no lane has more valid ones (see scan_span_packed)
	const int i = r - 1;
	if (i != 0) {
		const uint32_t e = D.bwd ? (i == 1 ? w[1] : (i == 2 ? w[5] : w[9])) : (i == 1 ? w[4] : (i == 2 ? w[8] : w[12]));
		w[1] = i == 1 ? w[5] : (i == 2 ? w[9] : w[13]);
		w[2] = i == 1 ? w[6] : (i == 2 ? w[10] : w[14]);
		w[3] = i == 1 ? w[7] : (i == 2 ? w[11] : w[15]);
		w[4] = i == 1 ? w[8] : (i == 2 ? w[12] : w[16]);
		w[0] = e;
	}
	const int cl = nit - 1;
	if ((A.variant & 4u) == 0 && __ballot(len - 16 * cl > 8) == 0)
		chunk(J0Tag<8>{}, cl, 0);
	else
		chunk(J0Tag<16>{}, cl, 0);
}

// k in 16..31 with a compile-time specialisation: packed streams (the quad
// loop unless A.variant bit 3 or a memory ablation); otherwise the general
// rolling scan.
template <int K, bool HAS_LO, int ABL = 0, bool SAFE = false>
__device__ __forceinline__ void scan_any(const VcKernelArgs &A, const uint32_t *__restrict__ s32,
                                         uint64_t wmax, uint64_t off, int len, int c_lo, int c_hi,
                                         int vlo, int vhi, int nit, const uint32_t *__restrict__ filt,
                                         WaveQueue &Q, uint32_t &tl, int lane)
{
	if constexpr (K >= VC_FLANK_MIN_K && (ABL & VC_KV_FLANK) != 0 && !HAS_LO && (ABL & (2 | 8 | 16 | 32)) == 0) {
		// flank kernels, whole reads, -DVC_SCAN_BWD: odd lanes scan backwards
		// (A/B only: same time as every lane forwards in the same code, and that
		// code is 10 % slower than the quad loop)
		if constexpr (VC_SCAN_FB) {
			scan_span_quad_fb<K, ABL, SAFE>(A, s32, wmax, off, len, nit, filt, Q, tl, lane);
			return;
		}
	}
	if constexpr (K >= 16) {
		if constexpr ((ABL & (2 | 8 | 16)) == 0) {
#ifdef VC_ABLATION
			if ((A.variant & 8u) == 0)   // ablation builds: A.variant bit 3 = the pair loop
#endif
			{
				scan_span_quad<K, HAS_LO, ABL, SAFE>(A, s32, wmax, off, len, c_lo, vlo, vhi, nit, filt, Q, tl, lane);
				return;
			}
		}
		scan_span_packed<K, HAS_LO, ABL, SAFE>(A, s32, wmax, off, len, c_lo, c_hi, vlo, vhi, nit, filt, Q, tl,
		                                       lane);
	} else
		scan_span<K, HAS_LO, ABL>(A, s32, wmax, off, len, c_lo, c_hi, vlo, vhi, nit, filt, Q, tl, lane);
}

__device__ __forceinline__ void load_filter(const VcKernelArgs &A, uint32_t *filt)
{
	const uint32_t nw = A.fwords;        // a multiple of 4
	const uint4 *src = reinterpret_cast<const uint4 *>(A.filter);
	uint4 *dst = reinterpret_cast<uint4 *>(filt);
	for (uint32_t i = threadIdx.x; i < nw / 4u; i += blockDim.x) dst[i] = src[i];
	if (threadIdx.x < 4) filt[nw + threadIdx.x] = 0u;     // the zero word(s)
	// flank_bits_u8 addresses the filter from LDS address 0 (the kernels have
	// no static LDS, so the dynamic array starts there; folds at compile time)
	if (lds_base(filt) != 0u) __builtin_trap();
	__syncthreads();
}

// ---------------------------------------------------------------------------
// kernel 1: whole reads, one lane per read
// ---------------------------------------------------------------------------

template <int K, int ABL = 0>
__global__ void __launch_bounds__(VC_BLOCK)
vc_count_reads_kernel(VcKernelArgs A)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	uint32_t *filt = smem;
	const int lane = threadIdx.x & (WAVE - 1);
	const int wave = threadIdx.x / WAVE;
	WaveQueue Q;
	Q.q = reinterpret_cast<uint64_t *>(smem + vc_filter_lds_words(A.fwords)) + wave * A.qcap;
	Q.n = 0;
	Q.pend = false;
	load_filter(A, filt);

	const uint32_t *s32 = reinterpret_cast<const uint32_t *>(A.seq);
	const uint64_t wmax = A.seq_words ? A.seq_words - 1 : 0;
	unsigned long long tally = 0;

	// The lengths and offsets of the next read group are requested before
	// this group is scanned (one load each, index clamped, so the compiler's
	// count of loads in flight stays exact) and used after its queue drain.
	const uint64_t rlast = A.n_reads - 1;
	uint64_t g = blockIdx.x;
	uint64_t r = g * (uint64_t)VC_BLOCK + threadIdx.x;
	uint32_t len_raw = A.lens[r < rlast ? r : rlast];
	uint64_t off_raw = A.offs[r < rlast ? r : rlast];
	while (g * (uint64_t)VC_BLOCK < A.n_reads) {
		int len = r < A.n_reads ? (int)len_raw : 0;
		const uint64_t off = off_raw + A.off_adj;
		if ((uint32_t)len > VC_LONG_READ) {
			const uint32_t slot = atomicAdd(A.nlong, 1u);
			if (slot < A.long_cap) A.longlist[slot] = (uint32_t)r;
			len = 0;
		}
		const uint64_t gn = g + gridDim.x;
		const uint64_t rn = gn * (uint64_t)VC_BLOCK + threadIdx.x;
		len_raw = A.lens[rn < rlast ? rn : rlast];
		off_raw = A.offs[rn < rlast ? rn : rlast];
		const int nch = (len + 15) >> 4;
		const int nit = wave_max_i32(nch);
		uint32_t tl = 0;
		// the packed scan loads dwords [off/4, off/4 + 8 ceil(nit/2) + 13) (lanes
		// past their span keep loading); groups clear of the buffer end skip the
		// per-load clamping
		bool clear = (off >> 2) + 8u * (uint64_t)((nit + 1) >> 1) + 13u <= wmax;
		if constexpr ((ABL & VC_KV_FLANK) != 0) {
			// backward lanes (scan_span_quad_fb) load dwords down to
			// (off + len - 16) / 4 - 4 (nit + 2) and up to (off + len) / 4
			const int64_t xb = ((int64_t)off + len - 16) >> 2;
			clear = clear && xb - 4 * (int64_t)(nit + 6) >= 0 && (uint64_t)(xb + 4) <= wmax;
		}
		if (K >= 16 && __builtin_amdgcn_ballot_w64(!clear) == 0)
			scan_any<K, false, ABL, true>(A, s32, wmax, off, len, 0, nch, 0, len, nit, filt, Q, tl, lane);
		else
			scan_any<K, false, ABL>(A, s32, wmax, off, len, 0, nch, 0, len, nit, filt, Q, tl, lane);
		tally += tl;
		// drain at a group end only once the queue holds more than 112 entries
		// (two per lane): each drain exposes one probe latency, so fewer, fuller
		// drains cost less (C2: -1.6 %, C5: +-0; ABL 64 = a drain per group)
		if constexpr ((ABL & 64) != 0) queue_flush<ABL>(A, Q, lane);
		else if ((int)Q.n > (int)A.qcap - 2 * WAVE) queue_flush<ABL>(A, Q, lane);
		g = gn;
		r = rn;
	}
	queue_flush<ABL>(A, Q, lane);
	const unsigned long long t = wave_sum_u64(tally);
	if (lane == 0 && t) atomicAdd(A.tally, t);
}

// ---------------------------------------------------------------------------
// kernel 2: long reads, every lane of the grid takes one segment
// ---------------------------------------------------------------------------

template <int K, int ABL = 0>
__global__ void __launch_bounds__(VC_BLOCK)
vc_count_long_kernel(VcKernelArgs A)
{
	const uint32_t nl_raw = *A.nlong;
	const uint32_t nl = nl_raw < A.long_cap ? nl_raw : A.long_cap;
	if (nl_raw > A.long_cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(A.flags, 1u);   // reported by vc_finish
	if (nl == 0) return;   // uniform over the grid
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	uint32_t *filt = smem;
	const int lane = threadIdx.x & (WAVE - 1);
	const int wave = threadIdx.x / WAVE;
	WaveQueue Q;
	Q.q = reinterpret_cast<uint64_t *>(smem + vc_filter_lds_words(A.fwords)) + wave * A.qcap;
	Q.n = 0;
	Q.pend = false;
	load_filter(A, filt);

	const uint32_t *s32 = reinterpret_cast<const uint32_t *>(A.seq);
	const uint64_t wmax = A.seq_words ? A.seq_words - 1 : 0;
	const int k = K ? K : A.k;
	unsigned long long tally = 0;
	const uint64_t stride = (uint64_t)gridDim.x * VC_BLOCK;

	for (uint32_t li = 0; li < nl; ++li) {
		const uint32_t r = A.longlist[li];
		const int len = (int)A.lens[r];
		const uint64_t off = A.offs[r] + A.off_adj;
		const uint64_t nseg = ((uint64_t)len + VC_LONG_SEG - 1) / VC_LONG_SEG;
		for (uint64_t s0 = (uint64_t)blockIdx.x * VC_BLOCK; s0 < nseg; s0 += stride) {
			const uint64_t s = s0 + threadIdx.x;
			int vlo = 0, vhi = 0, c_lo = 0, c_hi = 0;
			if (s < nseg) {
				const int64_t e0 = (int64_t)s * VC_LONG_SEG;
				const int64_t e1 = e0 + VC_LONG_SEG < len ? e0 + VC_LONG_SEG : len;
				vlo = (int)(e0 - (k - 1) > 0 ? e0 - (k - 1) : 0);
				vhi = (int)e1;
				c_lo = vlo >> 4;
				c_hi = (vhi + 15) >> 4;
			}
			const int nit = wave_max_i32(c_hi - c_lo);
			uint32_t tl = 0;
			scan_any<K, true, ABL>(A, s32, wmax, off, len, c_lo, c_hi, vlo, vhi, nit, filt, Q, tl, lane);
			tally += tl;
		}
	}
	queue_flush<ABL>(A, Q, lane);
	const unsigned long long t = wave_sum_u64(tally);
	if (lane == 0 && t) atomicAdd(A.tally, t);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------

template <int K, int ABL = 0>
static hipError_t launch_kw(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	const size_t lds = vc_lds_bytes(A->fwords, A->qcap);
	hipLaunchKernelGGL((vc_count_reads_kernel<K, ABL>), dim3(grid), dim3(VC_BLOCK), lds, st, *A);
	hipError_t e = hipGetLastError();
	if (e != hipSuccess || grid_long <= 0) return e;   // grid_long 0: the host knows there is no long read
	hipLaunchKernelGGL((vc_count_long_kernel<K, ABL & (VC_KV_FLANK | VC_KV_BIG)>), dim3(grid_long), dim3(VC_BLOCK),
	                   lds, st, *A);
	return hipGetLastError();
}

#ifdef VC_ABLATION
#ifdef VC_ABL_SHORT   // the drain decomposition only (compiles in a fraction of the time)
#define VC_ABL_LIST(X) X(1) X(2) X(4) X(7) X(1024) X(2048) X(4096)
#else
#define VC_ABL_LIST(X) X(1) X(2) X(4) X(3) X(5) X(6) X(7) X(8) X(12) X(16) X(20) X(64) X(1024) X(2048) X(4096)
#endif
#endif

template <int K>
static hipError_t launch_k_impl(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
#ifdef VC_ABLATION
	if constexpr (K == 21) {
		if (A->ablate) switch (A->ablate) {
#define VC_ABL_CASE(n)                                                                          \
	case n:                                                                                     \
		return A->flank ? launch_kw<21, n | VC_KV_FLANK>(A, grid, grid_long, st)                \
		     : A->big   ? launch_kw<21, n | VC_KV_BIG>(A, grid, grid_long, st)                  \
		                : launch_kw<21, n>(A, grid, grid_long, st);
			VC_ABL_LIST(VC_ABL_CASE)
#undef VC_ABL_CASE
		default: break;
		}
	}
#endif
	if constexpr (K >= VC_FLANK_MIN_K) {
		if (A->flank) return launch_kw<K, VC_KV_FLANK>(A, grid, grid_long, st);
		if (A->big) return launch_kw<K, VC_KV_BIG>(A, grid, grid_long, st);
	}
	return launch_kw<K>(A, grid, grid_long, st);
}

template <int K>
static hipError_t setup_k_impl(int lds)
{
	hipError_t e = hipFuncSetAttribute((const void *)vc_count_reads_kernel<K>,
	                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds);
	if (e == hipSuccess)
		e = hipFuncSetAttribute((const void *)vc_count_long_kernel<K>,
		                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
	if constexpr (K >= VC_FLANK_MIN_K) {
		if (e == hipSuccess)
			e = hipFuncSetAttribute((const void *)vc_count_reads_kernel<K, VC_KV_FLANK>,
			                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
		if (e == hipSuccess)
			e = hipFuncSetAttribute((const void *)vc_count_long_kernel<K, VC_KV_FLANK>,
			                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
		if (e == hipSuccess)
			e = hipFuncSetAttribute((const void *)vc_count_reads_kernel<K, VC_KV_BIG>,
			                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
		if (e == hipSuccess)
			e = hipFuncSetAttribute((const void *)vc_count_long_kernel<K, VC_KV_BIG>,
			                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
	}
#ifdef VC_ABLATION
	if constexpr (K == 21) {
#define VC_ABL_SET(n)                                                                           \
	if (e == hipSuccess)                                                                        \
		e = hipFuncSetAttribute((const void *)vc_count_reads_kernel<21, n>,                     \
		                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);               \
	if (e == hipSuccess)                                                                        \
		e = hipFuncSetAttribute((const void *)vc_count_reads_kernel<21, n | VC_KV_FLANK>,       \
		                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);               \
	if (e == hipSuccess)                                                                        \
		e = hipFuncSetAttribute((const void *)vc_count_reads_kernel<21, n | VC_KV_BIG>,         \
		                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
		VC_ABL_LIST(VC_ABL_SET)
#undef VC_ABL_SET
	}
#endif
	return e;
}

// Development builds of kernel variants (tools/ab_libs.sh, never the product):
// -DVC_DEV_ONLY=21 [-DVC_DEV_ONLY2=31] instantiates the packed kernels of
// those k only (k < 16 keeps the run-time-k kernel), so an A/B library builds
// in a minute instead of compiling all sixteen; other k fail to launch.
#ifndef VC_DEV_ONLY2
#define VC_DEV_ONLY2 VC_DEV_ONLY
#endif
template <int K>
static hipError_t launch_k(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
#ifdef VC_DEV_ONLY
	if constexpr (K != 0 && K != VC_DEV_ONLY && K != VC_DEV_ONLY2) return hipErrorNotSupported;
	else
#endif
		return launch_k_impl<K>(A, grid, grid_long, st);
}

template <int K>
static hipError_t setup_k(int lds)
{
#ifdef VC_DEV_ONLY
	if constexpr (K != 0 && K != VC_DEV_ONLY && K != VC_DEV_ONLY2) return hipSuccess;
	else
#endif
		return setup_k_impl<K>(lds);
}

#endif
