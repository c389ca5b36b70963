// vafc_gzip.cpp -- see vafc_gzip.h.
//
// Deflate (RFC 1951) and gzip (RFC 1952) are restated here from the formats;
// zlib (the reference's gzread, pinned by the system package) remains the
// decoder of record for every chunk whose speculative decode is not used.
#include "vafc_gzip.h"
#include "vafc.h"
#include "vafc_affinity.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <immintrin.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <time.h>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace {

double gz_now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}
std::atomic<uint64_t> prof_search_us{0}, prof_decode_us{0}, prof_resolve_us{0}, prof_crc_us{0};
// waits (VAFC_GZ_PROFILE): workers idle, the sequencer waiting for the next
// chunk / for queue room, the reader waiting for the next piece
std::atomic<uint64_t> prof_widle_us{0}, prof_seqwait_us{0}, prof_seqpush_us{0}, prof_rdwait_us{0};

constexpr uint32_t WSIZE = 32768;             // deflate history
constexpr uint16_t MARK = 0x8000;             // symbol = MARK | window index
constexpr size_t OUT_CAP = (size_t)64 << 20;  // symbols per speculative chunk
constexpr size_t PIECE_CAP = (size_t)16 << 20;  // bytes per zlib-fallback piece

inline uint32_t le32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

// ---------------------------------------------------------------------------
// bit input: LSB-first, 64-bit buffer refilled with whole unaligned words
// (the bits above `cnt` are always either zero or the true next bits)
// ---------------------------------------------------------------------------
struct BitIn {
	const uint8_t *p = nullptr;
	uint64_t n = 0;       // input bytes
	uint64_t pos = 0;     // next byte to load
	uint64_t buf = 0;
	unsigned cnt = 0;     // valid bits in buf

	void init(const uint8_t *p_, uint64_t n_, uint64_t bitoff)
	{
		p = p_;
		n = n_;
		pos = bitoff >> 3;
		buf = 0;
		cnt = 0;
		refill();
		drop((unsigned)(bitoff & 7));
	}
	inline void refill()
	{
		if (__builtin_expect(pos + 8 <= n, 1)) {
			uint64_t w;
			memcpy(&w, p + pos, 8);
			buf |= w << cnt;
			pos += (63 - cnt) >> 3;
			cnt |= 56;
		} else {
			while (cnt <= 56) {
				const uint64_t b = pos < n ? p[pos] : 0;
				buf |= b << cnt;
				++pos;
				cnt += 8;
			}
		}
	}
	inline uint64_t bitpos() const { return pos * 8 - cnt; }
	inline bool overrun() const { return bitpos() > n * 8; }
	inline void drop(unsigned k)
	{
		buf >>= k;
		cnt -= k;
	}
	inline uint32_t take(unsigned k)
	{
		const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1));
		drop(k);
		return v;
	}
};

// ---------------------------------------------------------------------------
// Huffman decoding tables.  Entry: bits 0-7 bits to consume, 8-12 extra bits
// (or sub-table index bits), 13-15 kind, 16-31 value.  A length or distance
// entry consumes its code AND its extra bits in one shift; the extra bits are
// read from the bit buffer before it (at the code length, bits - extra), so
// the next table lookup waits for one shift instead of two.
// ---------------------------------------------------------------------------
// K_LIT2: two literals in one literal/length table entry (value = first |
// second << 8, length = both codes): DNA literals have 2-3-bit codes, so most
// 11-bit lookups of FASTQ sequence text decode a pair.
enum : uint32_t { K_LIT = 0, K_LIT2 = 1, K_LEN = 2, K_EOB = 3, K_SUB = 4, K_BAD = 5 };
inline uint32_t mk(uint32_t len, uint32_t ext, uint32_t kind, uint32_t val)
{
	return len | ext << 8 | kind << 13 | val << 16;
}
inline uint32_t e_len(uint32_t e) { return e & 0xff; }
inline uint32_t e_ext(uint32_t e) { return (e >> 8) & 31; }
inline uint32_t e_kind(uint32_t e) { return (e >> 13) & 7; }
inline uint32_t e_val(uint32_t e) { return e >> 16; }

const uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
                            131, 163, 195, 227, 258};
const uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025,
                            1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12,
                          13, 13};
const uint8_t CL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

constexpr unsigned LROOT = 11, DROOT = 8, CROOT = 7;
constexpr size_t LTAB = (1u << LROOT) + 288 * 16;
constexpr size_t DTAB = (1u << DROOT) + 32 * 128;

enum Code { C_CL, C_LIT, C_DIST };

inline uint32_t sym_entry(Code c, unsigned s, unsigned len)
{
	if (c == C_LIT) {
		if (s < 256) return mk(len, 0, K_LIT, s);
		if (s == 256) return mk(len, 0, K_EOB, 0);
		if (s <= 285) return mk(len + LEXT[s - 257], LEXT[s - 257], K_LEN, LBASE[s - 257]);   // length: code + extra bits
		return mk(len, 0, K_BAD, 0);
	}
	if (c == C_DIST) return s < 30 ? mk(len + DEXT[s], DEXT[s], K_LIT, DBASE[s]) : mk(len, 0, K_BAD, 0);
	return mk(len, 0, K_LIT, s);
}

inline unsigned rev(unsigned x, unsigned n)
{
	unsigned r = 0;
	for (unsigned i = 0; i < n; ++i) r |= ((x >> i) & 1) << (n - 1 - i);
	return r;
}

// zlib's acceptance rules (inflate_table): over-subscribed codes are errors;
// an incomplete code-length code is an error; an incomplete literal/length or
// distance code is accepted only when its longest code has length 1; a code
// with no symbols at all is accepted (decoding from it is the error).
bool build(uint32_t *T, unsigned root, const uint8_t *lens, unsigned n, Code c)
{
	unsigned count[16] = {0};
	for (unsigned i = 0; i < n; ++i) count[lens[i]]++;
	count[0] = 0;
	unsigned maxlen = 15;
	while (maxlen && !count[maxlen]) --maxlen;
	const uint32_t bad = mk(1, 0, K_BAD, 0);
	for (unsigned i = 0; i < (1u << root); ++i) T[i] = bad;
	if (maxlen == 0) return c != C_CL;
	int left = 1;
	for (unsigned l = 1; l <= 15; ++l) {
		left <<= 1;
		left -= (int)count[l];
		if (left < 0) return false;
	}
	if (left > 0 && (c == C_CL || maxlen != 1)) return false;
	unsigned offs[16];
	offs[1] = 0;
	for (unsigned l = 1; l < 15; ++l) offs[l + 1] = offs[l] + count[l];
	uint16_t sorted[320];
	for (unsigned s = 0; s < n; ++s)
		if (lens[s]) sorted[offs[lens[s]]++] = (uint16_t)s;
	unsigned code = 0, idx = 0;
	const unsigned short_max = maxlen < root ? maxlen : root;
	for (unsigned l = 1; l <= short_max; ++l) {
		for (unsigned c2 = 0; c2 < count[l]; ++c2) {
			const unsigned s = sorted[idx++];
			const uint32_t e = sym_entry(c, s, l);
			for (unsigned k = rev(code, l); k < (1u << root); k += 1u << l) T[k] = e;
			++code;
		}
		code <<= 1;
	}
	if (maxlen <= root) return true;
	// longer codes: one sub-table per root prefix, sized for its longest code
	uint8_t ml[1u << LROOT];
	{
		unsigned cc = code;
		for (unsigned l = root + 1; l <= maxlen; ++l) {
			for (unsigned c2 = 0; c2 < count[l]; ++c2) ml[cc >> (l - root)] = (uint8_t)l, ++cc;
			cc <<= 1;
		}
	}
	unsigned next_sub = 1u << root, cur = ~0u, sub = 0, sbits = 0;
	for (unsigned l = root + 1; l <= maxlen; ++l) {
		for (unsigned c2 = 0; c2 < count[l]; ++c2) {
			const unsigned s = sorted[idx++];
			const unsigned pre = code >> (l - root);
			if (pre != cur) {
				cur = pre;
				sbits = ml[pre] - root;
				sub = next_sub;
				next_sub += 1u << sbits;
				for (unsigned i = 0; i < (1u << sbits); ++i) T[sub + i] = bad;
				T[rev(pre, root)] = mk(root, sbits, K_SUB, sub);
			}
			const unsigned lo = l - root;
			const uint32_t e = sym_entry(c, s, l);
			for (unsigned k = rev(code & ((1u << lo) - 1), lo); k < (1u << sbits); k += 1u << lo) T[sub + k] = e;
			++code;
		}
		code <<= 1;
	}
	return true;
}

// Literal/length root table: entries whose code leaves room for a second
// literal code within the root bits become K_LIT2 pairs.  The next code's
// entry is looked up on the bits after the first code (the higher root bits
// are unknown, so it must fit in the known ones).
void pair_literals(uint32_t *T, unsigned root)
{
	static thread_local uint32_t single[1u << LROOT];
	memcpy(single, T, ((size_t)1 << root) * sizeof(uint32_t));
	for (unsigned i = 0; i < (1u << root); ++i) {
		const uint32_t e = single[i];
		if (e_kind(e) != K_LIT) continue;
		const unsigned l1 = e_len(e);
		if (l1 >= root) continue;
		const uint32_t e2 = single[i >> l1];
		if (e_kind(e2) != K_LIT || e_len(e2) > root - l1) continue;
		T[i] = mk(l1 + e_len(e2), 0, K_LIT2, e_val(e) | e_val(e2) << 8);
	}
}

struct Tables {
	uint32_t lit[LTAB];
	uint32_t dist[DTAB];
};

const Tables &fixed_tables()
{
	static Tables *t = [] {
		Tables *f = new Tables;
		uint8_t l[288];
		for (int i = 0; i < 288; ++i) l[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
		build(f->lit, LROOT, l, 288, C_LIT);
		pair_literals(f->lit, LROOT);
		uint8_t d[32];
		memset(d, 5, sizeof d);
		build(f->dist, DROOT, d, 32, C_DIST);
		return f;
	}();
	return *t;
}

// Dynamic block header (RFC 1951 3.2.7) into T; false where zlib reports an error.
bool read_dynamic(BitIn &in, Tables &T)
{
	in.refill();
	const unsigned hlit = in.take(5) + 257, hdist = in.take(5) + 1, hclen = in.take(4) + 4;
	if (hlit > 286 || hdist > 30) return false;
	uint8_t cl[19] = {0};
	for (unsigned i = 0; i < hclen; ++i) {
		if (in.cnt < 3) in.refill();
		cl[CL_ORDER[i]] = (uint8_t)in.take(3);
	}
	uint32_t ct[1u << CROOT];
	if (!build(ct, CROOT, cl, 19, C_CL)) return false;
	uint8_t lens[320];
	unsigned i = 0;
	const unsigned total = hlit + hdist;
	while (i < total) {
		in.refill();
		const uint32_t e = ct[in.buf & ((1u << CROOT) - 1)];
		if (e_kind(e) == K_BAD) return false;
		in.drop(e_len(e));
		const unsigned s = e_val(e);
		if (s < 16) {
			lens[i++] = (uint8_t)s;
			continue;
		}
		unsigned rep;
		uint8_t v = 0;
		if (s == 16) {
			if (i == 0) return false;
			v = lens[i - 1];
			rep = 3 + in.take(2);
		} else if (s == 17) {
			rep = 3 + in.take(3);
		} else {
			rep = 11 + in.take(7);
		}
		if (i + rep > total) return false;
		memset(lens + i, v, rep);
		i += rep;
	}
	if (in.overrun() || lens[256] == 0) return false;
	if (!build(T.lit, LROOT, lens, hlit, C_LIT) || !build(T.dist, DROOT, lens + hlit, hdist, C_DIST)) return false;
	pair_literals(T.lit, LROOT);
	return true;
}

// ---------------------------------------------------------------------------
// speculative output.  Phase 1 writes 16-bit symbols: MARK | i names byte i
// of the 32 KiB window that precedes the chunk (i = 32768 - distance before
// the start).  Once the last 32 KiB of symbols hold no marker, no later
// back-reference can reach one, so phase 2 writes plain bytes: t[] is indexed
// by output position, its first `res` bytes are filled in later by resolving
// s[0..res) against the window, the rest are final when written.
// ---------------------------------------------------------------------------
// Large output buffers are backed by transparent huge pages where the kernel
// allows it (THP "madvise" mode): a chunk writes tens of MB into freshly
// grown buffers, and 4 KiB first-touch faults from many workers at once cost
// more than the decoding (VAFC_GZ_NOHUGE=1 turns this off, A/B).
const bool gz_huge = getenv("VAFC_GZ_NOHUGE") == nullptr;
void advise_huge(void *p, size_t n)
{
	if (!gz_huge) return;
	const uintptr_t H = (uintptr_t)2 << 20;
	const uintptr_t a = ((uintptr_t)p + H - 1) & ~(H - 1), b = ((uintptr_t)p + n) & ~(H - 1);
	if (b > a) madvise((void *)a, (size_t)(b - a), MADV_HUGEPAGE);
}

struct Out {
	uint16_t *s = nullptr;             // phase 1 symbols
	size_t ns = 0, caps = 0;
	uint8_t *t = nullptr;              // text by output position (phase 2)
	size_t nt = 0, capt = 0;
	bool wide = true;                  // in phase 1
	size_t res = 0;                    // t[0..res) still to be resolved from s
	int64_t floor = -(int64_t)WSIZE;   // lowest output index a back-reference may reach
	uint32_t min_mark = WSIZE;         // lowest window index referenced
	int64_t last_mark = -1;            // highest output index that may hold a marker
	~Out()
	{
		free(s);
		free(t);
	}
	size_t total() const { return wide ? ns : nt; }
	// bytes written (the buffers' caps are address space, faulted in as
	// written), with a huge page of slack for each
	size_t held() const { return ns * sizeof(uint16_t) + nt + ((size_t)4 << 20); }
	void release_buffers()
	{
		free(s);
		free(t);
		s = nullptr;
		t = nullptr;
		ns = nt = caps = capt = res = 0;
	}
	void reset(bool known_history)
	{
		ns = nt = res = 0;
		min_mark = WSIZE;
		last_mark = -1;
		floor = known_history ? 0 : -(int64_t)WSIZE;
		wide = !known_history;
	}
	static bool grow_buf(void **p, size_t *cap, size_t need, size_t elem)
	{
		if (need > OUT_CAP + 4096) return false;
		// the whole cap at once: beyond the mmap threshold, so the pages are
		// faulted in as written and nothing is ever copied by a regrow (a
		// chain of reallocs from 1 MiB cost as much as the decode for chunks
		// in fresh buffers, as a held share's are)
		size_t nc = *cap ? *cap : OUT_CAP + 4096;
		while (nc < need) nc *= 2;
		void *q = realloc(*p, nc * elem);
		if (!q) return false;
		advise_huge(q, nc * elem);
		*p = q;
		*cap = nc;
		return true;
	}
	bool room(size_t k)
	{
		if (wide) return caps - ns >= k || grow_buf((void **)&s, &caps, ns + k, 2);
		return capt - nt >= k || grow_buf((void **)&t, &capt, nt + k, 1);
	}
	// phase 1 -> 2: the last 32 KiB of symbols are literal bytes
	bool narrow()
	{
		if (capt < ns + 600 && !grow_buf((void **)&t, &capt, ns + ((size_t)1 << 20), 1)) return false;
		const size_t h = ns < WSIZE ? ns : WSIZE;
		for (size_t i = ns - h; i < ns; ++i) t[i] = (uint8_t)s[i];
		res = ns - h;
		nt = ns;
		wide = false;
		return true;
	}
	// end of chunk: everything not yet in t is resolved later
	bool finish()
	{
		if (!wide) return true;
		if (capt < ns + 64 && !grow_buf((void **)&t, &capt, ns + 64, 1)) return false;
		res = ns;
		nt = ns;
		return true;
	}
};

inline void copy_match8(uint8_t *dst, unsigned dist, unsigned len)
{
	const uint8_t *s = dst - dist;
	if (dist >= 16) {
		for (unsigned i = 0; i < len; i += 16) memcpy(dst + i, s + i, 16);
	} else if (dist >= 8) {
		for (unsigned i = 0; i < len; i += 8) memcpy(dst + i, s + i, 8);
	} else if (dist == 1) {
		memset(dst, s[0], len);
	} else {
		for (unsigned i = 0; i < len; ++i) dst[i] = s[i];
	}
}

// One Huffman-coded block body up to its end-of-block code.  Returns 1 at
// the end of the block, 0 on an error, 2 (phase 1 only) when the output has
// just switched to phase 2 and the block continues there.
//
// Phase 1, a match whose source is output (src >= 0) at distance >= 8: the
// first 16 symbols are copied unconditionally (two 16-byte moves; longer
// matches continue 8 at a time) and ORed to see whether a marker came along.
// Level-1 FASTQ is almost all matches (8 symbols on average, 85 % of them
// from a source that may hold markers: profiles/r03_gz_symbols.log), and the
// branches on the length and on the source's markers were the loop's
// unpredictable ones: +12 % on one thread of the box
// (profiles/r03_gz_ab_cp16.log).  The look may see up to 15 symbols past the
// source range, all of them output already: it can only move last_mark up,
// which is safe (it delays phase 2).  The same loop with the reader and the
// cursor in locals was 12 % slower on the box
// (profiles/r03_gz_ab_decoder_locals.log).
template <bool WIDE>
int decode_huff(BitIn &in, const Tables &T, Out &o)
{
	for (;;) {
		if (WIDE) {
			if (__builtin_expect((int64_t)o.ns - o.last_mark > (int64_t)WSIZE, 0)) return o.narrow() ? 2 : 0;
			if (__builtin_expect(o.caps - o.ns < 600, 0) && !o.room(600)) return 0;
		} else {
			if (__builtin_expect(o.capt - o.nt < 600, 0) && !o.room(600)) return 0;
		}
		if (__builtin_expect(in.pos > in.n + 16, 0)) return 0;
		in.refill();
		uint32_t e = T.lit[in.buf & ((1u << LROOT) - 1)];
		if (e_kind(e) == K_SUB) e = T.lit[e_val(e) + ((in.buf >> LROOT) & ((1u << e_ext(e)) - 1))];
		const uint64_t b0 = in.buf;   // a length's extra bits are read from here
		in.drop(e_len(e));
		if (e_kind(e) <= K_LIT2) {
			// one or two literals per entry, written as a pair (the second
			// slot of a single literal is overwritten next); up to three more
			// root entries without a refill: >= 56 bits after it, the first
			// code <= 15 bits, root literal entries <= 11 bits, and every
			// lookup has >= 11 valid bits
			size_t n = WIDE ? o.ns : o.nt;
			auto put = [&](uint32_t x) {
				const uint32_t v = e_val(x);
				if (WIDE) {
					o.s[n] = (uint16_t)(v & 0xFFu);
					o.s[n + 1] = (uint16_t)(v >> 8);
				} else {
					const uint16_t v16 = (uint16_t)v;
					memcpy(o.t + n, &v16, 2);
				}
				n += 1u + e_kind(x);
			};
			put(e);
#pragma GCC unroll 3
			for (int x = 0; x < 3; ++x) {
				const uint32_t e2 = T.lit[in.buf & ((1u << LROOT) - 1)];
				if (e_kind(e2) > K_LIT2) break;
				in.drop(e_len(e2));
				put(e2);
			}
			if (WIDE) o.ns = n;
			else o.nt = n;
			continue;
		}
		if (e_kind(e) == K_EOB) return in.overrun() ? 0 : 1;
		if (e_kind(e) != K_LEN) return 0;
		const unsigned lx = e_ext(e);
		const unsigned len = e_val(e) + (unsigned)((b0 >> (e_len(e) - lx)) & ((1u << lx) - 1));
		uint32_t d = T.dist[in.buf & ((1u << DROOT) - 1)];
		if (e_kind(d) == K_SUB) d = T.dist[e_val(d) + ((in.buf >> DROOT) & ((1u << e_ext(d)) - 1))];
		if (e_kind(d) == K_BAD) return 0;
		const uint64_t b1 = in.buf;
		in.drop(e_len(d));
		const unsigned dx = e_ext(d);
		const unsigned dist = e_val(d) + (unsigned)((b1 >> (e_len(d) - dx)) & ((1u << dx) - 1));
		if (!WIDE) {   // every source byte lies in t[nt - 32768, nt): literal text
			if ((int64_t)o.nt - (int64_t)dist < o.floor) return 0;
			copy_match8(o.t + o.nt, dist, len);
			o.nt += len;
			continue;
		}
		const int64_t src = (int64_t)o.ns - (int64_t)dist;
		uint16_t *dst = o.s + o.ns;
		if (__builtin_expect(src >= 0 && dist >= 8, 1)) {
			// 8 symbols per step, in order, each from a source that ends
			// before the step's destination starts (dist >= 8)
			const uint16_t *q = dst - dist;
			uint64_t a, b, c, f;
			memcpy(&a, q, 8);
			memcpy(&b, q + 4, 8);
			memcpy(dst, &a, 8);
			memcpy(dst + 4, &b, 8);
			memcpy(&c, q + 8, 8);
			memcpy(&f, q + 12, 8);
			memcpy(dst + 8, &c, 8);
			memcpy(dst + 12, &f, 8);
			uint64_t acc = a | b | c | f;
			for (unsigned i = 16; i < len; i += 8) {
				memcpy(&a, q + i, 8);
				memcpy(&b, q + i + 4, 8);
				memcpy(dst + i, &a, 8);
				memcpy(dst + i + 4, &b, 8);
				acc |= a | b;
			}
			const int64_t lm = (int64_t)o.ns + len - 1;
			o.last_mark = (acc & 0x8000800080008000ull) ? lm : o.last_mark;
		} else if (src >= 0) {
			const uint16_t *q = dst - dist;
			uint16_t acc = 0;
			for (unsigned i = 0; i < len; ++i) {
				const uint16_t v = q[i];
				dst[i] = v;
				acc |= v;
			}
			if (acc & MARK) o.last_mark = (int64_t)o.ns + len - 1;
		} else {
			if (src < o.floor) return 0;   // before the member's first byte
			const uint32_t m = (uint32_t)(src + WSIZE);
			if (m < o.min_mark) o.min_mark = m;
			for (unsigned i = 0; i < len; ++i) {
				const int64_t si = src + (int64_t)i;
				dst[i] = si < 0 ? (uint16_t)(MARK | (uint32_t)(si + WSIZE)) : o.s[si];
			}
			o.last_mark = (int64_t)o.ns + len - 1;
		}
		o.ns += len;
	}
}

// decode_huff<false> with the bit reader and the output cursor in locals:
// stores through the byte pointer may alias any memory, so fields of `in` and
// `o` would otherwise be reloaded after every literal written.  Same results.
int decode_huff_narrow(BitIn &in, const Tables &T, Out &o)
{
	const uint8_t *const p = in.p;
	const uint64_t n = in.n;
	uint64_t pos = in.pos, buf = in.buf;
	unsigned cnt = in.cnt;
	uint8_t *t = o.t;
	size_t nt = o.nt, capt = o.capt;
	const int64_t floor = o.floor;
	const uint32_t *const LT = T.lit, *const DT = T.dist;
	auto save = [&]() {
		in.pos = pos;
		in.buf = buf;
		in.cnt = cnt;
		o.nt = nt;
	};
	for (;;) {
		if (__builtin_expect(capt - nt < 600, 0)) {
			save();
			if (!o.room(600)) return 0;
			t = o.t;
			capt = o.capt;
		}
		if (__builtin_expect(pos > n + 16, 0)) {
			save();
			return 0;
		}
		if (__builtin_expect(pos + 8 <= n, 1)) {   // BitIn::refill
			uint64_t w;
			memcpy(&w, p + pos, 8);
			buf |= w << cnt;
			pos += (63 - cnt) >> 3;
			cnt |= 56;
		} else {
			while (cnt <= 56) {
				const uint64_t b = pos < n ? p[pos] : 0;
				buf |= b << cnt;
				++pos;
				cnt += 8;
			}
		}
		uint32_t e = LT[buf & ((1u << LROOT) - 1)];
		if (e_kind(e) == K_SUB) e = LT[e_val(e) + ((buf >> LROOT) & ((1u << e_ext(e)) - 1))];
		const uint64_t b0 = buf;   // a length's extra bits are read from here
		buf >>= e_len(e);
		cnt -= e_len(e);
		if (e_kind(e) <= K_LIT2) {   // see decode_huff
			uint16_t v16 = (uint16_t)e_val(e);
			memcpy(t + nt, &v16, 2);
			nt += 1u + e_kind(e);
#pragma GCC unroll 3
			for (int x = 0; x < 3; ++x) {
				const uint32_t e2 = LT[buf & ((1u << LROOT) - 1)];
				if (e_kind(e2) > K_LIT2) break;
				buf >>= e_len(e2);
				cnt -= e_len(e2);
				v16 = (uint16_t)e_val(e2);
				memcpy(t + nt, &v16, 2);
				nt += 1u + e_kind(e2);
			}
			continue;
		}
		if (e_kind(e) == K_EOB) {
			save();
			return in.overrun() ? 0 : 1;
		}
		if (e_kind(e) != K_LEN) {
			save();
			return 0;
		}
		const unsigned lx = e_ext(e);
		const unsigned len = e_val(e) + (unsigned)((b0 >> (e_len(e) - lx)) & ((1u << lx) - 1));
		uint32_t d = DT[buf & ((1u << DROOT) - 1)];
		if (e_kind(d) == K_SUB) d = DT[e_val(d) + ((buf >> DROOT) & ((1u << e_ext(d)) - 1))];
		if (e_kind(d) == K_BAD) {
			save();
			return 0;
		}
		const uint64_t b1 = buf;
		buf >>= e_len(d);
		cnt -= e_len(d);
		const unsigned dx = e_ext(d);
		const unsigned dist = e_val(d) + (unsigned)((b1 >> (e_len(d) - dx)) & ((1u << dx) - 1));
		// every source byte lies in t[nt - 32768, nt): literal text
		if (__builtin_expect((int64_t)nt - (int64_t)dist < floor, 0)) {
			save();
			return 0;
		}
		copy_match8(t + nt, dist, len);
		nt += len;
	}
}

int decode_huff_any(BitIn &in, const Tables &T, Out &o)
{
	if (o.wide) {
		const int r = decode_huff<true>(in, T, o);
		if (r != 2) return r;
	}
	return decode_huff_narrow(in, T, o);
}

// Stored block body; the 3 header bits are consumed.
bool decode_stored(BitIn &in, Out &o)
{
	const uint64_t byte = (in.bitpos() + 7) >> 3;
	if (byte + 4 > in.n) return false;
	const unsigned len = in.p[byte] | in.p[byte + 1] << 8, nlen = in.p[byte + 2] | in.p[byte + 3] << 8;
	if (len != (~nlen & 0xffffu) || byte + 4 + len > in.n) return false;
	if (!o.room((size_t)len + 600)) return false;
	const uint8_t *s = in.p + byte + 4;
	if (o.wide) {
		for (unsigned i = 0; i < len; ++i) o.s[o.ns + i] = s[i];
		o.ns += len;
	} else {
		memcpy(o.t + o.nt, s, len);
		o.nt += len;
	}
	in.init(in.p, in.n, (byte + 4 + len) * 8);
	return true;
}

// RFC 1952 member header at byte `off`: offset of its deflate data, or -1
// where zlib's inflate would report an error (or the header is cut short).
int64_t member_header(const uint8_t *p, uint64_t n, uint64_t off)
{
	uint64_t q = off;
	if (q + 10 > n || p[q] != 0x1f || p[q + 1] != 0x8b || p[q + 2] != 8) return -1;
	const unsigned flg = p[q + 3];
	if (flg & 0xe0) return -1;
	q += 10;
	if (flg & 4) {
		if (q + 2 > n) return -1;
		q += 2 + (p[q] | p[q + 1] << 8);
		if (q > n) return -1;
	}
	for (unsigned f = 8; f <= 16; f <<= 1) {
		if (!(flg & f)) continue;
		const uint8_t *z = q < n ? (const uint8_t *)memchr(p + q, 0, (size_t)(n - q)) : nullptr;
		if (!z) return -1;
		q = (uint64_t)(z - p) + 1;
	}
	if (flg & 2) {
		if (q + 2 > n) return -1;
		const uint32_t hc = (uint32_t)crc32(0, p + off, (uInt)(q - off)) & 0xffff;
		if (hc != (uint32_t)(p[q] | p[q + 1] << 8)) return -1;
		q += 2;
	}
	return (int64_t)q;
}

struct Event {
	uint64_t off;   // output offset at which a member ended
	uint32_t crc, isize;
};

// Speculative chunk decode: blocks from bit `start` until the first block
// start at or past `end_bit`, across member ends.
struct Chunk {
	uint64_t index = ~0ull;
	uint64_t nom_a = 0, nom_b = 0;    // nominal bit range
	int64_t start = -1;               // bit where decoding began; -1 none
	uint64_t end = 0;                 // where it stopped (a block start, or the stream end)
	bool ok = false, stream_end = false;
	std::vector<Event> events;
	Out out;
	bool busy = false;                // slot in use (decoding, or held until resolved)
	bool decoded = false;
	bool known = false;               // starts at the stream's first block (empty history, no search)
	bool end_dynamic = false;         // share scans: stop only at a dynamic block (one a search can find)
	std::unique_ptr<Tables> tab;      // allocated by the first decode (a held share keeps many chunks)
};

// After a final block: the member trailer, then the next member's header.
// Returns 1 to go on decoding at *in, 0 at the end of the stream, -1 on an
// error.
int member_end(const uint8_t *p, uint64_t n, BitIn &in, Chunk &C)
{
	Out &o = C.out;
	uint64_t byte = (in.bitpos() + 7) >> 3;
	if (byte + 8 > n) return -1;
	C.events.push_back({o.total(), le32(p + byte), le32(p + byte + 4)});
	byte += 8;
	if (n - byte < 2 || p[byte] != 0x1f || p[byte + 1] != 0x8b) {   // end, or trailing garbage
		C.stream_end = true;
		C.end = byte * 8;
		return 0;
	}
	const int64_t d = member_header(p, n, byte);
	if (d < 0) return -1;
	o.floor = (int64_t)o.total();
	in.init(p, n, (uint64_t)d * 8);
	return 1;
}

bool decode_blocks(const uint8_t *p, uint64_t n, BitIn &in, Chunk &C, bool first_checked)
{
	Out &o = C.out;
	bool first = first_checked;
	for (;;) {
		const uint64_t at = in.bitpos();
		if (at >= C.nom_b && !first) {
			in.refill();
			if (!C.end_dynamic || ((in.buf >> 1) & 3) == 2) {
				C.end = at;
				return o.finish();
			}
		}
		first = false;
		in.refill();
		const unsigned bfinal = in.take(1), btype = in.take(2);
		bool good;
		if (btype == 0) good = decode_stored(in, o);
		else if (btype == 1) good = decode_huff_any(in, fixed_tables(), o) == 1;
		else if (btype == 2) good = read_dynamic(in, *C.tab) && decode_huff_any(in, *C.tab, o) == 1;
		else good = false;
		if (!good) return false;
		if (!bfinal) continue;
		const int r = member_end(p, n, in, C);
		if (r < 0) return false;
		if (r == 0) return o.finish();
	}
}

// First 13 header bits that can start a dynamic block: BTYPE = 2, at most
// 286 literal/length and 30 distance codes (about 22 % of patterns).
const uint8_t *head13()
{
	static uint8_t *t = [] {
		uint8_t *x = new uint8_t[8192];
		for (unsigned w = 0; w < 8192; ++w) x[w] = (w & 6) == 4 && ((w >> 3) & 31) <= 29 && ((w >> 8) & 31) <= 29;
		return x;
	}();
	return t;
}

// Cheap tests on a candidate dynamic block header at bit b (whose first 13
// bits passed head13): a complete code-length code.
// Kraft sum (in units of 2^-7) of four 3-bit code lengths
const uint16_t *kraft4()
{
	static uint16_t *t = [] {
		uint16_t *x = new uint16_t[4096];
		for (unsigned w = 0; w < 4096; ++w) {
			unsigned k = 0;
			for (int i = 0; i < 4; ++i) {
				const unsigned l = (w >> (3 * i)) & 7;
				if (l) k += 128u >> l;
			}
			x[w] = (uint16_t)k;
		}
		return x;
	}();
	return t;
}

inline bool quick_dynamic(const uint8_t *p, uint64_t n, uint64_t b, uint64_t w)
{
	const unsigned hclen = (unsigned)((w >> 13) & 15) + 4;
	const uint64_t b2 = b + 17, byte2 = b2 >> 3;
	if (byte2 + 8 > n) return false;
	uint64_t w2;
	memcpy(&w2, p + byte2, 8);
	w2 >>= (b2 & 7);
	// the code-length code: hclen 3-bit lengths, which must form a complete code
	w2 &= hclen == 19 ? ~0ull >> 7 : ((1ull << (3 * hclen)) - 1);
	const uint16_t *K = kraft4();
	unsigned kraft = K[w2 & 4095];
	if (kraft > 128) return false;
	kraft += K[(w2 >> 12) & 4095];
	if (kraft > 128) return false;
	kraft += K[(w2 >> 24) & 4095] + K[(w2 >> 36) & 4095] + K[(w2 >> 48) & 511];
	return kraft == 128;
}

// Plausible block header at bit b (the block after a candidate): stored with
// matching LEN/NLEN, fixed, or a dynamic header that builds.
bool plausible_next(const uint8_t *p, uint64_t n, uint64_t b, Tables &scratch)
{
	BitIn in;
	in.init(p, n, b);
	in.take(1);
	const unsigned bt = in.take(2);
	if (bt == 1) return true;
	if (bt == 3) return false;
	if (bt == 0) {
		const uint64_t byte = (in.bitpos() + 7) >> 3;
		if (byte + 4 > n) return false;
		return (p[byte] | p[byte + 1] << 8) == (~(p[byte + 2] | p[byte + 3] << 8) & 0xffff);
	}
	return read_dynamic(in, scratch);
}

void decode_chunk(const uint8_t *p, uint64_t n, uint64_t first_bit, Chunk &C)
{
	if (!C.tab) C.tab.reset(new Tables);
	C.ok = C.stream_end = false;
	C.start = -1;
	C.events.clear();
	Out &o = C.out;
	BitIn in;
	if (C.known) {   // the stream's start: known (empty) history
		o.reset(true);
		C.start = (int64_t)first_bit;
		in.init(p, n, first_bit);
		C.ok = decode_blocks(p, n, in, C, true);
		return;
	}
	const uint64_t lim = std::min(C.nom_b, n * 8);
	Tables scratch;
	const double t0 = gz_now();
	const uint8_t *H = head13();
	uint64_t w8 = 0, wbyte = ~0ull;
	for (uint64_t b = C.nom_a; b < lim; ++b) {
		const uint64_t byte = b >> 3;
		if (byte + 24 > n) break;   // (a block start this close to the end is left to zlib)
		if (byte != wbyte) {   // one load serves the 8 bit offsets of a byte
			memcpy(&w8, p + byte, 8);
			wbyte = byte;
		}
		const uint64_t w = w8 >> (b & 7);
		if (!H[w & 8191] || !quick_dynamic(p, n, b, w)) continue;
		o.reset(false);
		C.events.clear();
		in.init(p, n, b);
		in.take(3);
		if (!read_dynamic(in, *C.tab) || decode_huff_any(in, *C.tab, o) != 1) continue;
		// the candidate block decoded; its header bit said whether it was final
		BitIn h;
		h.init(p, n, b);
		const bool final_blk = h.take(1);
		if (!final_blk && !plausible_next(p, n, in.bitpos(), scratch)) continue;
		C.start = (int64_t)b;
		const double t1 = gz_now();
		prof_search_us += (uint64_t)((t1 - t0) * 1e6);
		struct Acc {
			double t;
			~Acc() { prof_decode_us += (uint64_t)((gz_now() - t) * 1e6); }
		} acc{t1};
		if (final_blk) {   // continue through the trailer like decode_blocks
			const int r = member_end(p, n, in, C);
			if (r < 0) return;
			if (r == 0) {
				C.ok = o.finish();
				return;
			}
		}
		C.ok = decode_blocks(p, n, in, C, false);
		return;
	}
}

// ---------------------------------------------------------------------------
// resolved output handed to the reader
// ---------------------------------------------------------------------------
struct Piece {
	uint8_t *text = nullptr;          // owned (malloc); an accepted chunk's t[] is swapped in
	size_t n = 0, cap = 0;
	Chunk *src = nullptr;             // symbols still to resolve (accepted chunk)
	std::vector<uint8_t> window;      // the 32 KiB before src's first symbol
	std::vector<Event> events;
	std::vector<uint32_t> seg_crc;    // events.size() + 1 segments
	bool stream_end = false;
	bool ready = false, resolving = false;
	int lent = 0;                     // spans handed out with a hold (vc_gzp_span_hold), not yet released
	~Piece() { free(text); }
	bool reserve(size_t c)
	{
		if (c <= cap) return true;
		uint8_t *q = (uint8_t *)realloc(text, c);
		if (!q) return false;
		advise_huge(q, c);
		text = q;
		cap = c;
		return true;
	}
};

// t[0..res) of the source chunk from its symbols and the window; then the
// chunk's text buffer becomes the piece's (the piece's old buffer goes back
// to the chunk for reuse).
void resolve(Piece &P)
{
	Out &o = P.src->out;
	const uint16_t *s = o.s;
	uint8_t *t = o.t;
	const size_t n = o.res;
	// symbol -> byte: literals map to themselves, MARK | i to window byte i
	static thread_local std::unique_ptr<uint8_t[]> lut(new uint8_t[65536]);
	uint8_t *L = lut.get();
	for (int v = 0; v < 256; ++v) L[v] = (uint8_t)v;
	memcpy(L + MARK, P.window.data(), WSIZE);
	// 16 symbols at a time: all literals (one pack), a run of consecutive
	// window bytes (a back-reference chain that reaches the window: one
	// 16-byte copy), one window byte repeated (a run of it), else per symbol
	const uint8_t *W = P.window.data();
	const __m128i iota0 = _mm_setr_epi16(0, 1, 2, 3, 4, 5, 6, 7), iota1 = _mm_setr_epi16(8, 9, 10, 11, 12, 13, 14, 15);
	size_t i = 0;
	for (; i + 16 <= n; i += 16) {
		const __m128i v0 = _mm_loadu_si128((const __m128i *)(s + i));
		const __m128i v1 = _mm_loadu_si128((const __m128i *)(s + i + 8));
		if ((_mm_movemask_epi8(_mm_or_si128(v0, v1)) & 0xAAAA) == 0) {   // no symbol >= 256
			_mm_storeu_si128((__m128i *)(t + i), _mm_packus_epi16(v0, v1));
			continue;
		}
		const uint16_t f = s[i];
		if (f >= MARK && (uint32_t)(f - MARK) + 16u <= WSIZE) {
			const __m128i b = _mm_set1_epi16((short)f);
			const int run = _mm_movemask_epi8(_mm_and_si128(_mm_cmpeq_epi16(v0, _mm_add_epi16(b, iota0)),
			                                                _mm_cmpeq_epi16(v1, _mm_add_epi16(b, iota1))));
			if (run == 0xFFFF) {
				memcpy(t + i, W + (f - MARK), 16);
				continue;
			}
			const int same = _mm_movemask_epi8(_mm_and_si128(_mm_cmpeq_epi16(v0, b), _mm_cmpeq_epi16(v1, b)));
			if (same == 0xFFFF) {
				memset(t + i, W[f - MARK], 16);
				continue;
			}
		}
		for (int k = 0; k < 16; ++k) t[i + k] = L[s[i + k]];
	}
	for (; i < n; ++i) t[i] = L[s[i]];
	std::swap(P.text, o.t);
	std::swap(P.cap, o.capt);
	P.n = o.nt;
}

// CRC-32 (gzip's, zlib's crc32) by carry-less multiplication: four 128-bit
// lanes folded over 64-byte blocks, then one lane, then Barrett reduction
// (Gopal et al., "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ
// Instruction", Intel 2009; bit-reflected constants from its appendix).
// Pre- and post-inverted like zlib's; len a multiple of 16, at least 64.
__attribute__((target("pclmul,sse4.1"))) inline __m128i fold128(__m128i a, __m128i b, __m128i k)
{
	return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(a, k, 0x11), b), _mm_clmulepi64_si128(a, k, 0x00));
}

__attribute__((target("pclmul,sse4.1"))) uint32_t crc32_fold(uint32_t crc, const uint8_t *buf, uint64_t len)
{
	alignas(16) static const uint64_t k1k2[] = {0x0154442bd4ull, 0x01c6e41596ull};
	alignas(16) static const uint64_t k3k4[] = {0x01751997d0ull, 0x00ccaa009eull};
	alignas(16) static const uint64_t k5k0[] = {0x0163cd6124ull, 0};
	alignas(16) static const uint64_t poly[] = {0x01db710641ull, 0x01f7011641ull};
	crc = ~crc;
	__m128i x1 = _mm_loadu_si128((const __m128i *)(buf + 0x00));
	__m128i x2 = _mm_loadu_si128((const __m128i *)(buf + 0x10));
	__m128i x3 = _mm_loadu_si128((const __m128i *)(buf + 0x20));
	__m128i x4 = _mm_loadu_si128((const __m128i *)(buf + 0x30));
	x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
	__m128i x0 = _mm_load_si128((const __m128i *)k1k2);
	buf += 64;
	len -= 64;
	while (len >= 64) {
		const __m128i x5 = _mm_clmulepi64_si128(x1, x0, 0x00), x6 = _mm_clmulepi64_si128(x2, x0, 0x00);
		const __m128i x7 = _mm_clmulepi64_si128(x3, x0, 0x00), x8 = _mm_clmulepi64_si128(x4, x0, 0x00);
		x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
		x2 = _mm_clmulepi64_si128(x2, x0, 0x11);
		x3 = _mm_clmulepi64_si128(x3, x0, 0x11);
		x4 = _mm_clmulepi64_si128(x4, x0, 0x11);
		x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128((const __m128i *)(buf + 0x00)));
		x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128((const __m128i *)(buf + 0x10)));
		x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128((const __m128i *)(buf + 0x20)));
		x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128((const __m128i *)(buf + 0x30)));
		buf += 64;
		len -= 64;
	}
	x0 = _mm_load_si128((const __m128i *)k3k4);
	x1 = fold128(x1, x2, x0);
	x1 = fold128(x1, x3, x0);
	x1 = fold128(x1, x4, x0);
	while (len >= 16) {
		x1 = fold128(x1, _mm_loadu_si128((const __m128i *)buf), x0);
		buf += 16;
		len -= 16;
	}
	// 128 -> 64 bits
	x2 = _mm_clmulepi64_si128(x1, x0, 0x10);
	x3 = _mm_setr_epi32(~0, 0, ~0, 0);
	x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2);
	x0 = _mm_loadl_epi64((const __m128i *)k5k0);
	x2 = _mm_srli_si128(x1, 4);
	x1 = _mm_and_si128(x1, x3);
	x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x00), x2);
	// Barrett reduction to 32 bits
	x0 = _mm_load_si128((const __m128i *)poly);
	x2 = _mm_and_si128(x1, x3);
	x2 = _mm_clmulepi64_si128(x2, x0, 0x10);
	x2 = _mm_and_si128(x2, x3);
	x2 = _mm_clmulepi64_si128(x2, x0, 0x00);
	x1 = _mm_xor_si128(x1, x2);
	return ~(uint32_t)_mm_extract_epi32(x1, 1);
}

const bool have_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");

uint32_t vc_crc32(uint32_t c, const uint8_t *p, uint64_t n)
{
	if (have_clmul && n >= 64) {
		const uint64_t m = n & ~(uint64_t)15;
		c = crc32_fold(c, p, m);
		p += m;
		n -= m;
	}
	while (n) {   // zlib's length is 32-bit
		const uint64_t m = std::min<uint64_t>(n, (uint64_t)1 << 30);
		c = (uint32_t)crc32(c, p, (uInt)m);
		p += m;
		n -= m;
	}
	return c;
}

void piece_crcs(Piece &P)
{
	P.seg_crc.clear();
	uint64_t a = 0;
	for (const Event &e : P.events) {
		P.seg_crc.push_back(vc_crc32(0, P.text + a, e.off - a));
		a = e.off;
	}
	P.seg_crc.push_back(vc_crc32(0, P.text + a, P.n - a));
}

} // namespace

// How a VcGzParallel covers the stream (vafc_gzip.h, shares of one stream).
struct GzShareOpts {
	bool scan = false;                // vc_gzp_scan_share
	uint64_t begin = 0, end = UINT64_MAX;   // scan: the share's nominal bytes
	bool first_share = true;          // stream: from the stream's start
	uint64_t start_bit = 0;           // stream, later shares: the share's first block
	const uint8_t *window = nullptr;  // stream, later shares: the 32 KiB before it
	uint64_t text_len = UINT64_MAX;   // stream: the share's text (CRC accounting)
	uint64_t hold_bytes = 0;          // scan: keep the decoded share (at most this many bytes) for resume()
};

class VcGzParallel {
public:
	~VcGzParallel() { shutdown(); }
	bool start(const char *path, int threads, uint64_t chunk_bytes, const GzShareOpts *so = nullptr);
	// scan mode: wait for the scan's result
	void scan_result(VcGzShare *sh, uint16_t *wsym)
	{
		std::unique_lock<std::mutex> lk(mu_);
		cv_.wait(lk, [&] { return seq_done_; });
		*sh = share_;
		if (wsym) memcpy(wsym, wsym_.data(), WSIZE * sizeof(uint16_t));
	}
	void share_crc(VcGzShareCrc *out)
	{
		std::lock_guard<std::mutex> lk(mu_);
		*out = scrc_;
	}
	// scan mode: the scan kept every chunk of the share (vc_gzp_scan_share_hold)
	bool held() const { return held_; }
	// A held share: stream its text from the kept chunks with the now known
	// window before it (nullptr: the stream's first share), then on past its
	// end with zlib, in small pieces, as far as the reader asks.
	bool resume(const uint8_t *window, uint64_t text_len);
	int64_t read(uint8_t *dst, size_t n);
	int64_t span(const uint8_t **out, size_t maxn, void **hold = nullptr);
	void release(void *hold);
	void get_stats(VcGzStats *st)
	{
		std::lock_guard<std::mutex> lk(mu_);
		*st = stats;
	}

private:
	VcGzStats stats;                  // guarded by mu_ (out_bytes, members, crc_error: reader thread)
	// input
	int fd_ = -1;
	const uint8_t *p_ = nullptr;
	uint64_t n_ = 0, first_bit_ = 0, chunk_bits_ = 0, nchunks_ = 0;
	// shared state
	std::mutex mu_;
	std::condition_variable cv_;
	bool stop_ = false, seq_done_ = false;
	std::vector<std::unique_ptr<Chunk>> slots_;
	uint64_t next_decode_ = 0;
	std::deque<std::unique_ptr<Piece>> pieces_;
	std::vector<std::unique_ptr<Piece>> spare_;
	std::vector<std::unique_ptr<Piece>> lent_;    // read, but spans of them still held
	size_t max_pieces_ = 8;
	std::vector<std::thread> workers_;
	std::thread seq_;
	// sequencer state
	std::vector<uint8_t> window_ = std::vector<uint8_t>(WSIZE);
	uint64_t member_text_ = 0;        // bytes of the current member so far
	// reader state
	Piece *cur_ = nullptr;
	size_t rd_ = 0, ev_ = 0, seg_a_ = 0;
	bool spent_ = false;              // cur_ fully read (released at the next span)
	uint32_t mcrc_ = 0;
	uint64_t mlen_ = 0;
	bool done_ = false;
	// shares (vafc_gzip.h)
	bool known_start_ = true;         // chunk 0 starts at the stream's first block
	bool scan_ = false;               // scan mode: symbols of the share's last 32 KiB, no text
	uint64_t last_bit_ = 0;           // the chunks cover [first_bit_, last_bit_)
	VcGzShare share_;
	std::vector<uint16_t> wsym_ = std::vector<uint16_t>(WSIZE);
	uint64_t share_len_ = UINT64_MAX; // stream mode: CRC accounting stops at this text offset
	uint64_t pbase_ = 0;              // text offset of cur_'s first byte
	bool crc_stopped_ = false;
	VcGzShareCrc scrc_;
	bool hold_ = false, held_ = false;   // scan: keeping the share's chunks / kept all of them
	uint64_t hold_budget_ = 0, held_bytes_ = 0;
	bool continue_after_ = false;     // resumed share: zlib on past the last kept chunk
	uint64_t scan_pos_ = UINT64_MAX / 2;   // held scan: the chunk the scan waits for (bounds decode-ahead)
	uint64_t seq_first_ = UINT64_MAX;      // resumed share: the sequencer's first block (the share's start)
	int threads_ = 1;

	void worker();
	void sequencer();
	void scan_sequencer();
	void share_cut(const Piece &P, size_t cut);   // the CRC accounting reaches the share's end
	void stream_done_crc()   // the stream ended before the share's end: what is open is the tail
	{
		if (share_len_ == UINT64_MAX || crc_stopped_) return;
		std::lock_guard<std::mutex> lk(mu_);
		scrc_.tail_crc = mcrc_;
		scrc_.tail_len = mlen_;
		scrc_.complete = stats.crc_error ? 0u : 1u;
		crc_stopped_ = true;
	}
	bool fallback(uint64_t &expect, uint64_t nom_b, bool &ended, size_t piece_cap = PIECE_CAP);
	Piece *new_piece();
	bool push_piece(std::unique_ptr<Piece> P);   // waits for queue space; false on stop
	void window_append(const uint8_t *t, size_t n);
	void shutdown();
};

Piece *VcGzParallel::new_piece()
{
	std::lock_guard<std::mutex> lk(mu_);
	if (!spare_.empty()) {
		Piece *P = spare_.back().release();
		spare_.pop_back();
		P->n = 0;
		P->src = nullptr;
		P->events.clear();
		P->seg_crc.clear();
		P->stream_end = P->ready = P->resolving = false;
		return P;
	}
	return new Piece;
}

bool VcGzParallel::push_piece(std::unique_ptr<Piece> P)
{
	std::unique_lock<std::mutex> lk(mu_);
	const double w0 = gz_now();
	cv_.wait(lk, [&] { return stop_ || pieces_.size() < max_pieces_; });
	prof_seqpush_us += (uint64_t)((gz_now() - w0) * 1e6);
	if (stop_) return false;
	pieces_.push_back(std::move(P));
	cv_.notify_all();
	return true;
}

void VcGzParallel::window_append(const uint8_t *t, size_t n)
{
	uint8_t *w = window_.data();
	if (n >= WSIZE) {
		memcpy(w, t + n - WSIZE, WSIZE);
	} else if (n) {
		memmove(w, w + n, WSIZE - n);
		memcpy(w + WSIZE - n, t, n);
	}
}

void VcGzParallel::worker()
{
	for (;;) {
		std::unique_lock<std::mutex> lk(mu_);
		Piece *task = nullptr;
		Chunk *dec = nullptr;
		const double w0 = gz_now();
		cv_.wait(lk, [&] {
			if (stop_) return true;
			for (auto &P : pieces_)
				if (P->src && !P->resolving) {
					task = P.get();
					return true;
				}
			// a held share has a slot per chunk: decode at most a slot ring's
			// worth ahead of the scan, as the ring itself bounds ordinary runs
			if (next_decode_ < nchunks_ && next_decode_ < scan_pos_ + (uint64_t)threads_ + 2) {
				Chunk &C = *slots_[next_decode_ % slots_.size()];
				if (!C.busy) {
					dec = &C;
					return true;
				}
			}
			return false;
		});
		prof_widle_us += (uint64_t)((gz_now() - w0) * 1e6);
		if (stop_) return;
		if (task) {
			task->resolving = true;
			lk.unlock();
			const bool ok = true;
			{
				const double r0 = gz_now();
				resolve(*task);
				// a resumed share's chunk is never decoded again: its symbols and the
				// buffer the piece swapped in go now, spread over the workers, rather
				// than all at once when the share is closed
				if (continue_after_) task->src->out.release_buffers();
				const double r1 = gz_now();
				piece_crcs(*task);
				prof_resolve_us += (uint64_t)((r1 - r0) * 1e6);
				prof_crc_us += (uint64_t)((gz_now() - r1) * 1e6);
			}
			lk.lock();
			task->src->busy = false;
			task->src = nullptr;
			if (!ok) {   // out of memory: the stream ends before this piece
				task->n = 0;
				task->events.clear();
				task->seg_crc.assign(1, 0);
				task->stream_end = true;
			}
			task->ready = true;
			cv_.notify_all();
			continue;
		}
		const uint64_t j = next_decode_++;
		dec->busy = true;
		dec->decoded = false;
		dec->index = j;
		dec->known = j == 0 && known_start_;
		dec->end_dynamic = scan_;
		dec->nom_a = first_bit_ + j * chunk_bits_;
		dec->nom_b = j + 1 == nchunks_ ? last_bit_ : first_bit_ + (j + 1) * chunk_bits_;
		lk.unlock();
		decode_chunk(p_, n_, first_bit_, *dec);
		lk.lock();
		dec->decoded = true;
		cv_.notify_all();
	}
}

// zlib from the true boundary `expect` with the true history, until the first
// block start at or past nom_b, the end of the stream, or an error.  Output
// goes to pieces of at most PIECE_CAP bytes.  false only on stop / no memory.
bool VcGzParallel::fallback(uint64_t &expect, uint64_t nom_b, bool &ended, size_t piece_cap)
{
	z_stream zs;
	memset(&zs, 0, sizeof zs);
	if (inflateInit2(&zs, -15) != Z_OK) return false;
	uint64_t byte = expect >> 3;
	const unsigned sh = (unsigned)(expect & 7);
	if (sh) {
		inflatePrime(&zs, (int)(8 - sh), p_[byte] >> sh);
		++byte;
	}
	const size_t dict = (size_t)std::min<uint64_t>(member_text_, WSIZE);
	if (dict) inflateSetDictionary(&zs, window_.data() + WSIZE - dict, (uInt)dict);
	const uint8_t *in = p_ + byte;
	auto feed = [&]() {
		zs.next_in = (Bytef *)in;
		zs.avail_in = (uInt)std::min<uint64_t>(n_ - (uint64_t)(in - p_), (uint64_t)1 << 30);
	};
	feed();
	std::unique_ptr<Piece> P(new_piece());
	auto emit = [&](bool last) -> bool {
		P->stream_end = last;
		piece_crcs(*P);
		P->ready = true;
		return push_piece(std::move(P));
	};
	bool alive = P->reserve(piece_cap);
	while (alive) {
		if (P->n >= piece_cap) {   // piece full
			if (!emit(false)) {
				alive = false;
				break;
			}
			P.reset(new_piece());
			if (!P->reserve(piece_cap)) {
				alive = false;
				break;
			}
		}
		zs.next_out = P->text + P->n;
		zs.avail_out = (uInt)(piece_cap - P->n);
		const int ret = inflate(&zs, Z_BLOCK);
		const size_t made = (size_t)(zs.next_out - (P->text + P->n));
		window_append(P->text + P->n, made);
		P->n += made;
		member_text_ += made;
		in = zs.next_in;
		if (ret == Z_STREAM_END) {   // member end: trailer, then another member or the end
			uint64_t tb = (uint64_t)(in - p_);
			if (tb + 8 > n_) {   // trailer cut short: gzread's "unexpected end of file"
				ended = true;
				break;
			}
			P->events.push_back({P->n, le32(p_ + tb), le32(p_ + tb + 4)});
			tb += 8;
			const int64_t d = (n_ - tb >= 2 && p_[tb] == 0x1f && p_[tb + 1] == 0x8b) ? member_header(p_, n_, tb) : -1;
			if (d < 0) {   // no further member (trailing bytes ignored), or a header zlib rejects
				ended = true;
				break;
			}
			member_text_ = 0;
			inflateReset(&zs);
			in = p_ + d;
			feed();
			if ((uint64_t)d * 8 >= nom_b) {
				expect = (uint64_t)d * 8;
				break;
			}
			continue;
		}
		if (ret != Z_OK && ret != Z_BUF_ERROR) {   // corrupt data: the output so far, then the end
			ended = true;
			break;
		}
		if (zs.avail_in == 0) {
			if ((uint64_t)(in - p_) >= n_) {
				if (ret == Z_BUF_ERROR) {   // input exhausted inside the stream
					ended = true;
					break;
				}
			} else {
				feed();
			}
		} else if (ret == Z_BUF_ERROR && zs.avail_out != 0) {
			ended = true;   // no progress with input and room: treat as corrupt
			break;
		}
		if ((zs.data_type & 192) == 128) {   // at the start of a block (not after the final one)
			const uint64_t at = (uint64_t)(in - p_) * 8 - (uint64_t)(zs.data_type & 7);
			if (at >= nom_b) {
				expect = at;
				break;
			}
		}
	}
	inflateEnd(&zs);
	if (!alive) return false;
	if (P->n == 0 && P->events.empty() && !ended) {
		std::lock_guard<std::mutex> lk(mu_);
		spare_.push_back(std::move(P));
		return true;
	}
	return emit(ended);
}

void VcGzParallel::sequencer()
{
	uint64_t expect = seq_first_ != UINT64_MAX ? seq_first_ : first_bit_;
	bool ended = false;
	for (uint64_t j = 0; j < nchunks_ && !ended; ++j) {
		Chunk *C = slots_[j % slots_.size()].get();
		{
			std::unique_lock<std::mutex> lk(mu_);
			const double w0 = gz_now();
			cv_.wait(lk, [&] { return stop_ || (C->index == j && C->decoded); });
			prof_seqwait_us += (uint64_t)((gz_now() - w0) * 1e6);
			if (stop_) break;
		}
		if (expect >= C->nom_b) {
			std::lock_guard<std::mutex> lk(mu_);
			C->busy = false;
			++stats.skipped;  // under mu_
			cv_.notify_all();
			continue;
		}
		const uint64_t have = std::min<uint64_t>(member_text_, WSIZE);
		const bool take = C->ok && C->start >= 0 && (uint64_t)C->start == expect &&
		                  C->out.min_mark >= WSIZE - have;
		if (take) {
			std::unique_ptr<Piece> P(new_piece());
			P->src = C;
			P->window = window_;
			P->events = C->events;
			P->stream_end = C->stream_end;
			// the window after this chunk: its last 32 KiB, markers resolved
			const Out &o = C->out;
			const size_t n = o.nt;
			uint8_t tail[WSIZE];
			const size_t tn = std::min<size_t>(n, WSIZE);
			for (size_t i = 0; i < tn; ++i) {
				const size_t x = n - tn + i;
				if (x >= o.res) {
					tail[i] = o.t[x];
				} else {
					const uint16_t v = o.s[x];
					tail[i] = v < 256 ? (uint8_t)v : window_[v & (WSIZE - 1)];
				}
			}
			window_append(tail, tn);
			member_text_ = C->events.empty() ? member_text_ + n : n - C->events.back().off;
			expect = C->end;
			ended = C->stream_end;
			{
				std::lock_guard<std::mutex> lk(mu_);
				++stats.accepted;
			}
			if (!push_piece(std::move(P))) break;
			continue;
		}
		const uint64_t nom_b = C->nom_b;   // read before the slot goes back to the workers
		{
			std::lock_guard<std::mutex> lk(mu_);
			C->busy = false;
			++stats.fallback;
			cv_.notify_all();
		}
		if (!fallback(expect, nom_b, ended)) break;
	}
	// a resumed share: its last record may end in the next share, which no
	// chunk covers -- zlib on from the share's end in small pieces (the reader
	// stops after a few KiB, and the pass waits for each piece)
	if (continue_after_ && !ended && !stop_) fallback(expect, UINT64_MAX, ended, (size_t)256 << 10);
	std::lock_guard<std::mutex> lk(mu_);
	seq_done_ = true;
	cv_.notify_all();
}

// Scan mode: the chunks of the share in order, each taken only where it
// begins at the previous one's end (no zlib fallback: the history before the
// share is unknown); the share's last 32 KiB kept as symbols that name bytes
// of the window before the share (vafc_gzip.h).
void VcGzParallel::scan_sequencer()
{
	for (uint32_t i = 0; i < WSIZE; ++i) wsym_[i] = (uint16_t)(MARK | i);
	std::vector<uint16_t> tail(WSIZE);
	uint64_t expect = known_start_ ? first_bit_ : UINT64_MAX;
	if (known_start_) share_.start_bit = first_bit_;
	else member_text_ = WSIZE;        // a member open before the share: its history is the full window
	bool ok = true, ended = false;
	uint64_t len = 0;
	for (uint64_t j = 0; j < nchunks_ && ok && !ended; ++j) {
		Chunk *C = slots_[j % slots_.size()].get();
		{
			std::unique_lock<std::mutex> lk(mu_);
			if (slots_.size() >= nchunks_) {   // a slot per chunk (held, or over the budget since)
				scan_pos_ = j;
				cv_.notify_all();
			}
			cv_.wait(lk, [&] { return stop_ || (C->index == j && C->decoded); });
			if (stop_) {
				ok = false;
				break;
			}
		}
		// one slot per chunk (a held share): a chunk's buffers are freed with it
		const bool per_chunk = slots_.size() >= nchunks_;
		auto release = [&]() {
			if (per_chunk) C->out.release_buffers();
			std::lock_guard<std::mutex> lk(mu_);
			C->busy = false;
			cv_.notify_all();
		};
		if (expect == UINT64_MAX) {   // the share's first block: in the first chunk that found one
			if (C->start < 0) {
				release();
				continue;
			}
			expect = (uint64_t)C->start;
			share_.start_bit = expect;
		}
		if (expect >= C->nom_b) {
			release();
			continue;
		}
		const uint64_t have = std::min<uint64_t>(member_text_, WSIZE);
		if (!(C->ok && C->start >= 0 && (uint64_t)C->start == expect && C->out.min_mark >= WSIZE - have)) {
			ok = false;
			release();
			break;
		}
		const Out &o = C->out;
		const size_t n = o.nt;
		const size_t tn = std::min<size_t>(n, WSIZE);
		for (size_t i = 0; i < tn; ++i) {
			const size_t x = n - tn + i;
			const uint16_t v = x >= o.res ? (uint16_t)o.t[x] : o.s[x];
			tail[i] = v < 256 ? v : wsym_[v & (WSIZE - 1)];
		}
		if (tn == WSIZE) {
			memcpy(wsym_.data(), tail.data(), WSIZE * sizeof(uint16_t));
		} else if (tn) {
			memmove(wsym_.data(), wsym_.data() + tn, (WSIZE - tn) * sizeof(uint16_t));
			memcpy(wsym_.data() + WSIZE - tn, tail.data(), tn * sizeof(uint16_t));
		}
		len += n;
		member_text_ = C->events.empty() ? member_text_ + n : n - C->events.back().off;
		expect = C->end;
		ended = C->stream_end;
		if (hold_ && held_bytes_ + o.held() <= hold_budget_) {   // kept for resume(): stays busy
			held_bytes_ += o.held();
			continue;
		}
		if (hold_) {   // over the budget: the share will be decoded again; free what was kept
			hold_ = false;
			std::lock_guard<std::mutex> lk(mu_);
			for (uint64_t i = 0; i < j; ++i) {
				Chunk *K = slots_[i % slots_.size()].get();
				if (K->busy && K->index == i && K->decoded) {
					K->out.release_buffers();
					K->busy = false;
				}
			}
			cv_.notify_all();
		}
		release();
	}
	std::lock_guard<std::mutex> lk(mu_);
	held_ = hold_ && ok && share_.start_bit != UINT64_MAX;
	share_.ok = ok;
	share_.text_len = share_.start_bit == UINT64_MAX ? 0 : len;
	share_.end_bit = ended || share_.start_bit == UINT64_MAX ? UINT64_MAX : expect;
	seq_done_ = true;
	cv_.notify_all();
}

bool VcGzParallel::resume(const uint8_t *window, uint64_t text_len)
{
	{
		std::unique_lock<std::mutex> lk(mu_);
		cv_.wait(lk, [&] { return seq_done_; });
		if (!held_) return false;
	}
	if (seq_.joinable()) seq_.join();
	{   // workers read scan_ and may still be decoding chunks past a stream end
		std::lock_guard<std::mutex> lk(mu_);
		scan_ = false;
		continue_after_ = true;
		max_pieces_ = (size_t)threads_ + 4;
		seq_done_ = false;
	}
	share_len_ = text_len;
	if (window) {   // a later share: its history is the window before it
		memcpy(window_.data(), window, WSIZE);
		member_text_ = WSIZE;
	} else {
		member_text_ = 0;
	}
	seq_first_ = share_.start_bit;
	const VcCpuSet cpus = vc_affinity_get();
	seq_ = std::thread([this, cpus] {
		vc_affinity_bind(cpus);
		sequencer();
	});
	return true;
}

// The reader has delivered the share's last byte, at offset `cut` of piece P
// (inside the segment that starts at seg_a_): the CRC of the member still open
// there is the share's tail.
void VcGzParallel::share_cut(const Piece &P, size_t cut)
{
	const size_t part = cut - seg_a_;
	const uint32_t c = part ? vc_crc32(0, P.text + seg_a_, part) : 0;
	std::lock_guard<std::mutex> lk(mu_);
	scrc_.tail_crc = (uint32_t)crc32_combine(mcrc_, c, (z_off_t)part);
	scrc_.tail_len = mlen_ + part;
	scrc_.complete = 1;
	crc_stopped_ = true;
}

bool VcGzParallel::start(const char *path, int threads, uint64_t chunk_bytes, const GzShareOpts *so)
{
	fd_ = open(path, O_RDONLY);
	if (fd_ < 0) return false;
	struct stat sb;
	if (fstat(fd_, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_size < 18) return false;
	n_ = (uint64_t)sb.st_size;
	void *m = mmap(nullptr, (size_t)n_, PROT_READ, MAP_PRIVATE, fd_, 0);
	if (m == MAP_FAILED) return false;
	p_ = (const uint8_t *)m;
	madvise(m, (size_t)n_, MADV_SEQUENTIAL);
	const int64_t d = member_header(p_, n_, 0);
	if (d < 0) return false;
	first_bit_ = (uint64_t)d * 8;
	last_bit_ = n_ * 8;
	if (so && so->scan) {
		scan_ = true;
		hold_ = so->hold_bytes > 0;
		hold_budget_ = so->hold_bytes;
		if (hold_) scan_pos_ = 0;
		if (so->begin > 0) {   // a later share: its first block is searched for
			known_start_ = false;
			first_bit_ = std::max<uint64_t>(first_bit_, std::min<uint64_t>(so->begin, n_) * 8);
		}
		if (so->end < n_) last_bit_ = std::max<uint64_t>(first_bit_, so->end * 8);
		if (first_bit_ >= last_bit_) {   // nothing of the stream in the share
			share_.ok = true;
			seq_done_ = true;
			return true;
		}
	} else if (so) {
		share_len_ = so->text_len;
		if (!so->first_share) {
			if (so->start_bit >= n_ * 8 || !so->window) return false;
			known_start_ = false;
			first_bit_ = so->start_bit;
			memcpy(window_.data(), so->window, WSIZE);
			member_text_ = WSIZE;
		}
	}
	if (threads < 1) threads = 1;
	if (chunk_bytes == 0) {   // about four chunks per worker, 1..4 MiB each
		chunk_bytes = (last_bit_ - first_bit_) / 8 / (4 * (uint64_t)threads);
		chunk_bytes = std::max<uint64_t>((uint64_t)1 << 20, std::min<uint64_t>((uint64_t)4 << 20, chunk_bytes));
	}
	if (chunk_bytes < 1024) chunk_bytes = 1024;
	chunk_bits_ = chunk_bytes * 8;
	nchunks_ = (last_bit_ - first_bit_ + chunk_bits_ - 1) / chunk_bits_;
	if (nchunks_ == 0) nchunks_ = 1;
	stats.chunks = nchunks_;
	if (threads < 1) threads = 1;
	size_t extra = 2;
	if (const char *e = getenv("VAFC_GZ_SLOTS")) extra = (size_t)atoi(e);   // A/B knob: slots beyond the workers
	// a held share keeps every chunk (hold_budget_ bounds their buffers; a
	// chunk's decode tables are allocated by its first decode)
	slots_.resize(hold_ ? (size_t)nchunks_ + extra : (size_t)threads + extra);
	threads_ = threads;
	for (auto &s : slots_) s.reset(new Chunk);
	max_pieces_ = (size_t)threads + extra + 2;
	fixed_tables();
	const VcCpuSet cpus = vc_affinity_get();   // vc_count_file's placement (vafc_affinity.h)
	for (int t = 0; t < threads; ++t)
		workers_.emplace_back([this, cpus] {
			vc_affinity_bind(cpus);
			worker();
		});
	seq_ = std::thread([this, cpus] {
		vc_affinity_bind(cpus);
		if (scan_) scan_sequencer();
		else sequencer();
	});
	return true;
}

// The next bytes of the stream without a copy: *out points into the current
// piece, valid until the next call (the piece is released then).
int64_t VcGzParallel::span(const uint8_t **out, size_t maxn, void **hold)
{
	for (;;) {
		if (done_ || maxn == 0) return 0;
		if (cur_ && spent_) {   // release the piece the previous span pointed into
			const bool last = cur_->stream_end;
			pbase_ += cur_->n;
			{
				std::lock_guard<std::mutex> lk(mu_);
				std::unique_ptr<Piece> P = std::move(pieces_.front());
				pieces_.pop_front();
				if (P->lent > 0) lent_.push_back(std::move(P));   // back once every hold is released
				else spare_.push_back(std::move(P));
				cv_.notify_all();
			}
			cur_ = nullptr;
			if (last) {
				done_ = true;
				stream_done_crc();
				return 0;
			}
		}
		if (!cur_) {
			std::unique_lock<std::mutex> lk(mu_);
			const double w0 = gz_now();
			cv_.wait(lk, [&] { return (!pieces_.empty() && pieces_.front()->ready) || (seq_done_ && pieces_.empty()); });
			prof_rdwait_us += (uint64_t)((gz_now() - w0) * 1e6);
			if (pieces_.empty()) {
				done_ = true;
				lk.unlock();
				stream_done_crc();
				return 0;
			}
			cur_ = pieces_.front().get();
			rd_ = ev_ = seg_a_ = 0;
			spent_ = false;
		}
		Piece &P = *cur_;
		const size_t lim = ev_ < P.events.size() ? (size_t)P.events[ev_].off : P.n;
		if (rd_ < lim) {
			const size_t take = std::min(maxn, lim - rd_);
			// a share ends inside this segment: its tail is accounted as soon as
			// its last byte goes out (the reader may stop soon after)
			if (!crc_stopped_ && share_len_ != UINT64_MAX && pbase_ + lim > share_len_ &&
			    pbase_ + rd_ + take >= share_len_)
				share_cut(P, (size_t)(share_len_ - pbase_));
			*out = P.text + rd_;
			if (hold) {
				std::lock_guard<std::mutex> lk(mu_);
				++P.lent;
				*hold = &P;
			}
			rd_ += take;
			stats.out_bytes += take;
			return (int64_t)take;
		}
		// a segment is complete: its CRC joins the member's
		if (crc_stopped_) {   // past a share's end: another rank accounts for the rest
			seg_a_ = lim;
			if (ev_ < P.events.size()) {
				++ev_;
				continue;
			}
			spent_ = true;
			continue;
		}
		if (share_len_ != UINT64_MAX && pbase_ + lim > share_len_) {   // the share ends inside this segment
			share_cut(P, (size_t)(share_len_ - pbase_));
			continue;
		}
		const size_t seg = lim - seg_a_;
		mcrc_ = (uint32_t)crc32_combine(mcrc_, P.seg_crc[ev_], (z_off_t)seg);
		mlen_ += seg;
		seg_a_ = lim;
		if (ev_ < P.events.size()) {
			const Event &e = P.events[ev_];
			if (share_len_ != UINT64_MAX && scrc_.events == 0) {
				// a share's first member end: the member may have begun in an
				// earlier share, so its check is the caller's (vafc_gzip.h)
				std::lock_guard<std::mutex> lk(mu_);
				scrc_.head_crc = mcrc_;
				scrc_.head_len = mlen_;
				scrc_.head_expect_crc = e.crc;
				scrc_.head_expect_isize = e.isize;
				scrc_.events = 1;
			} else {
				if (mcrc_ != e.crc || (uint32_t)mlen_ != e.isize) {   // gzread stops at a failed check
					std::lock_guard<std::mutex> lk(mu_);
					stats.crc_error = 1;
					scrc_.crc_error = 1;
					done_ = true;
					return 0;
				}
				if (share_len_ != UINT64_MAX) {
					std::lock_guard<std::mutex> lk(mu_);
					++scrc_.events;
				}
			}
			++stats.members;
			mcrc_ = 0;
			mlen_ = 0;
			++ev_;
			if (share_len_ != UINT64_MAX && pbase_ + lim == share_len_) share_cut(P, lim);   // a member ends the share
			continue;
		}
		if (share_len_ != UINT64_MAX && pbase_ + lim == share_len_) {
			share_cut(P, lim);
			continue;
		}
		spent_ = true;
	}
}

int64_t VcGzParallel::read(uint8_t *dst, size_t n)
{
	size_t got = 0;
	while (got < n) {
		const uint8_t *p;
		const int64_t k = span(&p, n - got);
		if (k <= 0) break;
		memcpy(dst + got, p, (size_t)k);
		got += (size_t)k;
	}
	return (int64_t)got;
}

void VcGzParallel::release(void *hold)
{
	std::lock_guard<std::mutex> lk(mu_);
	Piece *P = static_cast<Piece *>(hold);
	if (--P->lent > 0) return;
	for (size_t i = 0; i < lent_.size(); ++i)
		if (lent_[i].get() == P) {   // already read: reusable now
			spare_.push_back(std::move(lent_[i]));
			lent_.erase(lent_.begin() + (long)i);
			cv_.notify_all();
			return;
		}
	// still the piece being read: it goes back when it is spent
}

void VcGzParallel::shutdown()
{
	if (getenv("VAFC_GZ_PROFILE"))
		fprintf(stderr,
		        "[gzp] thread-seconds: search %.3f decode %.3f resolve %.3f crc %.3f; waits: workers %.3f "
		        "sequencer-chunk %.3f sequencer-room %.3f reader %.3f\n",
		        prof_search_us * 1e-6, prof_decode_us * 1e-6, prof_resolve_us * 1e-6, prof_crc_us * 1e-6,
		        prof_widle_us * 1e-6, prof_seqwait_us * 1e-6, prof_seqpush_us * 1e-6, prof_rdwait_us * 1e-6);
	{
		std::lock_guard<std::mutex> lk(mu_);
		stop_ = true;
		cv_.notify_all();
	}
	if (seq_.joinable()) seq_.join();
	for (auto &t : workers_) t.join();
	workers_.clear();
	if (p_) munmap((void *)p_, (size_t)n_);
	p_ = nullptr;
	if (fd_ >= 0) close(fd_);
	fd_ = -1;
}

VcGzParallel *vc_gzp_open(const char *path, int threads, uint64_t chunk_bytes)
{
	VcGzParallel *g = new VcGzParallel;
	if (!g->start(path, threads, chunk_bytes)) {
		delete g;
		return nullptr;
	}
	return g;
}

int64_t vc_gzp_read(VcGzParallel *g, uint8_t *dst, size_t n) { return g->read(dst, n); }

int64_t vc_gzp_span(VcGzParallel *g, const uint8_t **p, size_t max) { return g->span(p, max); }

int64_t vc_gzp_span_hold(VcGzParallel *g, const uint8_t **p, size_t max, void **hold) { return g->span(p, max, hold); }

void vc_gzp_release(VcGzParallel *g, void *hold) { g->release(hold); }

void vc_gzp_stats(VcGzParallel *g, VcGzStats *st) { g->get_stats(st); }

void vc_gzp_close(VcGzParallel *g)
{
	const double t0 = gz_now();
	delete g;
	if (getenv("VAFC_GZ_PROFILE")) fprintf(stderr, "[gzp] close %.3f s\n", gz_now() - t0);
}

bool vc_gzp_scan_share(const char *path, int threads, uint64_t chunk_bytes, uint64_t begin, uint64_t end,
                       VcGzShare *sh, uint16_t *window_sym)
{
	GzShareOpts so;
	so.scan = true;
	so.begin = begin;
	so.end = end;
	VcGzParallel *g = new VcGzParallel;
	if (!g->start(path, threads, chunk_bytes, &so)) {
		delete g;
		return false;
	}
	g->scan_result(sh, window_sym);
	delete g;
	return true;
}

bool vc_gzp_scan_share_hold(const char *path, int threads, uint64_t chunk_bytes, uint64_t begin, uint64_t end,
                            uint64_t hold_bytes, VcGzShare *sh, uint16_t *window_sym, VcGzParallel **held)
{
	GzShareOpts so;
	so.scan = true;
	so.begin = begin;
	so.end = end;
	so.hold_bytes = hold_bytes;
	*held = nullptr;
	VcGzParallel *g = new VcGzParallel;
	if (!g->start(path, threads, chunk_bytes, &so)) {
		delete g;
		return false;
	}
	g->scan_result(sh, window_sym);
	if (g->held()) *held = g;
	else delete g;
	return true;
}

bool vc_gzp_resume_share(VcGzParallel *g, const uint8_t *window, uint64_t text_len)
{
	return g->resume(window, text_len);
}

VcGzParallel *vc_gzp_open_share(const char *path, int threads, uint64_t chunk_bytes, bool first_share,
                                uint64_t start_bit, const uint8_t *window, uint64_t text_len)
{
	GzShareOpts so;
	so.first_share = first_share;
	so.start_bit = start_bit;
	so.window = window;
	so.text_len = text_len;
	VcGzParallel *g = new VcGzParallel;
	if (!g->start(path, threads, chunk_bytes, &so)) {
		delete g;
		return nullptr;
	}
	return g;
}

void vc_gzp_share_crc(VcGzParallel *g, VcGzShareCrc *out) { g->share_crc(out); }

// ---------------------------------------------------------------------------
// host-only test hooks (C ABI): the whole decompressed stream, parallel and
// through gzread, into caller buffers
// ---------------------------------------------------------------------------
extern "C" int64_t vc_gz_inflate_parallel(const char *path, int threads, uint64_t chunk_bytes, uint8_t *out,
                                          uint64_t cap, uint64_t *stats6)
{
	VcGzParallel *g = vc_gzp_open(path, threads, chunk_bytes);
	if (!g) return -1;
	uint64_t tot = 0;
	for (;;) {   // spans: no copy unless the caller wants the bytes
		const uint8_t *q;
		const int64_t r = g->span(&q, (size_t)1 << 20);
		if (r <= 0) break;
		if (out && tot < cap) memcpy(out + tot, q, (size_t)std::min<uint64_t>((uint64_t)r, cap - tot));
		tot += (uint64_t)r;
	}
	if (stats6) {
		VcGzStats s;
		g->get_stats(&s);
		stats6[0] = s.chunks;
		stats6[1] = s.accepted;
		stats6[2] = s.skipped;
		stats6[3] = s.fallback;
		stats6[4] = s.members;
		stats6[5] = (uint64_t)s.crc_error;
	}
	vc_gzp_close(g);
	return (int64_t)tot;
}

extern "C" int64_t vc_gz_inflate_zlib(const char *path, uint8_t *out, uint64_t cap)
{
	gzFile f = gzopen(path, "r");
	if (!f) return -1;
	uint64_t tot = 0;
	std::vector<uint8_t> tmp((size_t)1 << 20);
	for (;;) {
		const int r = gzread(f, tmp.data(), (unsigned)tmp.size());
		if (r <= 0) break;
		if (out && tot < cap) memcpy(out + tot, tmp.data(), (size_t)std::min<uint64_t>((uint64_t)r, cap - tot));
		tot += (uint64_t)r;
	}
	gzclose(f);
	return (int64_t)tot;
}

extern "C" uint32_t vc_gz_crc32(uint32_t crc, const uint8_t *p, uint64_t n) { return vc_crc32(crc, p, n); }

extern "C" uint32_t vc_gz_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2)
{
	return (uint32_t)crc32_combine64(crc1, crc2, (z_off64_t)len2);
}

extern "C" void vc_gz_share_close(vc_gz_share *h)
{
	if (!h) return;
	if (h->g) vc_gzp_close(h->g);
	delete h;
}

extern "C" int vc_gz_share_scan(const char *path, uint64_t begin, uint64_t end, int n_threads, uint64_t chunk_bytes,
                                vc_gz_share_info *out, uint16_t *window_sym)
{
	if (!path || !out || end <= begin) return VC_EINVAL;
	VcGzShare sh;
	if (!vc_gzp_scan_share(path, n_threads < 1 ? 1 : n_threads, chunk_bytes, begin, end, &sh, window_sym))
		return VC_EIO;
	out->start_bit = sh.start_bit;
	out->end_bit = sh.end_bit;
	out->text_len = sh.text_len;
	out->ok = sh.ok ? 1u : 0u;
	out->ended = sh.start_bit != UINT64_MAX && sh.end_bit == UINT64_MAX ? 1u : 0u;
	return VC_OK;
}
