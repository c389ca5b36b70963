// vafc_fastq.cpp -- see vafc_fastq.h.
#include "vafc_fastq.h"
#include "vafc_gzip.h"

#include <ctype.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <unistd.h>
#include <immintrin.h>

// The first up to four '\n' in [p, e), in order, into nl[]; returns how many.
// One vector compare per 32 (16) bytes and a bit scan per line end, instead
// of a memchr call per line (the record fast path of next() asks for four).
__attribute__((target("avx2"))) static int newlines4_avx2(const uint8_t *p, const uint8_t *e, const uint8_t **nl)
{
	int n = 0;
	const __m256i NL = _mm256_set1_epi8('\n');
	for (; p + 32 <= e; p += 32) {
		uint32_t m = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_loadu_si256((const __m256i *)p), NL));
		while (m) {
			nl[n++] = p + __builtin_ctz(m);
			if (n == 4) return 4;
			m &= m - 1;
		}
	}
	for (; p < e; ++p)
		if (*p == '\n') {
			nl[n++] = p;
			if (n == 4) return 4;
		}
	return n;
}

static int newlines4_sse2(const uint8_t *p, const uint8_t *e, const uint8_t **nl)
{
	int n = 0;
	const __m128i NL = _mm_set1_epi8('\n');
	for (; p + 16 <= e; p += 16) {
		uint32_t m = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)p), NL));
		while (m) {
			nl[n++] = p + __builtin_ctz(m);
			if (n == 4) return 4;
			m &= m - 1;
		}
	}
	for (; p < e; ++p)
		if (*p == '\n') {
			nl[n++] = p;
			if (n == 4) return 4;
		}
	return n;
}

static int newlines4_memchr(const uint8_t *p, const uint8_t *e, const uint8_t **nl)
{
	int n = 0;
	while (n < 4 && p < e) {
		const uint8_t *q = (const uint8_t *)memchr(p, '\n', (size_t)(e - p));
		if (!q) break;
		nl[n++] = q;
		p = q + 1;
	}
	return n;
}

typedef int (*Newlines4Fn)(const uint8_t *, const uint8_t *, const uint8_t **);

// VAFC_NL_SCAN=memchr: one memchr per line (the A/B baseline).  Chosen while
// the library's constructors run, so the CPU model is initialised first
// (__builtin_cpu_supports may otherwise read it before libgcc has).
static Newlines4Fn pick_newlines4()
{
	__builtin_cpu_init();
	const char *e = getenv("VAFC_NL_SCAN");
	if (e && !strcmp(e, "memchr")) return newlines4_memchr;
	return __builtin_cpu_supports("avx2") ? newlines4_avx2 : newlines4_sse2;
}
static const Newlines4Fn newlines4 = pick_newlines4();

bool VcFastqReader::open(const char *path, size_t window)
{
	close();
	fp_ = gzopen(path, "r");
	if (!fp_) return false;
	gzbuffer(fp_, 1u << 20);
	cap_ = window;
	buf_ = (uint8_t *)malloc(cap_);
	b_ = e_ = 0;
	eof_ = false;
	hdr_ = 0;
	return buf_ != nullptr;
}

bool VcFastqReader::open_parallel(const char *path, int threads, uint64_t chunk_bytes, size_t window)
{
	close();
	if (threads >= 1) {
		if (!chunk_bytes) {   // 0: sized by the inflater from the file size
			const char *e = getenv("VAFC_GZ_CHUNK");   // test knob
			chunk_bytes = e && atoll(e) > 0 ? (uint64_t)atoll(e) : 0;
		}
		gzp_ = vc_gzp_open(path, threads, chunk_bytes);
	}
	if (!gzp_) return open(path, window);
	cap_ = 0;
	buf_ = nullptr;   // points into the inflater's pieces (not owned)
	b_ = e_ = 0;
	eof_ = false;
	hdr_ = 0;
	return true;
}

bool VcFastqReader::open_src(VcTextSource *src, uint64_t off, size_t window)
{
	// a worker reopens its reader for every piece: keep an owned window of
	// the same size (a fresh 1 MB malloc is an mmap, first-touch faults and
	// an munmap whose TLB shootdown stops every thread of the process)
	uint8_t *keep = nullptr;
	if (buf_ && !view_ && !gzp_ && cap_ == window) {
		keep = buf_;
		buf_ = nullptr;
	}
	close();
	src_ = src;
	foff_ = base_ = off;
	cap_ = window;
	buf_ = keep ? keep : (uint8_t *)malloc(cap_);
	b_ = e_ = 0;
	eof_ = false;
	hdr_ = 0;
	return buf_ != nullptr;
}

bool VcFastqReader::open_view(const uint8_t *p, uint64_t n, uint64_t off)
{
	close();
	view_ = true;
	buf_ = (uint8_t *)p;
	cap_ = (size_t)n;
	base_ = foff_ = off;
	b_ = 0;
	e_ = (size_t)n;
	eof_ = false;
	hdr_ = 0;
	return p != nullptr || n == 0;
}

void VcFastqReader::close()
{
	if (view_) {
		buf_ = nullptr;   // not owned
		view_ = false;
	}
	seqp_ = nullptr;
	if (fp_) gzclose(fp_);
	fp_ = nullptr;
	if (gzp_) {
		vc_gzp_close(gzp_);
		buf_ = nullptr;   // not owned
	}
	gzp_ = nullptr;
	src_ = nullptr;
	free(buf_);
	buf_ = nullptr;
}

bool VcFastqReader::refill()
{
	if (eof_) return false;
	if (view_) {   // the whole text is in the window already
		eof_ = true;
		b_ = e_;
		return false;
	}
	if (seqp_) {   // the window is about to be replaced: keep this record's sequence
		seq_.l = 0;
		seq_.append((const uint8_t *)seqp_, seql_);
		seqp_ = nullptr;
	}
	ssize_t n;
	if (src_) {
		if (refill_fn_) refill_fn_(refill_arg_);
		n = (ssize_t)src_->read(buf_, cap_, foff_);
		base_ = foff_;
		if (n > 0) foff_ += (uint64_t)n;
	} else if (gzp_) {   // the inflater's own buffer, no copy
		const uint8_t *q = nullptr;
		n = (ssize_t)vc_gzp_span(gzp_, &q, (size_t)1 << 30);
		if (n > 0) {
			buf_ = (uint8_t *)q;
			b_ = 0;
			e_ = (size_t)n;
			return true;
		}
	} else {
		n = gzread(fp_, buf_, (unsigned)cap_);
	}
	if (n <= 0) {
		eof_ = true;
		b_ = e_ = 0;
		return false;
	}
	b_ = 0;
	e_ = (size_t)n;
	return true;
}

int64_t VcFastqReader::peek_header()
{
	if (!hdr_) {   // the scan of next() (kseq.h:197-201)
		int c;
		do c = getc_(); while (c != -1 && c != '>' && c != '@');
		if (c == -1) return -1;
		hdr_ = c;
		hdr_pos_ = last_pos();
	}
	return (int64_t)hdr_pos_;
}

// Bytes up to the next '\n' (consumed, not stored) appended to dst; -1 only
// if the input was exhausted on entry (kseq.h:106).  Afterwards a trailing
// '\r' of the whole accumulated string is dropped when it is longer than one
// byte (kseq.h:146).
int VcFastqReader::line(VcByteBuf *dst)
{
	if (at_end()) return -1;
	for (;;) {
		const uint8_t *p = buf_ + b_;
		const size_t n = e_ - b_;
		const uint8_t *nl = (const uint8_t *)memchr(p, '\n', n);
		if (nl) {
			dst->append(p, (size_t)(nl - p));
			b_ += (size_t)(nl - p) + 1;
			break;
		}
		dst->append(p, n);
		b_ = e_;
		if (!refill()) break;
	}
	if (dst->l > 1 && dst->s[dst->l - 1] == '\r') --dst->l;
	return (int)dst->l;
}

// line() for the quality string, of which only the length matters: the
// length and the number of trailing '\r' of the accumulated string are kept
// instead of its bytes, with the same CR rule (kseq.h:146).
int VcFastqReader::qual_line(size_t *l, size_t *tcr)
{
	if (at_end()) return -1;
	for (;;) {
		const uint8_t *p = buf_ + b_;
		const size_t n = e_ - b_;
		const uint8_t *nl = (const uint8_t *)memchr(p, '\n', n);
		const size_t seg = nl ? (size_t)(nl - p) : n;
		if (seg) {
			size_t t = 0;
			while (t < seg && p[seg - 1 - t] == '\r') ++t;
			*tcr = t == seg ? *tcr + t : t;
			*l += seg;
		}
		if (nl) {
			b_ += seg + 1;
			break;
		}
		b_ = e_;
		if (!refill()) break;
	}
	if (*l > 1 && *tcr > 0) {
		--*l;
		--*tcr;
	}
	return (int)*l;
}

// Name token: up to an isspace() byte (KS_SEP_SPACE); the delimiter (or 0 at
// end of input) is returned through delim.
int VcFastqReader::token(int *delim)
{
	*delim = 0;
	if (at_end()) return -1;
	for (;;) {
		while (b_ < e_) {
			int c = buf_[b_++];
			if (isspace(c)) {
				*delim = c;
				return 0;
			}
			if (keep_name_) name_.push(c);
		}
		if (!refill()) return 0;
	}
}

void VcFastqReader::skip_line()
{
	for (;;) {
		const uint8_t *p = buf_ + b_;
		const uint8_t *nl = (const uint8_t *)memchr(p, '\n', e_ - b_);
		if (nl) {
			b_ += (size_t)(nl - p) + 1;
			return;
		}
		b_ = e_;
		if (!refill()) return;
	}
}

int VcFastqReader::next()
{
	int c, d;
	if (!hdr_ && peek_header() < 0) return -1;   // scan to a '>' or '@' (kseq.h:197-201)
	seq_.l = name_.l = 0;
	seqp_ = nullptr;
	static const bool inplace = !(getenv("VAFC_SEQ_INPLACE") && getenv("VAFC_SEQ_INPLACE")[0] == '0');   // A/B knob
	if (inplace && hdr_ == '@' && !keep_name_ && b_ < e_) {
		// A whole four-line FASTQ record inside the window, located by its
		// first four line ends and taken only if every step below would take the common
		// branch: the header's rest up to its '\n' (the name token and the
		// comment are discarded, kseq.h:203-204), one sequence line followed by
		// a '+' line, and one quality line at least as long as the sequence
		// (kseq.h:209-229, each line with line()'s CR rule).  Anything else --
		// a record that crosses the window, wrapped sequences or qualities,
		// names kept -- falls through to the byte-wise path below, nothing
		// consumed.
		const uint8_t *p = buf_ + b_, *e = buf_ + e_;
		const uint8_t *nl[4];
		if (newlines4(p, e, nl) == 4) {
			const uint8_t *n1 = nl[0], *n2 = nl[1], *n3 = nl[2], *n4 = nl[3];
			const uint8_t *sq = n1 + 1, *q = n3 + 1;
			if (*sq != '\n' && *sq != '>' && *sq != '+' && *sq != '@' && n2[1] == '+') {
				size_t sl = (size_t)(n2 - sq);
				if (sl > 1 && sq[sl - 1] == '\r') --sl;
				size_t ql = (size_t)(n4 - q);
				if (ql > 1 && q[ql - 1] == '\r') --ql;
				if (ql >= sl) {
					seqp_ = (const char *)sq;
					seql_ = sl;
					b_ = (size_t)(n4 + 1 - buf_);
					hdr_ = 0;
					return sl == ql ? (int)sl : -2;
				}
			}
		}
	}
	if (token(&d) < 0) return -1;
	if (d != '\n' && !at_end()) skip_line();          // comment (kseq.h:204)
	c = -1;
	if (inplace && b_ < e_) {
		// In place: a sequence of one line followed by a line starting with
		// '+', '>' or '@' is exactly what the loop below would collect (its
		// first byte, then line()'s rest of the line with the CR rule), so it
		// is handed out as a pointer into the window instead of being copied
		// (refill() copies it out before the window is replaced).
		const uint8_t *p = buf_ + b_;
		const uint8_t *nl = (const uint8_t *)memchr(p, '\n', e_ - b_);
		if (nl && nl + 1 < buf_ + e_ && *p != '\n' && *p != '>' && *p != '+' && *p != '@' &&
		    (nl[1] == '+' || nl[1] == '>' || nl[1] == '@')) {
			size_t l = (size_t)(nl - p);
			if (l > 1 && p[l - 1] == '\r') --l;
			seqp_ = (const char *)p;
			seql_ = l;
			b_ = (size_t)(nl - buf_) + 2;
			c = nl[1];
		}
	}
	// sequence lines until a line starts with '+', '>' or '@' (kseq.h:209-213)
	if (!seqp_)
		while ((c = getc_()) != -1 && c != '>' && c != '+' && c != '@') {
			if (c == '\n') continue;
			seq_.push(c);
			line(&seq_);
		}
	if (c == '>' || c == '@') {
		hdr_ = c;
		hdr_pos_ = last_pos();
	}
	const size_t sl = seq_len();
	if (c != '+') return (int)sl;                     // FASTA
	do c = getc_(); while (c != -1 && c != '\n');     // rest of the '+' line
	if (c == -1) return -2;
	size_t ql = 0, qcr = 0;
	while (qual_line(&ql, &qcr) >= 0 && ql < sl) {}
	hdr_ = 0;
	return sl == ql ? (int)sl : -2;
}
