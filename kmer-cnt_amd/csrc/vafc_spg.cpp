// vafc_spg.cpp -- the snp-pattern-gen side of the C ABI (SURVEY.md §8(f)
// rank 2): genome loading and candidate k-mer counting on the GPU.
//
// snp-pattern-gen counts, over every sequence of a reference genome, the
// canonical k-mers that are candidate keys (the ref and alt k-mers of the
// BED's SNPs) -- count_candidate_kmers, snp-pattern-gen.c:159-190.  That is
// the vaf-counter scan with a different decode and one counter per key:
//   * the genome is copied to HBM and counted in seq_nt4 mode
//     (vc_set_nt4_decode): every chunk takes the exact seq_nt4_table decode
//     that vaf-counter's kernels use only for a read's tail;
//   * the candidate keys become a key table whose value is the key's own
//     index, so counts[i] is the number of occurrences of keys[i];
//   * chromosomes (longer than 16,384 bases) take the segmented long-read
//     kernel.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include "vafc.h"
#include "vafc_fastq.h"
#include "vafc_gzip.h"
#include "vafc_internal.h"

struct vc_fasta {
	std::vector<std::string> names;
	std::vector<uint8_t> seq;          // sequential reader
	uint8_t *raw = nullptr;            // mapped loader: malloc'd, first touched by the copy threads
	size_t raw_bytes = 0;
	std::vector<uint64_t> offs;
	std::vector<uint32_t> lens;
	~vc_fasta() { free(raw); }
	const uint8_t *data() const { return raw ? raw : seq.data(); }
	size_t bytes() const { return raw ? raw_bytes : seq.size(); }
};

// Parallel load of a FASTA file (plain, or gzip through the parallel
// inflater into memory) whose records kseq reads as "header
// line, then sequence lines up to the next line starting with '>'"
// (kseq.h:192-232): the file is mapped, T threads find the record headers and
// then copy each record's bytes minus the newlines straight to their final
// place (per-segment counts, prefix sums, copies).  Anything this does not
// restate exactly -- a first byte other than '>', a '\r', a line starting
// with '+' or '@' (kseq's FASTQ separators) -- returns false and the caller
// reads the file with the sequential kseq-semantics reader instead.
static bool fasta_parse_buffer(const uint8_t *d, size_t n, int threads, vc_fasta *fa);

static bool fasta_load_mapped(const char *path, int threads, vc_fasta *fa)
{
	const int fd = open(path, O_RDONLY);
	if (fd < 0) return false;
	struct stat sb;
	if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_size < 2) {
		close(fd);
		return false;
	}
	const size_t n = (size_t)sb.st_size;
	uint8_t magic[2] = {0, 0};
	if (pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b) {
		// gzip: the parallel inflater (vafc_gzip.h, gzread's output) into memory,
		// then the same parallel parse
		close(fd);
		VcGzParallel *g = vc_gzp_open(path, threads, 0);
		if (!g) return false;
		size_t cap = n * 4 + (1u << 20), len = 0;
		uint8_t *buf = (uint8_t *)malloc(cap);
		bool ok = buf != nullptr;
		while (ok) {
			const uint8_t *p;
			const int64_t got = vc_gzp_span(g, &p, (size_t)1 << 30);
			if (got <= 0) break;
			if (len + (size_t)got > cap) {
				size_t nc = cap * 2;
				while (nc < len + (size_t)got) nc *= 2;
				uint8_t *nb = (uint8_t *)realloc(buf, nc);
				if (!nb) {
					ok = false;
					break;
				}
				buf = nb;
				cap = nc;
			}
			memcpy(buf + len, p, (size_t)got);
			len += (size_t)got;
		}
		vc_gzp_close(g);
		try {
			ok = ok && len >= 2 && fasta_parse_buffer(buf, len, threads, fa);
		} catch (...) {
			free(buf);
			throw;
		}
		free(buf);
		return ok;
	}
	void *map = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
	close(fd);
	if (map == MAP_FAILED) return false;
	madvise(map, n, MADV_SEQUENTIAL);
	bool ok;
	try {
		ok = fasta_parse_buffer((const uint8_t *)map, n, threads, fa);
	} catch (...) {
		munmap(map, n);
		throw;
	}
	munmap(map, n);
	return ok;
}

static bool fasta_parse_buffer(const uint8_t *d, size_t n, int threads, vc_fasta *fa)
{
	bool ok = d[0] == '>';
	const int T = threads;
	// pass 1: header starts and disqualifying bytes, per thread range
	std::vector<std::vector<size_t>> heads(T);
	std::vector<char> bad(T, 0);
	auto range = [&](int t, size_t &a, size_t &b) {
		a = n * (size_t)t / (size_t)T;
		b = n * (size_t)(t + 1) / (size_t)T;
	};
	if (ok) {
		std::vector<std::thread> th;
		for (int t = 0; t < T; ++t)
			th.emplace_back([&, t] {
				size_t a, b;
				range(t, a, b);
				if (memchr(d + a, '\r', b - a)) {
					bad[t] = 1;
					return;
				}
				if (t == 0) heads[t].push_back(0);
				// line starts in [a, b): positions p with d[p - 1] == '\n'
				const uint8_t *p = a ? d + a - 1 : d;
				const uint8_t *e = d + b - 1;     // a newline at b - 1 starts a line at b (next range)
				while (p < e && (p = (const uint8_t *)memchr(p, '\n', (size_t)(e - p))) != nullptr) {
					const uint8_t c = p[1];
					if (c == '>') heads[t].push_back((size_t)(p + 1 - d));
					else if (c == '+' || c == '@') {
						bad[t] = 1;
						return;
					}
					++p;
				}
			});
		for (auto &x : th) x.join();
		for (int t = 0; t < T; ++t) ok = ok && !bad[t];
	}
	if (!ok) return false;
	// records: header [h, he), body [he + 1, next header)
	std::vector<size_t> hs;
	for (auto &v : heads) hs.insert(hs.end(), v.begin(), v.end());
	const size_t R = hs.size();
	std::vector<size_t> bs(R), be(R);
	fa->names.reserve(R);
	for (size_t r = 0; r < R; ++r) {
		const uint8_t *nl = (const uint8_t *)memchr(d + hs[r], '\n', n - hs[r]);
		const size_t he = nl ? (size_t)(nl - d) : n;
		size_t q = hs[r] + 1;                    // name: up to the first isspace byte (kseq KS_SEP_SPACE)
		while (q < he && !(d[q] == ' ' || d[q] == '\t' || d[q] == '\v' || d[q] == '\f')) ++q;
		fa->names.emplace_back((const char *)d + hs[r] + 1, q - hs[r] - 1);
		bs[r] = he < n ? he + 1 : n;
		be[r] = r + 1 < R ? hs[r + 1] : n;
	}
	// segments: the pieces of the bodies inside each thread's range
	struct Seg { size_t rec, a, b, len, out; };
	std::vector<std::vector<Seg>> segs(T);
	for (int t = 0; t < T; ++t) {
		size_t a, b;
		range(t, a, b);
		for (size_t r = 0; r < R; ++r) {
			const size_t x = bs[r] > a ? bs[r] : a, y = be[r] < b ? be[r] : b;
			if (x < y) segs[t].push_back({r, x, y, 0, 0});
		}
	}
	auto run = [&](auto fn) {
		std::vector<std::thread> th;
		for (int t = 0; t < T; ++t) th.emplace_back([&, t] { fn(t); });
		for (auto &x : th) x.join();
	};
	run([&](int t) {                            // pass 2a: sequence bytes per segment
		for (Seg &s : segs[t]) {
			size_t nl = 0;
			for (const uint8_t *p = d + s.a, *e = d + s.b; (p = (const uint8_t *)memchr(p, '\n', (size_t)(e - p)));
			     ++p)
				++nl;
			s.len = s.b - s.a - nl;
		}
	});
	fa->lens.assign(R, 0);
	fa->offs.assign(R, 0);
	size_t total = 0;
	for (int t = 0; t < T; ++t)                 // segments are in file order
		for (Seg &s : segs[t]) fa->lens[s.rec] += (uint32_t)s.len;
	for (size_t r = 0; r < R; ++r) {
		fa->offs[r] = total;
		total += fa->lens[r];
	}
	std::vector<size_t> cur(fa->offs.begin(), fa->offs.end());
	for (int t = 0; t < T; ++t)
		for (Seg &s : segs[t]) {
			s.out = cur[s.rec];
			cur[s.rec] += s.len;
		}
	// no zero fill: the copy threads touch every page first, in parallel
	fa->raw = (uint8_t *)malloc(total ? total : 1);
	if (!fa->raw) throw std::bad_alloc();
	fa->raw_bytes = total;
	uint8_t *o = fa->raw;
	run([&](int t) {                            // pass 2b: copy without the newlines
		for (const Seg &s : segs[t]) {
			uint8_t *w = o + s.out;
			const uint8_t *p = d + s.a, *e = d + s.b;
			while (p < e) {
				const uint8_t *q = (const uint8_t *)memchr(p, '\n', (size_t)(e - p));
				const size_t l = (size_t)((q ? q : e) - p);
				memcpy(w, p, l);
				w += l;
				p += l + (q ? 1 : 0);
			}
		}
	});
	return true;
}

// load_fasta (snp-pattern-gen.c:67-103): every record, kseq semantics, until
// the first kseq_read < 0
extern "C" int vc_fasta_load(const char *path, vc_fasta **out)
{
	if (!path || !out) return VC_EINVAL;
	*out = nullptr;
	VcFastqReader rd;   // a gzip genome is inflated in parallel (vafc_gzip.h)
	const char *te = getenv("VAFC_THREADS");
	int threads = te && atoi(te) > 0 ? atoi(te) : (int)std::thread::hardware_concurrency();
	threads = threads < 1 ? 1 : (threads > 16 ? 16 : threads);
	if (!getenv("VAFC_FASTA_SEQUENTIAL")) {    // test knob: force the sequential reader
		vc_fasta *fa = new (std::nothrow) vc_fasta;
		if (!fa) return VC_ENOMEM;
		bool done = false;
		try {
			done = fasta_load_mapped(path, threads, fa);
		} catch (...) {
			delete fa;
			return VC_ENOMEM;
		}
		if (done) {
			*out = fa;
			return VC_OK;
		}
		delete fa;
	}
	if (!rd.open_parallel(path, threads)) return VC_EIO;
	rd.keep_names(true);
	vc_fasta *fa = new (std::nothrow) vc_fasta;
	if (!fa) return VC_ENOMEM;
	try {
		// a plain file's sequence bytes never exceed its size: reserve once
		// instead of growing a genome-sized vector by doubling (each growth
		// copies everything loaded so far)
		struct stat sb;
		uint8_t magic[2] = {0, 0};
		FILE *fp = fopen(path, "rb");
		if (fp) {
			const bool gz = fread(magic, 1, 2, fp) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
			if (!gz && fstat(fileno(fp), &sb) == 0 && S_ISREG(sb.st_mode)) fa->seq.reserve((size_t)sb.st_size);
			fclose(fp);
		}
		int ret;
		while ((ret = rd.next()) >= 0) {
			fa->names.emplace_back(rd.name(), rd.name_len());
			fa->offs.push_back(fa->seq.size());
			fa->lens.push_back((uint32_t)ret);
			fa->seq.insert(fa->seq.end(), (const uint8_t *)rd.seq(), (const uint8_t *)rd.seq() + ret);
		}
	} catch (...) {
		delete fa;
		return VC_ENOMEM;
	}
	*out = fa;
	return VC_OK;
}

extern "C" int vc_fasta_count(const vc_fasta *fa) { return fa ? (int)fa->names.size() : 0; }

extern "C" const char *vc_fasta_name(const vc_fasta *fa, int i)
{
	return fa && i >= 0 && (size_t)i < fa->names.size() ? fa->names[(size_t)i].c_str() : nullptr;
}

extern "C" const uint8_t *vc_fasta_seq(const vc_fasta *fa, int i, uint32_t *len)
{
	if (!fa || i < 0 || (size_t)i >= fa->names.size()) return nullptr;
	if (len) *len = fa->lens[(size_t)i];
	return fa->data() + fa->offs[(size_t)i];
}

extern "C" int vc_fasta_data(const vc_fasta *fa, const uint8_t **seq, size_t *bytes, const uint64_t **offs,
                             const uint32_t **lens)
{
	if (!fa) return VC_EINVAL;
	if (seq) *seq = fa->data();
	if (bytes) *bytes = fa->bytes();
	if (offs) *offs = fa->offs.data();
	if (lens) *lens = fa->lens.data();
	return VC_OK;
}

extern "C" void vc_fasta_free(vc_fasta *fa) { delete fa; }

#define SPGCK(call)                                                                          \
	do {                                                                                     \
		hipError_t e_ = (call);                                                              \
		if (e_ != hipSuccess) {                                                              \
			fprintf(stderr, "[E::vafc] %s failed: %s\n", #call, hipGetErrorString(e_));     \
			rc = VC_EHIP;                                                                    \
			goto done;                                                                       \
		}                                                                                    \
	} while (0)

extern "C" int vc_count_candidates(int k, const uint8_t *seq, size_t seq_bytes, const uint64_t *offs,
                                   const uint32_t *lens, uint64_t n_seqs, const uint64_t *keys, size_t n_keys,
                                   uint32_t *counts, int device)
{
	if (k < 1 || k > 31 || (n_keys && (!keys || !counts)) || (n_seqs && (!seq || !offs || !lens)))
		return VC_EINVAL;
	for (uint64_t i = 0; i < n_seqs; ++i)
		if (offs[i] + lens[i] > seq_bytes) return VC_EINVAL;
	if (n_keys == 0) return VC_OK;
	const uint32_t n_patterns = (uint32_t)((n_keys + 1) / 2);
	std::vector<uint32_t> vals(n_keys), all(2 * (size_t)n_patterns + 2, 0);
	for (size_t i = 0; i < n_keys; ++i) vals[i] = (uint32_t)i;
	vc_ctx *ctx = nullptr;
	int rc = vc_create(&ctx, k, keys, vals.data(), n_keys, n_patterns, device);
	if (rc != VC_OK) return rc;
	vc_set_nt4_decode(ctx, 1);
	uint8_t *d_seq = nullptr;
	uint64_t *d_offs = nullptr;
	uint32_t *d_lens = nullptr;
	if (n_seqs) {
		SPGCK(hipMalloc(&d_seq, seq_bytes + 16));
		SPGCK(hipMemcpy(d_seq, seq, seq_bytes, hipMemcpyHostToDevice));
		SPGCK(hipMalloc(&d_offs, n_seqs * sizeof(uint64_t)));
		SPGCK(hipMalloc(&d_lens, n_seqs * sizeof(uint32_t)));
		SPGCK(hipMemcpy(d_offs, offs, n_seqs * sizeof(uint64_t), hipMemcpyHostToDevice));
		SPGCK(hipMemcpy(d_lens, lens, n_seqs * sizeof(uint32_t), hipMemcpyHostToDevice));
		rc = vc_count_device(ctx, d_seq, seq_bytes, d_offs, d_lens, n_seqs, nullptr);
		if (rc != VC_OK) goto done;
	}
	rc = vc_finish(ctx, all.data(), nullptr);
	if (rc == VC_OK) memcpy(counts, all.data(), n_keys * sizeof(uint32_t));
done:
	if (d_seq) (void)hipFree(d_seq);
	if (d_offs) (void)hipFree(d_offs);
	if (d_lens) (void)hipFree(d_lens);
	vc_destroy(ctx);
	return rc;
}
