// vafc_ingest.cpp -- see vafc_ingest.h.
#include "vafc_ingest.h"
#include "vafc_affinity.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/mman.h>
#include <immintrin.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "vafc_fastq.h"
#include "vafc_gzip.h"

namespace {

struct Piece {
	uint64_t j = 0;               // piece index (the ring holds `slots` pieces)
	uint64_t a = 0, b = 0;        // nominal byte range [a, b)
	int64_t start = -1;           // header offset parsing began at; -1: no record found
	uint64_t end = 0;             // header offset of the first record at or past b; text size at EOF
	bool eof = false;             // the reader hit end of input inside this piece
	uint64_t n = 0, bytes = 0;    // accepted reads (len >= k) in the slot, their bases
	std::vector<uint64_t> errs;   // a -2 came after this many accepted reads
	VcSlotBuf buf;
	int rc = VC_OK;
	bool ready = false;
};

double ing_clock(clockid_t id)
{
	struct timespec ts;
	clock_gettime(id, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Per-thread tallies of the reads out of a plain file (the copy out of the
// page cache): seconds and bytes, reset by each worker when it starts.
struct IoTally {
	double read_s = 0;
	uint64_t read_bytes = 0;
};
thread_local IoTally io_tally;

ssize_t pread_full(int fd, uint8_t *p, size_t n, uint64_t off)
{
	size_t got = 0;
	while (got < n) {
		ssize_t r = pread(fd, p + got, n - got, (off_t)(off + got));
		if (r < 0 && errno == EINTR) continue;
		if (r <= 0) break;
		got += (size_t)r;
	}
	return (ssize_t)got;
}

// How accepted sequences reach the slot (VAFC_SLOT_COPY): 0 one memcpy per
// read as it is parsed; 1 the same copies deferred and done in batches of
// about 32 KiB (or before the reader's window is refilled), so their time is
// measured; 2 batches gathered in a small L1-resident stage and written to the
// slot with non-temporal stores, whole 64-byte lines only (the slot is read
// next by the DMA engine, not the CPU: regular stores first read every
// destination line from DRAM for ownership).
int slot_copy_mode()   // read once per pass (A/B passes in one process)
{
	const char *e = getenv("VAFC_SLOT_COPY");
	return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 2;
}

class SlotCopier {
public:
	explicit SlotCopier(int mode) : mode_(mode) {}
	void bind(uint8_t *dst) { dst_ = dst; }
	// sequence [src, src + len) goes to dst + at; in_window: src stays valid
	// until the reader's window is refilled (else: only until the next record)
	void add(const char *src, size_t len, uint64_t at, bool in_window)
	{
		if (mode_ == 0) {
			memcpy(dst_ + at, src, len);
			return;
		}
		if (!in_window || len > kStage / 2) {   // the reader's own copy, or a very long read
			flush();
			const double t0 = ing_clock(CLOCK_MONOTONIC);
			memcpy(dst_ + at, src, len);
			secs += ing_clock(CLOCK_MONOTONIC) - t0;
			bytes += len;
			return;
		}
		if (!ents_.empty() && (pend_ + len > kStage || at != d1_)) flush();
		if (ents_.empty()) d0_ = d1_ = at;
		ents_.push_back({(const uint8_t *)src, (uint32_t)len});
		d1_ += len;
		pend_ += len;
		if (pend_ >= kStage / 2) flush();
	}
	void flush()
	{
		if (ents_.empty()) return;
		const double t0 = ing_clock(CLOCK_MONOTONIC);
		uint8_t *d = dst_ + d0_;
		if (mode_ == 1) {
			for (const Ent &e : ents_) {
				memcpy(d, e.src, e.len);
				d += e.len;
			}
		} else {
			uint8_t *s = stage_;
			for (const Ent &e : ents_) {
				memcpy(s, e.src, e.len);
				s += e.len;
			}
			stream(d, stage_, pend_);
		}
		secs += ing_clock(CLOCK_MONOTONIC) - t0;
		bytes += pend_;
		ents_.clear();
		pend_ = 0;
	}
	// end of a piece: everything written and the streaming stores ordered
	// before the piece is handed to the main thread
	void finish()
	{
		flush();
		if (mode_ == 2) _mm_sfence();
	}
	static void refill_hook(void *self) { ((SlotCopier *)self)->flush(); }
	double secs = 0;
	uint64_t bytes = 0;

private:
	struct Ent {
		const uint8_t *src;
		uint32_t len;
	};
	static constexpr size_t kStage = (size_t)32 << 10;
	int mode_;
	uint8_t *dst_ = nullptr;
	std::vector<Ent> ents_;
	uint64_t d0_ = 0, d1_ = 0;
	size_t pend_ = 0;
	alignas(64) uint8_t stage_[kStage];

	// n bytes from s to d: the partial lines at either end with regular
	// stores, every whole 64-byte line of d in between with streaming stores
	__attribute__((target("avx2"))) static void stream_avx2(uint8_t *d, const uint8_t *s, size_t n)
	{
		const size_t head = (size_t)((64 - ((uintptr_t)d & 63)) & 63);
		if (n < head + 64) {
			memcpy(d, s, n);
			return;
		}
		memcpy(d, s, head);
		d += head;
		s += head;
		n -= head;
		for (; n >= 64; n -= 64, d += 64, s += 64) {
			const __m256i a = _mm256_loadu_si256((const __m256i *)s);
			const __m256i b = _mm256_loadu_si256((const __m256i *)(s + 32));
			_mm256_stream_si256((__m256i *)d, a);
			_mm256_stream_si256((__m256i *)(d + 32), b);
		}
		memcpy(d, s, n);
	}
	static void stream(uint8_t *d, const uint8_t *s, size_t n)
	{
		static const bool avx2 = __builtin_cpu_supports("avx2");
		if (avx2) stream_avx2(d, s, n);
		else memcpy(d, s, n);
	}
};

// A plain file through pread into each worker's window.  VAFC_MMAP=1 maps
// the file instead and the workers parse the page cache in place
// (VcTextSource::view): no copy, but on the box's tmpfs-cached C2 stream the
// page faults of 16 threads cost more than the copies they save -- the
// reader alone 34 against 57 GB/s of text, the CLI 12.7 against 20.5
// Gbases/s (profiles/r04g_mmap_ab.json).  Populating
// each piece's page table entries with one madvise(MADV_POPULATE_READ)
// before parsing it was worse still in round 5: 14.6 against 39.2 Gbases/s
// (profiles/r05m1_mmap_populate_bench.json).
class FdSource : public VcIngestSource {
public:
	FdSource(int fd, uint64_t size) : fd_(fd), size_(size)
	{
		const char *e = getenv("VAFC_MMAP");
		if (size_ > 0 && e && e[0] == '1') {
			void *m = mmap(nullptr, (size_t)size_, PROT_READ, MAP_SHARED, fd_, 0);
			if (m != MAP_FAILED) map_ = (const uint8_t *)m;
		}
	}
	~FdSource() override
	{
		if (map_) munmap((void *)map_, (size_t)size_);
	}
	int64_t read(uint8_t *p, size_t n, uint64_t off) override
	{
		const double t0 = ing_clock(CLOCK_MONOTONIC);
		int64_t got;
		if (!map_) {
			got = pread_full(fd_, p, n, off);
		} else if (off >= size_) {
			got = 0;
		} else {
			got = (int64_t)(size_ - off < n ? (size_t)(size_ - off) : n);
			memcpy(p, map_ + off, (size_t)got);
		}
		io_tally.read_s += ing_clock(CLOCK_MONOTONIC) - t0;
		io_tally.read_bytes += got > 0 ? (uint64_t)got : 0;
		return got;
	}
	const uint8_t *view(uint64_t off, uint64_t *avail) override
	{
		*avail = map_ && off < size_ ? size_ - off : 0;
		return map_ && off <= size_ ? map_ + off : nullptr;
	}
	bool longer_than(uint64_t off) override { return size_ > off; }

private:
	int fd_;
	uint64_t size_;
	const uint8_t *map_ = nullptr;
};

// A gzip file's text: a pump thread takes the inflater's output in order as
// held spans (the decoder's own buffers, no copy) and appends them to a list
// of blocks; readers wait for the bytes they need.  Blocks wholly before the
// release point are handed back to the decoder.  The pump stays at most
// about `window` bytes ahead of the release point unless a reader waits for
// more (a record longer than the window must still be read).
class GzSource : public VcIngestSource {
public:
	GzSource(VcGzParallel *g, uint64_t window, const uint8_t *prefix = nullptr, size_t np = 0) : g_(g), window_(window)
	{
		if (np) {   // bytes that precede the stream in the text (a gzip share's previous byte)
			Block *b = new Block;
			uint8_t *c = (uint8_t *)malloc(np);
			memcpy(c, prefix, np);
			b->p = c;
			b->len = np;
			blocks_.push_back(b);
			end_ = np;
		}
		pump_ = std::thread([this, cpus = vc_affinity_get()] {
			vc_affinity_bind(cpus);
			pump();
		});
	}
	~GzSource() override
	{
		abort();
		pump_.join();
		for (Block *b : blocks_) {
			drop(b);
		}
	}
	int64_t read(uint8_t *p, size_t n, uint64_t off) override
	{
		std::vector<std::pair<const uint8_t *, size_t>> seg;
		size_t got = 0;
		{
			std::unique_lock<std::mutex> lk(mu_);
			wait_for(lk, off + n);
			if (end_ <= off) return 0;
			got = (size_t)(end_ - off < n ? end_ - off : n);
			// the blocks holding [off, off + got); never freed under a reader
			// (release points lie before every offset still to be read)
			size_t need = got;
			uint64_t pos = off;
			for (Block *b : blocks_) {
				if (!need) break;
				if (b->off + b->len <= pos) continue;
				const size_t from = (size_t)(pos - b->off);
				const size_t take = b->len - from < need ? b->len - from : need;
				seg.emplace_back(b->p + from, take);
				pos += take;
				need -= take;
			}
		}
		size_t at = 0;
		for (auto &sg : seg) {
			memcpy(p + at, sg.first, sg.second);
			at += sg.second;
		}
		return (int64_t)got;
	}
	bool longer_than(uint64_t off) override
	{
		std::unique_lock<std::mutex> lk(mu_);
		wait_for(lk, off + 1);
		return end_ > off;
	}
	void release(uint64_t off) override
	{
		std::lock_guard<std::mutex> lk(mu_);
		if (off <= rel_) return;
		rel_ = off;
		while (blocks_.size() > 1 && blocks_.front()->off + blocks_.front()->len <= rel_) {
			drop(blocks_.front());
			blocks_.pop_front();
		}
		room_.notify_all();
	}
	void abort() override
	{
		std::lock_guard<std::mutex> lk(mu_);
		aborted_ = true;
		data_.notify_all();
		room_.notify_all();
	}

private:
	struct Block {             // a span of the inflater's output, held (not copied)
		uint64_t off = 0;      // text offset of p[0]
		size_t len = 0;
		const uint8_t *p = nullptr;
		void *hold = nullptr;  // vc_gzp_release'd once every piece before its end is parsed
	};
	VcGzParallel *g_;
	uint64_t window_;
	std::thread pump_;
	std::mutex mu_;
	std::condition_variable data_, room_;
	std::deque<Block *> blocks_;
	uint64_t end_ = 0, rel_ = 0;   // bytes produced; release point
	int waiting_ = 0;              // readers waiting for bytes not produced yet
	bool eof_ = false, aborted_ = false;

	void wait_for(std::unique_lock<std::mutex> &lk, uint64_t want)
	{
		while (end_ < want && !eof_ && !aborted_) {
			++waiting_;
			room_.notify_all();
			data_.wait(lk);
			--waiting_;
		}
	}
	const bool copy_ = getenv("VAFC_GZ_COPY") != nullptr;   // A/B: copy the spans (round-2 first design)
	void drop(Block *b)
	{
		if (b->hold) vc_gzp_release(g_, b->hold);
		else free((void *)b->p);
		delete b;
	}
	void pump()
	{
		for (;;) {
			{
				std::unique_lock<std::mutex> lk(mu_);
				room_.wait(lk, [&] { return aborted_ || end_ - rel_ < window_ || waiting_ > 0; });
				if (aborted_) break;
			}
			const uint8_t *q = nullptr;
			void *h = nullptr;
			const int64_t n = copy_ ? vc_gzp_span(g_, &q, (size_t)8 << 20)
			                        : vc_gzp_span_hold(g_, &q, (size_t)64 << 20, &h);
			if (n <= 0) break;
			Block *nb = new Block;
			if (copy_) {
				uint8_t *c = (uint8_t *)malloc((size_t)n);
				if (!c) {
					delete nb;
					break;
				}
				memcpy(c, q, (size_t)n);
				q = c;
			}
			nb->p = q;
			nb->len = (size_t)n;
			nb->hold = h;
			std::lock_guard<std::mutex> lk(mu_);
			nb->off = end_;
			blocks_.push_back(nb);
			end_ += (uint64_t)n;
			data_.notify_all();
		}
		std::lock_guard<std::mutex> lk(mu_);
		eof_ = true;
		data_.notify_all();
	}
};

const uint8_t *find_nl(const uint8_t *p, const uint8_t *e)
{
	return p < e ? (const uint8_t *)memchr(p, '\n', (size_t)(e - p)) : nullptr;
}

// First plausible record header in s[1, n) (s = the text from offset
// `from`), or -1 when none is decided inside those n bytes (at_eof: they end
// the text).  FASTQ: a line "@..." followed by a sequence line, a '+' line and
// a quality line of the same length, then '@' or end of input.  FASTA: any line
// starting with '>' or '@' (kseq ends a FASTA record at either).  A candidate is
// accepted or rejected only on bytes inside the buffer, so a longer buffer can
// only turn a -1 into an answer, never change an answer.
int64_t guess_in(const uint8_t *s, size_t n, uint64_t from, bool at_eof, bool fasta)
{
	const uint8_t *e = s + n;
	for (const uint8_t *p = s + 1; p < e; ++p) {
		if (p[-1] != '\n') {
			p = find_nl(p, e);
			if (!p) return -1;
			continue;   // p -> '\n'; the loop steps past it
		}
		if (fasta) {
			if (*p == '>' || *p == '@') return (int64_t)(from + (uint64_t)(p - s));
			continue;
		}
		if (*p != '@') continue;
		const uint8_t *n1 = find_nl(p, e);
		const uint8_t *n2 = n1 ? find_nl(n1 + 1, e) : nullptr;
		if (!n2) return -1;
		if (n2 + 1 >= e) {
			if (!at_eof) return -1;
			continue;
		}
		if (n2[1] != '+') continue;
		const uint8_t *n3 = find_nl(n2 + 1, e);
		if (!n3) return -1;
		const uint8_t *n4 = find_nl(n3 + 1, e);
		const uint8_t *qe = n4 ? n4 : (at_eof ? e : nullptr);
		if (!qe) return -1;
		if (qe - (n3 + 1) != n2 - (n1 + 1)) continue;
		if (n4 && n4 + 1 < e && n4[1] != '@') continue;
		if (n4 && n4 + 1 >= e && !at_eof) return -1;
		return (int64_t)(from + (uint64_t)(p - s));
	}
	return -1;
}

// First plausible record header at or after a (a > 0), or -1, looked for in
// the 1 MiB of text from a - 1.  Only a guess: the caller checks it against
// the previous piece's end.  The text is read in growing steps (16 KiB, 128
// KiB, 1 MiB) until guess_in decides: a FASTQ record is a few hundred bytes,
// and reading the whole MiB per piece was 6 % of the bytes the workers copied
// out of the page cache (round 6, profiles/r06a_split.json).
int64_t guess_record(VcTextSource &src, uint64_t a, bool fasta, std::vector<uint8_t> &tmp)
{
	const uint64_t from = a - 1;
	const size_t cap = (size_t)1 << 20;
	uint64_t avail = 0;
	const uint8_t *v = src.view(from, &avail);
	if (v) {
		const size_t got = (size_t)(avail < cap ? avail : cap);
		return got < 2 ? -1 : guess_in(v, got, from, got < cap, fasta);
	}
	tmp.resize(cap);
	size_t have = 0;
	for (size_t want = (size_t)16 << 10;; want = want * 8 < cap ? want * 8 : cap) {
		const int64_t got = src.read(tmp.data() + have, want - have, from + have);
		have += got > 0 ? (size_t)got : 0;
		const bool at_eof = have < want;   // a short read ends at the end of the text
		if (have < 2) return -1;
		const int64_t g = guess_in(tmp.data(), have, from, at_eof, fasta);
		if (g >= 0 || at_eof || want == cap) return g;
	}
}

// Parse records whose header lies in [start, P.b) (kseq semantics from a
// record boundary) into the piece's slot.
int parse_piece(VcTextSource &src, uint64_t start, int k, int slot, VcIngestSink &sink, VcFastqReader &rd,
                Piece &P, SlotCopier &cp)
{
	P.start = (int64_t)start;
	P.n = P.bytes = 0;
	P.errs.clear();
	P.eof = false;
	P.end = start;
	uint64_t avail = 0;
	const uint8_t *v = src.view(start, &avail);
	const char *we = getenv("VAFC_READER_WINDOW");   // test knob: the workers' window in bytes
	const size_t win = we && atoll(we) > 0 ? (size_t)atoll(we) : (size_t)1 << 20;
	if (!(v ? rd.open_view(v, avail, start) : rd.open_src(&src, start, win))) return VC_ENOMEM;
	cp.bind(P.buf.seq);
	rd.on_refill(SlotCopier::refill_hook, &cp);
	struct Unhook {   // every pending copy done and the hook gone, however the piece ends
		VcFastqReader &r;
		SlotCopier &c;
		~Unhook()
		{
			c.finish();
			r.on_refill(nullptr, nullptr);
		}
	} unhook{rd, cp};
	size_t used = 0;
	for (;;) {
		const int64_t h = rd.peek_header();
		if (h < 0) {
			P.eof = true;
			P.end = UINT64_MAX;   // nothing follows
			break;
		}
		if ((uint64_t)h >= P.b) {
			P.end = (uint64_t)h;
			break;
		}
		const int ret = rd.next();
		if (ret == -1) {
			P.eof = true;
			P.end = UINT64_MAX;
			break;
		}
		if (ret == -2) {
			P.errs.push_back(P.n);
			continue;
		}
		if (ret < k) continue;
		const size_t len = (size_t)ret;
		if (used + len > P.buf.cap_bytes || P.n + 1 > P.buf.cap_reads) {
			size_t nb = P.buf.cap_bytes, nr = P.buf.cap_reads;
			while (used + len > nb) nb = nb * 2 + len;
			while (P.n + 1 > nr) nr = nr * 2 + 1024;
			cp.flush();   // the pending sequences into the old buffers, which grow() copies
			int rc = sink.grow(slot, &P.buf, nb, nr, used, (size_t)P.n);
			if (rc != VC_OK) return rc;
			cp.bind(P.buf.seq);
		}
		cp.add(rd.seq(), len, used, rd.seq_in_window());
		P.buf.offs[P.n] = used;
		P.buf.lens[P.n] = (uint32_t)len;
		used += len;
		P.bytes += len;
		++P.n;
	}
	return VC_OK;
}

// The reference's block loop replayed over a piece's accepted reads and -2
// events (vaf-counter.c:486-517, kthread.c:97-128).  Returns how many of the
// piece's reads are counted; sets *stopped once the file has ended.
struct BlockState {
	int64_t sum = 0;
	int empty = 0;
	bool stopped = false;
};

uint64_t replay_blocks(const Piece &P, int block_bases, BlockState &S, vc_file_stats &st)
{
	uint64_t keep = 0;
	size_t e = 0;
	auto end_block = [&]() {
		if (S.sum == 0) {
			if (++S.empty >= 3) S.stopped = true;
		} else {
			++st.blocks;
		}
		S.sum = 0;
	};
	for (uint64_t i = 0; i <= P.n && !S.stopped; ++i) {
		while (e < P.errs.size() && P.errs[e] == i && !S.stopped) {
			end_block();
			++e;
		}
		if (S.stopped || i == P.n) break;
		const uint32_t len = P.buf.lens[i];
		S.sum += len;
		st.bases += len;
		st.seqs += 1;
		keep = i + 1;
		if (S.sum >= block_bases) {
			++st.blocks;
			S.sum = 0;
		}
	}
	if (P.eof && !S.stopped) {   // -1 repeats until the third empty block
		end_block();
		S.stopped = true;
	}
	return keep;
}

} // namespace

thread_local VcIngestProfile vc_ingest_last;

static double ing_now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int vc_ingest_text(VcIngestSource &src, int k, int block_bases, int threads, int slots, uint64_t piece_bytes,
                   VcIngestSink &sink, vc_file_stats &st, VcTextRange *range)
{
	// timings are always taken (a few clock reads per piece of megabytes);
	// VAFC_INGEST_PROFILE also prints them
	const bool prof_print = getenv("VAFC_INGEST_PROFILE") != nullptr;
	const int copy_mode = slot_copy_mode();
	vc_ingest_last = VcIngestProfile();
	double t_wait = 0, t_submit = 0, t_reparse = 0;
	std::atomic<uint64_t> t_parse_us{0}, t_slotwait_us{0}, t_acquire_us{0};
	const double t_begin = ing_now();
	if (threads < 1 || slots < threads + 1 || piece_bytes < 2) return VC_EINVAL;
	// the range [r0, r1) of the text (the whole text without one)
	const uint64_t r0 = range ? range->begin : 0, r1 = range ? range->end : UINT64_MAX;
	if (range) {
		if (r1 <= r0) return VC_EINVAL;
		range->first = r0 == 0 ? 0 : UINT64_MAX;
		range->next = UINT64_MAX;
		range->errs = 0;
		range->stopped = false;
	}
	if (!src.longer_than(r0)) {   // empty input / range past the end: nothing counted
		if (range) range->first = UINT64_MAX;
		return VC_OK;
	}
	if (!src.longer_than(0)) return VC_OK;   // empty input: three empty blocks, nothing counted
	bool fasta = false;
	if (range && range->format >= 0) {
		fasta = range->format == 1;
	} else {
		VcFastqReader rd;
		if (!rd.open_src(&src, 0, (size_t)1 << 16)) return VC_ENOMEM;
		const int64_t h = rd.peek_header();
		if (h < 0) {                  // no record at all
			if (range) range->first = UINT64_MAX;
			return VC_OK;
		}
		uint8_t c = 0;
		if (src.read(&c, 1, (uint64_t)h) == 1) fasta = c == '>';
	}
	// piece j lives in pcs[j % slots] and fills slot j % slots; a worker takes
	// piece j once piece j - slots has been released by the main thread
	std::vector<Piece> pcs((size_t)slots);
	std::mutex mu;
	std::condition_variable cv;
	uint64_t released = 0;            // pieces the main thread is done with
	uint64_t n_pieces = UINT64_MAX;   // known once a worker finds its piece past the end
	bool abort = false;
	std::atomic<uint64_t> next{0};

	const VcCpuSet cpus = vc_affinity_get();   // vc_count_file's placement (vafc_affinity.h)
	// the workers' own tallies, added up as each worker ends
	std::atomic<uint64_t> w_read_ns{0}, w_read_bytes{0}, w_copy_ns{0}, w_copy_bytes{0}, w_guess_ns{0};
	std::atomic<uint64_t> w_cpu_ns{0}, w_wall_ns{0};
	auto worker_loop = [&](VcFastqReader &rd, std::vector<uint8_t> &tmp, SlotCopier &cp) {
		for (;;) {
			const uint64_t j = next.fetch_add(1);
			const double w0 = ing_now();
			{
				std::unique_lock<std::mutex> lk(mu);
				cv.wait(lk, [&] { return abort || released + (uint64_t)slots > j; });
				if (abort || j >= n_pieces) return;
			}
			// piece j of the range: [r0 + j P, min(r0 + (j + 1) P, r1))
			const uint64_t pa = r0 + j * piece_bytes;
			if (pa >= r1 || !src.longer_than(pa)) {
				std::lock_guard<std::mutex> lk(mu);
				if (j < n_pieces) n_pieces = j;
				cv.notify_all();
				return;
			}
			const double w1 = ing_now();
			const int slot = (int)(j % (uint64_t)slots);
			Piece &P = pcs[(size_t)slot];
			P.j = j;
			P.a = pa;
			P.b = r1 - pa > piece_bytes ? pa + piece_bytes : r1;
			int rc = sink.acquire(slot, &P.buf);
			t_acquire_us += (uint64_t)((ing_now() - w1) * 1e6);
			if (rc == VC_OK) {
				const double g0 = ing_now();
				const int64_t g = P.a == 0 ? 0 : guess_record(src, P.a, fasta, tmp);
				w_guess_ns += (uint64_t)((ing_now() - g0) * 1e9);
				if (g >= 0) rc = parse_piece(src, (uint64_t)g, k, slot, sink, rd, P, cp);
				else P.start = -1;
			}
			{
				const double w2 = ing_now();
				t_slotwait_us += (uint64_t)((w1 - w0) * 1e6);
				t_parse_us += (uint64_t)((w2 - w1) * 1e6);
			}
			std::lock_guard<std::mutex> lk(mu);
			P.rc = rc;
			P.ready = true;
			cv.notify_all();
		}
	};
	auto worker = [&]() {
		vc_affinity_bind(cpus);
		const double c0 = ing_clock(CLOCK_THREAD_CPUTIME_ID), t0 = ing_now();
		io_tally = IoTally();
		VcFastqReader rd;
		std::vector<uint8_t> tmp;
		SlotCopier cp(copy_mode);
		worker_loop(rd, tmp, cp);
		w_read_ns += (uint64_t)(io_tally.read_s * 1e9);
		w_read_bytes += io_tally.read_bytes;
		w_copy_ns += (uint64_t)(cp.secs * 1e9);
		w_copy_bytes += cp.bytes;
		w_cpu_ns += (uint64_t)((ing_clock(CLOCK_THREAD_CPUTIME_ID) - c0) * 1e9);
		w_wall_ns += (uint64_t)((ing_now() - t0) * 1e9);
	};
	const double main_cpu0 = ing_clock(CLOCK_THREAD_CPUTIME_ID);
	std::vector<std::thread> pool;
	for (int t = 0; t < threads; ++t) pool.emplace_back(worker);

	int rc = VC_OK;
	BlockState S;
	uint64_t expect = 0;              // where the next record's header is
	uint64_t np = 0;
	VcFastqReader rd;
	SlotCopier mcp(copy_mode);   // the main thread's re-parses
	for (uint64_t j = 0;; ++j) {
		const int slot = (int)(j % (uint64_t)slots);
		Piece &P = pcs[(size_t)slot];
		const double m0 = ing_now();
		{
			std::unique_lock<std::mutex> lk(mu);
			cv.wait(lk, [&] { return (P.ready && P.j == j) || n_pieces <= j; });
			if (!(P.ready && P.j == j)) break;   // past the end of the text
		}
		np = j + 1;
		t_wait += ing_now() - m0;
		if (rc == VC_OK) rc = P.rc;
		if (j == 0 && r0 > 0) {
			// a range's first header is its first piece's guess; none found:
			// nothing is counted (the previous range's `next` tells whether
			// that is right)
			if (P.start < 0) {
				src.release(P.a);
				std::lock_guard<std::mutex> lk(mu);
				P.ready = false;
				released = 1;
				abort = true;
				cv.notify_all();
				break;
			}
			expect = (uint64_t)P.start;
			if (range) range->first = expect;
		}
		if (rc == VC_OK && !S.stopped && P.b > expect) {
			if (P.start < 0 || (uint64_t)P.start != expect) { // a wrong guess: parse from the true boundary
				const double r0 = ing_now();
				rc = parse_piece(src, expect, k, slot, sink, rd, P, mcp);
				t_reparse += ing_now() - r0;
			}
			if (rc == VC_OK) {
				expect = P.end;
				if (range) range->errs += P.errs.size();
				const uint64_t keep = replay_blocks(P, block_bases, S, st);
				if (keep) {
					const uint64_t bytes = (uint64_t)P.buf.offs[keep - 1] + P.buf.lens[keep - 1];
					const double s0 = ing_now();
					rc = sink.submit(slot, P.buf, keep, bytes);
					t_submit += ing_now() - s0;
				}
			}
		}
		// later reads start at the next piece's guess (one byte before it) or
		// at the next record boundary
		const uint64_t nxt = r0 + (j + 1) * piece_bytes - 1;
		src.release(expect < nxt ? expect : nxt);
		const bool done = rc != VC_OK || S.stopped;
		{
			std::lock_guard<std::mutex> lk(mu);
			P.ready = false;
			released = j + 1;
			if (done) abort = true;
			cv.notify_all();
		}
		if (done) break;   // workers see abort; pieces not yet taken are dropped
	}
	src.abort();   // wake workers still reading pieces that are no longer needed
	for (auto &t : pool) t.join();
	{
		VcIngestProfile &L = vc_ingest_last;
		L.total = ing_now() - t_begin;
		L.main_wait = t_wait;
		L.submit = t_submit;
		L.reparse = t_reparse;
		L.parse = (t_parse_us.load() - t_acquire_us.load()) * 1e-6;
		L.slot_wait = t_slotwait_us.load() * 1e-6;
		L.acquire = t_acquire_us.load() * 1e-6;
		L.pieces = np;
		L.threads = threads;
		L.read_s = w_read_ns.load() * 1e-9;
		L.read_bytes = w_read_bytes.load();
		L.copy_s = w_copy_ns.load() * 1e-9;
		L.copy_bytes = w_copy_bytes.load();
		L.guess_s = w_guess_ns.load() * 1e-9;
		L.worker_cpu = w_cpu_ns.load() * 1e-9;
		L.worker_wall = w_wall_ns.load() * 1e-9;
		L.main_cpu = ing_clock(CLOCK_THREAD_CPUTIME_ID) - main_cpu0;
		L.copy_mode = copy_mode;
	}
	if (prof_print) {
		const VcIngestProfile &L = vc_ingest_last;
		fprintf(stderr, "[ingest] %llu pieces, %d threads: total %.3f s; main: wait %.3f submit %.3f reparse %.3f "
		        "cpu %.3f; workers: parse %.3f slot-wait %.3f acquire %.3f (thread-seconds); parse split: read %.3f "
		        "(%.2f GB) copy %.3f (%.2f GB, mode %d) guess %.3f; workers cpu %.3f of wall %.3f\n",
		        (unsigned long long)np, threads, L.total, t_wait, t_submit, t_reparse, L.main_cpu, L.parse,
		        L.slot_wait, L.acquire, L.read_s, L.read_bytes / 1e9, L.copy_s, L.copy_bytes / 1e9, L.copy_mode,
		        L.guess_s, L.worker_cpu, L.worker_wall);
	}
	if (range) {
		range->stopped = S.stopped;
		range->next = S.stopped ? UINT64_MAX : expect;
		if (range->first == UINT64_MAX) range->next = UINT64_MAX;
		return rc;
	}
	if (rc == VC_OK && !S.stopped) {
		// the text ended inside a record the last piece never reached (cannot
		// happen: the last piece parses to the end of the text) -- be explicit
		rc = VC_EINVAL;
	}
	return rc;
}

int vc_ingest_plain(int fd, uint64_t size, int k, int block_bases, int threads, int slots,
                    uint64_t piece_bytes, VcIngestSink &sink, vc_file_stats &st, VcTextRange *range)
{
	FdSource src(fd, size);
	return vc_ingest_text(src, k, block_bases, threads, slots, piece_bytes, sink, st, range);
}

int vc_ingest_gzip(VcGzParallel *g, int k, int block_bases, int threads, int slots, uint64_t piece_bytes,
                   uint64_t window_bytes, VcIngestSink &sink, vc_file_stats &st)
{
	GzSource src(g, window_bytes);
	return vc_ingest_text(src, k, block_bases, threads, slots, piece_bytes, sink, st);
}

int vc_ingest_gzip_share(VcGzParallel *g, const uint8_t *prefix, size_t np, int k, int block_bases, int threads,
                         int slots, uint64_t piece_bytes, uint64_t window_bytes, VcIngestSink &sink, vc_file_stats &st,
                         VcTextRange *range)
{
	GzSource src(g, window_bytes, prefix, np);
	return vc_ingest_text(src, k, block_bases, threads, slots, piece_bytes, sink, st, range);
}

int vc_gz_text_format(const char *path)
{
	gzFile f = gzopen(path, "r");
	if (!f) return -1;
	uint8_t buf[1 << 16];
	int fmt = -1;
	for (size_t seen = 0; fmt < 0 && seen < ((size_t)1 << 20);) {
		const int n = gzread(f, buf, sizeof buf);
		if (n <= 0) break;
		for (int i = 0; i < n; ++i)
			if (buf[i] == '>' || buf[i] == '@') {
				fmt = buf[i] == '>' ? 1 : 0;
				break;
			}
		seen += (size_t)n;
	}
	gzclose(f);
	return fmt;
}

// ---------------------------------------------------------------------------
// host-only hook: the parallel ingest without a device (tests, ingest speed)
// ---------------------------------------------------------------------------

#include <fcntl.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <time.h>

namespace {

class HostSink : public VcIngestSink {
public:
	HostSink(int slots, uint64_t piece, uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out, size_t lens_cap)
		: bufs_((size_t)slots), piece_(piece), seq_out_(seq_out), seq_cap_(seq_cap), lens_out_(lens_out),
		  lens_cap_(lens_cap) {}
	~HostSink() override
	{
		for (auto &b : bufs_) {
			free(b.seq);
			free(b.offs);
			free(b.lens);
		}
	}
	int acquire(int slot, VcSlotBuf *b) override
	{
		VcSlotBuf &s = bufs_[(size_t)slot];
		if (!s.seq) {
			int rc = grow(slot, &s, (size_t)piece_ + (size_t)piece_ / 4 + 64, (size_t)piece_ / 64 + 64, 0, 0);
			if (rc != VC_OK) return rc;
		}
		*b = s;
		return VC_OK;
	}
	int grow(int slot, VcSlotBuf *b, size_t bytes, size_t reads, size_t, size_t) override
	{
		VcSlotBuf &s = bufs_[(size_t)slot];
		uint8_t *q = (uint8_t *)realloc(s.seq, bytes);
		uint64_t *o = (uint64_t *)realloc(s.offs, reads * sizeof(uint64_t));
		uint32_t *l = (uint32_t *)realloc(s.lens, reads * sizeof(uint32_t));
		if (q) s.seq = q;
		if (o) s.offs = o;
		if (l) s.lens = l;
		if (!q || !o || !l) return VC_ENOMEM;
		s.cap_bytes = bytes;
		s.cap_reads = reads;
		*b = s;
		return VC_OK;
	}
	int submit(int, const VcSlotBuf &b, uint64_t n, uint64_t bytes) override
	{
		if (seq_out_ && nb_ + bytes <= seq_cap_) memcpy(seq_out_ + nb_, b.seq, (size_t)bytes);
		for (uint64_t i = 0; i < n; ++i)
			if (lens_out_ && nr_ + i < lens_cap_) lens_out_[nr_ + i] = b.lens[i];
		nb_ += bytes;
		nr_ += n;
		return VC_OK;
	}

private:
	std::vector<VcSlotBuf> bufs_;
	uint64_t piece_;
	uint8_t *seq_out_;
	size_t seq_cap_;
	uint32_t *lens_out_;
	size_t lens_cap_;
	uint64_t nb_ = 0, nr_ = 0;
};

double mono_now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

} // namespace

extern "C" int vc_scan_file_parallel(const char *path, int k, int block_bases, int n_threads,
                                     uint64_t piece_bytes, vc_file_stats *st, uint8_t *seq_out, size_t seq_cap,
                                     uint32_t *lens_out, size_t lens_cap)
{
	if (!path || !st || n_threads < 1) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	const double t0 = mono_now();
	struct stat sb;
	if (stat(path, &sb) != 0) return VC_EIO;
	if (!S_ISREG(sb.st_mode)) {   // a FIFO: read once, by the sequential reader (as vc_count_file)
		VcFastqReader rd;
		if (!rd.open(path)) return VC_EIO;
		size_t nb = 0, nr = 0;
		const int rc = vc_block_loop(rd, k, block_bases, [&](const char *q, size_t l) {
			if (seq_out && nb + l <= seq_cap) memcpy(seq_out + nb, q, l);
			if (lens_out && nr < lens_cap) lens_out[nr] = (uint32_t)l;
			nb += l;
			++nr;
			return VC_OK;
		}, local);
		local.seconds = mono_now() - t0;
		*st = local;
		return rc;
	}
	const int fd = open(path, O_RDONLY);
	if (fd < 0) return VC_EIO;
	if (fstat(fd, &sb) != 0) {
		close(fd);
		return VC_EIO;
	}
	uint8_t magic[2] = {0, 0};
	if (pread_full(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b) {
		// gzip: n_threads inflate workers (piece_bytes compressed bytes per
		// chunk), the inflated text parsed by vc_gz_parse_threads workers in
		// pieces of $VAFC_INGEST_PIECE (default 16 MB) -- vc_count_file's reader
		close(fd);
		int rc;
		VcGzParallel *g = vc_gzp_open(path, vc_gz_inflate_threads(n_threads), piece_bytes);
		if (g) {
			const char *pe = getenv("VAFC_INGEST_PIECE");
			const uint64_t piece = pe && atoll(pe) >= 2 ? (uint64_t)atoll(pe) : ((uint64_t)16 << 20);
			const int parsers = vc_gz_parse_threads(n_threads);
			HostSink sink(parsers + 2, piece, seq_out, seq_cap, lens_out, lens_cap);
			rc = vc_ingest_gzip(g, k, block_bases, parsers, parsers + 2, piece, (uint64_t)(parsers + 4) * piece * 2,
			                    sink, local);
			vc_gzp_close(g);
		} else {   // the inflater declines the file: gzread, one thread
			VcFastqReader rd;
			if (!rd.open(path)) return VC_EIO;
			size_t nb = 0, nr = 0;
			rc = vc_block_loop(rd, k, block_bases, [&](const char *q, size_t l) {
				if (seq_out && nb + l <= seq_cap) memcpy(seq_out + nb, q, l);
				if (lens_out && nr < lens_cap) lens_out[nr] = (uint32_t)l;
				nb += l;
				++nr;
				return VC_OK;
			}, local);
		}
		local.seconds = mono_now() - t0;
		*st = local;
		return rc;
	}
	if (piece_bytes < 2) {
		close(fd);
		return VC_EINVAL;
	}
	const int slots = n_threads < 2 ? n_threads + 2 : 2 * n_threads;   // as vc_count_file's reader
	HostSink sink(slots, piece_bytes, seq_out, seq_cap, lens_out, lens_cap);
	const int rc = vc_ingest_plain(fd, (uint64_t)sb.st_size, k, block_bases, n_threads, slots,
	                               piece_bytes, sink, local);
	close(fd);
	local.seconds = mono_now() - t0;
	*st = local;
	return rc;
}

extern "C" int vc_scan_file_range(const char *path, int k, int block_bases, int n_threads, uint64_t piece_bytes,
                                  uint64_t begin, uint64_t end, vc_file_stats *st, vc_range_info *ri,
                                  uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out, size_t lens_cap)
{
	if (!path || !st || !ri || n_threads < 1 || piece_bytes < 2 || end <= begin) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	*ri = vc_range_info{UINT64_MAX, UINT64_MAX, 0, 0, 1};
	const double t0 = mono_now();
	struct stat sb;
	if (stat(path, &sb) != 0) return VC_EIO;
	const int fd = S_ISREG(sb.st_mode) ? open(path, O_RDONLY) : -1;   // a FIFO is opened once, below
	if (S_ISREG(sb.st_mode) && fd < 0) return VC_EIO;
	uint8_t magic[2] = {0, 0};
	const bool reg = fd >= 0 && fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
	if (!reg || (pread_full(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b)) {
		if (fd >= 0) close(fd);   // not split (vc_count_file_range): the first range takes the whole file
		int rc = VC_OK;
		if (begin == 0) {
			rc = vc_scan_file_parallel(path, k, block_bases, n_threads, piece_bytes, &local, seq_out, seq_cap,
			                           lens_out, lens_cap);
			if (rc == VC_OK) *ri = vc_range_info{0, UINT64_MAX, 0, 1, 1};
		}
		local.seconds = mono_now() - t0;
		*st = local;
		return rc;
	}
	const int slots = n_threads < 2 ? n_threads + 2 : 2 * n_threads;
	HostSink sink(slots, piece_bytes, seq_out, seq_cap, lens_out, lens_cap);
	VcTextRange R;
	R.begin = begin;
	R.end = end;
	const int rc = vc_ingest_plain(fd, (uint64_t)sb.st_size, k, block_bases, n_threads, slots, piece_bytes, sink,
	                               local, &R);
	close(fd);
	*ri = vc_range_info{R.first, R.next, R.errs, R.stopped ? 1u : 0u, 0u};
	local.seconds = mono_now() - t0;
	*st = local;
	return rc;
}

// The host-only count of one gzip share from an open inflater (closed here).
static int scan_gz_share_g(VcGzParallel *g, int fmt, int k, int first_share, const uint8_t *window, uint64_t text_len,
                           int block_bases, int parsers, vc_file_stats &local, vc_range_info *ri,
                           vc_gz_share_crc *crc, uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out,
                           size_t lens_cap)
{
	const char *pe = getenv("VAFC_INGEST_PIECE");
	const uint64_t piece = pe && atoll(pe) >= 2 ? (uint64_t)atoll(pe) : ((uint64_t)16 << 20);
	HostSink sink(parsers + 2, piece, seq_out, seq_cap, lens_out, lens_cap);
	const size_t np = first_share ? 0 : 1;
	VcTextRange R;
	R.begin = np;
	R.end = np + text_len;
	R.format = fmt;
	const int rc = vc_ingest_gzip_share(g, first_share ? nullptr : window + 32767, np, k, block_bases, parsers,
	                                    parsers + 2, piece, (uint64_t)(parsers + 4) * piece * 2, sink, local, &R);
	VcGzShareCrc c;
	vc_gzp_share_crc(g, &c);
	vc_gzp_close(g);
	*ri = vc_range_info{R.first == UINT64_MAX ? UINT64_MAX : R.first - np,
	                    R.next == UINT64_MAX ? UINT64_MAX : R.next - np - text_len, R.errs, R.stopped ? 1u : 0u, 0u};
	*crc = vc_gz_share_crc{c.events, c.head_crc, c.head_len, c.head_expect_crc, c.head_expect_isize, c.tail_crc,
	                       c.tail_len, c.crc_error, c.complete};
	return rc;
}

extern "C" int vc_scan_gz_share(const char *path, int k, int first_share, uint64_t start_bit, const uint8_t *window,
                                uint64_t text_len, int block_bases, int n_threads, vc_file_stats *st,
                                vc_range_info *ri, vc_gz_share_crc *crc, uint8_t *seq_out, size_t seq_cap,
                                uint32_t *lens_out, size_t lens_cap)
{
	if (!path || !st || !ri || !crc || n_threads < 1 || text_len == 0 || (!first_share && !window)) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	*ri = vc_range_info{UINT64_MAX, UINT64_MAX, 0, 0, 0};
	memset(crc, 0, sizeof *crc);
	const double t0 = mono_now();
	const int fmt = vc_gz_text_format(path);
	if (fmt < 0) return VC_EINVAL;
	const char *ce = getenv("VAFC_GZ_CHUNK");   // test knob: compressed bytes per chunk
	VcGzParallel *g = vc_gzp_open_share(path, vc_gz_inflate_threads(n_threads), ce ? (uint64_t)atoll(ce) : 0,
	                                    first_share != 0, start_bit, window, text_len);
	if (!g) return VC_EIO;
	const int rc = scan_gz_share_g(g, fmt, k, first_share, window, text_len, block_bases,
	                               vc_gz_parse_threads(n_threads), local, ri, crc, seq_out, seq_cap, lens_out,
	                               lens_cap);
	local.seconds = mono_now() - t0;
	*st = local;
	return rc;
}

extern "C" int vc_scan_gz_share_held(vc_gz_share *h, int k, int first_share, const uint8_t *window, uint64_t text_len,
                                     int block_bases, int n_threads, vc_file_stats *st, vc_range_info *ri,
                                     vc_gz_share_crc *crc, uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out,
                                     size_t lens_cap)
{
	if (!h || !h->g || !st || !ri || !crc || n_threads < 1 || text_len == 0 || (!first_share && !window))
		return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	*ri = vc_range_info{UINT64_MAX, UINT64_MAX, 0, 0, 0};
	memset(crc, 0, sizeof *crc);
	const double t0 = mono_now();
	if (h->format < 0) return VC_EINVAL;
	VcGzParallel *g = h->g;
	h->g = nullptr;   // counted once; scan_gz_share_g closes it
	if (!vc_gzp_resume_share(g, first_share ? nullptr : window, text_len)) {
		vc_gzp_close(g);
		return VC_EINVAL;
	}
	const int rc = scan_gz_share_g(g, h->format, k, first_share, window, text_len, block_bases,
	                               vc_gz_held_parse_threads(n_threads), local, ri, crc, seq_out, seq_cap, lens_out,
	                               lens_cap);
	local.seconds = mono_now() - t0;
	*st = local;
	return rc;
}

extern "C" uint64_t vc_ingest_profile(double *prof)
{
	const VcIngestProfile &L = vc_ingest_last;
	if (prof) {
		prof[0] = L.total;
		prof[1] = L.main_wait;
		prof[2] = L.submit;
		prof[3] = L.reparse;
		prof[4] = L.parse;
		prof[5] = L.slot_wait;
		prof[6] = L.acquire;
	}
	return L.pieces;
}

extern "C" uint64_t vc_ingest_profile_ex(double *prof, int n)
{
	const VcIngestProfile &L = vc_ingest_last;
	const double v[VC_INGEST_PROFILE_FIELDS] = {
		L.total, L.main_wait, L.submit, L.reparse, L.parse, L.slot_wait, L.acquire, L.read_s,
		(double)L.read_bytes, L.copy_s, (double)L.copy_bytes, L.guess_s, L.worker_cpu, L.worker_wall,
		L.main_cpu, (double)L.threads, (double)L.copy_mode};
	for (int i = 0; prof && i < n && i < VC_INGEST_PROFILE_FIELDS; ++i) prof[i] = v[i];
	return L.pieces;
}
