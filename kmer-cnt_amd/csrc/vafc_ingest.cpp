// vafc_ingest.cpp -- see vafc_ingest.h.
#include "vafc_ingest.h"
#include "vafc_affinity.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/mman.h>
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
		if (!map_) return pread_full(fd_, p, n, off);
		if (off >= size_) return 0;
		const size_t got = size_ - off < n ? (size_t)(size_ - off) : n;
		memcpy(p, map_ + off, got);
		return (int64_t)got;
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
	GzSource(VcGzParallel *g, uint64_t window) : g_(g), window_(window)
	{
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

// First plausible record header at or after a (a > 0), or -1.  FASTQ: a line
// "@..." followed by a sequence line, a '+' line and a quality line of the
// same length, then '@' or end of input.  FASTA: any line starting with '>'
// or '@' (kseq ends a FASTA record at either).  Only a guess: the caller
// checks it against the previous piece's end.
int64_t guess_record(VcTextSource &src, uint64_t a, bool fasta, std::vector<uint8_t> &tmp)
{
	const uint64_t from = a - 1;
	const size_t want = (size_t)1 << 20;
	uint64_t avail = 0;
	const uint8_t *s = src.view(from, &avail);
	int64_t got;
	if (s) {
		got = (int64_t)(avail < want ? avail : want);
	} else {
		tmp.resize(want);
		got = src.read(tmp.data(), want, from);
		s = tmp.data();
	}
	if (got < 2) return -1;
	const uint8_t *e = s + got;
	const bool at_eof = (size_t)got < want;   // a short read ends at the end of the text
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
		if (n2 + 1 >= e || n2[1] != '+') continue;
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

// Parse records whose header lies in [start, P.b) (kseq semantics from a
// record boundary) into the piece's slot.
int parse_piece(VcTextSource &src, uint64_t start, int k, int slot, VcIngestSink &sink, VcFastqReader &rd,
                Piece &P)
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
			int rc = sink.grow(slot, &P.buf, nb, nr, used, (size_t)P.n);
			if (rc != VC_OK) return rc;
		}
		memcpy(P.buf.seq + used, rd.seq(), len);
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
	{
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
	auto worker = [&]() {
		vc_affinity_bind(cpus);
		VcFastqReader rd;
		std::vector<uint8_t> tmp;
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
				const int64_t g = P.a == 0 ? 0 : guess_record(src, P.a, fasta, tmp);
				if (g >= 0) rc = parse_piece(src, (uint64_t)g, k, slot, sink, rd, P);
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
	std::vector<std::thread> pool;
	for (int t = 0; t < threads; ++t) pool.emplace_back(worker);

	int rc = VC_OK;
	BlockState S;
	uint64_t expect = 0;              // where the next record's header is
	uint64_t np = 0;
	VcFastqReader rd;
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
				rc = parse_piece(src, expect, k, slot, sink, rd, P);
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
	}
	if (prof_print)
		fprintf(stderr, "[ingest] %llu pieces, %d threads: total %.3f s; main: wait %.3f submit %.3f reparse %.3f; "
		        "workers: parse %.3f slot-wait %.3f acquire %.3f (thread-seconds)\n", (unsigned long long)np, threads,
		        vc_ingest_last.total, t_wait, t_submit, t_reparse, vc_ingest_last.parse, vc_ingest_last.slot_wait,
		        vc_ingest_last.acquire);
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
	const int fd = open(path, O_RDONLY);
	if (fd < 0) return VC_EIO;
	struct stat sb;
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
	const int fd = open(path, O_RDONLY);
	if (fd < 0) return VC_EIO;
	struct stat sb;
	uint8_t magic[2] = {0, 0};
	const bool reg = fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
	if (!reg || (pread_full(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b)) {
		close(fd);   // not split (vc_count_file_range): the first range takes the whole file
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
