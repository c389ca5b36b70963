// vafc_ingest.h -- parallel ingest of a FASTA/FASTQ text with the
// reference's exact semantics: a plain file read
// with pread, or a gzip file's text as the parallel inflater produces it.
//
// The reference reads a file with one kseq stream inside kt_pipeline step 0
// (vaf-counter.c:486-517, kseq.h:192-232).  Here the text is cut into pieces
// that worker threads parse concurrently:
//
//   * piece j covers the nominal byte range [j P, (j+1) P).  Its worker guesses
//     the first record header at or after j P (the FASTQ four-line shape, or
//     a line start with '>'/'@' in FASTA) and parses, with kseq semantics,
//     every record whose header lies before (j+1) P; the last record may run
//     past the piece.  It stops at the header of the first record at or past
//     (j+1) P and reports that offset (`end`).
//   * the main thread takes the pieces in file order.  A piece whose start
//     equals the previous piece's end began at a true record boundary in the
//     same reader state, so its records are exactly the reference's; a piece
//     wholly inside the previous piece's records is skipped; any other piece
//     (a wrong guess) is parsed again from the previous end.
//   * the block loop (blocks of >= -b bases, reads shorter than k skipped, a
//     -2 from the reader ends a block, the file ends at the third empty
//     block; vaf-counter.c:486-517, kthread.c:97-128) is replayed over the
//     accepted reads in order, so a file cut short by empty blocks counts
//     exactly the reads the reference counts.
//
// Accepted reads go straight into the sink's slot buffers (pinned memory for
// the GPU path); the sink is handed each piece in file order.
#ifndef VAFC_INGEST_H
#define VAFC_INGEST_H

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "vafc.h"
#include "vafc_fastq.h"

// The reference's per-file block loop.  kt_pipeline(3 workers) runs
// worker_pipeline's step 0 strictly in block order and each worker retires on
// the first empty block it reads, so a file ends at its third empty block
// (kthread.c:97-128, vaf-counter.c:486-517).  Reads shorter than k are
// skipped and not counted; a -1/-2 from the reader ends the current block.
template <class Sink>
inline int vc_block_loop(VcFastqReader &rd, int k, int block_bases, Sink &&sink, vc_file_stats &st)
{
	int empty = 0, rc = VC_OK;
	while (empty < 3 && rc == VC_OK) {
		int64_t sum = 0;
		int ret;
		while ((ret = rd.next()) >= 0) {
			if (ret < k) continue;
			if ((rc = sink(rd.seq(), (size_t)ret)) != VC_OK) break;
			sum += ret;
			st.bases += (uint64_t)ret;
			st.seqs += 1;
			if (sum >= block_bases) break;
		}
		if (sum == 0) ++empty;
		else ++st.blocks;
	}
	return rc;
}


struct VcSlotBuf {
	uint8_t *seq = nullptr;       // accepted reads, concatenated
	uint64_t *offs = nullptr;
	uint32_t *lens = nullptr;
	size_t cap_bytes = 0, cap_reads = 0;
};

class VcIngestSink {
public:
	virtual ~VcIngestSink() = default;
	// worker thread: slot `slot` may be written (its previous piece has been
	// consumed); fill *b with its buffers
	virtual int acquire(int slot, VcSlotBuf *b) = 0;
	// worker thread: enlarge slot buffers to at least (bytes, reads), keeping
	// the first `used_bytes` / `used_reads` entries
	virtual int grow(int slot, VcSlotBuf *b, size_t bytes, size_t reads, size_t used_bytes,
	                 size_t used_reads) = 0;
	// main thread, file order: the first n reads (bytes of sequence) of the slot
	// are accepted
	virtual int submit(int slot, const VcSlotBuf &b, uint64_t n, uint64_t bytes) = 0;
};

// The text the pieces are cut from.
class VcIngestSource : public VcTextSource {
public:
	// Whether the text is longer than off bytes (waits until that is known).
	virtual bool longer_than(uint64_t off) = 0;
	// No byte before off will be read again.
	virtual void release(uint64_t) {}
	// The pass ended early: wake and end every read (short reads from now on).
	virtual void abort() {}
};

// A byte range of the text (one rank's share of a file, vc_count_file_range):
// the records whose header lies in [first, end), where first is the header
// found at or after begin (begin = 0: the text's start; later: a guess, as for
// a piece, that only the previous range's `next` can confirm).  The block
// loop starts afresh at `first`.  Out: first (UINT64_MAX: no header found
// within the reader's look-ahead -- nothing was counted), next (the header of
// the first record at or past end; UINT64_MAX: the text ended first), errs
// (reader -2 returns met) and stopped (the block loop ended the text inside
// the range).  Consecutive ranges count exactly the whole text's reads iff each
// range's first equals the previous range's next and no range met a -2
// (without one, a block ends empty only at the end of the text).
struct VcTextRange {
	uint64_t begin = 0, end = UINT64_MAX;
	uint64_t first = 0, next = UINT64_MAX, errs = 0;
	bool stopped = false;
	int format = -1;   // 1 FASTA, 0 FASTQ, -1: from the text's first header (a gzip share starts mid-stream)
};

// Where the last vc_ingest_text pass of the calling thread spent its time
// (vc_ingest_profile, include/vafc.h): wall seconds, main-thread seconds
// waiting for the next piece, submitting pieces (the sink: H2D copies and
// kernel launches), re-parsing mis-guessed pieces; worker thread-seconds
// parsing, waiting for a slot the main thread has not released, and waiting
// in the sink's acquire (the slot's previous copy still in flight).
// The workers' parse splits further into the reads out of the source
// (pread: the copy out of the page cache), the batched sequence copies into
// the slots (VAFC_SLOT_COPY 1/2; 0 copies per read, untimed) and the record
// guesses; their CPU seconds against their wall seconds tell descheduled
// time (a CPU quota's throttling) from work.
struct VcIngestProfile {
	double total = 0, main_wait = 0, submit = 0, reparse = 0, parse = 0, slot_wait = 0, acquire = 0;
	double read_s = 0, copy_s = 0, guess_s = 0, worker_cpu = 0, worker_wall = 0, main_cpu = 0;
	uint64_t read_bytes = 0, copy_bytes = 0;
	uint64_t pieces = 0;
	int threads = 0, copy_mode = 0;
};
extern thread_local VcIngestProfile vc_ingest_last;

// Whole-text pass (range == NULL) or the records of one range.  threads >= 1
// parse workers, `slots` >= threads + 1 slot buffers owned by the sink (piece j
// uses slot j % slots), pieces of `piece_bytes`.  Fills st (bases, seqs,
// blocks; not seconds).
int vc_ingest_text(VcIngestSource &src, int k, int block_bases, int threads, int slots, uint64_t piece_bytes,
                   VcIngestSink &sink, vc_file_stats &st, VcTextRange *range = nullptr);

// An open plain file of `size` bytes (the whole text, or one range of it).
int vc_ingest_plain(int fd, uint64_t size, int k, int block_bases, int threads, int slots,
                    uint64_t piece_bytes, VcIngestSink &sink, vc_file_stats &st, VcTextRange *range = nullptr);

// A gzip file opened with vc_gzp_open (vafc_gzip.h; the caller closes it): a
// pump thread copies the inflated stream into a window of blocks that the
// parse workers read (at most about `window_bytes` buffered ahead of the
// oldest piece still needed, unless a worker waits for more).
class VcGzParallel;
// Parse workers for gzip input inflated by `threads` workers: the inflate
// is several times slower per byte than the parse ($VAFC_GZ_PARSERS overrides).
// One in four: at -t 16 the CLI's gzip pass ran 5.07-5.14 Gbases/s with 4
// parsers against 4.36-4.52 with 3 and 4.97-5.04 with 5 once the inflater's
// buffers stopped regrowing (profiles/r06u_gz_sweep.log; one in five before).
inline int vc_gz_parse_threads(int threads)
{
	const char *e = getenv("VAFC_GZ_PARSERS");
	const int n = e && atoi(e) > 0 ? atoi(e) : (threads + 2) / 4;
	return n < 1 ? 1 : n;
}
// Parse workers for a held gzip share (vc_count_gz_share_held): its chunks
// are already inflated, so the parse takes the inflaters' place: -t of them
// ($VAFC_GZ_PARSERS overrides, as above).
inline int vc_gz_held_parse_threads(int threads)
{
	const char *e = getenv("VAFC_GZ_PARSERS");
	const int n = e && atoi(e) > 0 ? atoi(e) : threads;
	return n < 1 ? 1 : n;
}
// Inflate workers for gzip input: -t of them, next to the parse workers
// (measured on a 16-CPU share: 16 inflate + 3 parse workers beat 13 + 3 and
// 11 + 3, profiles/r02_gz_sweep3.log); $VAFC_GZ_INFLATERS overrides.
inline int vc_gz_inflate_threads(int threads)
{
	const char *e = getenv("VAFC_GZ_INFLATERS");
	if (e && atoi(e) > 0) return atoi(e);
	return threads < 1 ? 1 : threads;
}
int vc_ingest_gzip(VcGzParallel *g, int k, int block_bases, int threads, int slots, uint64_t piece_bytes,
                   uint64_t window_bytes, VcIngestSink &sink, vc_file_stats &st);
// One share of a gzip stream (vafc_gzip.h, vc_gzp_open_share): the text is
// prefix[0..np) (the last byte before the share, so that the first piece's
// guess sees whether the share starts at a line start) followed by the
// share's stream; range covers [np, np + text_len).
int vc_ingest_gzip_share(VcGzParallel *g, const uint8_t *prefix, size_t np, int k, int block_bases, int threads,
                         int slots, uint64_t piece_bytes, uint64_t window_bytes, VcIngestSink &sink, vc_file_stats &st,
                         VcTextRange *range);
// FASTA (1) or FASTQ (0) by the first '>' or '@' of a gzip file's text (the
// first kseq_read's scan, kseq.h:197-201), -1 if none in its first MiB.
int vc_gz_text_format(const char *path);

#endif
