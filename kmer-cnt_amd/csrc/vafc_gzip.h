// vafc_gzip.h -- parallel gzip inflate with gzread's output (SURVEY.md §8(f)
// rank 1: "libdeflate/parallel gz").
//
// The reference reads .gz input through zlib's gzread inside kseq
// (vaf-counter.c:12,557; kseq.h:74-85), one thread per file.  This reader
// produces the same byte stream with `threads` inflate workers:
//
//   * the compressed file is cut into chunks of `chunk_bytes`.  The worker of
//     chunk j (j > 0) looks for the first bit offset in its chunk where a
//     dynamic-Huffman deflate block starts (header checks, then a trial decode
//     of the whole block) and decodes from there, without the 32 KiB history
//     it cannot know: a back-reference before the chunk start is emitted as a
//     16-bit marker naming the window position.  It stops at the first block
//     start at or past the chunk's end and reports that bit offset.
//   * a sequencer takes the chunks in file order.  A chunk whose start equals
//     the previous chunk's end began at a true block boundary, so its symbols
//     are exactly the stream's; its markers are resolved against the previous
//     32 KiB of output (by a worker, in parallel).  Any other chunk -- a wrong
//     guess, a stored or fixed-Huffman block at the boundary, an output larger
//     than the cap, corrupt or truncated data -- is inflated again by zlib
//     itself from the true boundary with the true window (inflatePrime +
//     inflateSetDictionary), so every byte delivered comes from a decode that
//     started at a verified position with the correct history.
//   * gzip members (RFC 1952) are followed across chunks: the CRC-32 and
//     length of every member are checked in order; output stops after a
//     member whose check fails, and at trailing bytes that are not a gzip
//     header -- gzread's rules.  (On corrupt input gzread also drops up to one
//     internal buffer of output before the error; that part is buffer-size
//     dependent in the reference too and is not reproduced.)
#ifndef VAFC_GZIP_H
#define VAFC_GZIP_H

#include <stddef.h>
#include <stdint.h>

struct VcGzStats {
	uint64_t chunks = 0;           // nominal chunks of the compressed file
	uint64_t accepted = 0;         // chunks whose speculative decode was used
	uint64_t skipped = 0;          // chunks wholly inside the previous chunk's blocks
	uint64_t fallback = 0;         // chunks inflated again by zlib from the true boundary
	uint64_t members = 0;          // gzip members whose check passed
	uint64_t out_bytes = 0;        // bytes delivered
	int crc_error = 0;             // a member's CRC-32 / ISIZE did not match
};

class VcGzParallel;

// nullptr if the file is not gzip, its first header is not one zlib accepts,
// or it cannot be mapped: the caller then reads it with gzread.  chunk_bytes
// 0: about four chunks per worker, 1 to 4 MiB of compressed input each.
VcGzParallel *vc_gzp_open(const char *path, int threads, uint64_t chunk_bytes);

// ---------------------------------------------------------------------------
// Shares of one gzip stream over several ranks (round 6; the torchrun driver,
// kmer-cnt_amd/vafc_dist.py).  Rank r's share is the text of the deflate
// blocks from the first dynamic block that starts at or after byte A_r of the
// file to the first dynamic block that starts at or after A_{r+1}.
//
//   1. scan (vc_gzp_scan_share): the share's chunks are decoded speculatively
//      as always, and instead of text the sequencer keeps the share's last
//      32 KiB as symbols: a literal byte, or MARK | i for byte i of the
//      unknown 32 KiB before the share (markers of each chunk are mapped
//      through the previous chunk's symbols, so they all name that one
//      window).  A chunk that cannot be taken (a wrong start, a stored or
//      fixed block at the boundary, corrupt data) fails the scan: without the
//      history zlib cannot redo it, and the caller counts the file whole.
//   2. the ranks exchange (start, end, text length, last-32 KiB symbols); the
//      window before share r+1 is share r's symbols resolved against the
//      window before share r, so every window follows from rank 0's, whose
//      history is known (empty).
//   3. stream (vc_gzp_open_share): each rank inflates from its start bit with
//      its now known window, through the ordinary sequencer (zlib fallback
//      included), and on past its share's end as far as the reader asks (the
//      last record of a share ends in the next one).  CRC-32 accounting covers
//      the share only: the member that was open at the share's start and the
//      one still open at its end are reported as partial CRCs for the caller
//      to combine across ranks (vc_gz_crc32_combine); members wholly inside
//      are checked as gzread checks them.
// ---------------------------------------------------------------------------
struct VcGzShare {
	uint64_t start_bit = UINT64_MAX;   // UINT64_MAX: no dynamic block starts in the share's bytes
	uint64_t end_bit = UINT64_MAX;     // UINT64_MAX: the stream ended inside the share
	uint64_t text_len = 0;             // bytes of text from start_bit to end_bit
	bool ok = false;                   // every chunk of the share decoded and chained
};
// begin/end: the share's nominal bytes [A_r, A_{r+1}) of the compressed file
// (begin 0: the stream's first member, whose history is known).  window_sym
// (WSIZE = 32768 entries): the share's last 32 KiB of text as symbols.  false
// if the file cannot be opened as gzip.
bool vc_gzp_scan_share(const char *path, int threads, uint64_t chunk_bytes, uint64_t begin, uint64_t end,
                       VcGzShare *sh, uint16_t *window_sym);

struct VcGzShareCrc {
	uint32_t events = 0;               // member ends met inside the share
	uint32_t head_crc = 0;             // CRC-32 of the share's text up to its first member end
	uint64_t head_len = 0;
	uint32_t head_expect_crc = 0, head_expect_isize = 0;   // that member's trailer
	uint32_t tail_crc = 0;             // after the last member end (the whole share if none)
	uint64_t tail_len = 0;
	uint32_t crc_error = 0;            // a member wholly inside the share failed its check
	uint32_t complete = 0;             // the accounting reached the share's end (or the stream's)
};
// Stream from start_bit with the 32 KiB `window` before it (first_share: the
// stream's start, window unused); text_len bounds the CRC accounting.
VcGzParallel *vc_gzp_open_share(const char *path, int threads, uint64_t chunk_bytes, bool first_share,
                                uint64_t start_bit, const uint8_t *window, uint64_t text_len);
void vc_gzp_share_crc(VcGzParallel *g, VcGzShareCrc *out);
// The scan of vc_gzp_scan_share keeping the share's decoded chunks (about 3
// bytes per byte of text, at most hold_bytes of buffers), so that the count
// resumes from them instead of inflating the share again: *held is the open
// inflater (close with vc_gzp_close), or nullptr when the share did not fit
// (or could not be scanned).  false if the file cannot be opened as gzip.
bool vc_gzp_scan_share_hold(const char *path, int threads, uint64_t chunk_bytes, uint64_t begin, uint64_t end,
                            uint64_t hold_bytes, VcGzShare *sh, uint16_t *window_sym, VcGzParallel **held);
// Stream a held share (as vc_gzp_open_share would from its start) with the
// window before it (nullptr: the stream's first share).
bool vc_gzp_resume_share(VcGzParallel *g, const uint8_t *window, uint64_t text_len);

// The C ABI's handle of a held share (include/vafc.h vc_gz_share_open).
struct vc_gz_share {
	VcGzParallel *g = nullptr;
	int format = -1;    // FASTA 1 / FASTQ 0 by the stream's first header (vc_gz_text_format)
	int threads = 1;
};
// Next bytes of the decompressed stream, in order: > 0 bytes, 0 at the end.
int64_t vc_gzp_read(VcGzParallel *g, uint8_t *dst, size_t n);
// The same without a copy: up to `max` next bytes at *p, valid until the next
// call on g.
int64_t vc_gzp_span(VcGzParallel *g, const uint8_t **p, size_t max);
// The same, but the bytes stay valid until vc_gzp_release(g, *hold) (any
// thread), so the caller can keep them without copying; the decoder reuses a
// piece's buffer only once every hold on it is released.
int64_t vc_gzp_span_hold(VcGzParallel *g, const uint8_t **p, size_t max, void **hold);
void vc_gzp_release(VcGzParallel *g, void *hold);
void vc_gzp_stats(VcGzParallel *g, VcGzStats *st);
void vc_gzp_close(VcGzParallel *g);

#endif
