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
