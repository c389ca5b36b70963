// vafc_fastq.h -- FASTA/FASTQ record reader with the reference's kseq_read
// semantics (kseq.h:101-149 ks_getuntil2, kseq.h:192-232 kseq_read), written
// for throughput: a large refillable window, memchr line scans, the sequence
// and quality of a record kept in reusable buffers.  zlib's gzread reads both
// plain and gzip input (vaf-counter.c:12,557).
//
// Return values of next(): >= 0 sequence length, -1 end of input, -2
// truncated or length-mismatched quality -- exactly kseq_read's.
#ifndef VAFC_FASTQ_H
#define VAFC_FASTQ_H

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

class VcGzParallel;

// Random-access view of an input text for the parallel reader
// (vafc_ingest.h): a plain file read with pread, or a gzip stream as it is
// being inflated.
class VcTextSource {
public:
	virtual ~VcTextSource() = default;
	// Up to n bytes at offset off into p, waiting until they exist; fewer
	// than n only at the end of the text (or after the source was aborted).
	virtual int64_t read(uint8_t *p, size_t n, uint64_t off) = 0;
	// The whole text from offset off on, in place (a memory-mapped file):
	// a pointer to byte off and, in *avail, the bytes from there to the end
	// of the text; nullptr if the source has no such view (read() then).
	virtual const uint8_t *view(uint64_t off, uint64_t *avail)
	{
		(void)off;
		*avail = 0;
		return nullptr;
	}
};

class VcByteBuf {
public:
	char *s = nullptr;
	size_t l = 0, m = 0;
	~VcByteBuf() { free(s); }
	void reserve(size_t n)
	{
		if (n <= m) return;
		size_t nm = m ? m : 256;
		while (nm < n) nm *= 2;
		s = (char *)realloc(s, nm);
		m = nm;
	}
	void push(int c) { reserve(l + 1); s[l++] = (char)c; }
	void append(const uint8_t *p, size_t n)
	{
		reserve(l + n);
		memcpy(s + l, p, n);
		l += n;
	}
};

class VcFastqReader {
public:
	VcFastqReader() = default;
	~VcFastqReader() { close(); }
	bool open(const char *path, size_t window = (size_t)4 << 20);
	// As open(), but a gzip file is inflated by `threads` workers
	// (vafc_gzip.h) with gzread's output; plain files and gzip files the
	// parallel inflater declines are read as open() reads them.
	bool open_parallel(const char *path, int threads, uint64_t chunk_bytes = 0,
	                   size_t window = (size_t)4 << 20);
	bool gz_parallel() const { return gzp_ != nullptr; }
	// Source for the parallel ingest: records from offset `off` of a text
	// source (not owned).  `off` must be where kseq would look for a
	// record's header.
	bool open_src(VcTextSource *src, uint64_t off, size_t window = (size_t)4 << 20);
	// As open_src, over text held in place (VcTextSource::view): p is the
	// byte at text offset `off`, n the bytes from there to the end of the
	// text.  Nothing is copied in.
	bool open_view(const uint8_t *p, uint64_t n, uint64_t off);
	void close();
	int next();
	// File offset of the next record's header character ('@' or '>'),
	// scanning forward like next() does; -1 at end of input.  next() then
	// parses that record.
	int64_t peek_header();
	// The record's sequence: a one-line sequence whose line ends inside the
	// current window is a pointer into the window (valid until the next
	// next() call), anything else the reader's own copy.
	const char *seq() const { return seqp_ ? seqp_ : seq_.s; }
	size_t seq_len() const { return seqp_ ? seql_ : seq_.l; }
	// keep record names (kseq's name: the header up to the first isspace byte)
	void keep_names(bool on) { keep_name_ = on; }
	// Called before an owned window (open_src) is overwritten by the next
	// source read: sequences handed out as pointers into it are still valid
	// inside the call (the parallel reader's batched slot copy, vafc_ingest.cpp).
	void on_refill(void (*fn)(void *), void *arg)
	{
		refill_fn_ = fn;
		refill_arg_ = arg;
	}
	// seq() points into the window (valid until the window is refilled)
	bool seq_in_window() const { return seqp_ != nullptr; }
	const char *name() const { return name_.s ? name_.s : ""; }
	size_t name_len() const { return name_.l; }

private:
	gzFile fp_ = nullptr;
	VcGzParallel *gzp_ = nullptr;   // parallel gzip source (open_parallel)
	VcTextSource *src_ = nullptr; // random-access source (open_src), not owned
	uint64_t foff_ = 0;           // text offset of the next source read
	uint64_t base_ = 0;           // text offset of buf_[0] (source reads)
	uint8_t *buf_ = nullptr;
	size_t cap_ = 0, b_ = 0, e_ = 0;
	bool view_ = false;           // buf_ is the caller's text (open_view), not owned
	const char *seqp_ = nullptr;  // this record's sequence in the window, else seq_
	size_t seql_ = 0;
	bool eof_ = false;
	int hdr_ = 0;                 // header char already consumed, 0 if none
	uint64_t hdr_pos_ = 0;        // its text offset (source reads)
	VcByteBuf seq_, name_;
	bool keep_name_ = false;
	void (*refill_fn_)(void *) = nullptr;
	void *refill_arg_ = nullptr;

	bool refill();
	inline int getc_()
	{
		if (b_ >= e_ && !refill()) return -1;
		return buf_[b_++];
	}
	inline uint64_t last_pos() const { return base_ + b_ - 1; }   // of the byte getc_ just returned
	inline bool at_end() { return b_ >= e_ && !refill(); }
	int line(VcByteBuf *dst);     // rest of a line, appended; CR rule on the whole string
	int qual_line(size_t *l, size_t *tcr);   // the same for a string kept as its length only
	int token(int *delim);        // up to an isspace() byte, discarded
	void skip_line();
};

#endif
