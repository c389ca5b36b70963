/*
 * vafc.h -- C ABI of the MI355X-native vaf-counter hot path (libvafc.so).
 *
 * The reference (gerbenvoshol/kmer-cnt, vaf-counter.c) is a monolithic C
 * program with no plugin/FFI API; its in-process seam is
 *
 *     void count_fastq_kmers(const char *fn, int k, int n_thread, int block_size,
 *                            kmer_cnt_t *kmer_map, pattern_db_t *db);   // vaf-counter.c:550
 *
 * fed by load_patterns() (vaf-counter.c:149) and create_combined_kmer_map()
 * (vaf-counter.c:198), with steps 1+2 of its pipeline (extract k-mers
 * vaf-counter.c:519-535, look up + increment vaf-counter.c:537-544) as the hot
 * path.  This header is that seam re-cut at a device boundary: plain pointers
 * and sizes, no torch or HIP types, C linkage.  Every entry point names the
 * reference interface it replaces.
 *
 * Counts layout: uint32 counts[2*n_patterns], REF of pattern i at [2i], ALT at
 * [2i+1] -- i.e. indexed by the reference's map value (i<<1)|is_alt
 * (vaf-counter.c:227,239).  Counts wrap modulo 2^32 exactly like the
 * reference's uint32 fields (vaf-counter.c:101-102,473-477).
 *
 * Errors: 0 = ok, <0 = VC_E* below; vc_strerror() gives text.  HIP failures
 * are reported, never silently degraded to a CPU path.
 */
#ifndef VAFC_H
#define VAFC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VAFC_VERSION_MAJOR 0
#define VAFC_VERSION_MINOR 1

enum {
	VC_OK = 0,
	VC_EINVAL = -1,      /* bad argument (k outside 1..31, NULL pointer, ...) */
	VC_ENOMEM = -2,      /* host allocation failed */
	VC_EHIP = -3,        /* HIP runtime / kernel launch error */
	VC_ENODEV = -4,      /* no usable GPU */
	VC_EIO = -5,         /* file could not be opened / read */
	VC_ETOOMANY = -6,    /* more than INT32_MAX>>1 patterns (vaf-counter.c:205-209) */
	VC_EFULL = -7        /* k-mer histogram: more distinct k-mers than the table holds */
};

typedef struct vc_ctx vc_ctx;
typedef struct vc_patterns vc_patterns;

/* ------------------------------------------------------------------ */
/* Pattern database -- replaces load_patterns (vaf-counter.c:149-184)  */
/* and create_combined_kmer_map (vaf-counter.c:198-252).               */
/* ------------------------------------------------------------------ */

/* Load patterns.txt (records "chr start end rsid ref alt ref_kmer alt_kmer",
 * read with the reference's fscanf conversion; reading stops at the first
 * record that does not convert completely).  Returns VC_EIO if the file
 * cannot be opened (the reference then exits 1, vaf-counter.c:624-627). */
int vc_patterns_load(const char *path, vc_patterns **out);
void vc_patterns_free(vc_patterns *db);
int vc_patterns_count(const vc_patterns *db);

/* Canonical 2-bit keys and values (i<<1)|is_alt in insertion order (ref of
 * pattern i, then alt of pattern i), first insert wins, keys of strings with a
 * non-ACGTU character among their first k skipped.  *keys / *vals are malloc'd
 * (caller frees with vc_free).  *n_collisions = duplicate inserts ignored. */
int vc_patterns_keys(const vc_patterns *db, int k, uint64_t **keys, uint32_t **vals,
                     size_t *n_keys, int *n_collisions);

/* Write the .vaf file (vaf-counter.c:653-681): header "# Average depth",
 * column line, one row per pattern in file order. counts as above. */
int vc_write_vaf(const vc_patterns *db, const uint32_t *counts, const char *path);

/* Field access for host-side mirrors (Python): returns 0 and fills the
 * pointers (valid until vc_patterns_free). */
int vc_pattern_fields(const vc_patterns *db, int i, const char **chr, int *start,
                      const char **rsid, char *ref, char *alt,
                      const char **ref_kmer, const char **alt_kmer);

void vc_free(void *p);

/* ------------------------------------------------------------------ */
/* Device counter -- replaces the kmer_cnt_t map + pattern_t counters  */
/* (vaf-counter.c:67,92-108) and steps 1+2 of worker_pipeline          */
/* (vaf-counter.c:519-544, worker_lookup :449-479).                    */
/* ------------------------------------------------------------------ */

/* Create a counter on HIP device `device` for k in 1..31 from (key, value)
 * pairs as produced by vc_patterns_keys (first occurrence of a key wins).
 * The static key table and its LDS prefilter are built on the host and copied
 * once to HBM.  Counts start at zero. */
int vc_create(vc_ctx **out, int k, const uint64_t *keys, const uint32_t *vals,
              size_t n_keys, uint32_t n_patterns, int device);
void vc_destroy(vc_ctx *ctx);

/* Count one block of host-resident reads (asynchronous; accumulates).
 * seq: raw read bytes exactly as the FASTA/Q parser returned them (the
 * position-dependent 2-bit decode of vaf-counter.c:261-291 is applied on the
 * device); read i is seq[offs[i] .. offs[i]+lens[i]).  The caller may reuse
 * its buffers as soon as the call returns (they are staged into pinned
 * memory).  Reads shorter than k contribute nothing. */
int vc_count_block(vc_ctx *ctx, const uint8_t *seq, size_t seq_bytes,
                   const uint64_t *offs, const uint32_t *lens, uint64_t n_reads);

/* The counter's own (non-blocking) stream as vc_count_device's `stream`. */
#define VC_STREAM_CTX ((void *)(intptr_t)-1)

/* Same for device-resident reads (HBM pointers, e.g. from torch or
 * hipMalloc); enqueued on `stream`, a hipStream_t: NULL is HIP's null stream,
 * ordered with the legacy default stream (torch's default stream) as for any
 * HIP API; VC_STREAM_CTX is the counter's own stream (vc_stream).  Whatever
 * the stream, the launch is ordered after the counter's earlier work on its
 * own stream (vc_reset, earlier batches) and before its later work (vc_finish,
 * the shard sum), so vc_finish needs no device-wide synchronisation.  No host
 * synchronisation.  seq_bytes bounds every device read. */
int vc_count_device(vc_ctx *ctx, const uint8_t *d_seq, size_t seq_bytes,
                    const uint64_t *d_offs, const uint32_t *d_lens, uint64_t n_reads,
                    void *stream);

/* Wait for all queued work; copy counts[2*n_patterns] and the number of valid
 * k-mers extracted (perf_stats_t.total_kmers_extracted, vaf-counter.c:388)
 * to the host.  Either output may be NULL. */
int vc_finish(vc_ctx *ctx, uint32_t *counts, uint64_t *kmers_extracted);

/* Zero counts and the k-mer tally (asynchronous on the ctx stream). */
int vc_reset(vc_ctx *ctx);

/* Device pointer of the uint32 counts[2*n_patterns] array (for a device-side
 * all-reduce across ranks, e.g. RCCL through torch.distributed). */
void *vc_device_counts(vc_ctx *ctx);
/* Count into caller-owned device buffers instead (uint32[2*n_patterns] and
 * one uint64), e.g. torch tensors that an RCCL all-reduce then sums across
 * ranks; NULL restores the ctx's own buffers.  Not zeroed by this call. */
int vc_bind_outputs(vc_ctx *ctx, void *d_counts, void *d_tally);
void *vc_device_tally(vc_ctx *ctx);
void *vc_stream(vc_ctx *ctx);

/* Kernel timing: when enabled, every count call records HIP events around
 * the k-mer kernel on the stream it runs on; vc_kernel_ms synchronises on the
 * last pair and returns its elapsed milliseconds (sum of both kernels). */
int vc_set_timing(vc_ctx *ctx, int enable);
int vc_kernel_ms(vc_ctx *ctx, float *ms);

/* Table/prefilter geometry, for reports: n_keys, table slots, filter bytes. */
int vc_table_info(const vc_ctx *ctx, uint64_t *n_keys, uint64_t *slots, uint64_t *filter_bytes);

/* ------------------------------------------------------------------ */
/* Multi-GPU counter -- the reference counts all     */
/* files into one set of counters in one process (vaf-counter.c:473-477,*/
/* 647-650) and writes them once (:653-681).                           */
/* ------------------------------------------------------------------ */

#define VC_MAX_SHARDS 64

/* A counter with one shard per entry of devices[0..n_devices): each shard
 * holds a replica of the static table and its own counts on its device (a
 * device may repeat: several shards on one GPU).  Host reads given to
 * vc_count_block / vc_count_file are dealt to the shards batch by batch,
 * round robin (the -b block loop and its stop rule still run once, in file
 * order); vc_count_device deals device batches the same way over the
 * shards that live on the device holding d_seq (VC_EINVAL if none does).
 * vc_finish reduces the shards -- same-device shards summed on their device,
 * then, when the shards span more than one device, one RCCL reduce (ncclSum
 * of the u32 counts and the u64 k-mer tally) to shard 0 over xGMI -- and
 * returns the totals, bit-identical
 * to a single device counting everything (u32 sums wrap like the
 * reference's counters).  vc_reset / vc_set_nt4_decode apply to every shard;
 * vc_bind_outputs, vc_device_counts, timing and vc_table_info to shard 0.
 * n_devices == 1 is vc_create.  With more than one distinct device,
 * librccl.so.1 ($VAFC_RCCL_LIB names another) is loaded before any device is
 * touched; if it cannot be loaded the call fails with VC_EHIP. */
int vc_create_multi(vc_ctx **out, int k, const uint64_t *keys, const uint32_t *vals, size_t n_keys,
                    uint32_t n_patterns, const int *devices, int n_devices);
/* Shards of a counter (1 for vc_create), and shard i's device and the host
 * batches it has counted so far. */
int vc_shard_count(const vc_ctx *ctx);
int vc_shard_info(const vc_ctx *ctx, int i, int *device, uint64_t *batches);

/* ------------------------------------------------------------------ */
/* Whole-file pass -- replaces count_fastq_kmers (vaf-counter.c:550).  */
/* ------------------------------------------------------------------ */

typedef struct {
	uint64_t bases;        /* bases of reads with len >= k (pipeline_t.total_bases) */
	uint64_t seqs;         /* reads with len >= k (pipeline_t.total_seqs) */
	uint64_t blocks;       /* non-empty -b blocks */
	double seconds;        /* wall time of this file */
} vc_file_stats;

/* Parse FASTA/FASTQ (plain or gzip) with kseq_read semantics (kseq.h:192-232)
 * under the reference's block loop: blocks of >= block_bases bases, reads
 * shorter than k skipped, a read error (-2) or EOF ends a block, the file ends
 * at the third empty block (vaf-counter.c:486-517, kthread.c:97-128).  Reads
 * are streamed to the device in large pinned batches.  Plain (uncompressed)
 * files of 32 MB or more are parsed by n_threads worker threads (the CLI's
 * -t; vafc_ingest.h) with identical results; gzip files are inflated by
 * n_threads workers (vafc_gzip.h, gzread's output) while (n_threads + 3) / 5
 * workers parse the inflated text in parallel (VAFC_GZ_PARSERS overrides);
 * small plain files use one reader thread.  Returns VC_EIO if the file cannot be opened (the reference
 * skips such files silently, vaf-counter.c:557). */
int vc_count_file(vc_ctx *ctx, const char *path, int block_bases, int n_threads,
                  vc_file_stats *st);

/* One rank's share of a file (one process per GPU, kmer-cnt_amd/vafc_dist.py):
 * the records of a plain FASTA/FASTQ file whose header lies in the byte range
 * [first, end), where first is the first record header at or after `begin`
 * (begin = 0: the file's start; later: the record shape found there, as the
 * parallel reader's pieces do, vafc_ingest.h).  Counted like vc_count_file,
 * the block loop starting afresh at `first`.  The reference counts a file in
 * one kseq stream (vaf-counter.c:486-517,550-582); consecutive ranges
 * [b_0 = 0, b_1), [b_1, b_2), ... count exactly its reads iff every range's
 * ri.first equals the previous range's ri.next and no range has ri.errs > 0
 * (a -2 from the reader ends a block, and the reference's third-empty-block
 * stop depends on the blocks before it).  The caller checks that and
 * otherwise counts the file whole in one range (begin = 0, end = UINT64_MAX,
 * which is vc_count_file's result).  gzip files (and anything but a regular
 * file) are not split: begin = 0 counts the whole file (ri.whole = 1),
 * begin > 0 counts nothing (ri.first = ri.next = UINT64_MAX, ri.whole = 1).
 * VC_EIO if the file cannot be opened. */
typedef struct {
	uint64_t first;     /* header offset counting began at; UINT64_MAX: none found, nothing counted */
	uint64_t next;      /* header offset of the first record at or past end; UINT64_MAX: the file ended */
	uint64_t errs;      /* reader -2 returns (truncated records) met in the range */
	uint32_t stopped;   /* the block loop ended the file inside the range */
	uint32_t whole;     /* 1: the file is not split by ranges (gzip, pipe) */
} vc_range_info;
int vc_count_file_range(vc_ctx *ctx, const char *path, uint64_t begin, uint64_t end, int block_bases,
                        int n_threads, vc_file_stats *st, vc_range_info *ri);
/* Host-only: the same range through the parallel reader without a device;
 * accepted read bytes / lengths copied out while they fit (as
 * vc_scan_file_parallel). */
int vc_scan_file_range(const char *path, int k, int block_bases, int n_threads, uint64_t piece_bytes,
                       uint64_t begin, uint64_t end, vc_file_stats *st, vc_range_info *ri, uint8_t *seq_out,
                       size_t seq_cap, uint32_t *lens_out, size_t lens_cap);

/* Where the calling thread's last pass through the parallel reader
 * (vc_count_file / vc_count_file_range on a plain or gzip file,
 * vc_scan_file_parallel, vc_scan_file_range) spent its time: prof[0..7) =
 * the reader's wall seconds; main-thread seconds waiting for the next piece,
 * submitting pieces (H2D copies and kernel launches), re-parsing mis-guessed
 * pieces; worker thread-seconds parsing, waiting for a slot the main thread
 * had not released, waiting for a slot's previous copy to leave it.  Returns
 * the pieces of that pass (0: none yet).  prof may be NULL. */
uint64_t vc_ingest_profile(double *prof);

/* The same pass's profile with the workers' parse split (round 6): the first
 * min(n, VC_INGEST_PROFILE_FIELDS) of prof[] = the seven fields above, then
 * the workers' seconds reading the source (pread: the copy out of the page
 * cache) and the bytes read, seconds copying accepted sequences into the slots
 * and the bytes copied (0 with VAFC_SLOT_COPY=0, which copies per read
 * untimed), seconds guessing record starts, the workers' CPU seconds and
 * wall seconds (CPU < wall: descheduled, e.g. a CPU quota's throttling), the
 * main thread's CPU seconds, the worker count and the slot-copy mode.
 * Returns the pieces of that pass. */
#define VC_INGEST_PROFILE_FIELDS 17
uint64_t vc_ingest_profile_ex(double *prof, int n);

/* Optional: allocate vc_count_file's parallel-reader buffers for n_threads
 * reader threads now (pinned host + device memory, about 20 MB per thread),
 * so that a later vc_count_file does not pay for the allocation.  Without
 * it, vc_count_file's workers allocate each buffer on its first use, while
 * the other workers parse.  The CLI does not call it (VAFC_RESERVE=1 makes
 * it, inside the counting timer). */
int vc_reserve_file_ingest(vc_ctx *ctx, int n_threads);

/* Host-only: the same reader + block loop without a device (no counting).
 * Accepted read bytes / lengths are copied out while they fit (either output
 * may be NULL).  Lets the reader semantics be checked on machines without a
 * GPU and measures host ingest speed. */
int vc_scan_file(const char *path, int k, int block_bases, vc_file_stats *st,
                 uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out, size_t lens_cap);

/* Host-only: vc_count_file's parallel reader for plain (uncompressed) files,
 * without a device: n_threads workers parse pieces of piece_bytes of the file
 * concurrently (vafc_ingest.h); accepted reads come out in file order, exactly
 * as vc_scan_file's.  Lets the parallel reader be checked without a GPU and
 * measures its speed.  gzip input: n_threads inflate workers with chunks of
 * piece_bytes compressed bytes (the reader of vc_count_file for .gz), the
 * block loop in the calling thread. */
int vc_scan_file_parallel(const char *path, int k, int block_bases, int n_threads, uint64_t piece_bytes,
                          vc_file_stats *st, uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out,
                          size_t lens_cap);

/* Host-only gzip inflate (test and speed hooks): the whole decompressed
 * stream of `path` -- through the parallel inflater (n_threads workers,
 * chunk_bytes compressed bytes per chunk; stats6 = chunks, accepted, skipped,
 * zlib fallbacks, members checked, CRC error) or through zlib's gzread --
 * written to out while it fits.  Returns the stream's length, or -1 if the
 * file cannot be opened (parallel: is not gzip). */
int64_t vc_gz_inflate_parallel(const char *path, int n_threads, uint64_t chunk_bytes, uint8_t *out,
                               uint64_t cap, uint64_t *stats6);
int64_t vc_gz_inflate_zlib(const char *path, uint8_t *out, uint64_t cap);
/* Host-only: zlib-compatible CRC-32 of p[0..n) continuing from crc (the
 * inflater's member check; PCLMULQDQ folding where the CPU has it). */
uint32_t vc_gz_crc32(uint32_t crc, const uint8_t *p, uint64_t n);
/* zlib's crc32_combine: the CRC-32 of A then B from crc(A), crc(B), len(B). */
uint32_t vc_gz_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* One gzip file over several ranks (round 6, kmer-cnt_amd/vafc_dist.py; the
 * reference reads it with one gzread, vaf-counter.c:557, kseq.h:74-85).
 * Rank r's share is the text of the deflate blocks from the first dynamic
 * block starting at or after byte A_r of the file up to the first dynamic
 * block starting at or after A_{r+1} (A_0 = 0: the stream's start).
 *
 * 1. vc_gz_share_scan: each rank decodes its share speculatively without
 *    the history before it and reports where the share starts and ends (bit
 *    offsets), its text length, and its last 32 KiB of text as symbols
 *    (window_sym, 32768 entries: a byte value < 256, or 0x8000 | i for byte i
 *    of the unknown 32 KiB before the share).  ok = 0: the share could not be
 *    decoded without that history (the caller counts the file whole).
 * 2. The shares chain iff each share's start_bit equals the previous
 *    (non-empty) share's end_bit; the 32 KiB before share r+1 is share r's
 *    window_sym with every 0x8000 | i replaced by byte i of the 32 KiB before
 *    share r (share 0's history is empty).
 * 3. vc_count_gz_share: the share's reads, counted from start_bit with that
 *    window: the records whose header lies in the share's text, the block
 *    loop starting afresh at the first, as vc_count_file_range does for a
 *    byte range of a plain file.  ri.first / ri.next are offsets in the
 *    share's own text / the next share's text, so consecutive shares are
 *    exact under the same chain rule (first == previous next, no -2).  crc
 *    reports the CRC-32 accounting of the share: members wholly inside are
 *    checked (crc_error), the member open at the share's start closes at its
 *    first member end (head_*, to be checked by the caller with the previous
 *    shares' tails) and the one open at its end is the tail. */
typedef struct {
	uint64_t start_bit;   /* UINT64_MAX: no dynamic block starts in the share's bytes (an empty share) */
	uint64_t end_bit;     /* UINT64_MAX: the stream ended inside the share */
	uint64_t text_len;    /* bytes of text from start_bit to end_bit */
	uint32_t ok;
	uint32_t ended;
} vc_gz_share_info;
int vc_gz_share_scan(const char *path, uint64_t begin, uint64_t end, int n_threads, uint64_t chunk_bytes,
                     vc_gz_share_info *out, uint16_t *window_sym);

typedef struct {
	uint32_t events;            /* member ends inside the share */
	uint32_t head_crc;          /* CRC-32 of the share's text up to its first member end */
	uint64_t head_len;
	uint32_t head_expect_crc;   /* that member's trailer (CRC-32, ISIZE) */
	uint32_t head_expect_isize;
	uint32_t tail_crc;          /* from the last member end (or the share's start) to the share's end */
	uint64_t tail_len;
	uint32_t crc_error;         /* a member wholly inside the share failed its check */
	uint32_t complete;          /* the accounting reached the share's end */
} vc_gz_share_crc;
/* first_share: the stream's start (start_bit and window unused).  Counts like
 * vc_count_file_range (NULL ri/crc not allowed); VC_EIO if the file cannot be
 * opened as gzip. */
int vc_count_gz_share(vc_ctx *ctx, const char *path, int first_share, uint64_t start_bit, const uint8_t *window,
                      uint64_t text_len, int block_bases, int n_threads, vc_file_stats *st, vc_range_info *ri,
                      vc_gz_share_crc *crc);
/* Host-only: the same reader without a device (accepted reads copied out
 * while they fit, as vc_scan_file_range). */
int vc_scan_gz_share(const char *path, int k, int first_share, uint64_t start_bit, const uint8_t *window,
                     uint64_t text_len, int block_bases, int n_threads, vc_file_stats *st, vc_range_info *ri,
                     vc_gz_share_crc *crc, uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out, size_t lens_cap);

/* One pass per share instead of two: vc_gz_share_open scans as
 * vc_gz_share_scan and keeps the share's decoded chunks (one to two bytes of
 * memory per byte of text: two for every symbol decoded while the chunk can
 * still refer to the unknown window, which in FASTQ is most of it; at most
 * hold_bytes),
 * so that the count resolves them with the window instead of inflating the
 * share again.  *held is NULL when the share did not fit in hold_bytes (or
 * could not be scanned): the caller then counts with vc_count_gz_share.  A
 * held share is counted once (vc_count_gz_share_held / vc_scan_gz_share_held,
 * same outputs as the unheld forms) and closed with vc_gz_share_close.  ctx:
 * the counter that will count the share (the scan's threads run on its GPU's
 * NUMA node, where the kept text is then read), or NULL. */
typedef struct vc_gz_share vc_gz_share;
int vc_gz_share_open(vc_ctx *ctx, const char *path, uint64_t begin, uint64_t end, int n_threads,
                     uint64_t chunk_bytes, uint64_t hold_bytes, vc_gz_share_info *out, uint16_t *window_sym,
                     vc_gz_share **held);
int vc_count_gz_share_held(vc_ctx *ctx, vc_gz_share *held, int first_share, const uint8_t *window, uint64_t text_len,
                           int block_bases, int n_threads, vc_file_stats *st, vc_range_info *ri, vc_gz_share_crc *crc);
int vc_scan_gz_share_held(vc_gz_share *held, int k, int first_share, const uint8_t *window, uint64_t text_len,
                          int block_bases, int n_threads, vc_file_stats *st, vc_range_info *ri, vc_gz_share_crc *crc,
                          uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out, size_t lens_cap);
void vc_gz_share_close(vc_gz_share *held);

/* Host-only: the kseq_read return value of every record until -1 (inclusive),
 * written while they fit; returns the number of calls made, or VC_EIO. */
int64_t vc_scan_records(const char *path, int32_t *rets, int64_t cap);

/* ------------------------------------------------------------------ */
/* snp-pattern-gen                            */
/* ------------------------------------------------------------------ */

/* A reference genome in host memory: records, names and sequences exactly
 * as load_fasta keeps them (snp-pattern-gen.c:67-103: kseq_read until the
 * first negative return; name = the header up to the first whitespace).
 * Sequences are stored back to back (vc_fasta_data gives the concatenated
 * view that vc_count_candidates takes).  Plain or gzip input. */
typedef struct vc_fasta vc_fasta;
int vc_fasta_load(const char *path, vc_fasta **out);   /* VC_EIO if unopenable; gzip inflated
                                                          by up to 16 threads (VAFC_THREADS) */
int vc_fasta_count(const vc_fasta *fa);
const char *vc_fasta_name(const vc_fasta *fa, int i);
const uint8_t *vc_fasta_seq(const vc_fasta *fa, int i, uint32_t *len);
int vc_fasta_data(const vc_fasta *fa, const uint8_t **seq, size_t *bytes, const uint64_t **offs,
                  const uint32_t **lens);
void vc_fasta_free(vc_fasta *fa);

/* ------------------------------------------------------------------ */
/* kc-c4: histogram of canonical k-mer occurrence counts               */
/* (kc-c4.c)                                   */
/* ------------------------------------------------------------------ */

/* A counter in histogram mode: every canonical k-mer (seq_nt4_table decode,
 * kc-c4.c:85-101) of the reads given to vc_count_block / vc_count_device /
 * vc_count_file is counted in a device hash table of `table_slots` slots
 * (16 B each, rounded up to a power of two, at most 40 % of free HBM; 0 =
 * that maximum).
 * Replaces kc-c4's kc_c4x_t sub-tables and count_file (kc-c4.c:56-66,
 * 170-182).  vc_reset clears the table; vc_finish returns the k-mers seen. */
int vc_kc_create(vc_ctx **out, int k, uint64_t table_slots, int device);
/* Count only the k-mers of partition `part` of `n_parts` (1..1024), by the
 * low 10 bits of hash64 (kc-c4.c:40-50): ((h & 1023) * n_parts) >> 10 ==
 * part, so a partition holds whole kc-c4 / yak sub-tables (kc-c4.c:74-83,
 * p >= 10): a set larger than the table is counted in n_parts passes, or on
 * n_parts GPUs, whose histograms add up.  n_parts = 1 counts everything.
 * Clears the table. */
int vc_kc_set_partition(vc_ctx *ctx, uint32_t n_parts, uint32_t part);
/* Slots of the table (after rounding). */
uint64_t vc_kc_slots(vc_ctx *ctx);
/* Synchronizes; hist[c] (c = 1..255, 256 entries) += the number of distinct
 * k-mers counted min(c, 255) times (print_hist, kc-c4.c:196-223); distinct
 * and kmers receive the table's distinct k-mers and the k-mers seen.
 * VC_EFULL (hist untouched) when the table ran out of room: count again
 * with more partitions or a larger table. */
int vc_kc_histogram(vc_ctx *ctx, uint64_t *hist, uint64_t *distinct, uint64_t *kmers);
/* General form: hist[min(c, n_bins - 1)] += 1 (n_bins 2..1024) for every key
 * counted c >= min_count times and not dropped by vc_yak_bloom_select;
 * *distinct = the keys added.  yak-count's histogram (yak-count.c:209-240,
 * 500-503) is n_bins 1024, min_count 1 (no filter) or 2 (after its shrink to
 * [2, 1023], :268-288). */
int vc_kc_histogram2(vc_ctx *ctx, uint64_t *hist, uint32_t n_bins, uint64_t min_count, uint64_t *distinct,
                     uint64_t *kmers);

/* yak-count -b (yak-count.c:440-452), pass 1 to pass 2.  Count file 1 with
 * first-occurrence tracking on (vc_kc_track_first, which also clears), then
 * vc_yak_bloom_select replays yak's per-sub-table blocked Bloom filters
 * (2^(bf_shift - pre) bits each, n_hash bits per k-mer, yak-count.c:71-108,
 * 150-176) over the stream order to find the keys yak would have inserted,
 * restarts their counts at 0 and drops the rest; later count calls (file 2)
 * then only count those keys (yak's create_new = 0).  Without a valid filter
 * (n_hash <= 0, or bf_shift - pre outside 9..55) every key stays.  A later
 * vc_reset returns to insert mode. */
int vc_kc_track_first(vc_ctx *ctx, int on);
int vc_yak_bloom_select(vc_ctx *ctx, int pre, int bf_shift, int n_hash);

/* Decode mode of a counter: on = seq_nt4_table at every position, the decode
 * of snp-pattern-gen (snp-pattern-gen.c:165), instead of vaf-counter's
 * position-dependent one (the default).  Applies to later count calls. */
int vc_set_nt4_decode(vc_ctx *ctx, int on);

/* count_candidate_kmers (snp-pattern-gen.c:159-190) on the GPU: counts[i]
 * (u32, wrapping like the reference's khash values) = the number of
 * canonical k-mers of all n_seqs sequences that equal keys[i].  Sequences
 * are decoded with seq_nt4_table at every position (no vaf-counter quirk);
 * any other byte ends the current window.  keys must be distinct canonical
 * k-mers; seq/offs/lens are host buffers (sequence i at seq + offs[i]). */
int vc_count_candidates(int k, const uint8_t *seq, size_t seq_bytes, const uint64_t *offs,
                        const uint32_t *lens, uint64_t n_seqs, const uint64_t *keys, size_t n_keys,
                        uint32_t *counts, int device);

/* ------------------------------------------------------------------ */
/* correlation-matrix: depth-aware Pearson between .vaf samples + tree  */
/* (correlation-matrix.c)                      */
/* ------------------------------------------------------------------ */

typedef struct vc_vafset vc_vafset;
int vc_vafset_create(vc_vafset **out);
void vc_vafset_free(vc_vafset *s);
/* load_vaf_file (correlation-matrix.c:25-90): fgets lines of at most 4095
 * bytes, '#' and "CHR" lines skipped, rows read with the reference's 9-field
 * sscanf conversion (vaf = field 9, depth = field 8), at most 100,000 rows
 * (then the reference's warning on stderr); name = basename cut at the first
 * ".vaf".  VC_EIO if the file cannot be opened (the reference exits 1). */
int vc_vafset_add(vc_vafset *s, const char *path);
/* The same for n files read by n_threads threads: files are appended in
 * order up to the first one that cannot be opened (*n_added = its index,
 * VC_EIO; VC_OK if all were); truncated[i] = 1 where the 100,000-row cap was
 * hit, for the caller to print the reference's warning in file order
 * (load_vaf_file prints it while loading, correlation-matrix.c:70-73). */
int vc_vafset_add_many(vc_vafset *s, const char *const *paths, int n, int n_threads, int *n_added,
                       uint8_t *truncated);
/* A sample from arrays (n <= 100,000 rows). */
int vc_vafset_add_arrays(vc_vafset *s, const char *name, const double *vaf, const int32_t *depth, int n);
int vc_vafset_count(const vc_vafset *s);
const char *vc_vafset_name(const vc_vafset *s, int i);
int vc_vafset_snps(const vc_vafset *s, int i);
/* calculate_correlation_matrix + pearson_correlation_depth_aware
 * (correlation-matrix.c:94-162) on the GPU: corr[i*n + j] (n = samples, row
 * major, symmetric, 1.0 on the diagonal) is bit-identical to the reference's
 * double: for i < j the rows [0, rows of sample i) that have depth >=
 * min_depth in both samples (rows past sample j's end count as vaf 0, depth
 * 0), 0.0 below min_snps of them.  kernel_ms (may be NULL) receives the
 * kernel time. */
int vc_corr_matrix(const vc_vafset *s, int min_snps, int min_depth, double *corr, int device, float *kernel_ms);
/* The same on arrays: sample i has n_snps[i] rows at vaf/depth + i*stride. */
int vc_corr_matrix_raw(const double *vaf, const int32_t *depth, const int32_t *n_snps, int n_samples,
                       size_t stride, int min_snps, int min_depth, double *corr, int device, float *kernel_ms);
/* The .corr file (correlation-matrix.c:350-366): header row of names, then
 * one row per sample, "%.6f" cells.  VC_EIO if it cannot be created. */
int vc_corr_write(const vc_vafset *s, const double *corr, const char *path);
/* build_tree (correlation-matrix.c:190-257): average linkage on 1 - r, the
 * same merge order, ties and "%.4f" text.  VC_EIO if it cannot be created. */
int vc_corr_tree(const vc_vafset *s, const double *corr, const char *path);

/* ------------------------------------------------------------------ */
/* Synthetic workload (bench / tests): the generator of vafc_synth.py,  */
/* evaluated on the device.                                            */
/* ------------------------------------------------------------------ */

/* Generate reads first..first+n_reads-1 (fixed length read_len) into device
 * buffers d_seq[n_reads*read_len], d_offs[n_reads], d_lens[n_reads].
 * d_windows: device [n_snp][2][301] ASCII SNP windows, d_dosage: [n_snp] u8. */
int vc_synth_reads(uint8_t *d_seq, uint64_t *d_offs, uint32_t *d_lens, uint64_t first,
                   uint64_t n_reads, uint32_t read_len, uint64_t seed, double f_snp,
                   const uint8_t *d_windows, const uint8_t *d_dosage, uint32_t n_snp,
                   void *stream);

/* Test hook: position-dependent 2-bit decode (vaf-counter.c:261-291) of
 * device-resident reads into d_codes (same offsets as d_seq; 0..3, 4 =
 * invalid) by the kernels' own decode path. */
int vc_debug_decode(const uint8_t *d_seq, size_t seq_bytes, const uint64_t *d_offs,
                    const uint32_t *d_lens, uint64_t n_reads, uint8_t *d_codes, void *stream);

const char *vc_strerror(int err);
int vc_version(void);
/* Hash of the sources this library was built from (16 hex digits: sha256 of
 * every file of kmer-cnt_amd/csrc in name order, then include/vafc.h).  The same string
 * is embedded as "VAFC_BUILD_ID=<hex>" in the library and every CLI, so a
 * checker can compare it with the tree without loading the binary. */
const char *vc_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
