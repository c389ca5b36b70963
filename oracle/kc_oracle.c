/*
 * kc_oracle.c -- CPU restatement of the reference kc-c4 k-mer histogram
 * (SURVEY.md §8(f) rank 3).
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/ and the CPU-baseline leg of tools/kc_bench.py may run
 *   anything built from this file, and only as the CHECKER.  The product
 *   (libvafc.so, the HIP kc-c4 CLI) never links it.
 *
 * Parity pinning: checked byte-for-byte (stdout) against the real reference
 * binary oracle/_ref/kc-c4, compiled from /root/reference/kc-c4.c by
 * oracle/Makefile, on the fixtures of tests/golden/kc/
 * (tests/golden/make_golden_kc.py).
 *
 * A literal, scalar statement of the reference program:
 *
 *   FASTA/Q records   kseq_read semantics             kseq.h:192-232 (vafc_oracle.c reader)
 *   block loop        l < k skipped, -b block bases,  kc-c4.c:133-155 + kthread.c:97-128
 *                     3-empty-block stop rule
 *   k-mers            seq_nt4_table, rolling          kc-c4.c:85-100
 *                     canonical, N restarts
 *   counting          one count per distinct          kc-c4.c:116-128 (10-bit saturating,
 *                     canonical k-mer                 min(c, 1023))
 *   histogram         i = 1..255: k-mers counted      kc-c4.c:206-234
 *                     min(c, 255) times
 *
 * The reference keys its 2^p sub-tables by hash64 of the canonical k-mer
 * (kc-c4.c:40-50, 96, 125); hash64 is invertible on 2k bits, so one count per
 * distinct canonical k-mer is what it computes.  This file keys directly by
 * the canonical k-mer.
 */
#include "vafc_oracle.c"

typedef struct {
	uint64_t *key;
	uint32_t *cnt;
	uint8_t *used;
	uint64_t mask, n;
} kctab_t;

static void kct_init(kctab_t *t)
{
	t->mask = (1u << 16) - 1;
	t->n = 0;
	t->key = (uint64_t*)calloc(t->mask + 1, 8);
	t->cnt = (uint32_t*)calloc(t->mask + 1, 4);
	t->used = (uint8_t*)calloc(t->mask + 1, 1);
}

static void kct_free(kctab_t *t)
{
	free(t->key); free(t->cnt); free(t->used);
}

static void kct_add(kctab_t *t, uint64_t y);

static void kct_grow(kctab_t *t)
{
	kctab_t o = *t;
	uint64_t i;
	t->mask = (o.mask << 1) | 1;
	t->n = 0;
	t->key = (uint64_t*)calloc(t->mask + 1, 8);
	t->cnt = (uint32_t*)calloc(t->mask + 1, 4);
	t->used = (uint8_t*)calloc(t->mask + 1, 1);
	for (i = 0; i <= o.mask; ++i) {
		if (!o.used[i]) continue;
		uint64_t j = mix64(o.key[i]) & t->mask;
		while (t->used[j]) j = (j + 1) & t->mask;
		t->used[j] = 1; t->key[j] = o.key[i]; t->cnt[j] = o.cnt[i]; ++t->n;
	}
	kct_free(&o);
}

/* ++count of canonical k-mer y, saturating at KC_MAX = 1023 (kc-c4.c:11-12,126) */
static void kct_add(kctab_t *t, uint64_t y)
{
	uint64_t i = mix64(y) & t->mask;
	while (t->used[i]) {
		if (t->key[i] == y) {
			if (t->cnt[i] < 1023) ++t->cnt[i];
			return;
		}
		i = (i + 1) & t->mask;
	}
	t->used[i] = 1; t->key[i] = y; t->cnt[i] = 1; ++t->n;
	if (t->n * 2 > t->mask) kct_grow(t);
}

/* count_seq_buf (kc-c4.c:85-100): seq_nt4_table at every position */
static uint64_t kc_seq(kctab_t *t, int k, const unsigned char *s, int len)
{
	uint64_t x0 = 0, x1 = 0, n = 0, mask = (1ULL << 2 * k) - 1;
	int sh = 2 * (k - 1), l = 0, i;
	for (i = 0; i < len; ++i) {
		int c = g_nt4[s[i]];
		if (c < 4) {
			x0 = (x0 << 2 | (uint64_t)c) & mask;
			x1 = x1 >> 2 | (uint64_t)(3 - c) << sh;
			if (++l >= k) { kct_add(t, x0 < x1 ? x0 : x1); ++n; }
		} else l = 0, x0 = x1 = 0;
	}
	return n;
}

/* print_hist's counts (kc-c4.c:206-231): hist[min(c, 255)] += 1 */
static void kct_hist(const kctab_t *t, uint64_t *hist)
{
	uint64_t i;
	for (i = 0; i < 256; ++i) hist[i] = 0;
	for (i = 0; i <= t->mask; ++i)
		if (t->used[i]) ++hist[t->cnt[i] < 255 ? t->cnt[i] : 255];
}

/* count_file (kc-c4.c:181-195) with the block loop of worker_pipeline step 0
 * (:133-155): the same 3-empty-block stop rule as vaf-counter's pipeline. */
static int kc_file(const char *fn, int k, int block_len, kctab_t *t, uint64_t *kmers)
{
	oreader_t r;
	int empty_blocks = 0;
	if (rd_open(&r, fn) < 0) return -1;
	while (empty_blocks < 3) {
		int sum_len = 0, ret;
		while ((ret = rd_record(&r)) >= 0) {
			int l = (int)r.seq.l;
			if (l < k) continue;
			*kmers += kc_seq(t, k, (const unsigned char*)r.seq.s, l);
			sum_len += l;
			if (sum_len >= block_len) break;
		}
		if (sum_len == 0) ++empty_blocks;
	}
	rd_close(&r);
	return 0;
}

/* ------------------------------------------------------------------------ */
/* ctypes API for tests/                                                      */
/* ------------------------------------------------------------------------ */

/* Histogram of the reads of a file; -1 if it cannot be opened.  hist has 256
 * entries (index 0 unused); *distinct and *kmers as the GPU path reports. */
int kco_hist_file(const char *fn, int k, int block_len, uint64_t *hist, uint64_t *distinct, uint64_t *kmers)
{
	kctab_t t;
	uint64_t km = 0;
	init_tables();
	kct_init(&t);
	if (kc_file(fn, k, block_len, &t, &km) < 0) { kct_free(&t); return -1; }
	kct_hist(&t, hist);
	if (distinct) *distinct = t.n;
	if (kmers) *kmers = km;
	kct_free(&t);
	return 0;
}

/* Histogram of reads given as one byte buffer + offsets/lengths (every read,
 * no block loop: the caller already applied it). */
int kco_hist_reads(int k, const uint8_t *seq, const uint64_t *offs, const uint32_t *lens, uint64_t n,
                   uint64_t *hist, uint64_t *distinct, uint64_t *kmers)
{
	kctab_t t;
	uint64_t km = 0, i;
	init_tables();
	kct_init(&t);
	for (i = 0; i < n; ++i) km += kc_seq(&t, k, seq + offs[i], (int)lens[i]);
	kct_hist(&t, hist);
	if (distinct) *distinct = t.n;
	if (kmers) *kmers = km;
	kct_free(&t);
	return 0;
}

#ifdef KC_ORACLE_MAIN
/* Same CLI as the reference (kc-c4.c:236-265): "k:p:b:t:", defaults 31 / 10 /
 * 10000000 / 4, usage on no input, -p < 10 rejected, 255 histogram lines. */
int main(int argc, char *argv[])
{
	int c, k = 31, p = 10, block = 10000000, n_thread = 4, i;
	uint64_t hist[256];
	kctab_t t;
	uint64_t km = 0;
	opterr = 0;
	while ((c = getopt(argc, argv, "k:p:b:t:")) >= 0) {
		if (c == 'k') k = atoi(optarg);
		else if (c == 'p') p = atoi(optarg);
		else if (c == 'b') block = atoi(optarg);
		else if (c == 't') n_thread = atoi(optarg);
	}
	if (argc - optind < 1) {
		fprintf(stderr, "Usage: kc-c4 [options] <in.fa>\n");
		fprintf(stderr, "Options:\n");
		fprintf(stderr, "  -k INT     k-mer size [%d]\n", k);
		fprintf(stderr, "  -p INT     prefix length [%d]\n", p);
		fprintf(stderr, "  -b INT     block size [%d]\n", block);
		fprintf(stderr, "  -t INT     number of worker threads [%d]\n", n_thread);
		return 1;
	}
	if (p < 10) {
		fprintf(stderr, "ERROR: -p should be at least %d\n", 10);
		return 1;
	}
	init_tables();
	kct_init(&t);
	if (kc_file(argv[optind], k, block, &t, &km) < 0) {
		fprintf(stderr, "ERROR: failed to open %s\n", argv[optind]);
		return 1;
	}
	kct_hist(&t, hist);
	for (i = 1; i < 256; ++i) printf("%d\t%ld\n", i, (long)hist[i]);
	kct_free(&t);
	return 0;
}
#endif
