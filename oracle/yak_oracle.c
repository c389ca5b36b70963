/*
 * yak_oracle.c -- CPU restatement of the reference yak-count k-mer histogram
 * (second program).
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/ may run anything built from this file, and only as the
 *   CHECKER.  The product (libvafc.so, the HIP yak-count CLI) never links it.
 *
 * Parity pinning: checked byte-for-byte (stdout, the final stderr line, exit
 * code) against the real reference binary oracle/_ref/yak-count, compiled
 * from /root/reference/yak-count.c by oracle/Makefile, on the fixtures of
 * tests/golden/yak/ (tests/golden/make_golden_yak.py).
 *
 * A literal, scalar statement of the reference program:
 *
 *   hash              yak_hash64 of the canonical k-mer   yak-count.c:47-57, 312-327
 *   sub-tables        low `pre` bits pick one; its key     yak-count.c:150-160
 *                     is hash >> pre
 *   Bloom filter      one blocked filter (2^(b-pre) bits,  yak-count.c:71-108, 115-121
 *                     512-bit blocks) per sub-table; a
 *                     k-mer enters the table only once all
 *                     its n_hash bits were already set
 *   counts            10-bit saturating (1023)             yak-count.c:161-170
 *   two passes        with -b: counts cleared, file 2 (or  yak-count.c:440-452, 186-202
 *                     1) recounted into existing keys,
 *                     keys outside [2, 1023] dropped
 *   histogram         i = 1..1023                          yak-count.c:209-240, 500-503
 *
 * k-mers are visited in stream order (reads in file order, positions in read
 * order).  The reference buffers them per sub-table and inserts each buffer in
 * order (:299-309, 353-359), and each sub-table owns its Bloom filter, so the
 * order that matters -- within one sub-table -- is the stream order.
 */
#include "vafc_oracle.c"

#define YO_MAXC 1023

static uint64_t yo_hash64(uint64_t key, uint64_t mask)
{
	key = (~key + (key << 21)) & mask;
	key = key ^ key >> 24;
	key = ((key + (key << 3)) + (key << 8)) & mask;
	key = key ^ key >> 14;
	key = ((key + (key << 2)) + (key << 4)) & mask;
	key = key ^ key >> 28;
	key = (key + (key << 31)) & mask;
	return key;
}

typedef struct {
	uint64_t *key;      /* full hash */
	uint32_t *cnt;
	uint8_t *used;
	uint64_t mask, n;
} yotab_t;

static void yot_init(yotab_t *t, uint64_t mask)
{
	t->mask = mask;
	t->n = 0;
	t->key = (uint64_t*)calloc(mask + 1, 8);
	t->cnt = (uint32_t*)calloc(mask + 1, 4);
	t->used = (uint8_t*)calloc(mask + 1, 1);
}

static void yot_free(yotab_t *t)
{
	free(t->key); free(t->cnt); free(t->used);
}

static int64_t yot_find(const yotab_t *t, uint64_t h)
{
	uint64_t i = mix64(h) & t->mask;
	while (t->used[i]) {
		if (t->key[i] == h) return (int64_t)i;
		i = (i + 1) & t->mask;
	}
	return -1 - (int64_t)i;
}

static void yot_grow(yotab_t *t)
{
	yotab_t o = *t;
	uint64_t i;
	yot_init(t, (o.mask << 1) | 1);
	for (i = 0; i <= o.mask; ++i) {
		if (!o.used[i]) continue;
		int64_t j = -1 - yot_find(t, o.key[i]);
		t->used[j] = 1; t->key[j] = o.key[i]; t->cnt[j] = o.cnt[i]; ++t->n;
	}
	yot_free(&o);
}

typedef struct {
	int k, pre, bf_shift, n_hash, create_new;
	int bf_on;                 /* per-sub-table filters exist (yak_ch_init + yak_bf_init) */
	uint8_t *bf;               /* 2^pre filters of 2^(bf_shift - pre) bits */
	yotab_t t;
} yak_t;

/* yak_bf_insert (yak-count.c:91-108) on sub-table s's filter; returns how many
 * of the n_hash bits were already set */
static int yo_bf_insert(yak_t *y, uint64_t s, uint64_t x)
{
	int ns = y->bf_shift - y->pre, xs = ns - 9, i, cnt = 0;
	uint64_t blk = x & ((1ULL << xs) - 1);
	int h1 = (int)(x >> xs & 511), h2 = (int)(x >> ns & 511), z = h1;
	uint8_t *p = y->bf + (s << (ns - 3)) + (blk << 6);
	if ((h2 & 31) == 0) h2 = (h2 + 1) & 511;
	for (i = 0; i < y->n_hash; ++i, z = (z + h2) & 511) {
		uint8_t u = (uint8_t)(1u << (z & 7));
		cnt += !!(p[z >> 3] & u);
		p[z >> 3] |= u;
	}
	return cnt;
}

/* yak_ch_insert_list (yak-count.c:150-176) for one k-mer hash */
static void yo_insert(yak_t *y, uint64_t h)
{
	uint64_t s = h & ((1ULL << y->pre) - 1), x = h >> y->pre;
	int64_t i;
	if (y->create_new) {
		if (y->bf_on && yo_bf_insert(y, s, x) != y->n_hash) return;
		i = yot_find(&y->t, h);
		if (i < 0) {
			i = -1 - i;
			y->t.used[i] = 1; y->t.key[i] = h; y->t.cnt[i] = 0; ++y->t.n;
		}
		if (y->t.cnt[i] < YO_MAXC) ++y->t.cnt[i];
		if (y->t.n * 2 > y->t.mask) yot_grow(&y->t);
	} else {
		i = yot_find(&y->t, h);
		if (i >= 0 && y->t.cnt[i] < YO_MAXC) ++y->t.cnt[i];
	}
}

static void yo_seq(yak_t *y, const unsigned char *s, int len)
{
	int k = y->k, sh = 2 * (k - 1), l = 0, i;
	uint64_t x0 = 0, x1 = 0, mask = (1ULL << 2 * k) - 1;
	for (i = 0; i < len; ++i) {
		int c = g_nt4[s[i]];
		if (c < 4) {
			x0 = (x0 << 2 | (uint64_t)c) & mask;
			x1 = x1 >> 2 | (uint64_t)(3 - c) << sh;
			if (++l >= k) yo_insert(y, yo_hash64(x0 < x1 ? x0 : x1, mask));
		} else l = 0, x0 = x1 = 0;
	}
}

/* yak_count (yak-count.c:420-438): the block loop of worker_pipeline step 0
 * (:334-351), the same 3-empty-block stop rule as the other programs */
static int yo_file(yak_t *y, const char *fn, int64_t chunk)
{
	oreader_t r;
	int empty_blocks = 0;
	if (rd_open(&r, fn) < 0) return -1;
	while (empty_blocks < 3) {
		int sum_len = 0, ret;
		while ((ret = rd_record(&r)) >= 0) {
			int l = (int)r.seq.l;
			if (l < y->k) continue;
			yo_seq(y, (const unsigned char*)r.seq.s, l);
			sum_len += l;
			if (sum_len >= chunk) break;
		}
		if (sum_len == 0) ++empty_blocks;
	}
	rd_close(&r);
	return 0;
}

/* yak_count_file + shrink + yak_ch_hist (yak-count.c:440-452, 209-288):
 * hist[1024]; *tot = distinct k-mers after shrinking.  -1: unopenable. */
int yko_hist(const char *fn1, const char *fn2, int k, int pre, int bf_shift, int n_hash, int64_t chunk,
             uint64_t *hist, uint64_t *tot)
{
	yak_t y;
	uint64_t i;
	init_tables();
	memset(&y, 0, sizeof(y));
	y.k = k, y.pre = pre, y.bf_shift = bf_shift, y.n_hash = n_hash, y.create_new = 1;
	y.bf_on = n_hash > 0 && bf_shift > pre && bf_shift - pre >= 9 && bf_shift - pre + 9 <= 64;
	if (y.bf_on) {
		y.bf = (uint8_t*)calloc(1, (size_t)1 << (bf_shift - 3));
		if (!y.bf) return -2;
	}
	yot_init(&y.t, (1u << 16) - 1);
	if (yo_file(&y, fn1, chunk) < 0) { free(y.bf); yot_free(&y.t); return -1; }
	if (bf_shift > 0) {
		free(y.bf);
		y.bf = 0; y.bf_on = 0;
		for (i = 0; i <= y.t.mask; ++i) y.t.cnt[i] = 0;
		y.create_new = 0;
		if (yo_file(&y, fn2 ? fn2 : fn1, chunk) < 0) { yot_free(&y.t); return -1; }
		for (i = 0; i <= y.t.mask; ++i)
			if (y.t.used[i] && (y.t.cnt[i] < 2 || y.t.cnt[i] > YO_MAXC)) { y.t.used[i] = 0; --y.t.n; }
	}
	for (i = 0; i < 1024; ++i) hist[i] = 0;
	for (i = 0; i <= y.t.mask; ++i)
		if (y.t.used[i]) ++hist[y.t.cnt[i]];
	if (tot) *tot = y.t.n;
	yot_free(&y.t);
	return 0;
}

#ifdef YAK_ORACLE_MAIN
/* Same CLI as the reference (yak-count.c:456-507): "k:p:K:t:b:H:". */
int main(int argc, char *argv[])
{
	int c, k = 31, pre = 10, bf_shift = 0, n_hash = 4, n_thread = 4, i;
	int64_t chunk = 10000000;
	uint64_t hist[1024], tot = 0;
	opterr = 0;
	while ((c = getopt(argc, argv, "k:p:K:t:b:H:")) >= 0) {
		if (c == 'k') k = atoi(optarg);
		else if (c == 'p') pre = atoi(optarg);
		else if (c == 'K') chunk = atoi(optarg);
		else if (c == 't') n_thread = atoi(optarg);
		else if (c == 'b') bf_shift = atoi(optarg);
		else if (c == 'H') n_hash = atoi(optarg);
	}
	if (argc - optind < 1) {
		fprintf(stderr, "Usage: yak-count [options] <in.fa> [in.fa]\n");
		fprintf(stderr, "Options:\n");
		fprintf(stderr, "  -k INT     k-mer size [%d]\n", k);
		fprintf(stderr, "  -p INT     prefix length [%d]\n", pre);
		fprintf(stderr, "  -b INT     set Bloom filter size to 2**INT bits; 0 to disable [%d]\n", bf_shift);
		fprintf(stderr, "  -H INT     use INT hash functions for Bloom filter [%d]\n", n_hash);
		fprintf(stderr, "  -t INT     number of worker threads [%d]\n", n_thread);
		fprintf(stderr, "  -K INT     chunk size [100m]\n");
		fprintf(stderr, "Note: -b37 is recommended for human reads\n");
		return 1;
	}
	if (pre < 10) {
		fprintf(stderr, "ERROR: -p should be at least %d\n", 10);
		return 1;
	}
	if (yko_hist(argv[optind], argc - optind >= 2 ? argv[optind + 1] : argv[optind], k, pre, bf_shift, n_hash,
	             chunk, hist, &tot) != 0) {
		fprintf(stderr, "ERROR: failed to count %s\n", argv[optind]);
		return 1;
	}
	fprintf(stderr, "[M::%s] %ld distinct k-mers after shrinking\n", "main", (long)tot);
	for (i = 1; i < 1024; ++i) printf("%d\t%lld\n", i, (long long)hist[i]);
	return 0;
}
#endif
