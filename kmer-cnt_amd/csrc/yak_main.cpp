// yak_main.cpp -- the `yak-count` command on top of libvafc.so (SURVEY.md
// §8(f) rank 3).
//
// Drop-in for the reference CLI (yak-count.c:456-507): same options
// "k:p:K:t:b:H:" (options may follow the inputs), defaults, usage text and -p
// check; the same 1023 histogram lines on stdout and the same final stderr
// line ("[M::main] N distinct k-mers after shrinking").  Counting runs on the
// GPU (device: $VAFC_DEVICE, default 0) in one device table
// ($VAFC_KC_SLOTS slots, default sized from the size of file 1, at most 40 %
// of free HBM):
//
//   * no filter (-b 0, the default): every canonical k-mer of file 1 (a
//     second file is ignored, as in yak_count_file), 10-bit saturating counts
//     (histogram bins min(c, 1023));
//   * -b with one input, or file 2 = file 1: yak's two passes keep exactly the
//     k-mers seen at least twice (a k-mer seen twice always passes its Bloom
//     filter; pass 2 recounts exactly; the shrink drops counts below 2), so
//     one pass with min_count 2 gives the same histogram;
//   * -b with two different inputs: pass 1 over file 1 records first
//     occurrences, vc_yak_bloom_select replays yak's Bloom filters to pick the
//     same keys, pass 2 counts those keys in file 2, the shrink keeps [2, 1023].
//
// When the distinct k-mers outgrow the table, the inputs are counted again in
// partitions of whole yak sub-tables whose histograms add up.
//
// Differences, all on failure or progress paths: the per-block "[M] processed"
// progress lines are not printed; an input that cannot be opened prints an
// error and exits 1 (the reference dereferences a null table, yak-count.c:497).
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "vafc.h"

// Table size from the input: at most one distinct k-mer per byte of the file
// (five per byte of gzip), so no partition pass is needed unless HBM caps it.
static uint64_t size_hint(const char *fn)
{
	struct stat sb;
	if (stat(fn, &sb) != 0 || sb.st_size <= 0) return 1 << 16;
	uint64_t b = (uint64_t)sb.st_size;
	const size_t n = strlen(fn);
	if (n > 3 && strcmp(fn + n - 3, ".gz") == 0) b *= 5;
	return b + b / 4 + (1 << 16);
}

static int fail(vc_ctx *ctx, const char *what, int rc)
{
	fprintf(stderr, "ERROR: %s (%s)\n", what, vc_strerror(rc));
	vc_destroy(ctx);
	return 1;
}

int main(int argc, char *argv[])
{
	int c, k = 31, pre = 10, bf_shift = 0, n_hash = 4, n_thread = 4;
	long long chunk = 10000000;
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
	if (k < 1 || k > 31) {
		// yak's 2-bit k-mers are undefined beyond 31 (YAK_MAX_KMER, 1ULL << 2k)
		fprintf(stderr, "ERROR: k-mer size must be in 1..31\n");
		return 1;
	}
	// the block loop compares an int sum with the chunk size (yak-count.c:350)
	const int block = chunk > 0x7fffffffLL ? 0x7fffffff : (int)chunk;
	const char *dev_env = getenv("VAFC_DEVICE");
	const int device = dev_env ? atoi(dev_env) : 0;
	const char *slots_env = getenv("VAFC_KC_SLOTS");
	const char *fn1 = argv[optind];
	const uint64_t slots = slots_env ? strtoull(slots_env, nullptr, 10) : size_hint(fn1);
	const char *fn2 = argc - optind >= 2 ? argv[optind + 1] : fn1;
	const bool two_pass = bf_shift > 0;
	const bool replay = two_pass && strcmp(fn1, fn2) != 0;   // Bloom replay + pass 2 over file 2

	vc_ctx *ctx = nullptr;
	int rc = vc_kc_create(&ctx, k, slots, device);
	if (rc == VC_OK) rc = vc_reserve_file_ingest(ctx, n_thread);
	if (rc != VC_OK) return fail(ctx, "failed to create the k-mer table", rc);

	uint64_t hist[1024];
	uint64_t tot = 0;
	uint32_t n_parts = 1;
	for (;;) {
		bool full = false;
		uint64_t kmers = 0;
		memset(hist, 0, sizeof hist);
		tot = 0;
		for (uint32_t part = 0; part < n_parts && !full; ++part) {
			vc_file_stats st;
			rc = vc_kc_set_partition(ctx, n_parts, part);
			if (rc == VC_OK && replay) rc = vc_kc_track_first(ctx, 1);
			if (rc == VC_OK) rc = vc_count_file(ctx, fn1, block, n_thread, &st);
			if (rc == VC_EIO) return fail(ctx, "failed to open the input", rc);
			if (rc == VC_OK) rc = vc_finish(ctx, nullptr, nullptr);
			if (rc == VC_OK && replay) {
				rc = vc_yak_bloom_select(ctx, pre, bf_shift, n_hash);
				if (rc == VC_OK) rc = vc_count_file(ctx, fn2, block, n_thread, &st);
				if (rc == VC_EIO) return fail(ctx, "failed to open the input", rc);
				if (rc == VC_OK) rc = vc_finish(ctx, nullptr, nullptr);
			}
			uint64_t distinct = 0;
			if (rc == VC_OK) rc = vc_kc_histogram2(ctx, hist, 1024, two_pass ? 2 : 1, &distinct, &kmers);
			if (rc == VC_EFULL) {
				full = true;
				rc = VC_OK;
			}
			if (rc != VC_OK) return fail(ctx, "counting failed", rc);
			tot += distinct;
		}
		if (!full) break;
		// every k-mer seen is at most one distinct k-mer: slices of 70 % of the
		// table always fit on average; double on a further overflow
		const uint64_t cap = vc_kc_slots(ctx) / 10 * 7;
		uint64_t want = cap ? (kmers + cap - 1) / cap : 2;
		if (want <= n_parts) want = (uint64_t)n_parts * 2;
		if (want > 1024) return fail(ctx, "k-mer table too small", VC_EFULL);
		n_parts = (uint32_t)want;
	}
	vc_destroy(ctx);
	fprintf(stderr, "[M::%s] %ld distinct k-mers after shrinking\n", "main", (long)tot);
	for (int i = 1; i < 1024; ++i) printf("%d\t%lld\n", i, (long long)hist[i]);
	return 0;
}
