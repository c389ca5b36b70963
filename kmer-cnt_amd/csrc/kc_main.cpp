// kc_main.cpp -- the `kc-c4` command on top of libvafc.so (SURVEY.md §8(f)
// rank 3).
//
// Drop-in for the reference CLI (kc-c4.c:236-265): same options "k:p:b:t:"
// (options may follow the input), same defaults, usage text and -p check, the
// same 255 histogram lines on stdout.  Counting runs on the GPU (device:
// $VAFC_DEVICE, default 0) in one device hash table; -p (the reference's
// sub-table count) does not change the output and only has its check kept.
// When the distinct k-mers outgrow the table ($VAFC_KC_SLOTS, default sized
// from free HBM) the file is counted again in hash partitions whose
// histograms add up (vc_kc_set_partition).  The table is sized from the input
// file (at most 40 % of free HBM).
//
// Differences, all on failure paths: an input that cannot be opened prints
// an error and exits 1 (the reference dereferences a null table,
// kc-c4.c:185,261); a GPU error prints it and exits 1.
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

int main(int argc, char *argv[])
{
	int c, k = 31, p = 10, block = 10000000, n_thread = 4;
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
	if (k < 1 || k > 31) {
		// the reference's 2-bit k-mers are undefined beyond 31 (1ULL << 2k)
		fprintf(stderr, "ERROR: k-mer size must be in 1..31\n");
		return 1;
	}
	const char *dev_env = getenv("VAFC_DEVICE");
	const int device = dev_env ? atoi(dev_env) : 0;
	const char *slots_env = getenv("VAFC_KC_SLOTS");
	const char *fn = argv[optind];
	const uint64_t slots = slots_env ? strtoull(slots_env, nullptr, 10) : size_hint(fn);

	vc_ctx *ctx = nullptr;
	int rc = vc_kc_create(&ctx, k, slots, device);
	if (rc == VC_OK) rc = vc_reserve_file_ingest(ctx, n_thread);
	if (rc != VC_OK) {
		fprintf(stderr, "ERROR: failed to create the k-mer table (%s)\n", vc_strerror(rc));
		vc_destroy(ctx);
		return 1;
	}
	uint64_t hist[256] = {0};
	uint32_t n_parts = 1;
	for (;;) {
		bool full = false;
		uint64_t kmers = 0;
		for (uint32_t part = 0; part < n_parts && !full; ++part) {
			rc = vc_kc_set_partition(ctx, n_parts, part);
			vc_file_stats st;
			if (rc == VC_OK) rc = vc_count_file(ctx, fn, block, n_thread, &st);
			if (rc == VC_EIO) {
				fprintf(stderr, "ERROR: failed to open %s\n", fn);
				vc_destroy(ctx);
				return 1;
			}
			if (rc == VC_OK) rc = vc_finish(ctx, nullptr, nullptr);
			uint64_t distinct = 0;
			if (rc == VC_OK) rc = vc_kc_histogram(ctx, hist, &distinct, &kmers);
			if (rc == VC_EFULL) {
				full = true;
				rc = VC_OK;
			}
			if (rc != VC_OK) {
				fprintf(stderr, "ERROR: counting failed (%s)\n", vc_strerror(rc));
				vc_destroy(ctx);
				return 1;
			}
		}
		if (!full) break;
		// every k-mer seen is at most one distinct k-mer: slices of 70 % of the
		// table always fit on average; double on a further overflow
		const uint64_t cap = vc_kc_slots(ctx) / 10 * 7;
		uint64_t want = cap ? (kmers + cap - 1) / cap : 2;
		if (want <= n_parts) want = (uint64_t)n_parts * 2;
		if (want > 1024) {
			fprintf(stderr, "ERROR: k-mer table too small\n");
			vc_destroy(ctx);
			return 1;
		}
		n_parts = (uint32_t)want;
		for (int i = 0; i < 256; ++i) hist[i] = 0;
	}
	vc_destroy(ctx);
	for (int i = 1; i < 256; ++i) printf("%d\t%ld\n", i, (long)hist[i]);
	return 0;
}
