// vaf_counter_main.cpp -- the `vaf-counter` command on top of libvafc.so.
//
// Drop-in for the reference CLI (vaf-counter.c:584-738): same options
// "k:p:o:t:b:v" (options may follow the input files), same usage text, same
// stderr messages, same .vaf output and exit codes.  The counting phase runs
// on the GPU (device: $VAFC_DEVICE, default 0), or on several: $VAFC_DEVICES
// is a comma-separated device list, one shard per entry (vc_create_multi:
// batches dealt round robin, one RCCL reduce before the .vaf is written).
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <vector>

#include "vafc.h"

static double now_s()
{
	struct timespec ts;
	clock_gettime(CLOCK_REALTIME, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void usage(int k, int n_thread, int block)
{
	fprintf(stderr, "Usage: vaf-counter [options] -p <patterns.txt> -o <output.vaf> <reads.fq> [reads2.fq ...]\n");
	fprintf(stderr, "Options:\n");
	fprintf(stderr, "  -k INT    k-mer length [%d]\n", k);
	fprintf(stderr, "  -p FILE   input pattern file\n");
	fprintf(stderr, "  -o FILE   output VAF file\n");
	fprintf(stderr, "  -t INT    number of threads [%d]\n", n_thread);
	fprintf(stderr, "  -b INT    block size [%d]\n", block);
	fprintf(stderr, "  -v        verbose mode (report performance statistics)\n");
}

int main(int argc, char *argv[])
{
	int c, k = 21, n_thread = 4, block = 10000000, verbose = 0;
	const char *pattern_fn = nullptr, *out_fn = nullptr;
	opterr = 0;
	while ((c = getopt(argc, argv, "k:p:o:t:b:v")) >= 0) {
		if (c == 'k') k = atoi(optarg);
		else if (c == 'p') pattern_fn = optarg;
		else if (c == 'o') out_fn = optarg;
		else if (c == 't') n_thread = atoi(optarg);
		else if (c == 'b') block = atoi(optarg);
		else if (c == 'v') verbose = 1;
	}
	if (!pattern_fn || !out_fn || argc - optind < 1) {
		usage(k, n_thread, block);
		return 1;
	}
	if (k < 1 || k > 31) {
		// The reference's 2-bit k-mers are undefined beyond 31 (1ULL << 2k).
		fprintf(stderr, "Error: k-mer length must be in 1..31\n");
		return 1;
	}
	const char *dev_env = getenv("VAFC_DEVICE");
	std::vector<int> devices(1, dev_env ? atoi(dev_env) : 0);
	if (const char *ds = getenv("VAFC_DEVICES")) {
		std::vector<int> v;
		for (const char *p = ds; *p;) {
			char *e = nullptr;
			const long d = strtol(p, &e, 10);
			if (e == p) break;
			v.push_back((int)d);
			p = *e == ',' ? e + 1 : e;
			if (*e != ',') break;
		}
		if (!v.empty()) devices = v;
	}

	const double t_start = now_s();
	fprintf(stderr, "[M::%s] Loading patterns...\n", "main");
	double t = now_s();
	vc_patterns *db = nullptr;
	if (vc_patterns_load(pattern_fn, &db) != VC_OK) {
		fprintf(stderr, "Error: failed to load pattern file\n");
		return 1;
	}
	const double t_load = now_s() - t;
	const int n = vc_patterns_count(db);
	fprintf(stderr, "[M::%s] Loaded %d patterns in %.3f sec\n", "main", n, t_load);

	fprintf(stderr, "[M::%s] Creating k-mer map...\n", "main");
	t = now_s();
	uint64_t *keys = nullptr;
	uint32_t *vals = nullptr;
	size_t n_keys = 0;
	int n_coll = 0;
	int rc = vc_patterns_keys(db, k, &keys, &vals, &n_keys, &n_coll);
	if (rc == VC_ETOOMANY)
		fprintf(stderr, "Error: too many patterns (%d), maximum is %d\n", n, 0x7fffffff >> 1);
	if (rc != VC_OK) {
		fprintf(stderr, "Error: failed to create k-mer map\n");
		vc_patterns_free(db);
		return 1;
	}
	if (n_coll > 0)
		fprintf(stderr, "[W::%s] Warning: %d k-mer collisions detected. "
		        "Some patterns may have overlapping k-mers.\n", "create_combined_kmer_map", n_coll);
	vc_ctx *ctx = nullptr;
	rc = vc_create_multi(&ctx, k, keys, vals, n_keys, (uint32_t)n, devices.data(), (int)devices.size());
	vc_free(keys);
	vc_free(vals);
	if (rc != VC_OK) {
		fprintf(stderr, "Error: failed to create k-mer map (%s)\n", vc_strerror(rc));
		vc_destroy(ctx);
		vc_patterns_free(db);
		return 1;
	}
	const double t_map = now_s() - t;
	uint64_t tk = 0, tslots = 0, fbytes = 0;
	vc_table_info(ctx, &tk, &tslots, &fbytes);
	if (verbose)
		fprintf(stderr, "[V::%s] Created k-mer map with %d entries in %.3f sec\n", "main", (int)tk, t_map);

	fprintf(stderr, "[M::%s] Counting k-mers in FASTQ files with %d threads...\n", "main", n_thread);
	t = now_s();
	// the reader's pinned buffers are allocated inside the counting timer, as
	// the reference allocates its per-block buffers inside it (vaf-counter.c:489-503):
	// by vc_count_file's workers, each slot on its first use, overlapping the
	// other workers' parsing (VAFC_RESERVE=1: all of them up front, as before)
	rc = getenv("VAFC_RESERVE") && getenv("VAFC_RESERVE")[0] == '1' ? vc_reserve_file_ingest(ctx, n_thread) : VC_OK;
	const double t_reserved = now_s();
	if (rc != VC_OK) {
		fprintf(stderr, "Error: counting failed (%s)\n", vc_strerror(rc));
		vc_destroy(ctx);
		vc_patterns_free(db);
		return 1;
	}
	uint64_t tot_bases = 0, tot_seqs = 0;
	for (int i = optind; i < argc; ++i) {
		fprintf(stderr, "[M::%s] Processing %s...\n", "main", argv[i]);
		vc_file_stats st;
		rc = vc_count_file(ctx, argv[i], block, n_thread, &st);
		if (rc == VC_EIO) continue;   // unopenable input is skipped silently (vaf-counter.c:557)
		if (rc != VC_OK) {
			fprintf(stderr, "Error: counting failed on %s (%s)\n", argv[i], vc_strerror(rc));
			vc_destroy(ctx);
			vc_patterns_free(db);
			return 1;
		}
		tot_bases += st.bases;
		tot_seqs += st.seqs;
		if (verbose)
			fprintf(stderr, "[V::%s] Processed %s: %llu sequences, %llu bases in %.2f sec (%.2f Mbases/sec)\n",
			        "count_fastq_kmers", argv[i], (unsigned long long)st.seqs,
			        (unsigned long long)st.bases, st.seconds, st.bases / st.seconds / 1e6);
	}
	std::vector<uint32_t> counts(2 * (size_t)n + 2, 0);
	uint64_t kmers = 0;
	const double t_read = now_s();
	rc = vc_finish(ctx, counts.data(), &kmers);
	const double t_count = now_s() - t;
	// VAFC_PHASES=1: the counting timer split into the reader's buffer
	// allocation (pinned slots of every shard), the reading and counting of
	// the files, and vc_finish (the last batches, the shard sum / RCCL reduce
	// and the copy of the counts to the host)
	if (getenv("VAFC_PHASES"))
		fprintf(stderr, "[P::main] shards %d threads %d: reserve %.4f s, read+count %.4f s, finish %.4f s, "
		        "counting %.4f s\n", (int)devices.size(), n_thread, t_reserved - t, t_read - t_reserved,
		        now_s() - t_read, t_count);
	if (rc != VC_OK) {
		fprintf(stderr, "Error: counting failed (%s)\n", vc_strerror(rc));
		vc_destroy(ctx);
		vc_patterns_free(db);
		return 1;
	}
	uint64_t tot_ref = 0, tot_alt = 0;
	for (int i = 0; i < n; ++i) {
		tot_ref += counts[2 * (size_t)i];
		tot_alt += counts[2 * (size_t)i + 1];
	}
	const double avg = (double)(tot_ref + tot_alt) / (n > 0 ? n : 1);

	fprintf(stderr, "[M::%s] Writing VAF file...\n", "main");
	t = now_s();
	if (vc_write_vaf(db, counts.data(), out_fn) != VC_OK) {
		fprintf(stderr, "Error: failed to open output file\n");
		vc_destroy(ctx);
		vc_patterns_free(db);
		return 1;
	}
	const double t_write = now_s() - t;
	fprintf(stderr, "[M::%s] Done. Average depth: %.2f\n", "main", avg);

	if (verbose) {
		const double total = now_s() - t_start;
		// the reference reports its khashl geometry: 3n rounded up to a power of two
		unsigned want = (unsigned)n * 3u, bits = 0, x = want;
		while ((x >>= 1) != 0) ++bits;
		if (want & (want - 1)) ++bits;
		if (bits < 2) bits = 2;
		const unsigned cap = 1u << bits;
		fprintf(stderr, "\n=== Performance Statistics ===\n");
		fprintf(stderr, "Total runtime:           %.3f sec\n", total);
		fprintf(stderr, "  Pattern loading:       %.3f sec (%.1f%%)\n", t_load, 100.0 * t_load / total);
		fprintf(stderr, "  K-mer map creation:    %.3f sec (%.1f%%)\n", t_map, 100.0 * t_map / total);
		fprintf(stderr, "  K-mer counting:        %.3f sec (%.1f%%)\n", t_count, 100.0 * t_count / total);
		fprintf(stderr, "  Output writing:        %.3f sec (%.1f%%)\n", t_write, 100.0 * t_write / total);
		fprintf(stderr, "\nThroughput:\n");
		fprintf(stderr, "  Sequences processed:   %llu\n", (unsigned long long)tot_seqs);
		fprintf(stderr, "  Bases processed:       %llu (%.2f Mbases)\n", (unsigned long long)tot_bases, tot_bases / 1e6);
		fprintf(stderr, "  K-mers extracted:      %llu (%.2f million)\n", (unsigned long long)kmers, kmers / 1e6);
		if (t_count > 0) {
			fprintf(stderr, "  Speed:                 %.2f Mbases/sec\n", tot_bases / t_count / 1e6);
			fprintf(stderr, "  K-mer throughput:      %.2f million k-mers/sec\n", kmers / t_count / 1e6);
		}
		fprintf(stderr, "\nMemory:\n");
		fprintf(stderr, "  Patterns:              %d\n", n);
		fprintf(stderr, "  Hash table entries:    %d\n", (int)tk);
		fprintf(stderr, "  Hash table capacity:   %d\n", (int)cap);
		fprintf(stderr, "  Hash table load:       %.1f%%\n", 100.0 * tk / cap);
		fprintf(stderr, "\nOptimizations:\n");
		fprintf(stderr, "  SIMD:                  MI355X HIP (gfx950), LDS prefilter %llu KiB, device table %llu slots\n",
		        (unsigned long long)(fbytes >> 10), (unsigned long long)tslots);
		if (devices.size() > 1)
			fprintf(stderr, "  Shards:                %d (RCCL reduce of the counts)\n", (int)devices.size());
		fprintf(stderr, "  Threads:               %d workers\n", n_thread);
		fprintf(stderr, "==============================\n");
	}
	vc_destroy(ctx);
	vc_patterns_free(db);
	return 0;
}
