// corr_main.cpp -- drop-in correlation-matrix CLI
// over libvafc.so: the reference's options (-o -t -M -m -d, options may
// follow the files), messages, outputs and exit codes
// (correlation-matrix.c:259-409); the pairwise correlations run on the GPU
// (vc_corr_matrix).  No CPU fallback: without a GPU it reports the error and
// exits 1.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "vafc.h"

static void usage(int min_snps, int min_depth)
{
	fputs("Usage: correlation-matrix -o <output.corr> [-t] [-M MODE] [-m INT] [-d INT] <sample1.vaf> <sample2.vaf> "
	      "[sample3.vaf ...]\n"
	      "Options:\n"
	      "  -o FILE    output correlation matrix file\n"
	      "  -t         build tree/dendrogram (outputs to <output.tree>)\n"
	      "  -M MODE    preset mode: 'matched' (same individual, depth≥5, SNPs≥10),\n"
	      "                          'unmatched' (related/unrelated, depth≥1, SNPs≥20),\n"
	      "                          'strict' (high confidence, depth≥10, SNPs≥30)\n",
	      stderr);
	fprintf(stderr, "  -m INT     minimum SNPs with sufficient depth required [%d]\n", min_snps);
	fprintf(stderr, "  -d INT     minimum depth per SNP [%d]\n", min_depth);
	fputs("\nNote: -m and -d override preset mode values\n", stderr);
}

int main(int argc, char **argv)
{
	const char *out = nullptr, *mode = nullptr;
	bool tree = false, own_m = false, own_d = false;
	int min_snps = 20, min_depth = 1, c;
	opterr = 0;
	while ((c = getopt(argc, argv, "o:tm:d:M:")) >= 0) {
		switch (c) {
		case 'o': out = optarg; break;
		case 't': tree = true; break;
		case 'm': min_snps = atoi(optarg); own_m = true; break;
		case 'd': min_depth = atoi(optarg); own_d = true; break;
		case 'M': mode = optarg; break;
		default: break;   // unknown options are ignored, as ketopt's '?' is
		}
	}
	if (mode) {   // presets, correlation-matrix.c:282-306
		const char *label = nullptr;
		int pd = 0, ps = 0;
		if (!strcmp(mode, "matched")) label = "matched", pd = 5, ps = 10;
		else if (!strcmp(mode, "unmatched") || !strcmp(mode, "default")) label = "unmatched", pd = 1, ps = 20;
		else if (!strcmp(mode, "strict")) label = "strict", pd = 10, ps = 30;
		if (!label) {
			fprintf(stderr, "Error: unknown mode '%s'. Valid modes: matched, unmatched, strict\n", mode);
			return 1;
		}
		if (!own_d) min_depth = pd;
		if (!own_m) min_snps = ps;
		fprintf(stderr, "[M::main] Using '%s' mode: min_depth=%d, min_snps=%d\n", label, min_depth, min_snps);
	}
	const int n = argc - optind;
	if (!out || n < 2) {
		usage(min_snps, min_depth);
		return 1;
	}
	fprintf(stderr, "[M::main] Loading %d VAF files...\n", n);
	vc_vafset *set = nullptr;
	if (vc_vafset_create(&set) != VC_OK) {
		fprintf(stderr, "Error: failed to allocate memory\n");
		return 1;
	}
	// files are read in parallel; the messages come out in file order, as the
	// reference's sequential loop prints them (correlation-matrix.c:329-335)
	std::vector<uint8_t> truncated(n, 0);
	int added = 0;
	const int lrc = vc_vafset_add_many(set, (const char *const *)(argv + optind), n,
	                                   (int)std::thread::hardware_concurrency() < 16
	                                       ? (int)std::thread::hardware_concurrency() : 16,
	                                   &added, truncated.data());
	for (int i = 0; i < added; ++i) {
		if (truncated[i]) fprintf(stderr, "Warning: too many SNPs (max %d), truncating\n", 100000);
		fprintf(stderr, "[M::main] Loaded %s: %d SNPs\n", vc_vafset_name(set, i), vc_vafset_snps(set, i));
	}
	if (lrc != VC_OK) {
		fprintf(stderr, "Error: failed to load %s\n", argv[optind + added]);
		return 1;
	}
	fprintf(stderr, "[M::main] Computing correlation matrix...\n");
	std::vector<double> corr((size_t)n * n);
	int rc = vc_corr_matrix(set, min_snps, min_depth, corr.data(), 0, nullptr);
	if (rc != VC_OK) {
		fprintf(stderr, "Error: correlation on the GPU failed: %s\n", vc_strerror(rc));
		return 1;
	}
	fprintf(stderr, "[M::main] Writing correlation matrix...\n");
	if (vc_corr_write(set, corr.data(), out) != VC_OK) {
		fprintf(stderr, "Error: failed to open output file\n");
		return 1;
	}
	fprintf(stderr, "[M::main] Correlation matrix written to %s\n", out);
	if (tree) {
		// <out> with its first ".corr" and everything after it replaced by
		// ".tree", else <out>.tree; at most 511 bytes (the reference's buffer)
		std::string tn(out);
		if (tn.size() > 511) tn.resize(511);
		const size_t p = tn.find(".corr");
		if (p != std::string::npos) tn = tn.substr(0, p) + ".tree";
		else tn += ".tree";
		fprintf(stderr, "[M::main] Building dendrogram...\n");
		if (vc_corr_tree(set, corr.data(), tn.c_str()) == VC_OK)
			fprintf(stderr, "[M::main] Dendrogram written to %s\n", tn.c_str());
	}
	vc_vafset_free(set);
	return 0;
}
