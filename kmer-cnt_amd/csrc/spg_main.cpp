// spg_main.cpp -- the `snp-pattern-gen` command on top of libvafc.so.
//
// Drop-in for the reference tool (snp-pattern-gen.c:219-367): same options
// "k:b:f:o:" (options may follow other arguments), same messages, same
// pattern file and exit codes.  The genome pass -- counting the candidate
// k-mers over every chromosome -- runs on the GPU (vc_count_candidates,
// device $VAFC_DEVICE, default 0); BED parsing, k-mer extraction and the
// selection stay on the host as in the reference.
#include <getopt.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "vafc.h"

namespace {

// seq_nt4_table (snp-pattern-gen.c:30-47)
struct Nt4 {
	uint8_t t[256];
	Nt4()
	{
		memset(t, 4, sizeof(t));
		for (int i = 0; i < 4; ++i) t[i] = (uint8_t)i;
		const char *up = "ACGT", *lo = "acgt";
		for (int i = 0; i < 4; ++i) t[(uint8_t)up[i]] = t[(uint8_t)lo[i]] = (uint8_t)i;
		t['U'] = t['u'] = 3;
	}
};
const Nt4 NT4;

struct Snp {
	char chr[256];
	int start, end;
	char rsid[256];
	char ref, alt;
};

bool next_snp(FILE *fp, Snp &s)   // the reference's fscanf record (snp-pattern-gen.c:267,309)
{
	return fscanf(fp, "%254s%d%d%254s %c %c", s.chr, &s.start, &s.end, s.rsid, &s.ref, &s.alt) == 6;
}

// 2-bit key of k characters, UINT64_MAX on any non-ACGTU (snp-pattern-gen.c:129-139)
uint64_t key_of(const char *s, int k)
{
	uint64_t x = 0;
	for (int i = 0; i < k; ++i) {
		const uint8_t c = NT4.t[(uint8_t)s[i]];
		if (c >= 4) return UINT64_MAX;
		x = x << 2 | c;
	}
	return x;
}

uint64_t canonical(uint64_t x, int k)   // snp-pattern-gen.c:141-157
{
	uint64_t r = 0, y = x;
	for (int i = 0; i < k; ++i, y >>= 2) r = r << 2 | (3 - (y & 3));
	return x < r ? x : r;
}

class Genome {
public:
	explicit Genome(vc_fasta *fa) : fa_(fa)
	{
		for (int i = 0; i < vc_fasta_count(fa); ++i) by_name_.emplace(vc_fasta_name(fa, i), i);   // first wins
	}
	// the first chromosome of that name (find_seq, snp-pattern-gen.c:118-126)
	const uint8_t *find(const char *chr, uint32_t *len) const
	{
		auto it = by_name_.find(chr);
		return it == by_name_.end() ? nullptr : vc_fasta_seq(fa_, it->second, len);
	}

private:
	vc_fasta *fa_;
	std::unordered_map<std::string, int> by_name_;
};

// ref / alt k-mer strings around a SNP; false if out of range or not all
// ACGTU (extract_snp_kmer, snp-pattern-gen.c:192-217)
bool snp_kmers(const uint8_t *seq, uint32_t len, int pos, char alt, int k, char *ref_kmer, char *alt_kmer)
{
	const int flank = k / 2, start = pos - flank;
	if (start < 0 || (int64_t)start + k > (int64_t)len) return false;
	for (int i = 0; i < k; ++i)
		if (NT4.t[seq[start + i]] >= 4) return false;
	memcpy(ref_kmer, seq + start, (size_t)k);
	memcpy(alt_kmer, seq + start, (size_t)k);
	ref_kmer[k] = alt_kmer[k] = 0;
	alt_kmer[flank] = alt;
	return true;
}

void usage(int k)
{
	fprintf(stderr, "Usage: snp-pattern-gen -k %d -b <snps.bed> -f <ref.fa> -o <patterns.txt>\n", k);
	fprintf(stderr, "Options:\n");
	fprintf(stderr, "  -k INT    k-mer length (must be odd) [%d]\n", k);
	fprintf(stderr, "  -b FILE   input BED file with SNPs\n");
	fprintf(stderr, "  -f FILE   input reference genome FASTA file\n");
	fprintf(stderr, "  -o FILE   output pattern file\n");
}

} // namespace

int main(int argc, char *argv[])
{
	int c, k = 21;
	const char *bed_fn = nullptr, *fasta_fn = nullptr, *out_fn = nullptr;
	opterr = 0;
	while ((c = getopt(argc, argv, "k:b:f:o:")) >= 0) {
		if (c == 'k') k = atoi(optarg);
		else if (c == 'b') bed_fn = optarg;
		else if (c == 'f') fasta_fn = optarg;
		else if (c == 'o') out_fn = optarg;
	}
	if (k % 2 == 0) {
		fprintf(stderr, "Error: k must be odd\n");
		return 1;
	}
	if (!bed_fn || !fasta_fn || !out_fn) {
		usage(k);
		return 1;
	}
	if (k < 1 || k > 31) {   // 2-bit keys in 64 bits; the reference is undefined beyond 31
		fprintf(stderr, "Error: k-mer length must be in 1..31\n");
		return 1;
	}
	const char *dev_env = getenv("VAFC_DEVICE");
	const int device = dev_env ? atoi(dev_env) : 0;

	fprintf(stderr, "[M::%s] Loading reference genome...\n", "main");
	vc_fasta *fa = nullptr;
	if (vc_fasta_load(fasta_fn, &fa) != VC_OK) {
		fprintf(stderr, "Error: failed to load FASTA file\n");
		return 1;
	}
	fprintf(stderr, "[M::%s] Loaded %d sequences\n", "main", vc_fasta_count(fa));
	const Genome genome(fa);

	// pass 1: candidate keys, in first-seen order (snp-pattern-gen.c:259-296)
	fprintf(stderr, "[M::%s] Generating candidate k-mers from BED file...\n", "main");
	FILE *bed = fopen(bed_fn, "r");
	if (!bed) {
		fprintf(stderr, "Error: failed to open BED file\n");
		vc_fasta_free(fa);
		return 1;
	}
	std::unordered_map<uint64_t, uint32_t> index;
	std::vector<uint64_t> keys;
	char ref_kmer[128], alt_kmer[128];
	Snp snp;
	auto add_key = [&](uint64_t key) {
		if (index.emplace(key, (uint32_t)keys.size()).second) keys.push_back(key);
	};
	while (next_snp(bed, snp)) {
		uint32_t len = 0;
		const uint8_t *seq = genome.find(snp.chr, &len);
		if (!seq || !snp_kmers(seq, len, snp.start, snp.alt, k, ref_kmer, alt_kmer)) continue;
		const uint64_t re = key_of(ref_kmer, k), ae = key_of(alt_kmer, k);
		if (re == UINT64_MAX || ae == UINT64_MAX) continue;
		add_key(canonical(re, k));
		add_key(canonical(ae, k));
	}
	fclose(bed);
	fprintf(stderr, "[M::%s] Generated %d candidate k-mers\n", "main", (int)keys.size());

	// pass 2: the genome scan, on the GPU (snp-pattern-gen.c:159-190)
	fprintf(stderr, "[M::%s] Counting candidate k-mers in genome...\n", "main");
	std::vector<uint32_t> counts(keys.size() + 1, 0);
	{
		const uint8_t *gs = nullptr;
		size_t gbytes = 0;
		const uint64_t *goffs = nullptr;
		const uint32_t *glens = nullptr;
		vc_fasta_data(fa, &gs, &gbytes, &goffs, &glens);
		const int rc = vc_count_candidates(k, gs, gbytes, goffs, glens, (uint64_t)vc_fasta_count(fa),
		                                   keys.data(), keys.size(), counts.data(), device);
		if (rc != VC_OK) {
			fprintf(stderr, "Error: candidate counting failed (%s)\n", vc_strerror(rc));
			vc_fasta_free(fa);
			return 1;
		}
	}
	fprintf(stderr, "[M::%s] Finished counting k-mers\n", "main");

	// pass 3: SNPs whose ref k-mer occurs once and alt k-mer never (snp-pattern-gen.c:306-355)
	bed = fopen(bed_fn, "r");
	if (!bed) {
		fprintf(stderr, "Error: failed to open BED file\n");
		vc_fasta_free(fa);
		return 1;
	}
	FILE *out = fopen(out_fn, "w");
	if (!out) {
		fprintf(stderr, "Error: failed to open output file\n");
		fclose(bed);
		vc_fasta_free(fa);
		return 1;
	}
	fprintf(stderr, "[M::%s] Processing SNPs...\n", "main");
	int n_total = 0, n_unique = 0;
	auto count_of = [&](uint64_t key, uint32_t *v) {
		auto it = index.find(key);
		if (it == index.end()) return false;
		*v = counts[it->second];
		return true;
	};
	while (next_snp(bed, snp)) {
		++n_total;
		uint32_t len = 0;
		const uint8_t *seq = genome.find(snp.chr, &len);
		if (!seq) {
			fprintf(stderr, "Warning: chromosome %s not found\n", snp.chr);
			continue;
		}
		if (!snp_kmers(seq, len, snp.start, snp.alt, k, ref_kmer, alt_kmer)) continue;
		const uint64_t re = key_of(ref_kmer, k), ae = key_of(alt_kmer, k);
		if (re == UINT64_MAX || ae == UINT64_MAX) continue;
		uint32_t rv = 0, av = 0;
		if (count_of(canonical(re, k), &rv) && rv == 1 && count_of(canonical(ae, k), &av) && av == 0) {
			fprintf(out, "%s\t%d\t%d\t%s\t%c\t%c\t%s\t%s\n", snp.chr, snp.start, snp.end, snp.rsid, snp.ref,
			        snp.alt, ref_kmer, alt_kmer);
			++n_unique;
		}
	}
	fprintf(stderr, "[M::%s] Total SNPs: %d, Unique k-mer pairs: %d\n", "main", n_total, n_unique);
	fclose(bed);
	fclose(out);
	vc_fasta_free(fa);
	return 0;
}
