// vafc_spg.cpp -- the snp-pattern-gen side of the C ABI (SURVEY.md §8(f)
// rank 2): genome loading and candidate k-mer counting on the GPU.
//
// snp-pattern-gen counts, over every sequence of a reference genome, the
// canonical k-mers that are candidate keys (the ref and alt k-mers of the
// BED's SNPs) -- count_candidate_kmers, snp-pattern-gen.c:159-190.  That is
// the vaf-counter scan with a different decode and one counter per key:
//   * the genome is copied to HBM and counted in seq_nt4 mode
//     (vc_set_nt4_decode): every chunk takes the exact seq_nt4_table decode
//     that vaf-counter's kernels use only for a read's tail;
//   * the candidate keys become a key table whose value is the key's own
//     index, so counts[i] is the number of occurrences of keys[i];
//   * chromosomes (longer than 16,384 bases) take the segmented long-read
//     kernel.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "vafc.h"
#include "vafc_fastq.h"
#include "vafc_internal.h"

struct vc_fasta {
	std::vector<std::string> names;
	std::vector<uint8_t> seq;
	std::vector<uint64_t> offs;
	std::vector<uint32_t> lens;
};

// load_fasta (snp-pattern-gen.c:67-103): every record, kseq semantics, until
// the first kseq_read < 0
extern "C" int vc_fasta_load(const char *path, vc_fasta **out)
{
	if (!path || !out) return VC_EINVAL;
	*out = nullptr;
	VcFastqReader rd;   // a gzip genome is inflated in parallel (vafc_gzip.h)
	const char *te = getenv("VAFC_THREADS");
	int threads = te && atoi(te) > 0 ? atoi(te) : (int)std::thread::hardware_concurrency();
	threads = threads < 1 ? 1 : (threads > 16 ? 16 : threads);
	if (!rd.open_parallel(path, threads)) return VC_EIO;
	rd.keep_names(true);
	vc_fasta *fa = new (std::nothrow) vc_fasta;
	if (!fa) return VC_ENOMEM;
	try {
		int ret;
		while ((ret = rd.next()) >= 0) {
			fa->names.emplace_back(rd.name(), rd.name_len());
			fa->offs.push_back(fa->seq.size());
			fa->lens.push_back((uint32_t)ret);
			fa->seq.insert(fa->seq.end(), (const uint8_t *)rd.seq(), (const uint8_t *)rd.seq() + ret);
		}
	} catch (...) {
		delete fa;
		return VC_ENOMEM;
	}
	*out = fa;
	return VC_OK;
}

extern "C" int vc_fasta_count(const vc_fasta *fa) { return fa ? (int)fa->names.size() : 0; }

extern "C" const char *vc_fasta_name(const vc_fasta *fa, int i)
{
	return fa && i >= 0 && (size_t)i < fa->names.size() ? fa->names[(size_t)i].c_str() : nullptr;
}

extern "C" const uint8_t *vc_fasta_seq(const vc_fasta *fa, int i, uint32_t *len)
{
	if (!fa || i < 0 || (size_t)i >= fa->names.size()) return nullptr;
	if (len) *len = fa->lens[(size_t)i];
	return fa->seq.data() + fa->offs[(size_t)i];
}

extern "C" int vc_fasta_data(const vc_fasta *fa, const uint8_t **seq, size_t *bytes, const uint64_t **offs,
                             const uint32_t **lens)
{
	if (!fa) return VC_EINVAL;
	if (seq) *seq = fa->seq.data();
	if (bytes) *bytes = fa->seq.size();
	if (offs) *offs = fa->offs.data();
	if (lens) *lens = fa->lens.data();
	return VC_OK;
}

extern "C" void vc_fasta_free(vc_fasta *fa) { delete fa; }

#define SPGCK(call)                                                                          \
	do {                                                                                     \
		hipError_t e_ = (call);                                                              \
		if (e_ != hipSuccess) {                                                              \
			fprintf(stderr, "[E::vafc] %s failed: %s\n", #call, hipGetErrorString(e_));     \
			rc = VC_EHIP;                                                                    \
			goto done;                                                                       \
		}                                                                                    \
	} while (0)

extern "C" int vc_count_candidates(int k, const uint8_t *seq, size_t seq_bytes, const uint64_t *offs,
                                   const uint32_t *lens, uint64_t n_seqs, const uint64_t *keys, size_t n_keys,
                                   uint32_t *counts, int device)
{
	if (k < 1 || k > 31 || (n_keys && (!keys || !counts)) || (n_seqs && (!seq || !offs || !lens)))
		return VC_EINVAL;
	for (uint64_t i = 0; i < n_seqs; ++i)
		if (offs[i] + lens[i] > seq_bytes) return VC_EINVAL;
	if (n_keys == 0) return VC_OK;
	const uint32_t n_patterns = (uint32_t)((n_keys + 1) / 2);
	std::vector<uint32_t> vals(n_keys), all(2 * (size_t)n_patterns + 2, 0);
	for (size_t i = 0; i < n_keys; ++i) vals[i] = (uint32_t)i;
	vc_ctx *ctx = nullptr;
	int rc = vc_create(&ctx, k, keys, vals.data(), n_keys, n_patterns, device);
	if (rc != VC_OK) return rc;
	vc_set_nt4_decode(ctx, 1);
	uint8_t *d_seq = nullptr;
	uint64_t *d_offs = nullptr;
	uint32_t *d_lens = nullptr;
	if (n_seqs) {
		SPGCK(hipMalloc(&d_seq, seq_bytes + 16));
		SPGCK(hipMemcpy(d_seq, seq, seq_bytes, hipMemcpyHostToDevice));
		SPGCK(hipMalloc(&d_offs, n_seqs * sizeof(uint64_t)));
		SPGCK(hipMalloc(&d_lens, n_seqs * sizeof(uint32_t)));
		SPGCK(hipMemcpy(d_offs, offs, n_seqs * sizeof(uint64_t), hipMemcpyHostToDevice));
		SPGCK(hipMemcpy(d_lens, lens, n_seqs * sizeof(uint32_t), hipMemcpyHostToDevice));
		rc = vc_count_device(ctx, d_seq, seq_bytes, d_offs, d_lens, n_seqs, nullptr);
		if (rc != VC_OK) goto done;
	}
	rc = vc_finish(ctx, all.data(), nullptr);
	if (rc == VC_OK) memcpy(counts, all.data(), n_keys * sizeof(uint32_t));
done:
	if (d_seq) (void)hipFree(d_seq);
	if (d_offs) (void)hipFree(d_offs);
	if (d_lens) (void)hipFree(d_lens);
	vc_destroy(ctx);
	return rc;
}
