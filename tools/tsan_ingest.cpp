// ThreadSanitizer driver for the host readers (tools only; no GPU): built with
// the reader sources by tools/tsan_gz.sh.  For a FASTQ file and its gzip form
// it checks that every threaded path hands over the same reads as the
// sequential reader (VcFastqReader, kseq's rules):
//   * the parallel reader over the plain file (vc_scan_file_parallel);
//   * the plain file in W byte ranges (vc_scan_file_range), concatenated;
//   * the gzip file in W shares, two pass (vc_gz_share_scan, vc_scan_gz_share)
//     and held (vc_gzp_scan_share_hold, vc_scan_gz_share_held), concatenated.
//
//   tsan_ingest PLAIN.fq GZ.fq.gz [threads] [world]
#include "vafc.h"
#include "vafc_fastq.h"
#include "vafc_gzip.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <string>
#include <vector>

struct Reads {
	std::vector<uint8_t> seq;
	std::vector<uint32_t> lens;
	uint64_t seqs = 0;
	void trim(const vc_file_stats &st)
	{
		uint64_t b = 0;
		for (uint64_t i = 0; i < st.seqs; ++i) b += lens[i];
		seq.resize(b);
		lens.resize(st.seqs);
		seqs = st.seqs;
	}
	void append(const Reads &o)
	{
		seq.insert(seq.end(), o.seq.begin(), o.seq.end());
		lens.insert(lens.end(), o.lens.begin(), o.lens.end());
		seqs += o.seqs;
	}
	bool operator==(const Reads &o) const { return seq == o.seq && lens == o.lens; }
};

static int fails = 0;

static void check(bool ok, const char *what)
{
	if (!ok) {
		fprintf(stderr, "FAIL: %s\n", what);
		++fails;
	}
}

static const int K = 21, BLOCK = 100000;
static size_t cap_seq, cap_lens;

// The sequential reader's records (every read of these well-formed files is
// longer than k, so the block loop of vc_scan_file would take them all).
static Reads sequential(const char *path)
{
	Reads r;
	VcFastqReader rd;
	if (!rd.open(path)) return r;
	while (rd.next() >= 0) {
		r.seq.insert(r.seq.end(), (const uint8_t *)rd.seq(), (const uint8_t *)rd.seq() + rd.seq_len());
		r.lens.push_back((uint32_t)rd.seq_len());
		++r.seqs;
	}
	return r;
}

static void alloc(Reads &r)
{
	r.seq.assign(cap_seq, 0);
	r.lens.assign(cap_lens, 0);
}

int main(int argc, char **argv)
{
	if (argc < 3) {
		fprintf(stderr, "usage: tsan_ingest PLAIN.fq GZ.fq.gz [threads] [world]\n");
		return 2;
	}
	const char *fq = argv[1], *gz = argv[2];
	const int T = argc > 3 ? atoi(argv[3]) : 4;
	const int W = argc > 4 ? atoi(argv[4]) : 3;
	struct stat sb;
	if (stat(fq, &sb) != 0) return 2;
	const uint64_t size = (uint64_t)sb.st_size;
	cap_seq = size + 4096;
	cap_lens = size / 8 + 64;
	vc_file_stats st;
	vc_range_info ri;

	const Reads ref = sequential(fq);
	check(ref.seqs > 0, "sequential");

	Reads par;
	alloc(par);
	check(vc_scan_file_parallel(fq, K, BLOCK, T, 1 << 16, &st, par.seq.data(), cap_seq, par.lens.data(), cap_lens) ==
	          VC_OK,
	      "parallel");
	par.trim(st);
	check(par == ref, "parallel reads == sequential");

	Reads ranges;
	for (int r = 0; r < W; ++r) {
		const uint64_t b = size * (uint64_t)r / (uint64_t)W, e = size * (uint64_t)(r + 1) / (uint64_t)W;
		Reads x;
		alloc(x);
		check(vc_scan_file_range(fq, K, BLOCK, T, 1 << 16, b, e, &st, &ri, x.seq.data(), cap_seq, x.lens.data(),
		                         cap_lens) == VC_OK,
		      "range");
		x.trim(st);
		ranges.append(x);
	}
	check(ranges == ref, "ranges concatenated == sequential");

	check(sequential(gz) == ref, "gz sequential == plain");

	struct stat gb;
	if (stat(gz, &gb) != 0) return 2;
	const uint64_t gsize = (uint64_t)gb.st_size;
	for (int held = 0; held < 2; ++held) {
		std::vector<vc_gz_share_info> info(W);
		std::vector<std::vector<uint16_t>> sym(W, std::vector<uint16_t>(32768));
		std::vector<vc_gz_share *> hs(W, nullptr);
		for (int r = 0; r < W; ++r) {
			const uint64_t b = gsize * (uint64_t)r / (uint64_t)W, e = gsize * (uint64_t)(r + 1) / (uint64_t)W;
			if (!held) {
				check(vc_gz_share_scan(gz, b, e, T, 16384, &info[r], sym[r].data()) == VC_OK, "share scan");
				continue;
			}
			VcGzShare sh;
			VcGzParallel *g = nullptr;
			check(vc_gzp_scan_share_hold(gz, T, 16384, b, e, 1ull << 32, &sh, sym[r].data(), &g), "held scan");
			info[r] = vc_gz_share_info{sh.start_bit, sh.end_bit, sh.text_len, sh.ok ? 1u : 0u,
			                           sh.start_bit != UINT64_MAX && sh.end_bit == UINT64_MAX ? 1u : 0u};
			if (g) {
				hs[r] = new vc_gz_share;
				hs[r]->g = g;
				hs[r]->format = 0;   // FASTQ
				hs[r]->threads = T;
			}
		}
		std::vector<uint8_t> before(32768, 0);
		Reads all;
		for (int r = 0; r < W; ++r) {
			if (info[r].start_bit == UINT64_MAX) continue;
			check(info[r].ok != 0, "share ok");
			const std::vector<uint8_t> win = before;
			for (int i = 0; i < 32768; ++i) {
				const uint16_t v = sym[r][i];
				before[i] = v < 256 ? (uint8_t)v : win[v & 32767];
			}
			Reads x;
			alloc(x);
			vc_gz_share_crc crc;
			int rc;
			if (hs[r]) {
				rc = vc_scan_gz_share_held(hs[r], K, r == 0, win.data(), info[r].text_len, BLOCK, T, &st, &ri, &crc,
				                           x.seq.data(), cap_seq, x.lens.data(), cap_lens);
			} else {
				check(!held, "held share kept");
				rc = vc_scan_gz_share(gz, K, r == 0, info[r].start_bit, win.data(), info[r].text_len, BLOCK, T, &st,
				                      &ri, &crc, x.seq.data(), cap_seq, x.lens.data(), cap_lens);
			}
			check(rc == VC_OK, held ? "held share count" : "share count");
			x.trim(st);
			all.append(x);
		}
		for (vc_gz_share *h : hs) vc_gz_share_close(h);
		check(all == ref, held ? "held shares == sequential" : "two-pass shares == sequential");
	}
	printf("%s + %s: %llu reads, %d threads, %d ranks: %s\n", fq, gz, (unsigned long long)ref.seqs, T, W,
	       fails ? "FAILED" : "ok");
	return fails ? 1 : 0;
}
