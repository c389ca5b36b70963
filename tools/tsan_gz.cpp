// ThreadSanitizer driver for the parallel inflater (tools only; host code, no
// GPU): built with the inflater's own source by tools/tsan_gz.sh.  For one
// gzip file it checks, against zlib's gzread output of the same file:
//   1. the whole stream through vc_gzp_open (speculative chunks, fallbacks);
//   2. the file in W shares, two pass: vc_gzp_scan_share, the windows chained
//      from the scans' symbols, then vc_gzp_open_share from each start;
//   3. the same shares held: vc_gzp_scan_share_hold, then vc_gzp_resume_share
//      (budget large), and with a budget that runs out (the scan frees what
//      it kept and reports no held share).
// Each share's stream must equal the reference text from its start for its
// text length (and go on past it, as the reader reads on into the next share).
//
//   tsan_gz FILE.gz [threads] [chunk_bytes] [world]
#include "vafc_gzip.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <vector>

static std::vector<uint8_t> zlib_text(const char *path)
{
	std::vector<uint8_t> out;
	gzFile f = gzopen(path, "r");
	if (!f) return out;
	std::vector<uint8_t> buf(1 << 20);
	for (;;) {
		const int r = gzread(f, buf.data(), (unsigned)buf.size());
		if (r <= 0) break;
		out.insert(out.end(), buf.begin(), buf.begin() + r);
	}
	gzclose(f);
	return out;
}

static int fails = 0;

static void check(bool ok, const char *what)
{
	if (!ok) {
		fprintf(stderr, "FAIL: %s\n", what);
		++fails;
	}
}

// Read n bytes (or to the end) from g and compare with ref[off, off + n).
static void read_compare(VcGzParallel *g, const std::vector<uint8_t> &ref, uint64_t off, uint64_t n, const char *what)
{
	uint64_t got = 0;
	bool same = true;
	while (got < n) {
		const uint8_t *p;
		const int64_t r = vc_gzp_span(g, &p, (size_t)(n - got));
		if (r <= 0) break;
		if (off + got + (uint64_t)r > ref.size() || memcmp(p, ref.data() + off + got, (size_t)r) != 0) same = false;
		got += (uint64_t)r;
	}
	check(same && got == n, what);
}

int main(int argc, char **argv)
{
	if (argc < 2) {
		fprintf(stderr, "usage: tsan_gz FILE.gz [threads] [chunk_bytes] [world]\n");
		return 2;
	}
	const char *path = argv[1];
	const int threads = argc > 2 ? atoi(argv[2]) : 4;
	const uint64_t chunk = argc > 3 ? strtoull(argv[3], nullptr, 10) : (16u << 10);
	const int world = argc > 4 ? atoi(argv[4]) : 3;
	const std::vector<uint8_t> ref = zlib_text(path);
	FILE *f = fopen(path, "rb");
	if (!f) return 2;
	fseek(f, 0, SEEK_END);
	const uint64_t size = (uint64_t)ftell(f);
	fclose(f);

	// 1. the whole stream
	{
		VcGzParallel *g = vc_gzp_open(path, threads, chunk);
		check(g != nullptr, "open");
		if (g) {
			read_compare(g, ref, 0, ref.size(), "whole stream");
			vc_gzp_close(g);
		}
	}

	// 2./3. shares: scan (plain or held), chain the windows, stream each share
	for (int mode = 0; mode < 3; ++mode) {   // 0 two pass, 1 held, 2 held with a budget that runs out
		std::vector<VcGzShare> sh(world);
		std::vector<std::vector<uint16_t>> sym(world, std::vector<uint16_t>(32768));
		std::vector<VcGzParallel *> held(world, nullptr);
		for (int r = 0; r < world; ++r) {
			const uint64_t b = size * (uint64_t)r / (uint64_t)world, e = size * (uint64_t)(r + 1) / (uint64_t)world;
			if (e <= b) continue;
			bool ok;
			if (mode == 0) ok = vc_gzp_scan_share(path, threads, chunk, b, e, &sh[r], sym[r].data());
			else ok = vc_gzp_scan_share_hold(path, threads, chunk, b, e, mode == 1 ? (1ull << 32) : (4ull << 20),
			                                 &sh[r], sym[r].data(), &held[r]);
			check(ok, "scan");
		}
		// chain: start of r == end of the previous non-empty share; windows
		std::vector<std::vector<uint8_t>> win(world, std::vector<uint8_t>(32768, 0));
		std::vector<uint8_t> before(32768, 0);
		uint64_t text_at = 0, prev_end = UINT64_MAX;
		bool chained = true;
		std::vector<uint64_t> text_off(world, 0);
		for (int r = 0; r < world; ++r) {
			if (sh[r].start_bit == UINT64_MAX) continue;
			if (!sh[r].ok || (prev_end != UINT64_MAX && sh[r].start_bit != prev_end)) chained = false;
			win[r] = before;
			text_off[r] = text_at;
			for (int i = 0; i < 32768; ++i) {
				const uint16_t v = sym[r][i];
				sym[r][i] = v < 256 ? v : before[v & 32767];
			}
			for (int i = 0; i < 32768; ++i) before[i] = (uint8_t)sym[r][i];
			text_at += sh[r].text_len;
			prev_end = sh[r].end_bit;
		}
		if (chained) check(text_at == ref.size(), "share lengths add up");
		for (int r = 0; r < world; ++r) {
			if (sh[r].start_bit == UINT64_MAX || !chained) {
				if (held[r]) vc_gzp_close(held[r]);
				continue;
			}
			const uint64_t more = sh[r].end_bit == UINT64_MAX ? 0 : 4096;   // read on into the next share
			const uint64_t n = std::min<uint64_t>(sh[r].text_len + more, ref.size() - text_off[r]);
			VcGzParallel *g = held[r];
			if (g) {
				check(vc_gzp_resume_share(g, r == 0 ? nullptr : win[r].data(), sh[r].text_len), "resume");
			} else {
				check(mode != 1, "held share kept");
				g = vc_gzp_open_share(path, threads, chunk, r == 0, sh[r].start_bit, win[r].data(), sh[r].text_len);
			}
			if (!g) {
				check(false, "open share");
				continue;
			}
			read_compare(g, ref, text_off[r], n, mode == 0 ? "two-pass share" : "held share");
			VcGzShareCrc crc;
			vc_gzp_share_crc(g, &crc);
			check(crc.crc_error == 0, "share crc");
			vc_gzp_close(g);
		}
	}
	printf("%s: %zu bytes of text, %d threads, chunk %llu, %d shares: %s\n", path, ref.size(), threads,
	       (unsigned long long)chunk, world, fails ? "FAILED" : "ok");
	return fails ? 1 : 0;
}
