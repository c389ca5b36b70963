// vafc_host.cpp -- host side of libvafc.so: the C ABI of include/vafc.h.
//
//   patterns      load_patterns / create_combined_kmer_map   vaf-counter.c:149-252
//   device ctx    static key table + LDS prefilter in HBM, counts, streams
//   count_block   host block -> pinned staging -> H2D -> kernels (async)
//   count_file    count_fastq_kmers: block loop + kseq reader  vaf-counter.c:482-582
//   shards        one table replica + counts per GPU, host batches dealt
//                 round robin, one RCCL reduce before the writer  
//   write_vaf     .vaf writer                                  vaf-counter.c:653-681
//
// Nothing here computes counts on the CPU: every k-mer goes through the HIP
// kernels in vafc_kernels.hip, and any HIP failure is returned as VC_EHIP.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <ctype.h>
#include <dlfcn.h>
#include <sched.h>
#include <fcntl.h>
#include <limits.h>
#include <math.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <unordered_map>
#include <vector>

#include "vafc.h"
#include "vafc_affinity.h"
#include "vafc_common.h"
#include "vafc_fastq.h"
#include "vafc_gzip.h"
#include "vafc_ingest.h"
#include "vafc_internal.h"
#include "vafc_kc.h"

#define HIPCK(call)                                                                         \
	do {                                                                                    \
		hipError_t e_ = (call);                                                             \
		if (e_ != hipSuccess) {                                                             \
			fprintf(stderr, "[E::vafc] %s failed: %s (%s:%d)\n", #call, hipGetErrorString(e_), \
			        __FILE__, __LINE__);                                                    \
			return VC_EHIP;                                                                 \
		}                                                                                   \
	} while (0)

// ---------------------------------------------------------------------------
// patterns
// ---------------------------------------------------------------------------

namespace {

struct Pattern {
	char chr[256];
	int start, end;
	char rsid[256];
	char ref, alt;
	char ref_kmer[128];
	char alt_kmer[128];
};

unsigned char g_nt4[256];
bool g_nt4_init = false;

void init_nt4()
{
	if (g_nt4_init) return;
	for (int i = 0; i < 256; ++i) g_nt4[i] = 4;
	for (int i = 0; i < 4; ++i) g_nt4[i] = (unsigned char)i;
	const char *acgt[4] = {"Aa", "Cc", "Gg", "TtUu"};
	for (int c = 0; c < 4; ++c)
		for (const char *p = acgt[c]; *p; ++p) g_nt4[(unsigned char)*p] = (unsigned char)c;
	g_nt4_init = true;
}

// 2-bit key of the first k characters (vaf-counter.c:117-127); UINT64_MAX if
// any of them is not A/C/G/T/U (either case) or a raw byte 0..3.
uint64_t string_key(const char *s, int k)
{
	uint64_t x = 0;
	for (int i = 0; i < k; ++i) {
		unsigned c = g_nt4[(unsigned char)s[i]];
		if (c > 3) return UINT64_MAX;
		x = (x << 2) | c;
	}
	return x;
}

uint64_t canonical(uint64_t x, int k)
{
	uint64_t r = 0, y = x;
	for (int i = 0; i < k; ++i, y >>= 2) r = (r << 2) | (3u - (y & 3u));
	return r < x ? r : x;
}

} // namespace

struct vc_patterns {
	std::vector<Pattern> a;
};

extern "C" int vc_patterns_load(const char *path, vc_patterns **out)
{
	if (!path || !out) return VC_EINVAL;
	*out = nullptr;
	FILE *fp = fopen(path, "r");
	if (!fp) return VC_EIO;
	vc_patterns *db = new (std::nothrow) vc_patterns;
	if (!db) {
		fclose(fp);
		return VC_ENOMEM;
	}
	// One record buffer reused across records, like the reference's local
	// pattern_t: a k-mer string shorter than k is followed by its NUL and by
	// bytes of earlier longer strings (the reference's buffer starts as
	// uninitialised stack; this one starts zeroed).
	Pattern rec;
	memset(&rec, 0, sizeof(rec));
	while (fscanf(fp, "%255s%d%d%255s %c %c%127s%127s", rec.chr, &rec.start, &rec.end, rec.rsid,
	              &rec.ref, &rec.alt, rec.ref_kmer, rec.alt_kmer) == 8)
		db->a.push_back(rec);
	fclose(fp);
	*out = db;
	return VC_OK;
}

extern "C" void vc_patterns_free(vc_patterns *db) { delete db; }

extern "C" int vc_patterns_count(const vc_patterns *db) { return db ? (int)db->a.size() : 0; }

extern "C" int vc_pattern_fields(const vc_patterns *db, int i, const char **chr, int *start,
                                 const char **rsid, char *ref, char *alt, const char **ref_kmer,
                                 const char **alt_kmer)
{
	if (!db || i < 0 || (size_t)i >= db->a.size()) return VC_EINVAL;
	const Pattern &p = db->a[(size_t)i];
	if (chr) *chr = p.chr;
	if (start) *start = p.start;
	if (rsid) *rsid = p.rsid;
	if (ref) *ref = p.ref;
	if (alt) *alt = p.alt;
	if (ref_kmer) *ref_kmer = p.ref_kmer;
	if (alt_kmer) *alt_kmer = p.alt_kmer;
	return VC_OK;
}

extern "C" void vc_free(void *p) { free(p); }

extern "C" int vc_patterns_keys(const vc_patterns *db, int k, uint64_t **keys, uint32_t **vals,
                                size_t *n_keys, int *n_collisions)
{
	if (!db || !keys || !vals || !n_keys || k < 1 || k > 31) return VC_EINVAL;
	const size_t n = db->a.size();
	if (n > (size_t)(INT32_MAX >> 1)) return VC_ETOOMANY;   // vaf-counter.c:205-209
	init_nt4();
	uint64_t *K = (uint64_t *)malloc((2 * n + 1) * sizeof(uint64_t));
	uint32_t *V = (uint32_t *)malloc((2 * n + 1) * sizeof(uint32_t));
	if (!K || !V) {
		free(K);
		free(V);
		return VC_ENOMEM;
	}
	std::unordered_map<uint64_t, uint32_t> seen;
	seen.reserve(2 * n + 1);
	size_t m = 0;
	int coll = 0;
	for (size_t i = 0; i < n; ++i) {
		for (int allele = 0; allele < 2; ++allele) {
			const char *s = allele ? db->a[i].alt_kmer : db->a[i].ref_kmer;
			uint64_t x = string_key(s, k);
			if (x == UINT64_MAX) continue;
			uint64_t c = canonical(x, k);
			uint32_t v = ((uint32_t)i << 1) | (uint32_t)allele;
			if (seen.emplace(c, v).second) {
				K[m] = c;
				V[m] = v;
				++m;
			} else {
				++coll;                     // first insert wins (khashl.h:218)
			}
		}
	}
	*keys = K;
	*vals = V;
	*n_keys = m;
	if (n_collisions) *n_collisions = coll;
	return VC_OK;
}

extern "C" int vc_write_vaf(const vc_patterns *db, const uint32_t *counts, const char *path)
{
	if (!db || !path) return VC_EINVAL;
	const size_t n = db->a.size();
	uint64_t tot_ref = 0, tot_alt = 0;
	for (size_t i = 0; i < n; ++i) {
		tot_ref += counts ? counts[2 * i] : 0;
		tot_alt += counts ? counts[2 * i + 1] : 0;
	}
	const double avg = (double)(tot_ref + tot_alt) / (n > 0 ? (double)n : 1.0);
	FILE *fp = fopen(path, "w");
	if (!fp) return VC_EIO;
	setvbuf(fp, nullptr, _IOFBF, 1 << 20);
	fprintf(fp, "# Average depth: %.2f\n", avg);
	fprintf(fp, "CHR\tPOS\tRSID\tREF\tALT\tREF_COUNT\tALT_COUNT\tTOTAL_COUNT\tVAF\n");
	for (size_t i = 0; i < n; ++i) {
		const Pattern &p = db->a[i];
		const uint32_t rc = counts ? counts[2 * i] : 0, ac = counts ? counts[2 * i + 1] : 0;
		const uint32_t tot = rc + ac;                       // u32 wrap, as the reference
		const double vaf = tot > 0 ? (double)ac / tot : 0.0;
		fprintf(fp, "%s\t%d\t%s\t%c\t%c\t%u\t%u\t%u\t%.4f\n", p.chr, p.start, p.rsid, p.ref, p.alt, rc,
		        ac, tot, vaf);
	}
	return fclose(fp) == 0 ? VC_OK : VC_EIO;
}

// ---------------------------------------------------------------------------
// device context
// ---------------------------------------------------------------------------

namespace {

struct Slot {
	uint8_t *h_seq = nullptr;     // pinned
	uint64_t *h_offs = nullptr;
	uint32_t *h_lens = nullptr;
	uint8_t *d_seq = nullptr;
	uint64_t *d_offs = nullptr;
	uint32_t *d_lens = nullptr;
	size_t cap_bytes = 0, cap_reads = 0;
	hipEvent_t done = nullptr;
	hipEvent_t copied = nullptr;  // parallel reader: the slot's H2D copies (copy stream) are done
	bool pending = false;
	void *map = nullptr;          // one registered mapping holds h_seq, h_offs, h_lens (slot_alloc_mapped)
	size_t map_len = 0;
	bool d_one = false;           // d_offs, d_lens point into d_seq's allocation
};

} // namespace

struct vc_ctx {
	int dev = 0, k = 21;
	uint32_t n_patterns = 0;
	uint64_t n_keys = 0;
	hipStream_t st = nullptr;
	int n_cu = 256;
	vc_slot_t *d_table = nullptr;
	int ablate = 0;                   // kernel ablation variant (libvafc_abl.so only)
	uint32_t variant = 0;             // kernel A/B experiment knobs ($VAFC_VARIANT, tools/ab.py)
	int nt4 = 0;                      // seq_nt4 decode everywhere (vc_set_nt4_decode)
	uint32_t tbits = 0;
	uint32_t *d_filter = nullptr;
	uint32_t wbits = 0;
	uint32_t *d_l2f = nullptr;             // second-level filter (large key sets only)
	uint32_t l2bits = 0;
	uint32_t fsh = 0;
	uint32_t flank = 0;                    // the filter is the flank bitmap (vafc_common.h)
	uint32_t big = 0;                      // the filter is the large-panel Bloom filter (vc_big_word)
	uint32_t fwords = 0;                   // LDS filter words
	uint32_t qcap = VC_QCAP;               // LDS queue entries per wave
	uint32_t *d_counts = nullptr;          // active outputs (own or bound)
	unsigned long long *d_tally = nullptr;
	uint32_t *own_counts = nullptr;
	unsigned long long *own_tally = nullptr;
	uint32_t *d_nlong = nullptr;
	uint32_t *d_flags = nullptr;           // kernel error flags (VcKernelArgs::flags)
	uint8_t *d_pad = nullptr;              // 64 B staging for inputs under 16 B (kernels load 16 B)
	uint32_t *d_long = nullptr;
	uint32_t long_cap = 0;
	Slot slot[2];
	int cur = 0;
	std::vector<Slot> islot;               // parallel ingest (vc_count_file on plain files)
	hipStream_t cst = nullptr;             // the parallel reader's H2D copies (created on first use)
	bool ingest_warm = false;              // a parallel-reader pass has completed: its slots are pinned
	bool timing = false, timed = false;
	hipEvent_t t0 = nullptr, t1 = nullptr;
	// vc_count_device on a stream other than st: st's work so far -> that
	// stream (ev_in), and the launch -> st (ev_out), so that vc_reset, vc_finish
	// and the shard sum, all on st, stay ordered with it (created on first use)
	hipEvent_t ev_in = nullptr, ev_out = nullptr;
	VcCpuSet cpus;                    // the GPUs' NUMA-node CPUs for the reader threads (gpu_cpus)
	int cpus_threads = -1;            // the thread count cpus was computed for
	struct Kc *kc = nullptr;               // histogram mode (vc_kc_create)
	// multi-GPU (vc_create_multi): this ctx is shard 0; rep[i - 1] is shard i
	std::vector<vc_ctx *> rep;
	std::vector<int> lead;                 // per shard: the first shard on the same device
	std::vector<ncclComm_t> comms;         // one rank per distinct device, rank 0 = shard 0
	std::vector<int> comm_shard;           // the shard each rank reduces
	uint64_t rr = 0;                       // host batches dealt so far (round robin)
	uint64_t batches = 0;                  // batches counted by this shard (vc_shard_info)
};

static inline int n_shards(const vc_ctx *c) { return 1 + (int)c->rep.size(); }
static inline vc_ctx *shard_at(vc_ctx *c, int i) { return i == 0 ? c : c->rep[(size_t)i - 1]; }
// The shard that takes the next host batch.
static inline vc_ctx *next_shard(vc_ctx *c) { return shard_at(c, (int)(c->rr++ % (uint64_t)n_shards(c))); }

// kc-c4 histogram mode: the device hash table and its bookkeeping
struct Kc {
	unsigned long long *d_table = nullptr;   // 2 * slots
	uint64_t slots = 0;
	uint32_t tbits = 0;
	uint32_t n_parts = 1, part = 0;
	unsigned long long *d_stats = nullptr;   // k-mers, distinct, overflow
	unsigned long long *d_hist = nullptr;    // up to 1024 bins + the slots counted
	uint32_t *d_nlong = nullptr, *d_long = nullptr;
	uint64_t *d_segstart = nullptr;
	uint32_t long_cap = 0;
	uint64_t *d_first = nullptr;             // first-occurrence stamps (vc_kc_track_first)
	bool track_first = false, lookup_only = false;
	uint64_t read_base = 0;                  // reads launched since the last reset
};

static int ensure_long_cap(vc_ctx *c, uint64_t seq_bytes)
{
	uint64_t need = seq_bytes / (VC_LONG_READ + 1) + 1;
	if (need <= c->long_cap) return VC_OK;
	if (need > 0xFFFFFFFFull) need = 0xFFFFFFFFull;
	HIPCK(hipStreamSynchronize(c->st));
	if (c->d_long) HIPCK(hipFree(c->d_long));
	c->d_long = nullptr;
	HIPCK(hipMalloc(&c->d_long, need * sizeof(uint32_t)));
	c->long_cap = (uint32_t)need;
	return VC_OK;
}

extern "C" int vc_create(vc_ctx **out, int k, const uint64_t *keys, const uint32_t *vals,
                         size_t n_keys, uint32_t n_patterns, int device)
{
	if (!out || k < 1 || k > 31 || (n_keys && (!keys || !vals))) return VC_EINVAL;
	*out = nullptr;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VC_ENODEV;
	if (device < 0 || device >= ndev) return VC_EINVAL;
	HIPCK(hipSetDevice(device));
	HIPCK(vc_kernel_setup());

	vc_ctx *c = new (std::nothrow) vc_ctx;
	if (!c) return VC_ENOMEM;
	c->dev = device;
	c->k = k;
	c->n_patterns = n_patterns;
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
		c->n_cu = prop.multiProcessorCount;

	// exact table: 16-byte {key, value} slots, linear probing, load <= 1/2
	uint32_t tbits = 4;
	while (((uint64_t)1 << tbits) < 2 * (uint64_t)n_keys + 2) ++tbits;
	const uint64_t tslots = (uint64_t)1 << tbits;
	std::vector<vc_slot_t> tab(tslots, vc_slot_t{VC_EMPTY_KEY, 0u, 0u});
	// LDS prefilter: >= 24 bits per key, 1 KiB .. 128 KiB, 2 bits per key
	uint32_t wbits = 8;
	while (wbits < VC_MAX_FILTER_WBITS && ((uint64_t)32 << wbits) < 24 * (uint64_t)n_keys) ++wbits;
	const uint32_t fsh = vc_filter_shift(k, wbits);
	std::vector<uint32_t> fw((size_t)1 << wbits, 0);
	// second level: >= 40 bits per key, up to 2 MiB, when the LDS filter saturates
	uint32_t l2bits = 0;
	if (n_keys > VC_L2F_MIN_KEYS) {
		uint64_t bpk = 40;                                   // filter bits per key
		if (const char *e = getenv("VAFC_L2F_BITS_PER_KEY")) bpk = strtoull(e, nullptr, 10);   // A/B knob
		l2bits = 12;
		while (l2bits < VC_L2F_MAX_BITS && ((uint64_t)32 << l2bits) < bpk * (uint64_t)n_keys) ++l2bits;
	}
	std::vector<uint32_t> l2w(l2bits ? (size_t)1 << l2bits : 0, 0);
	uint64_t inserted = 0;
	for (size_t i = 0; i < n_keys; ++i) {
		const uint64_t key = keys[i];
		if (key == VC_EMPTY_KEY) continue;
		const uint32_t h = vc_hash(key);
		uint32_t s = vc_table_slot(h, tbits);
		bool dup = false;
		while (tab[s].key != VC_EMPTY_KEY) {
			if (tab[s].key == key) { dup = true; break; }
			s = (s + 1) & (uint32_t)(tslots - 1);
		}
		if (dup) continue;             // first occurrence wins
		tab[s].key = key;
		tab[s].val = vals[i];
		const uint32_t flo = (uint32_t)key, rlo = (uint32_t)vc_revcomp(key, k);
		fw[vc_filter_word(flo, rlo, fsh, wbits)] |= vc_filter_mask(flo, rlo);
		if (l2bits) l2w[vc_hash(key) >> (32 - l2bits)] |= vc_l2f_mask(vc_hash2(key));
		++inserted;
	}
	// flank bitmap instead of the Bloom filter (vafc_common.h) for k >= 21 and
	// no second level, when a random window's pass rate (about the fourth
	// power of the bitmap's density) stays under 1 %; VAFC_FILTER=bloom|flank forces
	// one (A/B and tests; flank only where k allows it)
	{
		const char *fe = getenv("VAFC_FILTER");
		const bool force_bloom = fe && !strcmp(fe, "bloom"), force_flank = fe && !strcmp(fe, "flank");
		// large panels, k >= 21: the 144 KiB Bloom filter (vafc_common.h
		// vc_big_word; the queues shrink to VC_BIG_QCAP); VAFC_FILTER=bloom128
		// keeps the 128 KiB power-of-two filter (A/B and tests)
		const bool force_b128 = fe && !strcmp(fe, "bloom128");
		if (k >= VC_FLANK_MIN_K && l2bits && !force_b128) {
			std::vector<uint32_t> fbig(VC_BIG_FILTER_WORDS, 0);
			for (const vc_slot_t &e : tab)
				if (e.key != VC_EMPTY_KEY) {
					const uint32_t flo = (uint32_t)e.key, rlo = (uint32_t)vc_revcomp(e.key, k);
					fbig[vc_big_word(flo, rlo, VC_BIG_FILTER_WORDS)] |= vc_filter_mask(flo, rlo);
				}
			fw.swap(fbig);
			c->big = 1;
			c->qcap = VC_BIG_QCAP;
#ifndef VC_BIG_RAWQ
			// the big kernels queue both strands' low words: key the second
			// level by them (vc_l2s_*) instead of the canonical k-mer
			std::fill(l2w.begin(), l2w.end(), 0u);
			for (const vc_slot_t &e : tab)
				if (e.key != VC_EMPTY_KEY) {
					const uint32_t flo = (uint32_t)e.key, rlo = (uint32_t)vc_revcomp(e.key, k);
					l2w[vc_l2s_hash(flo, rlo) >> (32 - l2bits)] |= vc_l2f_mask(vc_l2s_hash2(flo, rlo));
				}
#endif
		}
		if (k >= VC_FLANK_MIN_K && !l2bits && !force_bloom) {
			std::vector<uint32_t> fb((size_t)1 << VC_FLANK_WBITS, 0);
			for (const vc_slot_t &e : tab)
				if (e.key != VC_EMPTY_KEY) {
					vc_flank_mark(fb.data(), e.key, k);
					vc_flank_mark(fb.data(), vc_revcomp(e.key, k), k);
				}
			uint64_t set = 0;
			for (uint32_t w : fb) set += (uint64_t)__builtin_popcount(w);
			const double dens = (double)set / (double)((uint64_t)1 << (2 * VC_FLANK_BASES));
			if (force_flank || dens * dens * dens * dens <= 0.01) {
				fw.swap(fb);
				wbits = VC_FLANK_WBITS;
				c->flank = 1;
			}
		}
	}
	c->n_keys = inserted;
	c->tbits = tbits;
	c->wbits = wbits;
	c->fwords = (uint32_t)fw.size();
	c->l2bits = l2bits;
	c->fsh = fsh;
	c->ablate = getenv("VAFC_ABLATE") ? atoi(getenv("VAFC_ABLATE")) : 0;
	c->variant = getenv("VAFC_VARIANT") ? (uint32_t)atoi(getenv("VAFC_VARIANT")) : 0u;

	int rc = VC_OK;
#define TRY(call)                                                                        \
	do {                                                                                 \
		hipError_t e_ = (call);                                                          \
		if (e_ != hipSuccess) {                                                          \
			fprintf(stderr, "[E::vafc] %s failed: %s\n", #call, hipGetErrorString(e_)); \
			rc = VC_EHIP;                                                                \
			goto fail;                                                                   \
		}                                                                                \
	} while (0)
	TRY(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
	TRY(hipMalloc(&c->d_table, tslots * sizeof(vc_slot_t)));
	TRY(hipMalloc(&c->d_filter, fw.size() * sizeof(uint32_t)));
	TRY(hipMalloc(&c->own_counts, (2 * (size_t)n_patterns + 2) * sizeof(uint32_t)));
	TRY(hipMalloc(&c->own_tally, sizeof(unsigned long long)));
	c->d_counts = c->own_counts;
	c->d_tally = c->own_tally;
	TRY(hipMalloc(&c->d_nlong, sizeof(uint32_t)));
	TRY(hipMalloc(&c->d_flags, sizeof(uint32_t)));
	TRY(hipMemset(c->d_flags, 0, sizeof(uint32_t)));
	TRY(hipMalloc(&c->d_pad, 64));
	TRY(hipMemset(c->d_pad, 0, 64));
	TRY(hipMemcpy(c->d_table, tab.data(), tslots * sizeof(vc_slot_t), hipMemcpyHostToDevice));
	TRY(hipMemcpy(c->d_filter, fw.data(), fw.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
	if (l2bits) {
		TRY(hipMalloc(&c->d_l2f, l2w.size() * sizeof(uint32_t)));
		TRY(hipMemcpy(c->d_l2f, l2w.data(), l2w.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
	}
	TRY(hipMemset(c->d_counts, 0, (2 * (size_t)n_patterns + 2) * sizeof(uint32_t)));
	TRY(hipMemset(c->d_tally, 0, sizeof(unsigned long long)));
	TRY(hipEventCreate(&c->t0));
	TRY(hipEventCreate(&c->t1));
	for (auto &s : c->slot) TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
	if ((rc = ensure_long_cap(c, (uint64_t)1 << 30)) != VC_OK) goto fail;
#undef TRY
	*out = c;
	return VC_OK;
fail:
	vc_destroy(c);
	return rc;
}

static void free_slot(Slot &s)
{
	if (s.map) {
		(void)hipHostUnregister(s.map);
		munmap(s.map, s.map_len);
	} else {
		if (s.h_seq) (void)hipHostFree(s.h_seq);
		if (s.h_offs) (void)hipHostFree(s.h_offs);
		if (s.h_lens) (void)hipHostFree(s.h_lens);
	}
	if (s.d_seq) (void)hipFree(s.d_seq);
	if (!s.d_one) {
		if (s.d_offs) (void)hipFree(s.d_offs);
		if (s.d_lens) (void)hipFree(s.d_lens);
	}
	s.map = nullptr;
	s.map_len = 0;
	s.d_one = false;
	s.h_seq = nullptr;
	s.h_offs = nullptr;
	s.h_lens = nullptr;
	s.d_seq = nullptr;
	s.d_offs = nullptr;
	s.d_lens = nullptr;
	s.cap_bytes = s.cap_reads = 0;
	s.pending = false;
}

static void rccl_comms_destroy(vc_ctx *c);

extern "C" void vc_destroy(vc_ctx *c)
{
	if (!c) return;
	rccl_comms_destroy(c);
	for (vc_ctx *r : c->rep) vc_destroy(r);
	c->rep.clear();
	(void)hipSetDevice(c->dev);
	if (c->st) (void)hipStreamSynchronize(c->st);
	for (auto &s : c->slot) {
		free_slot(s);
		if (s.done) (void)hipEventDestroy(s.done);
	}
	for (auto &s : c->islot) {
		free_slot(s);
		if (s.done) (void)hipEventDestroy(s.done);
		if (s.copied) (void)hipEventDestroy(s.copied);
	}
	if (c->cst) (void)hipStreamDestroy(c->cst);
	if (c->t0) (void)hipEventDestroy(c->t0);
	if (c->t1) (void)hipEventDestroy(c->t1);
	if (c->ev_in) (void)hipEventDestroy(c->ev_in);
	if (c->ev_out) (void)hipEventDestroy(c->ev_out);
	if (c->d_table) (void)hipFree(c->d_table);
	if (c->d_filter) (void)hipFree(c->d_filter);
	if (c->d_l2f) (void)hipFree(c->d_l2f);
	if (c->own_counts) (void)hipFree(c->own_counts);
	if (c->own_tally) (void)hipFree(c->own_tally);
	if (c->d_nlong) (void)hipFree(c->d_nlong);
	if (c->d_flags) (void)hipFree(c->d_flags);
	if (c->d_pad) (void)hipFree(c->d_pad);
	if (c->d_long) (void)hipFree(c->d_long);
	if (c->kc) {
		Kc &K = *c->kc;
		for (void *q : {(void *)K.d_table, (void *)K.d_stats, (void *)K.d_hist, (void *)K.d_nlong, (void *)K.d_long,
		                (void *)K.d_segstart, (void *)K.d_first})
			if (q) (void)hipFree(q);
		delete c->kc;
	}
	if (c->st) (void)hipStreamDestroy(c->st);
	delete c;
}

// Enqueue the two counting kernels over device-resident reads on stream st.
static int kc_launch(vc_ctx *c, const uint8_t *d_seq, size_t seq_bytes, const uint64_t *d_offs,
                     const uint32_t *d_lens, uint64_t n_reads, hipStream_t st)
{
	Kc &K = *c->kc;
	const uint64_t need = seq_bytes / (KC_LONG + 1) + 1;
	if (need > K.long_cap) {
		HIPCK(hipStreamSynchronize(st));
		if (K.d_long) HIPCK(hipFree(K.d_long));
		if (K.d_segstart) HIPCK(hipFree(K.d_segstart));
		K.d_long = nullptr;
		K.d_segstart = nullptr;
		const uint64_t cap = need < 0xFFFFFFF0ull ? need : 0xFFFFFFF0ull;
		HIPCK(hipMalloc(&K.d_long, cap * sizeof(uint32_t)));
		HIPCK(hipMalloc(&K.d_segstart, (cap + 1) * sizeof(uint64_t)));
		K.long_cap = (uint32_t)cap;
	}
	KcArgs A;
	A.seq = d_seq;
	A.offs = d_offs;
	A.lens = d_lens;
	A.n_reads = n_reads;
	A.table = K.d_table;
	A.tmask = K.slots - 1;
	A.tbits = K.tbits;
	A.n_parts = K.n_parts;
	A.part = K.part;
	A.first = K.track_first && !K.lookup_only ? K.d_first : nullptr;
	A.read_base = K.read_base;
	A.lookup_only = K.lookup_only ? 1 : 0;
	K.read_base += n_reads;
	A.k = c->k;
	A.kmask = ((uint64_t)1 << (2 * c->k)) - 1;
	A.stats = K.d_stats;
	A.nlong = K.d_nlong;
	A.longlist = K.d_long;
	A.long_cap = K.long_cap;
	A.segstart = K.d_segstart;
	const uint64_t blocks = (n_reads + KC_THREADS - 1) / KC_THREADS;
	const uint64_t maxg = (uint64_t)c->n_cu * 16;
	const int grid = (int)(blocks < maxg ? blocks : maxg);
	if (c->timing) HIPCK(hipEventRecord(c->t0, st));
	HIPCK(vc_launch_kc(&A, grid, st));
	if (c->timing) {
		HIPCK(hipEventRecord(c->t1, st));
		c->timed = true;
	}
	return VC_OK;
}

// Whether any of n host-side read lengths takes the long-read kernel.
static bool any_long(const uint32_t *lens, uint64_t n)
{
	uint32_t m = 0;
	for (uint64_t i = 0; i < n; ++i) m = lens[i] > m ? lens[i] : m;
	return m > VC_LONG_READ;
}

// may_long = false: the caller knows no read is longer than VC_LONG_READ (a
// host batch), so the long-read kernel and its list reset are not launched.
static int launch(vc_ctx *c, const uint8_t *d_seq, size_t seq_bytes, const uint64_t *d_offs,
                  const uint32_t *d_lens, uint64_t n_reads, hipStream_t st, bool may_long = true)
{
	if (n_reads == 0) return VC_OK;
	if (c->kc) return kc_launch(c, d_seq, seq_bytes, d_offs, d_lens, n_reads, st);
	if (n_reads > 0xFFFFFFFFull) return VC_EINVAL;   // the long-read list holds u32 read indices
	int rc = ensure_long_cap(c, seq_bytes);
	if (rc != VC_OK) return rc;
	VcKernelArgs A;
	const uintptr_t p = (uintptr_t)d_seq;
	A.seq = (const uint8_t *)(p & ~(uintptr_t)3);
	A.off_adj = (uint64_t)(p & 3u);
	A.seq_words = (seq_bytes + A.off_adj + 3) / 4;
	const bool tiny = A.seq_words < 4;     // the scan loads whole 16-byte quads
	if (tiny) {
		HIPCK(hipMemcpyAsync(c->d_pad, d_seq, seq_bytes, hipMemcpyDeviceToDevice, st));
		A.seq = c->d_pad;
		A.off_adj = 0;
		A.seq_words = 16;
	}
	A.offs = d_offs;
	A.lens = d_lens;
	A.n_reads = n_reads;
	A.table = c->d_table;
	A.tbits = c->tbits;
	A.tmask = (uint32_t)(((uint64_t)1 << c->tbits) - 1);
	A.filter = c->d_filter;
	A.wbits = c->wbits;
	A.fsh = c->fsh;
	A.flank = c->flank;
	A.big = c->big;
	A.fwords = c->fwords;
	A.qcap = c->qcap;
	A.l2f = c->d_l2f;
	A.l2bits = c->l2bits;
	A.ablate = c->ablate;
	A.variant = c->variant;
	A.nt4 = (uint32_t)c->nt4;
	A.k = c->k;
	A.kmask = ((uint64_t)1 << (2 * c->k)) - 1;
	A.counts = c->d_counts;
	A.tally = c->d_tally;
	A.nlong = c->d_nlong;
	A.longlist = c->d_long;
	A.long_cap = c->long_cap;
	A.flags = c->d_flags;
	uint64_t groups = (n_reads + VC_BLOCK - 1) / VC_BLOCK;
	int grid = (int)(groups < (uint64_t)c->n_cu ? groups : (uint64_t)c->n_cu);
	if (may_long) HIPCK(hipMemsetAsync(c->d_nlong, 0, sizeof(uint32_t), st));
	if (c->timing) HIPCK(hipEventRecord(c->t0, st));
	HIPCK(vc_launch_count(&A, grid, may_long ? c->n_cu : 0, st));
	if (tiny) HIPCK(hipStreamSynchronize(st));   // d_pad is reused by the next tiny call
	if (c->timing) {
		HIPCK(hipEventRecord(c->t1, st));
		c->timed = true;
	}
	return VC_OK;
}

extern "C" int vc_set_nt4_decode(vc_ctx *c, int on)
{
	if (!c) return VC_EINVAL;
	c->nt4 = on ? 1 : 0;
	for (vc_ctx *r : c->rep) r->nt4 = c->nt4;
	return VC_OK;
}

extern "C" int vc_count_device(vc_ctx *c, const uint8_t *d_seq, size_t seq_bytes,
                               const uint64_t *d_offs, const uint32_t *d_lens, uint64_t n_reads,
                               void *stream)
{
	if (!c || (n_reads && (!d_seq || !d_offs || !d_lens))) return VC_EINVAL;
	if (!c->rep.empty() && n_reads) {
		// a multi-shard counter deals device batches round robin, like host
		// batches, over the shards that live on the device holding the reads
		int d = c->dev;
		hipPointerAttribute_t at;
		if (hipPointerGetAttributes(&at, d_seq) == hipSuccess && at.type == hipMemoryTypeDevice) d = at.device;
		(void)hipGetLastError();   // a host pointer is not an error here
		vc_ctx *sh = nullptr;
		for (int i = 0; i < n_shards(c) && !sh; ++i) {
			vc_ctx *x = next_shard(c);
			if (x->dev == d) sh = x;
		}
		if (!sh) return VC_EINVAL;
		c = sh;
		++c->batches;
	}
	HIPCK(hipSetDevice(c->dev));
	// NULL is HIP's null stream (ordered with the legacy default stream, which
	// is torch's default stream), as for every HIP API; VC_STREAM_CTX is the
	// counter's own non-blocking stream
	const hipStream_t st = stream == VC_STREAM_CTX ? c->st : (hipStream_t)stream;
	if (st == c->st) return launch(c, d_seq, seq_bytes, d_offs, d_lens, n_reads, st);
	if (!c->ev_in) HIPCK(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
	if (!c->ev_out) HIPCK(hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming));
	HIPCK(hipEventRecord(c->ev_in, c->st));           // e.g. a vc_reset before this call
	HIPCK(hipStreamWaitEvent(st, c->ev_in, 0));
	const int rc = launch(c, d_seq, seq_bytes, d_offs, d_lens, n_reads, st);
	if (rc != VC_OK) return rc;
	HIPCK(hipEventRecord(c->ev_out, st));
	HIPCK(hipStreamWaitEvent(c->st, c->ev_out, 0));   // vc_finish waits on c->st only
	return VC_OK;
}

static int slot_reserve(Slot &s, size_t bytes, size_t reads)
{
	if (bytes <= s.cap_bytes && reads <= s.cap_reads) return VC_OK;
	if (s.pending) HIPCK(hipEventSynchronize(s.done));
	s.pending = false;
	size_t nb = s.cap_bytes > bytes ? s.cap_bytes : bytes + bytes / 4 + 4096;
	size_t nr = s.cap_reads > reads ? s.cap_reads : reads + reads / 4 + 1024;
	free_slot(s);
	HIPCK(hipHostMalloc(&s.h_seq, nb, hipHostMallocDefault));
	HIPCK(hipHostMalloc(&s.h_offs, nr * sizeof(uint64_t), hipHostMallocDefault));
	HIPCK(hipHostMalloc(&s.h_lens, nr * sizeof(uint32_t), hipHostMallocDefault));
	HIPCK(hipMalloc(&s.d_seq, nb));
	HIPCK(hipMalloc(&s.d_offs, nr * sizeof(uint64_t)));
	HIPCK(hipMalloc(&s.d_lens, nr * sizeof(uint32_t)));
	s.cap_bytes = nb;
	s.cap_reads = nr;
	return VC_OK;
}

// Wait until a slot's previous batch has left its pinned buffers.
static int slot_acquire(vc_ctx *c, Slot **out)
{
	Slot &s = c->slot[c->cur];
	if (s.pending) {
		HIPCK(hipEventSynchronize(s.done));
		s.pending = false;
	}
	*out = &s;
	return VC_OK;
}

// H2D copy of a filled slot + kernels; the slot is released by its event.
static int slot_submit(vc_ctx *c, Slot &s, size_t bytes, uint64_t n_reads)
{
	if (n_reads) {
		HIPCK(hipMemcpyAsync(s.d_seq, s.h_seq, bytes, hipMemcpyHostToDevice, c->st));
		HIPCK(hipMemcpyAsync(s.d_offs, s.h_offs, n_reads * sizeof(uint64_t), hipMemcpyHostToDevice, c->st));
		HIPCK(hipMemcpyAsync(s.d_lens, s.h_lens, n_reads * sizeof(uint32_t), hipMemcpyHostToDevice, c->st));
		int rc = launch(c, s.d_seq, bytes, s.d_offs, s.d_lens, n_reads, c->st, any_long(s.h_lens, n_reads));
		if (rc != VC_OK) return rc;
		HIPCK(hipEventRecord(s.done, c->st));
		s.pending = true;
		++c->batches;
	}
	c->cur ^= 1;
	return VC_OK;
}

extern "C" int vc_count_block(vc_ctx *c, const uint8_t *seq, size_t seq_bytes, const uint64_t *offs,
                              const uint32_t *lens, uint64_t n_reads)
{
	if (!c || (n_reads && (!seq || !offs || !lens))) return VC_EINVAL;
	if (n_reads == 0) return VC_OK;
	for (uint64_t i = 0; i < n_reads; ++i)
		if (offs[i] + lens[i] > seq_bytes) return VC_EINVAL;
	c = next_shard(c);
	HIPCK(hipSetDevice(c->dev));
	Slot *s;
	int rc = slot_acquire(c, &s);
	if (rc == VC_OK) rc = slot_reserve(*s, seq_bytes, n_reads);
	if (rc != VC_OK) return rc;
	memcpy(s->h_seq, seq, seq_bytes);
	memcpy(s->h_offs, offs, n_reads * sizeof(uint64_t));
	memcpy(s->h_lens, lens, n_reads * sizeof(uint32_t));
	return slot_submit(c, *s, seq_bytes, n_reads);
}

static int reduce_shards(vc_ctx *c);

extern "C" int vc_finish(vc_ctx *c, uint32_t *counts, uint64_t *kmers)
{
	if (!c) return VC_EINVAL;
	if (!c->kc)
		for (int i = 0; i < n_shards(c); ++i) {   // kernel error flags (a sync point anyway)
			vc_ctx *sh = shard_at(c, i);
			uint32_t f = 0;
			HIPCK(hipSetDevice(sh->dev));
			// the shard's stream also waits for its launches on caller
			// streams (vc_count_device), so this covers every batch without
			// waiting on the caller's unrelated work on the device
			HIPCK(hipStreamSynchronize(sh->st));
			HIPCK(hipMemcpy(&f, sh->d_flags, sizeof f, hipMemcpyDeviceToHost));
			if (f & 1u) {
				fprintf(stderr, "[E::vafc] more reads longer than %d bases than the long-read list holds "
				        "(overlapping device reads?): counts incomplete\n", VC_LONG_READ);
				return VC_EINVAL;
			}
		}
	if (!c->rep.empty()) {
		int rc = reduce_shards(c);
		if (rc != VC_OK) return rc;
	}
	HIPCK(hipSetDevice(c->dev));
	HIPCK(hipStreamSynchronize(c->st));
	for (auto &s : c->slot) s.pending = false;
	if (c->kc) {   // histogram mode: the k-mers seen (vc_kc_histogram gives the rest)
		if (kmers) {
			unsigned long long st[3];
			HIPCK(hipMemcpy(st, c->kc->d_stats, sizeof st, hipMemcpyDeviceToHost));
			*kmers = st[0];
		}
		return VC_OK;
	}
	if (counts)
		HIPCK(hipMemcpy(counts, c->d_counts, 2 * (size_t)c->n_patterns * sizeof(uint32_t),
		                hipMemcpyDeviceToHost));
	if (kmers) {
		unsigned long long t = 0;
		HIPCK(hipMemcpy(&t, c->d_tally, sizeof(t), hipMemcpyDeviceToHost));
		*kmers = t;
	}
	return VC_OK;
}

extern "C" int vc_reset(vc_ctx *c)
{
	if (!c) return VC_EINVAL;
	HIPCK(hipSetDevice(c->dev));
	if (c->kc) {
		Kc &K = *c->kc;
		HIPCK(hipMemsetAsync(K.d_table, 0, K.slots * 16, c->st));
		HIPCK(hipMemsetAsync(K.d_stats, 0, 3 * sizeof(unsigned long long), c->st));
		if (K.track_first) HIPCK(hipMemsetAsync(K.d_first, 0xFF, K.slots * 8, c->st));
		K.read_base = 0;
		K.lookup_only = false;
		return VC_OK;
	}
	HIPCK(hipMemsetAsync(c->d_counts, 0, 2 * (size_t)c->n_patterns * sizeof(uint32_t), c->st));
	HIPCK(hipMemsetAsync(c->d_tally, 0, sizeof(unsigned long long), c->st));
	HIPCK(hipMemsetAsync(c->d_flags, 0, sizeof(uint32_t), c->st));
	for (vc_ctx *r : c->rep) {
		int rc = vc_reset(r);
		if (rc != VC_OK) return rc;
	}
	return VC_OK;
}

extern "C" void *vc_device_counts(vc_ctx *c) { return c ? (void *)c->d_counts : nullptr; }
extern "C" int vc_bind_outputs(vc_ctx *c, void *d_counts, void *d_tally)
{
	if (!c) return VC_EINVAL;
	c->d_counts = d_counts ? (uint32_t *)d_counts : c->own_counts;
	c->d_tally = d_tally ? (unsigned long long *)d_tally : c->own_tally;
	return VC_OK;
}

extern "C" void *vc_device_tally(vc_ctx *c) { return c ? (void *)c->d_tally : nullptr; }
extern "C" void *vc_stream(vc_ctx *c) { return c ? (void *)c->st : nullptr; }

extern "C" int vc_set_timing(vc_ctx *c, int enable)
{
	if (!c) return VC_EINVAL;
	c->timing = enable != 0;
	c->timed = false;
	return VC_OK;
}

extern "C" int vc_kernel_ms(vc_ctx *c, float *ms)
{
	if (!c || !ms) return VC_EINVAL;
	if (!c->timed) return VC_EINVAL;
	HIPCK(hipEventSynchronize(c->t1));
	HIPCK(hipEventElapsedTime(ms, c->t0, c->t1));
	return VC_OK;
}

extern "C" int vc_table_info(const vc_ctx *c, uint64_t *n_keys, uint64_t *slots, uint64_t *filter_bytes)
{
	if (!c) return VC_EINVAL;
	if (n_keys) *n_keys = c->n_keys;
	if (slots) *slots = (uint64_t)1 << c->tbits;
	if (filter_bytes) *filter_bytes = (uint64_t)4 * c->fwords;
	return VC_OK;
}

// ---------------------------------------------------------------------------
// multi-GPU shards.  The reference counts every block of
// every file into one set of u32 counters (vaf-counter.c:473-477, files in
// order :647-650) and writes them once (:653-681).  Here each shard (one per
// entry of the device list) holds a replica of the static table and its own
// counts; host batches are dealt round robin over the shards, the block loop
// and its stop rule still run once, in file order, on the host.  vc_finish
// reduces: shards sharing a device are summed on it (vc_shard_add_kernel),
// then one RCCL reduce (sum) of the per-device vectors to shard 0 over xGMI.
// u32 addition modulo 2^32 commutes, so the result is bit-identical to one
// device counting everything.
// ---------------------------------------------------------------------------

namespace {

// RCCL, loaded on first use so that single-GPU users do not need it.
struct RcclApi {
	bool tried = false, ok = false;
	decltype(&ncclCommInitAll) comm_init_all = nullptr;
	decltype(&ncclCommDestroy) comm_destroy = nullptr;
	decltype(&ncclReduce) reduce = nullptr;
	decltype(&ncclGroupStart) group_start = nullptr;
	decltype(&ncclGroupEnd) group_end = nullptr;
	decltype(&ncclGetErrorString) error_string = nullptr;
};
RcclApi g_rccl;
std::mutex g_rccl_mu;

const RcclApi *rccl()
{
	std::lock_guard<std::mutex> lk(g_rccl_mu);
	if (g_rccl.tried) return g_rccl.ok ? &g_rccl : nullptr;
	g_rccl.tried = true;
	// VAFC_RCCL_LIB names another library (tests point it at a missing file
	// to exercise the RCCL-missing path)
	const char *env = getenv("VAFC_RCCL_LIB");
	void *h = dlopen(env && *env ? env : "librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
	if (!h && !(env && *env)) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
	if (!h) {
		fprintf(stderr, "[E::vafc] cannot load RCCL: %s\n", dlerror());
		return nullptr;
	}
	RcclApi &R = g_rccl;
	R.comm_init_all = (decltype(R.comm_init_all))dlsym(h, "ncclCommInitAll");
	R.comm_destroy = (decltype(R.comm_destroy))dlsym(h, "ncclCommDestroy");
	R.reduce = (decltype(R.reduce))dlsym(h, "ncclReduce");
	R.group_start = (decltype(R.group_start))dlsym(h, "ncclGroupStart");
	R.group_end = (decltype(R.group_end))dlsym(h, "ncclGroupEnd");
	R.error_string = (decltype(R.error_string))dlsym(h, "ncclGetErrorString");
	R.ok = R.comm_init_all && R.comm_destroy && R.reduce && R.group_start && R.group_end && R.error_string;
	if (!R.ok) fprintf(stderr, "[E::vafc] RCCL lacks the symbols vafc needs\n");
	return R.ok ? &R : nullptr;
}

} // namespace

#define NCCK(R, call)                                                                               \
	do {                                                                                            \
		ncclResult_t e_ = (call);                                                                   \
		if (e_ != ncclSuccess) {                                                                    \
			fprintf(stderr, "[E::vafc] %s failed: %s (%s:%d)\n", #call, (R)->error_string(e_),      \
			        __FILE__, __LINE__);                                                            \
			return VC_EHIP;                                                                         \
		}                                                                                           \
	} while (0)

static void rccl_comms_destroy(vc_ctx *c)
{
	if (c->comms.empty()) return;
	const RcclApi *R = rccl();
	if (R)
		for (ncclComm_t m : c->comms) (void)R->comm_destroy(m);
	c->comms.clear();
	c->comm_shard.clear();
}

extern "C" int vc_create_multi(vc_ctx **out, int k, const uint64_t *keys, const uint32_t *vals, size_t n_keys,
                               uint32_t n_patterns, const int *devices, int n_devices)
{
	if (!out || !devices || n_devices < 1 || n_devices > VC_MAX_SHARDS) return VC_EINVAL;
	*out = nullptr;
	// RCCL is needed only to reduce across distinct devices (shards that share
	// a device are summed on it); load it before any device is touched, so a
	// missing library fails fast and leaves nothing to free
	int n_distinct = 0;
	for (int i = 0; i < n_devices; ++i) {
		bool seen = false;
		for (int j = 0; j < i; ++j) seen = seen || devices[j] == devices[i];
		n_distinct += seen ? 0 : 1;
	}
	if (n_distinct > 1 && !rccl()) return VC_EHIP;
	vc_ctx *c = nullptr;
	int rc = vc_create(&c, k, keys, vals, n_keys, n_patterns, devices[0]);
	if (rc != VC_OK) return rc;
	c->lead.assign(1, 0);
	for (int i = 1; i < n_devices; ++i) {
		vc_ctx *r = nullptr;
		if ((rc = vc_create(&r, k, keys, vals, n_keys, n_patterns, devices[i])) != VC_OK) {
			vc_destroy(c);
			return rc;
		}
		c->rep.push_back(r);
		int l = i;
		for (int j = 0; j < i; ++j)
			if (devices[j] == devices[i]) {
				l = j;
				break;
			}
		c->lead.push_back(l);
	}
	if (n_distinct > 1) {
		// one RCCL rank per distinct device; rank 0 is shard 0 (the reduce root)
		const RcclApi *R = rccl();
		std::vector<int> devs;
		for (int i = 0; i < n_devices; ++i)
			if (c->lead[(size_t)i] == i) {
				devs.push_back(devices[i]);
				c->comm_shard.push_back(i);
			}
		c->comms.assign(devs.size(), nullptr);
		const ncclResult_t e = R->comm_init_all(c->comms.data(), (int)devs.size(), devs.data());
		if (e != ncclSuccess) {
			fprintf(stderr, "[E::vafc] ncclCommInitAll over %d devices failed: %s\n", (int)devs.size(),
			        R->error_string(e));
			c->comms.clear();
			vc_destroy(c);
			return VC_EHIP;
		}
	}
	*out = c;
	return VC_OK;
}

// All shards' counts (and k-mer tallies) into shard 0; the other shards
// restart from zero, so the sum over shards is unchanged and vc_finish may be
// called again.
static int reduce_shards(vc_ctx *c)
{
	const int N = n_shards(c);
	const size_t n = 2 * (size_t)c->n_patterns;
	for (int i = 0; i < N; ++i) {   // every batch counted
		vc_ctx *sh = shard_at(c, i);
		HIPCK(hipSetDevice(sh->dev));
		HIPCK(hipStreamSynchronize(sh->st));
	}
	for (int i = 0; i < N; ++i) {   // same-device shards into the device's first shard
		const int l = c->lead[(size_t)i];
		if (l == i) continue;
		vc_ctx *L = shard_at(c, l), *S = shard_at(c, i);
		HIPCK(hipSetDevice(L->dev));
		HIPCK(vc_launch_shard_add(L->d_counts, S->d_counts, n, L->d_tally, S->d_tally, L->st));
	}
	if (c->comms.size() <= 1) {   // one distinct device: the on-device sum is the whole sum
		HIPCK(hipSetDevice(c->dev));
		HIPCK(hipStreamSynchronize(c->st));
		return VC_OK;
	}
	const RcclApi *R = rccl();
	if (!R) return VC_EHIP;
	NCCK(R, R->group_start());
	// every enqueue goes in, and the group is always closed, before an error
	// is returned: an open group would leave RCCL's thread-local state pending
	// for the next collective or for ncclCommDestroy in vc_destroy
	ncclResult_t first = ncclSuccess;
	for (size_t j = 0; j < c->comms.size() && first == ncclSuccess; ++j) {
		vc_ctx *L = shard_at(c, c->comm_shard[j]);
		(void)hipSetDevice(L->dev);   // the rank's device (its comm and stream live there)
		// in place on every rank: sendbuff == recvbuff; non-root ranks' buffers
		// are left as they were (zeroed below)
		if (n) first = R->reduce(L->d_counts, L->d_counts, n, ncclUint32, ncclSum, 0, c->comms[j], L->st);
		if (first == ncclSuccess)
			first = R->reduce(L->d_tally, L->d_tally, 1, ncclUint64, ncclSum, 0, c->comms[j], L->st);
	}
	const ncclResult_t ge = R->group_end();
	if (first == ncclSuccess) first = ge;
	if (first != ncclSuccess) {
		fprintf(stderr, "[E::vafc] RCCL reduce of the shard counts failed: %s\n", R->error_string(first));
		return VC_EHIP;
	}
	for (size_t j = 1; j < c->comms.size(); ++j) {   // non-root ranks restart from zero
		vc_ctx *L = shard_at(c, c->comm_shard[j]);
		HIPCK(hipSetDevice(L->dev));
		HIPCK(hipMemsetAsync(L->d_counts, 0, n * sizeof(uint32_t), L->st));
		HIPCK(hipMemsetAsync(L->d_tally, 0, sizeof(unsigned long long), L->st));
	}
	for (size_t j = 0; j < c->comms.size(); ++j) {
		vc_ctx *L = shard_at(c, c->comm_shard[j]);
		HIPCK(hipSetDevice(L->dev));
		HIPCK(hipStreamSynchronize(L->st));
	}
	return VC_OK;
}

extern "C" int vc_shard_count(const vc_ctx *c) { return c ? n_shards(c) : 0; }

extern "C" int vc_shard_info(const vc_ctx *c, int i, int *device, uint64_t *batches)
{
	if (!c || i < 0 || i >= n_shards(c)) return VC_EINVAL;
	const vc_ctx *sh = shard_at(const_cast<vc_ctx *>(c), i);
	if (device) *device = sh->dev;
	if (batches) *batches = sh->batches;
	return VC_OK;
}

// ---------------------------------------------------------------------------
// whole-file pass (count_fastq_kmers, vaf-counter.c:550-582)
// ---------------------------------------------------------------------------

#ifndef VC_BATCH_BYTES
#define VC_BATCH_BYTES ((size_t)64 << 20)
#endif

namespace {

// Accepted reads are written straight into a pinned slot; a full slot is
// shipped to the device and the other slot is filled meanwhile.  With several
// shards each batch goes to the next shard (its own slots, stream and device).
struct BatchWriter {
	vc_ctx *c;
	vc_ctx *sh = nullptr;         // shard of the open slot
	Slot *s = nullptr;
	size_t bytes = 0, limit = VC_BATCH_BYTES;
	uint64_t n = 0;
	int err = VC_OK;

	explicit BatchWriter(vc_ctx *ctx) : c(ctx)
	{
		const char *e = getenv("VAFC_BATCH_BYTES");   // test knob: smaller batches
		if (e && atoll(e) >= 1) limit = (size_t)atoll(e);
	}

	int open_slot()
	{
		sh = next_shard(c);
		if (hipSetDevice(sh->dev) != hipSuccess) return VC_EHIP;
		int rc = slot_acquire(sh, &s);
		if (rc == VC_OK) rc = slot_reserve(*s, VC_BATCH_BYTES, VC_BATCH_BYTES / 64);
		bytes = 0;
		n = 0;
		return rc;
	}
	int flush()
	{
		if (!s) return VC_OK;
		int rc = slot_submit(sh, *s, bytes, n);
		s = nullptr;
		bytes = 0;
		n = 0;
		return rc;
	}
	int add(const char *seq, size_t len)
	{
		if (!s && (err = open_slot()) != VC_OK) return err;
		if (bytes + len > s->cap_bytes || n + 1 > s->cap_reads || (n > 0 && bytes + len > limit)) {
			if (n > 0) {
				if ((err = flush()) != VC_OK) return err;
				if ((err = open_slot()) != VC_OK) return err;
			}
			if (len > s->cap_bytes && (err = slot_reserve(*s, len, 1)) != VC_OK) return err;
		}
		memcpy(s->h_seq + bytes, seq, len);
		s->h_offs[n] = bytes;
		s->h_lens[n] = (uint32_t)len;
		bytes += len;
		++n;
		return VC_OK;
	}
};

double wall_now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

} // namespace

// ---------------------------------------------------------------------------
// parallel ingest of plain files (vafc_ingest.h): pieces parsed by -t worker
// threads straight into pinned slots, shipped to the device in file order
// ---------------------------------------------------------------------------

#ifndef VC_PIECE_BYTES
#define VC_PIECE_BYTES ((uint64_t)16 << 20)
#endif
#ifndef VC_PIECE_BYTES_WARM
#define VC_PIECE_BYTES_WARM ((uint64_t)32 << 20)
#endif

static int ingest_slot_alloc(Slot &s, uint64_t piece);
static size_t ingest_slot_bytes(uint64_t piece);

namespace {

// Slot g of the reader lives on shard g % N (slot index g / N there), so the
// pieces of a file go round robin over the shards.
class DeviceSink : public VcIngestSink {
public:
	DeviceSink(vc_ctx *c, uint64_t piece) : c_(c), n_(n_shards(c)), piece_(piece) {}
	int acquire(int slot, VcSlotBuf *b) override
	{
		vc_ctx *sh;
		Slot &s = at(slot, &sh);
		HIPCK(hipSetDevice(sh->dev));
		if (s.pending) {
			HIPCK(hipEventSynchronize(s.done));
			s.pending = false;
		}
		// first use of the slot (reserve_ingest_slots, alloc = false), or
		// buffers sized for smaller pieces than this pass's
		if (!s.h_seq || s.cap_bytes < ingest_slot_bytes(piece_)) {
			const int rc = ingest_slot_alloc(s, piece_);
			if (rc != VC_OK) return rc;
		}
		fill(s, b);
		return VC_OK;
	}
	int grow(int slot, VcSlotBuf *b, size_t bytes, size_t reads, size_t used_bytes, size_t used_reads) override
	{
		vc_ctx *sh;
		Slot &s = at(slot, &sh);
		HIPCK(hipSetDevice(sh->dev));
		Slot n;
		n.done = s.done;
		n.copied = s.copied;
		if (hipHostMalloc(&n.h_seq, bytes, hipHostMallocDefault) != hipSuccess ||
		    hipHostMalloc(&n.h_offs, reads * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
		    hipHostMalloc(&n.h_lens, reads * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
		    hipMalloc(&n.d_seq, bytes) != hipSuccess || hipMalloc(&n.d_offs, reads * sizeof(uint64_t)) != hipSuccess ||
		    hipMalloc(&n.d_lens, reads * sizeof(uint32_t)) != hipSuccess) {
			free_slot(n);
			return VC_EHIP;
		}
		n.cap_bytes = bytes;
		n.cap_reads = reads;
		memcpy(n.h_seq, s.h_seq, used_bytes);
		memcpy(n.h_offs, s.h_offs, used_reads * sizeof(uint64_t));
		memcpy(n.h_lens, s.h_lens, used_reads * sizeof(uint32_t));
		free_slot(s);
		s = n;
		fill(s, b);
		return VC_OK;
	}
	// The copies go on the shard's copy stream and the kernels on its own
	// stream, ordered by one event per slot: the DMA engine streams the pieces
	// back to back instead of waiting for each piece's kernel.  A slot's next
	// copy comes after the worker has waited for its `done` (the kernel that
	// read its device buffers).
	int submit(int slot, const VcSlotBuf &, uint64_t n, uint64_t bytes) override
	{
		vc_ctx *sh;
		Slot &s = at(slot, &sh);
		HIPCK(hipSetDevice(sh->dev));
		if (!sh->cst) HIPCK(hipStreamCreateWithFlags(&sh->cst, hipStreamNonBlocking));
		if (!s.copied) HIPCK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
		HIPCK(hipMemcpyAsync(s.d_seq, s.h_seq, bytes, hipMemcpyHostToDevice, sh->cst));
		HIPCK(hipMemcpyAsync(s.d_offs, s.h_offs, n * sizeof(uint64_t), hipMemcpyHostToDevice, sh->cst));
		HIPCK(hipMemcpyAsync(s.d_lens, s.h_lens, n * sizeof(uint32_t), hipMemcpyHostToDevice, sh->cst));
		HIPCK(hipEventRecord(s.copied, sh->cst));
		HIPCK(hipStreamWaitEvent(sh->st, s.copied, 0));
		int rc = launch(sh, s.d_seq, bytes, s.d_offs, s.d_lens, n, sh->st, any_long(s.h_lens, n));
		if (rc != VC_OK) return rc;
		HIPCK(hipEventRecord(s.done, sh->st));
		s.pending = true;
		++sh->batches;
		return VC_OK;
	}

private:
	vc_ctx *c_;
	int n_;
	uint64_t piece_;
	Slot &at(int slot, vc_ctx **sh)
	{
		*sh = shard_at(c_, slot % n_);
		return (*sh)->islot[(size_t)(slot / n_)];
	}
	static void fill(const Slot &s, VcSlotBuf *b)
	{
		b->seq = s.h_seq;
		b->offs = s.h_offs;
		b->lens = s.h_lens;
		b->cap_bytes = s.cap_bytes;
		b->cap_reads = s.cap_reads;
	}
};

} // namespace

// Plain files of at least this size take the parallel reader.
#ifndef VC_PARALLEL_MIN_BYTES
#define VC_PARALLEL_MIN_BYTES ((uint64_t)32 << 20)
#endif

static int clamp_threads(int n) { return n < 1 ? 1 : (n > 64 ? 64 : n); }

// Pinned + device buffers of the parallel reader's slots (2 x threads slots of
// one piece each: sequence bytes at about half a FASTQ piece, growing on
// demand for FASTA), rounded up to a multiple of the shards and spread over
// them.  Returns the reader's slot count (> 0) or an error (< 0).
static int reserve_ingest_slots(vc_ctx *c, size_t slots, bool alloc);

static int reserve_ingest(vc_ctx *c, int threads, bool alloc)
{
	const int N = n_shards(c);
	// two slots per worker: a piece that finishes late holds back only its
	// own slot while the others parse ahead (threads + 2 slots left the
	// workers waiting for slots 2-3x as long: profiles/r04l_slots_ab.json)
	const char *e = getenv("VAFC_INGEST_SLOTS");   // A/B knob: the reader's slot count (> threads)
	const int want = e && atoi(e) > threads ? atoi(e) : (threads < 2 ? threads + 2 : 2 * threads);
	const int slots = (want + N - 1) / N * N;
	for (int i = 0; i < N; ++i) {
		vc_ctx *sh = shard_at(c, i);
		HIPCK(hipSetDevice(sh->dev));
		int rc = reserve_ingest_slots(sh, (size_t)(slots / N), alloc);
		if (rc != VC_OK) return rc;
	}
	return slots;
}

// One slot's buffers.  FASTQ: at most half of a piece's records' text is
// sequence (the quality line is as long); FASTA and long records grow the slot.
static size_t ingest_slot_bytes(uint64_t piece) { return (size_t)piece / 2 + ((size_t)256 << 10); }

// A slot's pinned buffers as one anonymous mapping on transparent huge pages,
// touched and registered with hipHostRegister, and its device buffers as one
// allocation: pinning 32 slots of a 16 MB piece took 0.018 s this way against
// 0.041-0.057 s as three hipHostMalloc + three hipMalloc each, at the same
// 52 GB/s H2D (tools/pin_probe.hip, profiles/r06b_pin_probe.log).  The CLI pins
// its slots inside the counting timer, as the reference allocates its block
// buffers inside it.  VAFC_PIN=malloc keeps hipHostMalloc (A/B).
static int slot_alloc_mapped(Slot &s, size_t bytes, size_t reads)
{
	const size_t huge = (size_t)2 << 20;
	const size_t ob = (bytes + 63) / 64 * 64, lb = ob + reads * sizeof(uint64_t);
	const size_t need = lb + reads * sizeof(uint32_t);
	const size_t len = (need + huge - 1) / huge * huge;
	void *m = mmap(nullptr, len + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (m == MAP_FAILED) return VC_ENOMEM;
	// the 2 MB-aligned part only (the slack before and after goes back)
	uint8_t *a = (uint8_t *)(((uintptr_t)m + huge - 1) / huge * huge);
	if (a > (uint8_t *)m) munmap(m, (size_t)(a - (uint8_t *)m));
	const size_t tail = (size_t)((uint8_t *)m + len + huge - (a + len));
	if (tail) munmap(a + len, tail);
	madvise(a, len, MADV_HUGEPAGE);
	for (size_t i = 0; i < len; i += 4096) a[i] = 0;   // fault the pages in (huge pages where granted)
	if (hipHostRegister(a, len, hipHostRegisterDefault) != hipSuccess) {
		(void)hipGetLastError();
		munmap(a, len);
		return VC_EHIP;
	}
	uint8_t *d = nullptr;
	if (hipMalloc(&d, need) != hipSuccess) {
		(void)hipGetLastError();
		(void)hipHostUnregister(a);
		munmap(a, len);
		return VC_EHIP;
	}
	s.map = a;
	s.map_len = len;
	s.h_seq = a;
	s.h_offs = (uint64_t *)(a + ob);
	s.h_lens = (uint32_t *)(a + lb);
	s.d_seq = d;
	s.d_offs = (uint64_t *)(d + ob);
	s.d_lens = (uint32_t *)(d + lb);
	s.d_one = true;
	s.cap_bytes = bytes;
	s.cap_reads = reads;
	return VC_OK;
}

static int ingest_slot_alloc(Slot &s, uint64_t piece)
{
	static const bool use_malloc = getenv("VAFC_PIN") && !strcmp(getenv("VAFC_PIN"), "malloc");
	if (use_malloc) return slot_reserve(s, ingest_slot_bytes(piece), (size_t)piece / 256 + 4096);
	const size_t bytes = ingest_slot_bytes(piece), reads = (size_t)piece / 256 + 4096;
	if (bytes <= s.cap_bytes && reads <= s.cap_reads) return VC_OK;
	if (s.pending) HIPCK(hipEventSynchronize(s.done));
	s.pending = false;
	free_slot(s);
	return slot_alloc_mapped(s, bytes + bytes / 4 + 4096, reads + reads / 4 + 1024);
}

// alloc = false: only the slot records and their events; each slot's buffers
// are then allocated by the worker that first fills it (DeviceSink::acquire),
// so pinning them overlaps the other workers' parsing instead of preceding it.
static int reserve_ingest_slots(vc_ctx *c, size_t slots, bool alloc)
{
	if (c->islot.size() < slots) {
		HIPCK(hipStreamSynchronize(c->st));
		const size_t old = c->islot.size();
		c->islot.resize(slots);
		for (size_t i = old; i < slots; ++i)
			HIPCK(hipEventCreateWithFlags(&c->islot[i].done, hipEventDisableTiming));
	}
	for (size_t i = 0; alloc && i < slots; ++i) {
		Slot &s = c->islot[i];
		if (s.h_seq) continue;
		int rc = ingest_slot_alloc(s, VC_PIECE_BYTES);
		if (rc != VC_OK) return rc;
	}
	return VC_OK;
}

extern "C" int vc_reserve_file_ingest(vc_ctx *c, int n_threads)
{
	if (!c) return VC_EINVAL;
	const int rc = reserve_ingest(c, clamp_threads(n_threads), true);
	return rc < 0 ? rc : VC_OK;
}

static int count_file_parallel(vc_ctx *c, int fd, uint64_t size, int block_bases, int n_threads,
                               vc_file_stats &st, VcTextRange *range = nullptr)
{
	const int threads = clamp_threads(n_threads);
	const int slots = reserve_ingest(c, threads, false);
	if (slots < 0) return slots;
	// pieces of 16 MB while the counter's slots are first pinned (the pinning
	// is paid inside the pass, by the workers); once a pass has pinned them,
	// later passes and files use 32 MB pieces (the slots grow once): half the
	// copies, kernels and events per byte (profiles/r05i_*: 39.7-40.5 against
	// 35.5-36.1 Gbases/s in one process; in a fresh CLI process the 32 MB
	// slots' pinning made the pass 40 % slower, profiles/r05i_cli_piece_ab.json)
	const char *pe = getenv("VAFC_INGEST_PIECE");          // test knob: piece size in bytes
	const uint64_t piece = pe && atoll(pe) >= 2 ? (uint64_t)atoll(pe)
	                                            : (c->ingest_warm ? VC_PIECE_BYTES_WARM : VC_PIECE_BYTES);
	DeviceSink sink(c, piece);
	const int rc = vc_ingest_plain(fd, size, c->k, block_bases, threads, slots, piece, sink, st, range);
	if (rc == VC_OK) c->ingest_warm = true;
	return rc;
}

// gzip input: the text the parallel inflater produces (n_threads workers) is
// parsed by the parallel reader's workers, fewer of them (vc_gz_parse_threads).
static int count_file_gzip(vc_ctx *c, VcGzParallel *g, int block_bases, int n_threads, vc_file_stats &st)
{
	const int parsers = vc_gz_parse_threads(clamp_threads(n_threads));
	const int slots = reserve_ingest(c, parsers, false);
	if (slots < 0) return slots;
	const char *pe = getenv("VAFC_INGEST_PIECE");          // test knob: piece size in bytes
	const uint64_t piece = pe && atoll(pe) >= 2 ? (uint64_t)atoll(pe) : VC_PIECE_BYTES;
	DeviceSink sink(c, piece);
	return vc_ingest_gzip(g, c->k, block_bases, parsers, slots, piece, (uint64_t)(slots + 2) * piece * 2, sink, st);
}

// Wait for every shard's queued batches.
static int sync_shards(vc_ctx *c)
{
	for (int i = 0; i < n_shards(c); ++i) {
		vc_ctx *sh = shard_at(c, i);
		HIPCK(hipSetDevice(sh->dev));
		HIPCK(hipStreamSynchronize(sh->st));
	}
	return hipSetDevice(c->dev) == hipSuccess ? VC_OK : VC_EHIP;
}

// CPUs of the NUMA node(s) the counter's GPUs hang off (sysfs, from each
// device's PCI bus id), within this process's affinity mask (vafc_affinity.h).
// Off when VAFC_NUMA=0, when sysfs says nothing, or when the node offers fewer
// CPUs of the mask than the reader has threads (or than the whole mask).
static VcCpuSet gpu_cpus(vc_ctx *c, int threads)
{
	if (c->cpus_threads == threads) return c->cpus;
	VcCpuSet out;
	const char *ne = getenv("VAFC_NUMA");
	cpu_set_t mask;
	CPU_ZERO(&out.set);
	if (!(ne && !strcmp(ne, "0")) && sched_getaffinity(0, sizeof mask, &mask) == 0) {
		bool any_node = false, bad = false;
		for (int i = 0; i < n_shards(c) && !bad; ++i) {
			char bus[64] = {0}, path[256], buf[4096];
			if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, shard_at(c, i)->dev) != hipSuccess) {
				(void)hipGetLastError();
				bad = true;
				break;
			}
			for (char *q = bus; *q; ++q) *q = (char)tolower((unsigned char)*q);
			snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
			FILE *f = fopen(path, "r");
			int node = -1;
			if (!f || fscanf(f, "%d", &node) != 1) node = -1;
			if (f) fclose(f);
			if (node < 0) {
				bad = true;
				break;
			}
			snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
			f = fopen(path, "r");
			size_t n = f ? fread(buf, 1, sizeof buf - 1, f) : 0;
			if (f) fclose(f);
			buf[n] = 0;
			for (char *q = buf; *q;) {   // "0-63,128-191"
				char *e;
				const long a = strtol(q, &e, 10);
				if (e == q) break;
				long b = a;
				if (*e == '-') b = strtol(e + 1, &e, 10);
				for (long x = a; x <= b && x < CPU_SETSIZE; ++x) CPU_SET((int)x, &out.set);
				any_node = true;
				q = *e == ',' ? e + 1 : e;
				if (*e != ',') break;
			}
		}
		if (!bad && any_node) {
			CPU_AND(&out.set, &out.set, &mask);
			const int have = CPU_COUNT(&out.set);
			out.on = have >= threads && have < CPU_COUNT(&mask);
		}
	}
	c->cpus = out;
	c->cpus_threads = threads;
	return out;
}

extern "C" int vc_count_file(vc_ctx *c, const char *path, int block_bases, int n_threads,
                             vc_file_stats *st)
{
	if (!c || !path) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	const double t0 = wall_now();
	HIPCK(hipSetDevice(c->dev));
	// a path that is not a regular file (a FIFO, a device) is opened exactly
	// once, by the sequential reader below: opening it here only to look at
	// it would let a pipe's writer see its reader go away
	struct stat sb;
	if (stat(path, &sb) != 0) return VC_EIO;
	const int fd = S_ISREG(sb.st_mode) ? open(path, O_RDONLY) : -1;
	if (S_ISREG(sb.st_mode) && fd < 0) return VC_EIO;
	uint8_t magic[2] = {0, 0};
	const bool reg = fd >= 0 && fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
	const bool gz = reg && pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
	const bool plain = reg && !gz;
	// the reader threads spawned below run on the GPU's NUMA node when it has
	// a CPU for each of them: the parse workers, or for gzip the inflaters,
	// the parsers of the inflated text, the pump and the block loop
	const int t = clamp_threads(n_threads);
	VcAffinityScope placement(gpu_cpus(c, gz ? vc_gz_inflate_threads(t) + vc_gz_parse_threads(t) + 2 : t));
	{
		const char *me = getenv("VAFC_INGEST_MIN");        // test knob: smallest file for the parallel reader
		const uint64_t min_bytes = me ? (uint64_t)atoll(me) : VC_PARALLEL_MIN_BYTES;
		if (plain && (uint64_t)sb.st_size >= min_bytes && sb.st_size > 0) {
			int rc = count_file_parallel(c, fd, (uint64_t)sb.st_size, block_bases, n_threads, local);
			close(fd);
			if (rc == VC_OK) rc = sync_shards(c);
			local.seconds = wall_now() - t0;
			if (st) *st = local;
			return rc;
		}
		if (fd >= 0) close(fd);
		if (gz) {   // parallel inflate + parallel parse (falls through if the inflater declines the file)
			const char *ce = getenv("VAFC_GZ_CHUNK");            // test knob: compressed bytes per chunk
			VcGzParallel *g = vc_gzp_open(path, vc_gz_inflate_threads(clamp_threads(n_threads)),
			                              ce ? (uint64_t)atoll(ce) : 0);
			if (g) {
				int rc = count_file_gzip(c, g, block_bases, n_threads, local);
				vc_gzp_close(g);
				if (rc == VC_OK) rc = sync_shards(c);
				local.seconds = wall_now() - t0;
				if (st) *st = local;
				return rc;
			}
		}
	}
	VcFastqReader rd;   // small plain files, pipes, gzip the inflater declines
	if (!rd.open_parallel(path, clamp_threads(n_threads))) return VC_EIO;
	BatchWriter bw(c);
	int rc = vc_block_loop(rd, c->k, block_bases,
	                    [&bw](const char *s, size_t l) { return bw.add(s, l); }, local);
	if (rc == VC_OK) rc = bw.flush();
	if (rc == VC_OK) rc = sync_shards(c);
	local.seconds = wall_now() - t0;
	if (st) *st = local;
	return rc;
}

extern "C" int vc_count_file_range(vc_ctx *c, const char *path, uint64_t begin, uint64_t end, int block_bases,
                                   int n_threads, vc_file_stats *st, vc_range_info *ri)
{
	if (!c || !path || !ri || end <= begin) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	*ri = vc_range_info{UINT64_MAX, UINT64_MAX, 0, 0, 1};
	const double t0 = wall_now();
	struct stat sb;
	if (stat(path, &sb) != 0) return VC_EIO;
	// not a regular file (a FIFO): never opened here, so vc_count_file's
	// reader is its only reader (a pipe is read once, as the reference does)
	const int fd = S_ISREG(sb.st_mode) ? open(path, O_RDONLY) : -1;
	if (S_ISREG(sb.st_mode) && fd < 0) return VC_EIO;
	uint8_t magic[2] = {0, 0};
	const bool reg = fd >= 0 && fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
	const bool gz = reg && pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
	if (!reg || gz) {   // not split: the first range counts the whole file
		if (fd >= 0) close(fd);
		if (begin > 0) {
			if (st) *st = local;
			return VC_OK;
		}
		const int rc = vc_count_file(c, path, block_bases, n_threads, st);
		if (rc == VC_OK) *ri = vc_range_info{0, UINT64_MAX, 0, 1, 1};
		return rc;
	}
	int rc = hipSetDevice(c->dev) == hipSuccess ? VC_OK : VC_EHIP;
	VcTextRange R;
	R.begin = begin;
	R.end = end;
	if (rc == VC_OK) {
		VcAffinityScope placement(gpu_cpus(c, clamp_threads(n_threads)));
		rc = count_file_parallel(c, fd, (uint64_t)sb.st_size, block_bases, n_threads, local, &R);
	}
	close(fd);
	if (rc == VC_OK) rc = sync_shards(c);
	*ri = vc_range_info{R.first, R.next, R.errs, R.stopped ? 1u : 0u, 0u};
	local.seconds = wall_now() - t0;
	if (st) *st = local;
	return rc;
}

// One share of a gzip file (include/vafc.h, vafc_gzip.h): the inflater (from
// the share's first block with its known window, or a held share resumed),
// the parallel reader over the share's text as a range (plus the previous
// byte, for the first guess).  Takes g and closes it.
static int count_gz_share_g(vc_ctx *c, VcGzParallel *g, int fmt, int parsers, int first_share,
                            const uint8_t *window, uint64_t text_len, int block_bases, vc_file_stats &local,
                            vc_range_info *ri, vc_gz_share_crc *crc)
{
	int rc = reserve_ingest(c, parsers, false);
	VcTextRange R;
	const size_t np = first_share ? 0 : 1;
	if (rc >= 0) {
		const int slots = rc;
		const char *pe = getenv("VAFC_INGEST_PIECE");          // test knob: piece size in bytes
		const uint64_t piece = pe && atoll(pe) >= 2 ? (uint64_t)atoll(pe) : VC_PIECE_BYTES;
		DeviceSink sink(c, piece);
		R.begin = np;
		R.end = np + text_len;
		R.format = fmt;
		rc = vc_ingest_gzip_share(g, first_share ? nullptr : window + 32767, np, c->k, block_bases, parsers, slots,
		                          piece, (uint64_t)(slots + 2) * piece * 2, sink, local, &R);
	}
	VcGzShareCrc sc;
	vc_gzp_share_crc(g, &sc);
	vc_gzp_close(g);
	if (rc == VC_OK) rc = sync_shards(c);
	*ri = vc_range_info{R.first == UINT64_MAX ? UINT64_MAX : R.first - np,
	                    R.next == UINT64_MAX ? UINT64_MAX : R.next - np - text_len, R.errs, R.stopped ? 1u : 0u, 0u};
	*crc = vc_gz_share_crc{sc.events, sc.head_crc, sc.head_len, sc.head_expect_crc, sc.head_expect_isize,
	                       sc.tail_crc, sc.tail_len, sc.crc_error, sc.complete};
	return rc;
}

extern "C" int vc_count_gz_share(vc_ctx *c, const char *path, int first_share, uint64_t start_bit,
                                 const uint8_t *window, uint64_t text_len, int block_bases, int n_threads,
                                 vc_file_stats *st, vc_range_info *ri, vc_gz_share_crc *crc)
{
	if (!c || !path || !ri || !crc || text_len == 0 || (!first_share && !window)) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	*ri = vc_range_info{UINT64_MAX, UINT64_MAX, 0, 0, 0};
	memset(crc, 0, sizeof *crc);
	const double t0 = wall_now();
	HIPCK(hipSetDevice(c->dev));
	const int fmt = vc_gz_text_format(path);
	if (fmt < 0) return VC_EINVAL;
	const int t = clamp_threads(n_threads);
	VcAffinityScope placement(gpu_cpus(c, vc_gz_inflate_threads(t) + vc_gz_parse_threads(t) + 2));
	const char *ce = getenv("VAFC_GZ_CHUNK");   // test knob: compressed bytes per chunk
	VcGzParallel *g = vc_gzp_open_share(path, vc_gz_inflate_threads(t), ce ? (uint64_t)atoll(ce) : 0,
	                                    first_share != 0, start_bit, window, text_len);
	if (!g) return VC_EIO;
	const int rc = count_gz_share_g(c, g, fmt, vc_gz_parse_threads(t), first_share, window, text_len, block_bases,
	                                local, ri, crc);
	local.seconds = wall_now() - t0;
	if (st) *st = local;
	return rc;
}

extern "C" int vc_gz_share_open(vc_ctx *c, const char *path, uint64_t begin, uint64_t end, int n_threads,
                                uint64_t chunk_bytes, uint64_t hold_bytes, vc_gz_share_info *out,
                                uint16_t *window_sym, vc_gz_share **held)
{
	if (!path || !out || !held || end <= begin) return VC_EINVAL;
	*held = nullptr;
	const int t = n_threads < 1 ? 1 : n_threads;
	// the scan's threads where the count's will run (the GPU's NUMA node):
	// the chunks they keep are first touched there, so the count reads them
	// from local memory
	VcCpuSet none;
	CPU_ZERO(&none.set);
	if (c) HIPCK(hipSetDevice(c->dev));
	const int ct = clamp_threads(t);
	VcAffinityScope placement(c ? gpu_cpus(c, vc_gz_inflate_threads(ct) + vc_gz_parse_threads(ct) + 2) : none);
	VcGzShare sh;
	VcGzParallel *g = nullptr;
	if (!vc_gzp_scan_share_hold(path, t, chunk_bytes, begin, end, hold_bytes, &sh, window_sym, &g)) return VC_EIO;
	out->start_bit = sh.start_bit;
	out->end_bit = sh.end_bit;
	out->text_len = sh.text_len;
	out->ok = sh.ok ? 1u : 0u;
	out->ended = sh.start_bit != UINT64_MAX && sh.end_bit == UINT64_MAX ? 1u : 0u;
	if (g) {
		vc_gz_share *h = new vc_gz_share;
		h->g = g;
		h->format = vc_gz_text_format(path);
		h->threads = t;
		*held = h;
	}
	return VC_OK;
}

extern "C" int vc_count_gz_share_held(vc_ctx *c, vc_gz_share *h, int first_share, const uint8_t *window,
                                      uint64_t text_len, int block_bases, int n_threads, vc_file_stats *st,
                                      vc_range_info *ri, vc_gz_share_crc *crc)
{
	if (!c || !h || !h->g || !ri || !crc || text_len == 0 || (!first_share && !window)) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	*ri = vc_range_info{UINT64_MAX, UINT64_MAX, 0, 0, 0};
	memset(crc, 0, sizeof *crc);
	const double t0 = wall_now();
	HIPCK(hipSetDevice(c->dev));
	if (h->format < 0) return VC_EINVAL;
	const int t = clamp_threads(n_threads);
	VcAffinityScope placement(gpu_cpus(c, vc_gz_inflate_threads(t) + vc_gz_parse_threads(t) + 2));
	VcGzParallel *g = h->g;
	h->g = nullptr;   // counted once; count_gz_share_g closes it
	if (!vc_gzp_resume_share(g, first_share ? nullptr : window, text_len)) {
		vc_gzp_close(g);
		return VC_EINVAL;
	}
	const int rc = count_gz_share_g(c, g, h->format, vc_gz_held_parse_threads(t), first_share, window, text_len,
	                                block_bases, local, ri, crc);
	local.seconds = wall_now() - t0;
	if (st) *st = local;
	return rc;
}

extern "C" int vc_scan_file(const char *path, int k, int block_bases, vc_file_stats *st,
                            uint8_t *seq_out, size_t seq_cap, uint32_t *lens_out, size_t lens_cap)
{
	if (!path || !st) return VC_EINVAL;
	vc_file_stats local = {0, 0, 0, 0.0};
	const double t0 = wall_now();
	VcFastqReader rd;
	if (!rd.open(path)) return VC_EIO;
	size_t nb = 0, nr = 0;
	int rc = vc_block_loop(rd, k, block_bases, [&](const char *s, size_t l) {
		if (seq_out && nb + l <= seq_cap) memcpy(seq_out + nb, s, l);
		if (lens_out && nr < lens_cap) lens_out[nr] = (uint32_t)l;
		nb += l;
		++nr;
		return VC_OK;
	}, local);
	local.seconds = wall_now() - t0;
	*st = local;
	return rc;
}

extern "C" int64_t vc_scan_records(const char *path, int32_t *rets, int64_t cap)
{
	if (!path) return VC_EINVAL;
	VcFastqReader rd;
	if (!rd.open(path)) return VC_EIO;
	int64_t n = 0;
	int ret;
	do {
		ret = rd.next();
		if (n < cap && rets) rets[n] = ret;
		++n;
	} while (ret != -1);
	return n;
}

// ---------------------------------------------------------------------------
// synthetic reads, misc
// ---------------------------------------------------------------------------

extern "C" int vc_synth_reads(uint8_t *d_seq, uint64_t *d_offs, uint32_t *d_lens, uint64_t first,
                              uint64_t n_reads, uint32_t read_len, uint64_t seed, double f_snp,
                              const uint8_t *d_windows, const uint8_t *d_dosage, uint32_t n_snp,
                              void *stream)
{
	if (read_len < 1 || read_len > 301 || (n_snp && (!d_windows || !d_dosage))) return VC_EINVAL;
	double t = f_snp * 4294967296.0;
	uint64_t thr = t <= 0 ? 0 : (t >= 4294967296.0 ? (uint64_t)1 << 32 : (uint64_t)llround(t));
	HIPCK(vc_launch_synth(d_seq, d_offs, d_lens, first, n_reads, read_len, seed, thr, d_windows,
	                      d_dosage, n_snp, (hipStream_t)stream));
	return VC_OK;
}

// Test hook: device decode of whole reads to codes (0..3, 4 = invalid).
extern "C" int vc_debug_decode(const uint8_t *d_seq, size_t seq_bytes, const uint64_t *d_offs,
                               const uint32_t *d_lens, uint64_t n_reads, uint8_t *d_codes, void *stream)
{
	HIPCK(vc_launch_decode(d_seq, seq_bytes, d_offs, d_lens, n_reads, d_codes, (hipStream_t)stream));
	return VC_OK;
}

// ---------------------------------------------------------------------------
// kc-c4 histogram mode (vafc_kc.hip)
// ---------------------------------------------------------------------------

extern "C" int vc_kc_create(vc_ctx **out, int k, uint64_t table_slots, int device)
{
	if (!out) return VC_EINVAL;
	*out = nullptr;
	vc_ctx *c = nullptr;
	int rc = vc_create(&c, k, nullptr, nullptr, 0, 0, device);
	if (rc != VC_OK) return rc;
	Kc *K = new (std::nothrow) Kc;
	if (!K) {
		vc_destroy(c);
		return VC_ENOMEM;
	}
	c->kc = K;
	// at most 40 % of free HBM (rounded down to a power of two), so first-
	// occurrence stamps and yak's scratch table still fit beside it
	size_t fr = 0, tot = 0;
	if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = (size_t)1 << 30;
	uint32_t cap_bits = 10;
	while (cap_bits < 40 && ((uint64_t)32 << cap_bits) <= (uint64_t)(fr * 0.4)) ++cap_bits;
	uint32_t tbits = cap_bits;
	if (table_slots) {
		tbits = 10;
		while (tbits < cap_bits && ((uint64_t)1 << tbits) < table_slots) ++tbits;
	}
	K->tbits = tbits;
	K->slots = (uint64_t)1 << tbits;
	if (hipMalloc(&K->d_table, K->slots * 16) != hipSuccess || hipMalloc(&K->d_stats, 3 * 8) != hipSuccess ||
	    hipMalloc(&K->d_hist, 1025 * 8) != hipSuccess || hipMalloc(&K->d_nlong, 4) != hipSuccess) {
		vc_destroy(c);
		return VC_EHIP;
	}
	rc = vc_reset(c);
	if (rc == VC_OK && hipStreamSynchronize(c->st) != hipSuccess) rc = VC_EHIP;
	if (rc != VC_OK) {
		vc_destroy(c);
		return rc;
	}
	*out = c;
	return VC_OK;
}

extern "C" int vc_kc_set_partition(vc_ctx *c, uint32_t n_parts, uint32_t part)
{
	if (!c || !c->kc || n_parts == 0 || n_parts > 1024 || part >= n_parts) return VC_EINVAL;
	HIPCK(hipSetDevice(c->dev));
	HIPCK(hipStreamSynchronize(c->st));
	c->kc->n_parts = n_parts;
	c->kc->part = part;
	return vc_reset(c);
}

extern "C" uint64_t vc_kc_slots(vc_ctx *c) { return c && c->kc ? c->kc->slots : 0; }

// hist[0..n_bins) on the host += the device histogram; *counted = slots in it
static int kc_hist(vc_ctx *c, uint64_t *hist, uint32_t n_bins, uint64_t min_count, uint64_t *counted)
{
	Kc &K = *c->kc;
	HIPCK(hipMemsetAsync(K.d_hist, 0, 1025 * 8, c->st));
	const uint64_t blocks = (K.slots + 255) / 256;
	const uint64_t maxg = (uint64_t)c->n_cu * 8;
	HIPCK(vc_launch_kc_hist(K.d_table, K.slots, K.d_hist, n_bins, min_count, (int)(blocks < maxg ? blocks : maxg),
	                        c->st));
	std::vector<unsigned long long> h(n_bins + 1);
	HIPCK(hipMemcpyAsync(h.data(), K.d_hist, (n_bins + 1) * 8, hipMemcpyDeviceToHost, c->st));
	HIPCK(hipStreamSynchronize(c->st));
	if (hist)
		for (uint32_t i = 0; i < n_bins; ++i) hist[i] += h[i];
	if (counted) *counted = h[n_bins];
	return VC_OK;
}

extern "C" int vc_kc_histogram2(vc_ctx *c, uint64_t *hist, uint32_t n_bins, uint64_t min_count, uint64_t *distinct,
                                uint64_t *kmers)
{
	if (!c || !c->kc || n_bins < 2 || n_bins > 1024) return VC_EINVAL;
	Kc &K = *c->kc;
	HIPCK(hipSetDevice(c->dev));
	HIPCK(hipStreamSynchronize(c->st));
	unsigned long long st[3];
	HIPCK(hipMemcpy(st, K.d_stats, sizeof st, hipMemcpyDeviceToHost));
	if (kmers) *kmers = st[0];
	if (distinct) *distinct = st[1];
	if (st[2] || st[1] > K.slots / 100 * 85) return VC_EFULL;
	uint64_t counted = 0;
	int rc = kc_hist(c, hist, n_bins, min_count, &counted);
	if (rc == VC_OK && distinct) *distinct = counted;
	return rc;
}

extern "C" int vc_kc_histogram(vc_ctx *c, uint64_t *hist, uint64_t *distinct, uint64_t *kmers)
{
	return vc_kc_histogram2(c, hist, 256, 1, distinct, kmers);
}

extern "C" int vc_kc_track_first(vc_ctx *c, int on)
{
	if (!c || !c->kc) return VC_EINVAL;
	Kc &K = *c->kc;
	HIPCK(hipSetDevice(c->dev));
	HIPCK(hipStreamSynchronize(c->st));
	if (on && !K.d_first && hipMalloc(&K.d_first, K.slots * 8) != hipSuccess) {
		K.d_first = nullptr;
		return VC_ENOMEM;
	}
	K.track_first = on != 0;
	return vc_reset(c);
}

extern "C" int vc_yak_bloom_select(vc_ctx *c, int pre, int bf_shift, int n_hash)
{
	if (!c || !c->kc || pre < 0 || pre > 40) return VC_EINVAL;
	Kc &K = *c->kc;
	HIPCK(hipSetDevice(c->dev));
	HIPCK(hipStreamSynchronize(c->st));
	unsigned long long st[3];
	HIPCK(hipMemcpy(st, K.d_stats, sizeof st, hipMemcpyDeviceToHost));
	if (st[2] || st[1] > K.slots / 100 * 85) return VC_EFULL;
	// yak_ch_init / yak_bf_init (yak-count.c:71-80, 115-121): filters exist only
	// for n_hash > 0 and 9 <= bf_shift - pre <= 55
	const int ns = bf_shift - pre;
	const bool bf_on = n_hash > 0 && bf_shift > pre && ns >= 9 && ns + 9 <= 64;
	if (bf_on && !K.track_first) return VC_EINVAL;
	YakBloom B;
	B.table = K.d_table;
	B.counts_out = K.d_table;
	B.first = K.d_first;
	B.slots = K.slots;
	B.pre = (uint32_t)pre;
	B.ns = bf_on ? (uint32_t)ns : 9;
	B.n_hash = bf_on ? (uint32_t)n_hash : 0;
	B.wtab = nullptr;
	B.wslots = 1;
	B.wbits = 0;
	B.overflow = K.d_stats + 2;
	if (bf_on) {
		uint64_t singles = 0;
		std::vector<uint64_t> h(2, 0);
		int rc = kc_hist(c, h.data(), 2, 1, nullptr);   // h[1]: keys seen exactly once
		if (rc != VC_OK) return rc;
		singles = h[1];
		uint32_t wbits = 10;
		while (wbits < 48 && ((uint64_t)1 << wbits) < 2 * singles * (uint64_t)n_hash) ++wbits;
		B.wbits = wbits;
		B.wslots = (uint64_t)1 << wbits;
		// no room for the scratch table: report full, so the caller counts
		// again in more partitions (fewer singletons per pass)
		if (hipMalloc(&B.wtab, B.wslots * 16) != hipSuccess) return VC_EFULL;
		HIPCK(hipMemsetAsync(B.wtab, 0, B.wslots * 16, c->st));
	}
	const uint64_t blocks = (K.slots + 255) / 256;
	const uint64_t maxg = (uint64_t)c->n_cu * 8;
	hipError_t e = vc_launch_yak_select(&B, (int)(blocks < maxg ? blocks : maxg), c->st);
	if (e == hipSuccess) e = hipStreamSynchronize(c->st);
	if (B.wtab) (void)hipFree(B.wtab);
	if (e != hipSuccess) return VC_EHIP;
	HIPCK(hipMemcpy(st, K.d_stats, sizeof st, hipMemcpyDeviceToHost));
	if (st[2]) return VC_EFULL;
	K.lookup_only = true;
	return VC_OK;
}

extern "C" const char *vc_strerror(int err)
{
	switch (err) {
	case VC_OK: return "ok";
	case VC_EINVAL: return "invalid argument";
	case VC_ENOMEM: return "out of host memory";
	case VC_EHIP: return "HIP runtime error";
	case VC_ENODEV: return "no HIP device";
	case VC_EIO: return "file could not be opened";
	case VC_ETOOMANY: return "too many patterns";
	case VC_EFULL: return "k-mer table full";
	default: return "unknown error";
	}
}

extern "C" int vc_version(void) { return VAFC_VERSION_MAJOR * 100 + VAFC_VERSION_MINOR; }
