// vafc_kernels.hip -- dispatch of the counting kernels on k (the K = 16..31
// instantiations live in vafc_kernels_kNN.hip, k < 16 runs the run-time-k
// kernel instantiated here), plus the decode test hook and the synthetic
// read generator.
#include "vafc_scan.h"

#define VC_K_LIST(X) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) \
	X(30) X(31)
#define VC_K_DECL(k)                                                                         \
	hipError_t vc_launch_k##k(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st); \
	hipError_t vc_setup_k##k(int lds);
VC_K_LIST(VC_K_DECL)
#undef VC_K_DECL

// ---------------------------------------------------------------------------
// debug kernel: position-dependent decode of whole reads (tests only)
// ---------------------------------------------------------------------------

__global__ void vc_decode_kernel(const uint8_t *seq, uint64_t seq_bytes, const uint64_t *offs,
                                 const uint32_t *lens, uint64_t n_reads, uint8_t *codes)
{
	const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (r >= n_reads) return;
	const uint32_t *s32 = reinterpret_cast<const uint32_t *>(seq);
	const uint64_t nw = (seq_bytes + 3) / 4;
	const uint64_t wmax = nw ? nw - 1 : 0;
	const int len = (int)lens[r];
	const uint64_t off = offs[r];
	const int tail_c = (len & 15) ? (len >> 4) : -1;
	for (int c = 0; 16 * c < len; ++c) {
		uint64_t addr = off + 16ull * c;
		uint64_t wi = addr >> 2;
		uint32_t sh = (uint32_t)(addr & 3u);
		uint32_t w[5];
		for (int j = 0; j < 5; ++j) w[j] = ldw(s32, wi + j, wmax);
		for (int m = 0; m < 4; ++m) {
			uint32_t b = __builtin_amdgcn_alignbyte(w[m + 1], w[m], sh);
			uint32_t t = (c == tail_c) ? dec_tail(b) : dec_head(b);
			for (int i = 0; i < 4; ++i) {
				int p = 16 * c + 4 * m + i;
				if (p < len) {
					uint32_t cb = (t >> (8 * i)) & 0xFFu;
					codes[off + p] = (cb & 4u) ? 4u : (uint8_t)(cb & 3u);
				}
			}
		}
	}
}

// ---------------------------------------------------------------------------
// synthetic reads (vafc_synth.py on the device)
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint64_t h64(uint64_t seed, uint64_t item, uint64_t draw)
{
	uint64_t z = seed * 0x9E3779B97F4A7C15ull + item * 0xD1B54A32D192ED03ull + draw * 0xABC98388FB8FAC03ull;
	z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
	z ^= z >> 27; z *= 0x94D049BB133111EBull;
	z ^= z >> 31;
	return z;
}

__global__ void vc_synth_kernel(uint8_t *seq, uint64_t *offs, uint32_t *lens, uint64_t first,
                                uint64_t n_reads, uint32_t L, uint64_t seed, uint64_t thr,
                                const uint8_t *win, const uint8_t *dosage, uint32_t n_snp)
{
	const uint64_t total = n_reads * (uint64_t)L;
	const uint64_t THR_N = 4294967ull, THR_SUB = 25769803ull;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t rd = i / L;
		const uint32_t p = (uint32_t)(i - rd * L);
		const uint64_t ri = first + rd;
		const uint64_t r0 = h64(seed, ri, 0), r1 = h64(seed, ri, 1);
		const uint64_t r2 = h64(seed, ri, 2), r3 = h64(seed, ri, 3);
		const bool rc = (r3 & 1ull) != 0;
		const uint32_t q = rc ? L - 1u - p : p;
		const uint64_t r = h64(seed, ri, 16ull + q);
		uint32_t base = (uint32_t)(r & 3ull);
		const bool is_snp = n_snp > 0 && (r0 >> 32) < thr;
		if (is_snp) {
			const uint64_t snp = ((r1 >> 32) * (uint64_t)n_snp) >> 32;
			const uint32_t g = dosage[snp];
			const bool alt = g == 2u || (g == 1u && (r1 & 1ull));
			const uint64_t nstart = 301u - L + 1u;
			const uint64_t start = ((r2 >> 32) * nstart) >> 32;
			const uint8_t ch = win[(snp * 2u + (alt ? 1u : 0u)) * 301u + start + q];
			base = ch == 'A' ? 0u : ch == 'C' ? 1u : ch == 'G' ? 2u : 3u;
		}
		const uint64_t u = r >> 32;
		if (u >= THR_N && u < THR_SUB) base = (base + 1u + (uint32_t)(((r >> 2) & 0xFFFFull) % 3ull)) & 3u;
		uint8_t out;
		if (u < THR_N) out = 'N';
		else {
			if (rc) base ^= 3u;
			out = "ACGT"[base];
		}
		seq[i] = out;
		if (p == 0) { offs[rd] = rd * (uint64_t)L; lens[rd] = L; }
	}
}

// ---------------------------------------------------------------------------
// multi-shard reduction, step 1: shards that share a device are summed into
// the device's first shard (u32 adds wrap like the reference's counters) and
// restart from zero; the devices' sums then go through RCCL (vafc_host.cpp)
// ---------------------------------------------------------------------------

__global__ void vc_shard_add_kernel(uint32_t *dst, uint32_t *src, uint64_t n, unsigned long long *dst_tally,
                                    unsigned long long *src_tally)
{
	const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	for (uint64_t i = gid; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		dst[i] += src[i];
		src[i] = 0u;
	}
	if (gid == 0) {
		*dst_tally += *src_tally;
		*src_tally = 0ull;
	}
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------

extern "C" hipError_t vc_launch_shard_add(uint32_t *dst, uint32_t *src, uint64_t n, unsigned long long *dst_tally,
                                          unsigned long long *src_tally, hipStream_t st)
{
	uint64_t blocks = (n + 255) / 256;
	if (blocks < 1) blocks = 1;
	if (blocks > 1024) blocks = 1024;
	hipLaunchKernelGGL(vc_shard_add_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dst, src, n, dst_tally,
	                   src_tally);
	return hipGetLastError();
}

extern "C" hipError_t vc_launch_count(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	switch (A->k) {
#define VC_K_CASE(k) case k: return vc_launch_k##k(A, grid, grid_long, st);
		VC_K_LIST(VC_K_CASE)
#undef VC_K_CASE
	default: return launch_k<0>(A, grid, grid_long, st);
	}
}

extern "C" hipError_t vc_kernel_setup(void)
{
	// the largest dynamic LDS any launch asks for: the 128 KiB filter with full
	// queues, or the large-panel filter with short ones (exactly 160 KiB)
	const size_t l128 = vc_lds_bytes(1u << VC_MAX_FILTER_WBITS, VC_QCAP);
	const size_t lbig = vc_lds_bytes(VC_BIG_FILTER_WORDS, VC_BIG_QCAP);
	const int lds = (int)(l128 > lbig ? l128 : lbig);
	hipError_t e = setup_k<0>(lds);
#define VC_K_SET(k) if (e == hipSuccess) e = vc_setup_k##k(lds);
	VC_K_LIST(VC_K_SET)
#undef VC_K_SET
	return e;
}

extern "C" hipError_t vc_launch_decode(const uint8_t *seq, uint64_t seq_bytes, const uint64_t *offs,
                                       const uint32_t *lens, uint64_t n_reads, uint8_t *codes,
                                       hipStream_t st)
{
	const int blk = 256;
	const int grid = (int)((n_reads + blk - 1) / blk);
	if (grid == 0) return hipSuccess;
	hipLaunchKernelGGL(vc_decode_kernel, dim3(grid), dim3(blk), 0, st, seq, seq_bytes, offs, lens,
	                   n_reads, codes);
	return hipGetLastError();
}

extern "C" hipError_t vc_launch_synth(uint8_t *seq, uint64_t *offs, uint32_t *lens, uint64_t first,
                                      uint64_t n_reads, uint32_t L, uint64_t seed, uint64_t thr,
                                      const uint8_t *win, const uint8_t *dosage, uint32_t n_snp,
                                      hipStream_t st)
{
	const uint64_t total = n_reads * (uint64_t)L;
	if (total == 0) return hipSuccess;
	uint64_t blocks = (total + 255) / 256;
	if (blocks > 65536) blocks = 65536;
	hipLaunchKernelGGL(vc_synth_kernel, dim3((unsigned)blocks), dim3(256), 0, st, seq, offs, lens,
	                   first, n_reads, L, seed, thr, win, dosage, n_snp);
	return hipGetLastError();
}
