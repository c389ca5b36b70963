// vafc_corr.hip -- correlation-matrix on the GPU:
// depth-aware Pearson correlation of every pair of .vaf samples
// (correlation-matrix.c:94-162), plus the host side of the tool: the .vaf
// loader (:25-90), the .corr writer (:350-366) and the UPGMA-like tree
// (:190-257).
//
// The reference runs, for every pair i < j, three sequential passes over
// the rows [0, n_i) of sample i (n_i = rows of the LOWER-indexed sample; the
// higher one's rows past its end read as vaf 0.0, depth 0):
//   count of rows valid in both (depth >= min_depth), then the two sums of
//   VAFs in row order, the means, then the centred products summed in row
//   order.  Double arithmetic, every operation separately rounded.
// The output is printed with %.6f, and the tree compares distances exactly,
// so the device reproduces the reference's doubles bit for bit: one lane per
// pair keeps the reference's summation order; FP contraction is off; invalid
// rows contribute exactly nothing (terms times a 1.0 / 0.0 validity factor,
// see the kernel; pairs whose sums turn NaN are recounted by the x86-NaN
// kernel).  The host finishes each pair from the device sums with the
// reference's formula (sqrt, epsilon branch).
//
// Layout (HBM): x[n_samples][P] doubles (P = rows padded to CH, zero past a
// sample's end), and two validity bitmaps per sample, u32 words of 32 rows:
//   lo[s] -- rows r < n_s with depth >= min_depth (sample s as the lower index
//            of a pair: bounds the pair's row range to n_s),
//   hi[s] -- rows r < P with (r < n_s ? depth : 0) >= min_depth (sample s as
//            the higher index: the reference's zero rows past its end).
// A pair's valid rows are lo[a] & hi[b].
//
// Kernel: a 256-thread block owns a tile of TA = 32 lower samples x TB = 64
// higher samples (tiles entirely below the diagonal exit); lane l of wave w
// takes b = b0 + l and a = a0 + 8w .. 8w + 7, i.e. eight pairs.  Rows are
// staged CH = 64 at a time through LDS: the b rows transposed (row-major in
// the lane index, conflict-free), the a rows as broadcasts (one address per
// wave).  Each pair is a sequential scan, so there is no cross-lane
// reduction and no reassociation.  FP64 VALU-bound: per pair and valid row
// 2 adds (pass 1), 2 subtracts, 3 multiplies and 3 adds (pass 2).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <new>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "vafc.h"

#define CORR_CAP 100000   // correlation-matrix.c:8 MAX_SNPS
#define CORR_LINE 4096    // correlation-matrix.c:9 MAX_LINE

namespace {

#ifndef CORR_TA
#define CORR_TA 32
#endif
constexpr int TA = CORR_TA, TB = 64, CH = 64, NT = 256, PA = TA / (NT / 64);

struct CorrArgs {
	const double *x;          // [n][P]
	const uint32_t *lo, *hi;  // [n][P / 32]
	int n, P, words;
	int *cnt;                 // [n][n], pairs a < b
	double *sx, *sy, *sxy, *sxx, *syy;
};

__global__ void __launch_bounds__(NT) corr_pairs_kernel(CorrArgs A)
{
#pragma clang fp contract(off)
	const int a0 = blockIdx.y * TA, b0 = blockIdx.x * TB;
	if (a0 >= b0 + TB - 1 || a0 >= A.n) return;       // no pair a < b in this tile (uniform)
	__shared__ double xa[TA][CH + 2];                    // a rows, row-major in the row index
	__shared__ double xb[CH][TB + 1];                    // b rows, transposed (+1: write conflicts)
	__shared__ uint32_t wa[TA][CH / 32], wb[TB][CH / 32];
	const int t = threadIdx.x, lb = t & 63, ag = (t >> 6) * PA;
	const int b = b0 + lb;

	int cnt[PA];
	double s1[PA], s2[PA], mx[PA], my[PA], pxy[PA], pxx[PA], pyy[PA];
#pragma unroll
	for (int r = 0; r < PA; ++r) {
		cnt[r] = 0;
		s1[r] = s2[r] = 0.0;
		pxy[r] = pxx[r] = pyy[r] = 0.0;
	}
	for (int pass = 0; pass < 2; ++pass) {
		for (int c0 = 0; c0 < A.P; c0 += CH) {
			__syncthreads();
			for (int e = t; e < TB * CH; e += NT) {
				const int row = e / CH, s = e % CH, bb = b0 + row;
				xb[s][row] = bb < A.n ? A.x[(size_t)bb * A.P + c0 + s] : 0.0;
			}
			for (int e = t; e < TA * CH; e += NT) {
				const int row = e / CH, s = e % CH, aa = a0 + row;
				xa[row][s] = aa < A.n ? A.x[(size_t)aa * A.P + c0 + s] : 0.0;
			}
			if (t < TB * (CH / 32)) {
				const int row = t / (CH / 32), w = t % (CH / 32), bb = b0 + row;
				wb[row][w] = bb < A.n ? A.hi[(size_t)bb * A.words + c0 / 32 + w] : 0u;
			} else if (t < TB * (CH / 32) + TA * (CH / 32)) {
				const int u = t - TB * (CH / 32), row = u / (CH / 32), w = u % (CH / 32), aa = a0 + row;
				wa[row][w] = aa < A.n ? A.lo[(size_t)aa * A.words + c0 / 32 + w] : 0u;
			}
			__syncthreads();
#pragma unroll
			for (int w = 0; w < CH / 32; ++w) {
				const uint32_t mb = wb[lb][w];
				uint32_t m[PA];
#pragma unroll
				for (int r = 0; r < PA; ++r) {
					m[r] = wa[ag + r][w] & mb;
					if (pass == 0) cnt[r] += __popc(m[r]);
				}
				uint32_t any = 0;
#pragma unroll
				for (int r = 0; r < PA; ++r) any |= m[r];
				if (!__any(any != 0u)) continue;
				for (int s = 0; s < 32; ++s) {
					const double y = xb[w * 32 + s][lb];
#pragma unroll
					for (int r = 0; r < PA; ++r) {
						// branch-free: terms are multiplied by the row's validity
						// f = 1.0 / 0.0.  A valid row is unchanged (x * 1 = x, so
						// fma(x, f, s) rounds s + x once, as the reference's add); an
						// invalid finite row adds +-0.0, which leaves every sum as it
						// is (a sum starts at +0.0 and never becomes -0.0 under
						// round-to-nearest).  An invalid inf / NaN row turns the sums
						// NaN: such pairs are recounted by corr_pairs_x86_kernel.
						const double f = (double)((m[r] >> s) & 1u);
						const double x = xa[ag + r][w * 32 + s];
						if (pass == 0) {
							s1[r] = __fma_rn(x, f, s1[r]);             // correlation-matrix.c:107-112
							s2[r] = __fma_rn(y, f, s2[r]);
						} else {
							const double dx = (x - mx[r]) * f, dy = (y - my[r]) * f;   // :118-125
							const double p = dx * dy, q = dx * dx, u = dy * dy;
							pxy[r] = pxy[r] + p;
							pxx[r] = pxx[r] + q;
							pyy[r] = pyy[r] + u;
						}
					}
				}
			}
		}
		if (pass == 0) {
#pragma unroll
			for (int r = 0; r < PA; ++r) {                // :113-114 (unused when no row is valid)
				mx[r] = cnt[r] ? s1[r] / (double)cnt[r] : 0.0;
				my[r] = cnt[r] ? s2[r] / (double)cnt[r] : 0.0;
			}
		}
	}
#pragma unroll
	for (int r = 0; r < PA; ++r) {
		const int a = a0 + ag + r;
		if (a < b && b < A.n) {
			const size_t o = (size_t)a * A.n + b;
			A.cnt[o] = cnt[r];
			A.sx[o] = s1[r];
			A.sy[o] = s2[r];
			A.sxy[o] = pxy[r];
			A.sxx[o] = pxx[r];
			A.syy[o] = pyy[r];
		}
	}
}

// NaN signs.  The reference's sums only turn NaN on "nan"/"inf" VAF text, and
// what it prints then ("nan" or "-nan") is the sign of an x86 NaN: an SSE
// add/sub/mul/div returns its first operand if that is a NaN, else its second
// if that is one, else (inf - inf, 0 * inf) the default NaN, which is
// negative.  The first operands follow the reference's code
// (correlation-matrix.c:108-125 as compiled: sum + x, x - mean, dx * dy,
// sum + product, sum / count).  The fast kernel keeps the GPU's NaNs; pairs
// that come back with a NaN sum are counted again by this kernel, one lane
// per pair, with every operation's NaN chosen the x86 way.
__device__ __forceinline__ double x86_nan(double r, double a, double b)
{
	if (!isnan(r)) return r;
	if (isnan(a)) return a;
	if (isnan(b)) return b;
	return __longlong_as_double((long long)0xFFF8000000000000ull);
}

__global__ void __launch_bounds__(64) corr_pairs_x86_kernel(CorrArgs A, const int2 *pairs, int n_pairs)
{
#pragma clang fp contract(off)
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_pairs) return;
	const int a = pairs[i].x, b = pairs[i].y;
	const double *xa = A.x + (size_t)a * A.P, *xb = A.x + (size_t)b * A.P;
	const uint32_t *la = A.lo + (size_t)a * A.words, *hb = A.hi + (size_t)b * A.words;
	int cnt = 0;
	double s1 = 0.0, s2 = 0.0;
	for (int r = 0; r < A.P; ++r) {
		if (!((la[r >> 5] & hb[r >> 5]) >> (r & 31) & 1u)) continue;
		++cnt;
		s1 = x86_nan(s1 + xa[r], s1, xa[r]);
		s2 = x86_nan(s2 + xb[r], s2, xb[r]);
	}
	const double c = (double)cnt;
	const double mx = cnt ? x86_nan(s1 / c, s1, c) : 0.0, my = cnt ? x86_nan(s2 / c, s2, c) : 0.0;
	double pxy = 0.0, pxx = 0.0, pyy = 0.0;
	for (int r = 0; r < A.P; ++r) {
		if (!((la[r >> 5] & hb[r >> 5]) >> (r & 31) & 1u)) continue;
		const double dx = x86_nan(xa[r] - mx, xa[r], mx), dy = x86_nan(xb[r] - my, xb[r], my);
		const double p = x86_nan(dx * dy, dx, dy), q = x86_nan(dx * dx, dx, dx), u = x86_nan(dy * dy, dy, dy);
		pxy = x86_nan(pxy + p, pxy, p);
		pxx = x86_nan(pxx + q, pxx, q);
		pyy = x86_nan(pyy + u, pyy, u);
	}
	const size_t o = (size_t)a * A.n + b;
	A.sxy[o] = pxy;
	A.sxx[o] = pxx;
	A.syy[o] = pyy;
}

}  // namespace

// ---------------------------------------------------------------------------
// sample set + loader (correlation-matrix.c:25-90)
// ---------------------------------------------------------------------------

struct vc_vafset {
	std::vector<std::string> name;
	std::vector<std::vector<double>> x;
	std::vector<std::vector<int32_t>> d;
};

extern "C" int vc_vafset_create(vc_vafset **out)
{
	if (!out) return VC_EINVAL;
	*out = new (std::nothrow) vc_vafset();
	return *out ? VC_OK : VC_ENOMEM;
}

extern "C" void vc_vafset_free(vc_vafset *s) { delete s; }

extern "C" int vc_vafset_count(const vc_vafset *s) { return s ? (int)s->name.size() : 0; }

extern "C" const char *vc_vafset_name(const vc_vafset *s, int i)
{
	return s && i >= 0 && i < (int)s->name.size() ? s->name[i].c_str() : nullptr;
}

extern "C" int vc_vafset_snps(const vc_vafset *s, int i)
{
	return s && i >= 0 && i < (int)s->name.size() ? (int)s->x[i].size() : VC_EINVAL;
}

// One .vaf file; *truncated = the 100,000-row cap was hit (the caller prints
// the reference's warning).  false if the file cannot be opened.
// load_vaf_file's body on an opened file (closed here)
static void vaf_load_fp(FILE *fp, const char *path, std::string &nm, std::vector<double> &x,
                        std::vector<int32_t> &d, bool &truncated)
{
	truncated = false;
	// sample name: basename, at most 255 bytes, cut at the first ".vaf"
	const char *base = strrchr(path, '/');
	nm.assign(base ? base + 1 : path);
	if (nm.size() > 255) nm.resize(255);
	const size_t cut = nm.find(".vaf");
	if (cut != std::string::npos) nm.resize(cut);
	char line[CORR_LINE];
	while (fgets(line, sizeof line, fp)) {          // lines past 4095 bytes arrive in pieces, as there
		if (line[0] == '#' || strncmp(line, "CHR", 3) == 0) continue;
		char f1[256], f3[256], c1, c2;
		int pos, nref, nalt, tot;
		double v;
		if (sscanf(line, "%255s\t%d\t%255s\t%c\t%c\t%d\t%d\t%d\t%lf", f1, &pos, f3, &c1, &c2, &nref, &nalt, &tot,
		           &v) != 9)
			continue;
		if (x.size() >= CORR_CAP) {
			truncated = true;
			break;
		}
		x.push_back(v);
		d.push_back(tot);
	}
	fclose(fp);
}

static bool vaf_load_one(const char *path, std::string &nm, std::vector<double> &x, std::vector<int32_t> &d,
                         bool &truncated)
{
	FILE *fp = fopen(path, "r");
	if (!fp) return false;
	vaf_load_fp(fp, path, nm, x, d, truncated);
	return true;
}

extern "C" int vc_vafset_add(vc_vafset *s, const char *path)
{
	if (!s || !path) return VC_EINVAL;
	std::string nm;
	std::vector<double> x;
	std::vector<int32_t> d;
	bool trunc;
	if (!vaf_load_one(path, nm, x, d, trunc)) return VC_EIO;
	if (trunc) fprintf(stderr, "Warning: too many SNPs (max %d), truncating\n", CORR_CAP);
	s->name.push_back(nm);
	s->x.push_back(std::move(x));
	s->d.push_back(std::move(d));
	return VC_OK;
}

extern "C" int vc_vafset_add_many(vc_vafset *s, const char *const *paths, int n, int n_threads, int *n_added,
                                  uint8_t *truncated)
{
	if (!s || n < 0 || (n && (!paths || !truncated))) return VC_EINVAL;
	std::vector<std::string> nm(n);
	std::vector<std::vector<double>> x(n);
	std::vector<std::vector<int32_t>> d(n);
	std::vector<char> tr(n, 0);
	// The files are opened here, in order, up to the first that cannot be
	// opened, as the reference's loop does (correlation-matrix.c:304,329-335;
	// nothing after it is opened: a FIFO named after a missing file must not
	// block).  At most W files are open and not yet parsed at any time (the
	// workers close each one once parsed), so any number of inputs works under
	// the usual 1,024-descriptor limit, like the reference's one-at-a-time loop.
	const int T = n_threads < 1 ? 1 : (n_threads > 64 ? 64 : n_threads);
	const int W = 2 * T < 64 ? 2 * T : 64;
	std::vector<FILE *> fp((size_t)n, nullptr);
	std::mutex mu;
	std::condition_variable cv;
	int opened = 0, handed = 0, parsed = 0;
	bool closed = false;                           // no more files will be opened
	std::vector<std::thread> th;
	for (int t = 0; t < T && t < n; ++t)
		th.emplace_back([&] {
			for (;;) {
				int i;
				{
					std::unique_lock<std::mutex> lk(mu);
					cv.wait(lk, [&] { return handed < opened || closed; });
					if (handed >= opened) return;  // closed and nothing left
					i = handed++;
				}
				bool trunc = false;
				vaf_load_fp(fp[(size_t)i], paths[i], nm[i], x[i], d[i], trunc);   // closes the file
				tr[i] = trunc;
				{
					std::lock_guard<std::mutex> lk(mu);
					++parsed;
				}
				cv.notify_all();
			}
		});
	for (int i = 0; i < n; ++i) {
		{
			std::unique_lock<std::mutex> lk(mu);
			cv.wait(lk, [&] { return opened - parsed < W; });
		}
		FILE *f = fopen(paths[i], "r");
		if (!f) break;
		{
			std::lock_guard<std::mutex> lk(mu);
			fp[(size_t)i] = f;
			++opened;
		}
		cv.notify_all();
	}
	{
		std::lock_guard<std::mutex> lk(mu);
		closed = true;
	}
	cv.notify_all();
	for (auto &t : th) t.join();
	const int m = opened;
	int i = 0;
	for (; i < m; ++i) {                           // in order, up to the first file that failed
		truncated[i] = (uint8_t)tr[i];
		s->name.push_back(std::move(nm[i]));
		s->x.push_back(std::move(x[i]));
		s->d.push_back(std::move(d[i]));
	}
	if (n_added) *n_added = i;
	return i == n ? VC_OK : VC_EIO;
}

extern "C" int vc_vafset_add_arrays(vc_vafset *s, const char *name, const double *vaf, const int32_t *depth, int n)
{
	if (!s || !name || n < 0 || n > CORR_CAP || (n && (!vaf || !depth))) return VC_EINVAL;
	s->name.emplace_back(name);
	s->x.emplace_back(vaf, vaf + n);
	s->d.emplace_back(depth, depth + n);
	return VC_OK;
}

// ---------------------------------------------------------------------------
// the matrix
// ---------------------------------------------------------------------------

#define CCK(x)                                   \
	do {                                         \
		if ((x) != hipSuccess) {                 \
			rc = VC_EHIP;                        \
			goto done;                           \
		}                                        \
	} while (0)

// The x86 NaN of an operation whose first operand is a (see x86_nan above);
// this host is x86-64, so a NaN from two non-NaN operands is already the
// default one -- only the choice between two NaN operands is pinned here.
static inline double host_nan(double r, double a, double b)
{
	return isnan(r) ? (isnan(a) ? a : (isnan(b) ? b : r)) : r;
}

// correlation-matrix.c:113-142, from the device sums, operands in the
// reference's order (denominator sqrt(sum_y2) * sqrt(sum_x2); epsilon branch
// sum_x2 * sum_y2)
static double corr_finish(int cnt, double sxy, double sxx, double syy, int min_snps)
{
	if (cnt < min_snps) return 0.0;
	const double dx = sqrt(sxx), dy = sqrt(syy);
	if (dx < 1e-10 || dy < 1e-10) {
		const double s = sqrt(host_nan(sxx * syy, sxx, syy));
		const double e = host_nan(s + 0.00001, s, 0.00001);
		return host_nan(sxy / e, sxy, e);
	}
	const double d = host_nan(dy * dx, dy, dx);
	return host_nan(sxy / d, sxy, d);
}

extern "C" int vc_corr_matrix_raw(const double *vaf, const int32_t *depth, const int32_t *n_snps, int n_samples,
                                  size_t stride, int min_snps, int min_depth, double *corr, int device,
                                  float *kernel_ms)
{
	if (n_samples < 0 || (n_samples && (!vaf || !depth || !n_snps || !corr))) return VC_EINVAL;
	const int n = n_samples;
	int maxn = 0;
	for (int i = 0; i < n; ++i) {
		if (n_snps[i] < 0 || (size_t)n_snps[i] > stride) return VC_EINVAL;
		maxn = n_snps[i] > maxn ? n_snps[i] : maxn;
	}
	if (kernel_ms) *kernel_ms = 0.f;
	for (int i = 0; i < n; ++i) corr[(size_t)i * n + i] = 1.0;      // :156
	if (n < 2) return VC_OK;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VC_ENODEV;
	if (device < 0 || device >= ndev) return VC_EINVAL;
	const int P = ((maxn > 0 ? maxn : 1) + CH - 1) / CH * CH, words = P / 32;
	const size_t nn = (size_t)n * n;
	std::vector<double> hx((size_t)n * P, 0.0);
	std::vector<uint32_t> hlo((size_t)n * words, 0u), hhi((size_t)n * words, 0u);
	for (int s = 0; s < n; ++s) {
		const double *xs = vaf + (size_t)s * stride;
		const int32_t *ds = depth + (size_t)s * stride;
		for (int r = 0; r < P; ++r) {
			const int dep = r < n_snps[s] ? ds[r] : 0;
			if (r < n_snps[s]) hx[(size_t)s * P + r] = xs[r];
			if (dep >= min_depth) {
				hhi[(size_t)s * words + r / 32] |= 1u << (r % 32);
				if (r < n_snps[s]) hlo[(size_t)s * words + r / 32] |= 1u << (r % 32);
			}
		}
	}
	std::vector<int> hc(nn, 0);
	std::vector<double> hs(3 * nn, 0.0);
	int rc = VC_OK;
	CorrArgs A{};
	hipEvent_t e0 = nullptr, e1 = nullptr;
	void *dbuf[9] = {}, *dpairs = nullptr;
	std::vector<int2> nanp;
	CCK(hipSetDevice(device));
	CCK(hipMalloc(&dbuf[0], hx.size() * sizeof(double)));
	CCK(hipMalloc(&dbuf[1], hlo.size() * sizeof(uint32_t)));
	CCK(hipMalloc(&dbuf[2], hhi.size() * sizeof(uint32_t)));
	CCK(hipMalloc(&dbuf[3], nn * sizeof(int)));
	for (int i = 4; i < 9; ++i) CCK(hipMalloc(&dbuf[i], nn * sizeof(double)));
	CCK(hipMemcpy(dbuf[0], hx.data(), hx.size() * sizeof(double), hipMemcpyHostToDevice));
	CCK(hipMemcpy(dbuf[1], hlo.data(), hlo.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
	CCK(hipMemcpy(dbuf[2], hhi.data(), hhi.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
	A.x = (const double *)dbuf[0];
	A.lo = (const uint32_t *)dbuf[1];
	A.hi = (const uint32_t *)dbuf[2];
	A.n = n;
	A.P = P;
	A.words = words;
	A.cnt = (int *)dbuf[3];
	A.sx = (double *)dbuf[4];
	A.sy = (double *)dbuf[5];
	A.sxy = (double *)dbuf[6];
	A.sxx = (double *)dbuf[7];
	A.syy = (double *)dbuf[8];
	CCK(hipEventCreate(&e0));
	CCK(hipEventCreate(&e1));
	CCK(hipEventRecord(e0, 0));
	hipLaunchKernelGGL(corr_pairs_kernel, dim3((n + TB - 1) / TB, (n + TA - 1) / TA), dim3(NT), 0, 0, A);
	CCK(hipGetLastError());
	CCK(hipEventRecord(e1, 0));
	CCK(hipEventSynchronize(e1));
	if (kernel_ms) CCK(hipEventElapsedTime(kernel_ms, e0, e1));
	CCK(hipMemcpy(hc.data(), A.cnt, nn * sizeof(int), hipMemcpyDeviceToHost));
	CCK(hipMemcpy(hs.data(), A.sxy, nn * sizeof(double), hipMemcpyDeviceToHost));
	CCK(hipMemcpy(hs.data() + nn, A.sxx, nn * sizeof(double), hipMemcpyDeviceToHost));
	CCK(hipMemcpy(hs.data() + 2 * nn, A.syy, nn * sizeof(double), hipMemcpyDeviceToHost));
	for (int i = 0; i < n; ++i)
		for (int j = i + 1; j < n; ++j) {
			const size_t o = (size_t)i * n + j;
			if (hc[o] >= min_snps && (isnan(hs[o]) || isnan(hs[nn + o]) || isnan(hs[2 * nn + o])))
				nanp.push_back(make_int2(i, j));
		}
	if (!nanp.empty()) {
		CCK(hipMalloc(&dpairs, nanp.size() * sizeof(int2)));
		CCK(hipMemcpy(dpairs, nanp.data(), nanp.size() * sizeof(int2), hipMemcpyHostToDevice));
		hipLaunchKernelGGL(corr_pairs_x86_kernel, dim3(((int)nanp.size() + 63) / 64), dim3(64), 0, 0, A,
		                   (const int2 *)dpairs, (int)nanp.size());
		CCK(hipGetLastError());
		CCK(hipMemcpy(hs.data(), A.sxy, nn * sizeof(double), hipMemcpyDeviceToHost));
		CCK(hipMemcpy(hs.data() + nn, A.sxx, nn * sizeof(double), hipMemcpyDeviceToHost));
		CCK(hipMemcpy(hs.data() + 2 * nn, A.syy, nn * sizeof(double), hipMemcpyDeviceToHost));
	}
	for (int i = 0; i < n; ++i)
		for (int j = i + 1; j < n; ++j) {
			const size_t o = (size_t)i * n + j;
			const double r = corr_finish(hc[o], hs[o], hs[nn + o], hs[2 * nn + o], min_snps);
			corr[o] = r;
			corr[(size_t)j * n + i] = r;                       // :160
		}
done:
	for (void *p : dbuf)
		if (p) (void)hipFree(p);
	if (dpairs) (void)hipFree(dpairs);
	if (e0) (void)hipEventDestroy(e0);
	if (e1) (void)hipEventDestroy(e1);
	return rc;
}

extern "C" int vc_corr_matrix(const vc_vafset *s, int min_snps, int min_depth, double *corr, int device,
                              float *kernel_ms)
{
	if (!s || !corr) return VC_EINVAL;
	const int n = (int)s->name.size();
	size_t stride = 1;
	for (int i = 0; i < n; ++i) stride = s->x[i].size() > stride ? s->x[i].size() : stride;
	std::vector<double> x((size_t)n * stride, 0.0);
	std::vector<int32_t> d((size_t)n * stride, 0), ns(n);
	for (int i = 0; i < n; ++i) {
		ns[i] = (int32_t)s->x[i].size();
		std::copy(s->x[i].begin(), s->x[i].end(), x.begin() + (size_t)i * stride);
		std::copy(s->d[i].begin(), s->d[i].end(), d.begin() + (size_t)i * stride);
	}
	return vc_corr_matrix_raw(x.data(), d.data(), ns.data(), n, stride, min_snps, min_depth, corr, device,
	                          kernel_ms);
}

// ---------------------------------------------------------------------------
// writers (correlation-matrix.c:350-366, 190-257)
// ---------------------------------------------------------------------------

extern "C" int vc_corr_write(const vc_vafset *s, const double *corr, const char *path)
{
	if (!s || !corr || !path) return VC_EINVAL;
	FILE *fp = fopen(path, "w");
	if (!fp) return VC_EIO;
	const int n = (int)s->name.size();
	fputs("Sample", fp);
	for (int i = 0; i < n; ++i) fprintf(fp, "\t%s", s->name[i].c_str());
	fputc('\n', fp);
	for (int i = 0; i < n; ++i) {
		fputs(s->name[i].c_str(), fp);
		for (int j = 0; j < n; ++j) fprintf(fp, "\t%.6f", corr[(size_t)i * n + j]);
		fputc('\n', fp);
	}
	fclose(fp);
	return VC_OK;
}

// Average-linkage merging on d = 1 - r: each step takes the first strictly
// smallest distance in (i, j > i) scan order among active samples (none
// below 1e10: stop), prints it halved, averages row j into row i and retires j.
extern "C" int vc_corr_tree(const vc_vafset *s, const double *corr, const char *path)
{
	if (!s || !corr || !path) return VC_EINVAL;
	FILE *fp = fopen(path, "w");
	if (!fp) return VC_EIO;
	const int n = (int)s->name.size();
	std::vector<double> d((size_t)n * n);
	for (size_t i = 0; i < d.size(); ++i) d[i] = 1.0 - corr[i];
	std::vector<int> act;                         // active samples, ascending
	for (int i = 0; i < n; ++i) act.push_back(i);
	fputs("# Simple dendrogram (UPGMA-like clustering)\n# Format: (Sample1:distance, Sample2:distance)\n", fp);
	while (act.size() > 1) {
		int bi = -1, bj = -1;
		double best = 1e10;
		for (size_t p = 0; p < act.size(); ++p) {
			const double *row = &d[(size_t)act[p] * n];
			for (size_t q = p + 1; q < act.size(); ++q)
				if (row[act[q]] < best) {
					best = row[act[q]];
					bi = act[p];
					bj = act[q];
				}
		}
		if (bi < 0) break;
		fprintf(fp, "Cluster: %s (%.4f) <-> %s (%.4f)\n", s->name[bi].c_str(), best / 2, s->name[bj].c_str(),
		        best / 2);
		for (int k : act) {
			if (k == bi || k == bj) continue;
			const double v = (d[(size_t)bi * n + k] + d[(size_t)bj * n + k]) / 2.0;
			d[(size_t)bi * n + k] = v;
			d[(size_t)k * n + bi] = v;
		}
		for (size_t p = 0; p < act.size(); ++p)
			if (act[p] == bj) {
				act.erase(act.begin() + p);
				break;
			}
	}
	fclose(fp);
	return VC_OK;
}
