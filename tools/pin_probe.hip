// Pinning cost of the parallel reader's slots (tools only): 32 slots of one
// 16 MB piece each (8.25 MB of sequence + offsets + lengths), allocated
//   A  as the reader does: 3 hipHostMalloc + 3 hipMalloc per slot
//   B  one hipHostMalloc + one hipMalloc per slot (the three arrays in one)
//   C  per slot one 2 MB-aligned mmap with MADV_HUGEPAGE, touched, then
//      hipHostRegister (transparent huge pages: 512x fewer pages to pin/map)
//   D  as C without MADV_HUGEPAGE (4 KiB pages)
// and the H2D copy rate out of each kind of memory.
//   hipcc --offload-arch=gfx950 -O2 tools/pin_probe.hip -o tools/bin/pin_probe && tools/bin/pin_probe
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

static const size_t SLOTS = 32, SEQ = ((size_t)16 << 20) / 2 + ((size_t)256 << 10), NR = ((size_t)16 << 20) / 256 + 4096;

static void *map_huge(size_t n, bool huge)
{
	const size_t al = (size_t)2 << 20;
	const size_t m = (n + al - 1) / al * al;
	void *p = mmap(nullptr, m + al, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (p == MAP_FAILED) return nullptr;
	uint8_t *q = (uint8_t *)(((uintptr_t)p + al - 1) / al * al);
	if (huge) madvise(q, m, MADV_HUGEPAGE);
	memset(q, 0, m);
	return q;
}

static double h2d(void *h, void *d, size_t n)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	float best = 1e9f;
	for (int i = 0; i < 5; ++i) {
		(void)hipEventRecord(a, 0);
		(void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, 0);
		(void)hipEventRecord(b, 0);
		(void)hipEventSynchronize(b);
		float ms;
		(void)hipEventElapsedTime(&ms, a, b);
		if (ms < best) best = ms;
	}
	(void)hipEventDestroy(a);
	(void)hipEventDestroy(b);
	return n / (best * 1e-3) / 1e9;
}

int main()
{
	CK(hipSetDevice(0));
	CK(hipFree(nullptr));
	const size_t per = SEQ + NR * 12;
	for (int rep = 0; rep < 3; ++rep) {
		double t[8];
		std::vector<void *> h, d;
		t[0] = now();
		for (size_t i = 0; i < SLOTS; ++i) {
			void *p;
			CK(hipHostMalloc(&p, SEQ, hipHostMallocDefault)); h.push_back(p);
			CK(hipHostMalloc(&p, NR * 8, hipHostMallocDefault)); h.push_back(p);
			CK(hipHostMalloc(&p, NR * 4, hipHostMallocDefault)); h.push_back(p);
			CK(hipMalloc(&p, SEQ)); d.push_back(p);
			CK(hipMalloc(&p, NR * 8)); d.push_back(p);
			CK(hipMalloc(&p, NR * 4)); d.push_back(p);
		}
		t[1] = now();
		const double gA = h2d(h[0], d[0], SEQ);
		for (void *p : h) CK(hipHostFree(p));
		for (void *p : d) CK(hipFree(p));
		h.clear();
		d.clear();
		t[2] = now();
		for (size_t i = 0; i < SLOTS; ++i) {
			void *p;
			CK(hipHostMalloc(&p, per, hipHostMallocDefault)); h.push_back(p);
			CK(hipMalloc(&p, per)); d.push_back(p);
		}
		t[3] = now();
		for (void *p : h) CK(hipHostFree(p));
		for (void *p : d) CK(hipFree(p));
		h.clear();
		std::vector<void *> hv;
		for (int huge = 1; huge >= 0; --huge) {
			t[4 + 2 * (1 - huge)] = now();
			for (size_t i = 0; i < SLOTS; ++i) {
				void *p = map_huge(per, huge);
				if (!p) return 1;
				CK(hipHostRegister(p, per, hipHostRegisterDefault));
				hv.push_back(p);
			}
			t[5 + 2 * (1 - huge)] = now();
			void *dd;
			CK(hipMalloc(&dd, per));
			const double g = h2d(hv[0], dd, SEQ);
			CK(hipFree(dd));
			printf("%s: %.1f GB/s H2D; ", huge ? "C (THP + register)" : "D (4K + register)", g);
			for (void *p : hv) {
				CK(hipHostUnregister(p));
				munmap(p, per);   // the aligned part only; the probe leaks the slack
			}
			hv.clear();
		}
		printf("\nA per-slot 3+3 allocations %.4f s (H2D %.1f GB/s) | B 1+1 per slot %.4f s | "
		       "C THP mmap+touch+register %.4f s | D 4K mmap+touch+register %.4f s  (%zu slots, %.0f MB pinned)\n",
		       t[1] - t[0], gA, t[3] - t[2], t[5] - t[4], t[7] - t[6], SLOTS, SLOTS * per / 1e6);
	}
	return 0;
}
