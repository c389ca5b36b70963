// Pinned-slot allocation cost (tools only): the parallel reader's 18 slots
// allocated as the reader does (per slot: 3 hipHostMalloc + 3 hipMalloc)
// against one hipHostMalloc + one hipMalloc of the same total, and the
// per-slot form from 4 threads at once.
//   hipcc --offload-arch=gfx950 -O2 tools/alloc_probe.hip -o alloc_probe && ./alloc_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

int main()
{
	const size_t slots = 18, nb = (size_t)(16 << 20) * 5 / 8 + (1 << 20), nr = (16 << 20) / 256 + 4096;
	const size_t b = nb + nb / 4 + 4096, r = nr + nr / 4 + 1024;
	CK(hipSetDevice(0));
	CK(hipFree(nullptr));
	for (int rep = 0; rep < 3; ++rep) {
		std::vector<void *> h, d;
		double t0 = now();
		for (size_t i = 0; i < slots; ++i) {
			void *p;
			CK(hipHostMalloc(&p, b, hipHostMallocDefault)); h.push_back(p);
			CK(hipHostMalloc(&p, r * 8, hipHostMallocDefault)); h.push_back(p);
			CK(hipHostMalloc(&p, r * 4, hipHostMallocDefault)); h.push_back(p);
		}
		double t1 = now();
		for (size_t i = 0; i < slots; ++i) {
			void *p;
			CK(hipMalloc(&p, b)); d.push_back(p);
			CK(hipMalloc(&p, r * 8)); d.push_back(p);
			CK(hipMalloc(&p, r * 4)); d.push_back(p);
		}
		double t2 = now();
		for (void *p : h) CK(hipHostFree(p));
		for (void *p : d) CK(hipFree(p));
		double t3 = now();
		void *H, *D;
		CK(hipHostMalloc(&H, slots * (b + r * 12), hipHostMallocDefault));
		double t4 = now();
		CK(hipMalloc(&D, slots * (b + r * 12)));
		double t5 = now();
		CK(hipHostFree(H));
		CK(hipFree(D));
		std::vector<std::thread> th;
		std::vector<void *> hh(slots * 3);
		double t6 = now();
		for (int w = 0; w < 4; ++w)
			th.emplace_back([&, w] {
				for (size_t i = w; i < slots; i += 4) {
					(void)hipHostMalloc(&hh[3 * i], b, hipHostMallocDefault);
					(void)hipHostMalloc(&hh[3 * i + 1], r * 8, hipHostMallocDefault);
					(void)hipHostMalloc(&hh[3 * i + 2], r * 4, hipHostMallocDefault);
				}
			});
		for (auto &t : th) t.join();
		double t7 = now();
		for (void *p : hh) CK(hipHostFree(p));
		printf("per-slot: host %.4f s, device %.4f s, free %.4f s | one block: host %.4f s, device %.4f s | per-slot host, 4 threads %.4f s (%.0f MB pinned)\n",
		       t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t7 - t6, slots * (b + r * 12) / 1e6);
	}
	return 0;
}
