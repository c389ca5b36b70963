// pinned_copy.cpp -- host write rate into the staging buffers the ingest path
// uses (tools only): 150-byte records copied one by one, as BatchWriter::add
// does, into hipHostMalloc memory (default, non-coherent) vs malloc'd memory.
//   hipcc -O3 -o tools/pinned_copy tools/pinned_copy.cpp && tools/pinned_copy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double run(unsigned char *dst, const unsigned char *src, size_t bytes)
{
	const size_t rec = 150, stride = 311;      // FASTQ: 150 bases of every 311 bytes
	const size_t n = bytes / rec;
	double best = 1e30;
	for (int rep = 0; rep < 5; ++rep) {
		const double t0 = now();
		for (size_t i = 0; i < n; ++i) memcpy(dst + i * rec, src + i * stride, rec);
		const double t = now() - t0;
		best = t < best ? t : best;
	}
	return bytes / best / 1e9;
}

int main()
{
	const size_t bytes = (size_t)64 << 20;
	unsigned char *src = (unsigned char *)malloc(bytes * 311 / 150 + 4096);
	memset(src, 'A', bytes * 311 / 150 + 4096);
	unsigned char *m = (unsigned char *)malloc(bytes);
	memset(m, 0, bytes);
	unsigned char *p1 = nullptr, *p2 = nullptr, *p3 = nullptr;
	if (hipHostMalloc((void **)&p1, bytes, hipHostMallocDefault) != hipSuccess ||
	    hipHostMalloc((void **)&p2, bytes, hipHostMallocNonCoherent) != hipSuccess ||
	    hipHostMalloc((void **)&p3, bytes, hipHostMallocWriteCombined) != hipSuccess) {
		fprintf(stderr, "hipHostMalloc failed\n");
		return 1;
	}
	memset(p1, 0, bytes);
	memset(p2, 0, bytes);
	memset(p3, 0, bytes);
	printf("malloc                    %.2f GB/s of sequence bytes\n", run(m, src, bytes));
	printf("hipHostMallocDefault      %.2f GB/s\n", run(p1, src, bytes));
	printf("hipHostMallocNonCoherent  %.2f GB/s\n", run(p2, src, bytes));
	printf("hipHostMallocWriteCombined %.2f GB/s\n", run(p3, src, bytes));
	return 0;
}
