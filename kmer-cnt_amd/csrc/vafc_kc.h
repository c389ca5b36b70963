// vafc_kc.h -- argument block and launchers of the kc-c4 kernels
// (vafc_kc.hip), shared with the host library.  Not part of the C ABI.
#ifndef VAFC_KC_H
#define VAFC_KC_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define KC_THREADS 256
#define KC_LONG 4096          // reads longer than this are cut into segments
#define KC_SEG 1024           // bases per long-read segment (plus a k-1 halo)
#define KC_MAX_PROBE 1024     // a longer probe sequence marks the table full

struct KcArgs {
	const uint8_t *seq;
	const uint64_t *offs;
	const uint32_t *lens;
	uint64_t n_reads;
	unsigned long long *table;   // 2 * slots: key (hash64 + 1, 0 = empty), count
	uint64_t tmask;
	uint32_t tbits;
	uint32_t n_parts, part;      // count k-mers with (lo32(hash64) * n_parts) >> 32 == part
	int k;
	uint64_t kmask;
	unsigned long long *stats;   // [0] k-mers seen, [1] distinct inserted, [2] overflow
	uint32_t *nlong;
	uint32_t *longlist;
	uint32_t long_cap;
	uint64_t *segstart;          // long_cap + 1
};

#ifdef __cplusplus
extern "C" {
#endif
hipError_t vc_launch_kc(const KcArgs *A, int grid, hipStream_t st);
hipError_t vc_launch_kc_hist(const unsigned long long *table, uint64_t slots, unsigned long long *hist, int grid,
                             hipStream_t st);
#ifdef __cplusplus
}
#endif

#endif
