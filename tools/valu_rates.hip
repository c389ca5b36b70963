// valu_rates.hip -- issue cost of the VALU instructions the counting kernel
// uses, measured on the device (tools only, never shipped).  Every wave runs
// 8 independent chains of one instruction (inline asm, so the compiler keeps
// exactly that instruction), W waves per SIMD on every CU (W = 1, 2, 4, 8:
// blocks of 256 / 512 / 1024 threads, one per CU, or two 1024-thread blocks
// per CU); the time per instruction per SIMD is kernel time / (W waves *
// instructions per wave).  Round 6 added the occupancy sweep: is the 2.7-3.0
// cycles measured at 4 waves per SIMD an occupancy artefact (the guide gives
// 2 cycles per wave64 VALU instruction on a 32-wide SIMD)?
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rates tools/valu_rates.hip && tools/valu_rates [W ...]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 16384

#define CHAIN8(INS)                                                                                    \
	asm volatile(INS : "+v"(a0) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a1) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a2) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a3) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a4) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a5) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a6) : "v"(s0), "v"(s1));                                                  \
	asm volatile(INS : "+v"(a7) : "v"(s0), "v"(s1));

#define KERNEL(NAME, INS)                                                                              \
	__global__ void __launch_bounds__(1024) NAME(unsigned *out, unsigned seed)                         \
	{                                                                                                  \
		unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
		         a6 = a0 + 6, a7 = a0 + 7;                                                             \
		unsigned s0 = seed * 3u + threadIdx.x, s1 = seed ^ 0x55u;                                      \
		for (int i = 0; i < ITERS; ++i) {                                                              \
			CHAIN8(INS)                                                                                \
		}                                                                                              \
		out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;          \
	}

KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL(k_and_b32, "v_and_b32 %0, %0, %1")
KERNEL(k_lshrrev_b32, "v_lshrrev_b32 %0, %1, %0")
KERNEL(k_lshl_or_b32, "v_lshl_or_b32 %0, %0, %1, %2")
KERNEL(k_alignbit_b32, "v_alignbit_b32 %0, %0, %1, %2")
KERNEL(k_alignbyte_b32, "v_alignbyte_b32 %0, %0, %1, %2")
KERNEL(k_bitop3_b32, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x48")
KERNEL(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_perm_b32, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_bfe_u32, "v_bfe_u32 %0, %0, %1, %2")
KERNEL(k_and_or_b32, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_or3_b32, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_add_f32, "v_add_f32 %0, %0, %1")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_pk_lshrrev_b16, "v_pk_lshrrev_b16 %0, %1, %0")
KERNEL(k_xad_u32, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, %1, %2")
KERNEL(k_cndmask_vcc, "v_cndmask_b32 %0, %0, %1, vcc")

typedef void (*kfn)(unsigned *, unsigned);

int main(int argc, char **argv)
{
	int cus = 0;
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
	int clk_khz = 0;
	hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
	unsigned *out;
	hipMalloc(&out, (size_t)2 * cus * 1024 * 4);
	struct { const char *name; kfn f; } ks[] = {
		{"v_add_u32", k_add_u32}, {"v_and_b32", k_and_b32}, {"v_lshrrev_b32", k_lshrrev_b32},
		{"v_lshl_or_b32", k_lshl_or_b32}, {"v_alignbit_b32", k_alignbit_b32}, {"v_alignbyte_b32", k_alignbyte_b32},
		{"v_bitop3_b32", k_bitop3_b32}, {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_lo_u32", k_mul_lo_u32},
		{"v_perm_b32", k_perm_b32}, {"v_bfe_u32", k_bfe_u32}, {"v_and_or_b32", k_and_or_b32},
		{"v_or3_b32", k_or3_b32}, {"v_add_f32", k_add_f32}, {"v_fma_f32", k_fma_f32},
		{"v_pk_add_u16", k_pk_add_u16}, {"v_pk_lshrrev_b16", k_pk_lshrrev_b16},
		{"v_xad_u32", k_xad_u32}, {"v_lshl_add_u32", k_lshl_add_u32}, {"v_cndmask_b32", k_cndmask_vcc},
	};
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	int ws[8] = {1, 2, 4, 8}, nw = 4;
	if (argc > 1) {
		nw = 0;
		for (int i = 1; i < argc && nw < 8; ++i) ws[nw++] = atoi(argv[i]);
	}
	printf("CUs %d, reported clock %.0f MHz, %d instructions per wave per kernel\n", cus, clk_khz / 1e3, ITERS * 8);
	printf("%-18s", "cycles/instr/SIMD");
	for (int w = 0; w < nw; ++w) printf("  W=%d waves/SIMD", ws[w]);
	printf("\n");
	for (auto &k : ks) {
		printf("%-18s", k.name);
		for (int w = 0; w < nw; ++w) {
			const int W = ws[w];
			// W waves per SIMD = 4 W per CU: one block of 256 W threads per CU up
			// to 1024, else 4W/16 blocks of 1024 per CU
			const int threads = W <= 4 ? 256 * W : 1024, blocks = W <= 4 ? cus : cus * (W / 4);
			float best = 1e30f;
			for (int rep = 0; rep < 5; ++rep) {
				hipEventRecord(e0, 0);
				hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (unsigned)rep);
				hipEventRecord(e1, 0);
				hipEventSynchronize(e1);
				float ms;
				hipEventElapsedTime(&ms, e0, e1);
				if (rep && ms < best) best = ms;
			}
			const double instr_per_simd = (double)W * ITERS * 8;
			const double ns_per_instr = best * 1e6 / instr_per_simd;
			printf("  %7.2f (%6.3f ms)", ns_per_instr * 2.4, best);
		}
		printf("\n");
	}
	printf("(cycles at 2.4 GHz per wave-instruction per SIMD; kernel time in parentheses)\n");
	hipFree(out);
	return 0;
}
