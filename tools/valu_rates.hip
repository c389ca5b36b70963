// valu_rates.hip -- issue cost of the VALU instructions the counting kernel
// uses, measured on the device (tools only, never shipped).  Every wave runs
// 8 independent chains of one instruction (inline asm, so the compiler keeps
// exactly that instruction), 16 waves per CU (4 per SIMD) on every CU; the
// time per instruction per SIMD is kernel time / (4 waves * instructions per
// wave).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rates tools/valu_rates.hip && tools/valu_rates
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 4096

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

int main()
{
	int cus = 0;
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
	int clk_khz = 0;
	hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
	unsigned *out;
	const int blocks = cus;     // one 1024-thread block (16 waves = 4 per SIMD) per CU
	hipMalloc(&out, (size_t)blocks * 1024 * 4);
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
	printf("CUs %d, reported clock %.0f MHz, %d instructions per wave per kernel\n", cus, clk_khz / 1e3, ITERS * 8);
	for (auto &k : ks) {
		float best = 1e30f;
		for (int rep = 0; rep < 5; ++rep) {
			hipEventRecord(e0, 0);
			hipLaunchKernelGGL(k.f, dim3(blocks), dim3(1024), 0, 0, out, (unsigned)rep);
			hipEventRecord(e1, 0);
			hipEventSynchronize(e1);
			float ms;
			hipEventElapsedTime(&ms, e0, e1);
			if (rep && ms < best) best = ms;
		}
		const double instr_per_simd = 4.0 * ITERS * 8;     // 4 waves per SIMD
		const double ns_per_instr = best * 1e6 / instr_per_simd;
		printf("%-18s %8.3f ms  %.3f ns per wave-instruction per SIMD  (%.2f cycles at 2.4 GHz)\n", k.name, best,
		       ns_per_instr, ns_per_instr * 2.4);
	}
	hipFree(out);
	return 0;
}
