// ubench_valu.hip -- issue rate of the integer VALU / LDS instructions the
// SRTP kernels are built from, on gfx950.  Each wave runs ITERS x 8
// independent chains of one instruction; waves record s_memtime deltas.
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_valu.hip -o /tmp/ubv
//   /tmp/ubv            -> one line per instruction: cycles per wave-instr
//                          per SIMD at W waves/SIMD, and lane-ops/s chip-wide
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 2048

#define CH8(OP)                                                            \
	OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define DEFK(NAME, ASM)                                                    \
	__global__ void NAME(uint32_t *out, uint64_t *cyc, uint32_t s)         \
	{                                                                      \
		uint32_t a0 = threadIdx.x ^ s, a1 = a0 + 1, a2 = a0 + 2,           \
			 a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,           \
			 a7 = a0 + 7;                                                  \
		uint32_t b = s * 7 + threadIdx.x, c = s * 13;                      \
		__syncthreads();                                                   \
		uint64_t t0 = __builtin_amdgcn_s_memtime();                        \
		for (int i = 0; i < ITERS; i++) {                                  \
			CH8(ASM)                                                       \
		}                                                                  \
		uint64_t t1 = __builtin_amdgcn_s_memtime();                        \
		out[blockIdx.x * blockDim.x + threadIdx.x] =                       \
			a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                         \
		if ((threadIdx.x & 63) == 0)                                       \
			cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;  \
	}

#define A_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define A_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define A_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define A_ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
#define A_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
#define A_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b));
#define A_ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define A_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define A_BFE(x) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x));
#define A_PKADD(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
#define A_LSHL(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
#define A_LSHR(x) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x));
#define A_OR(x) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define A_AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define A_DPP(x) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
#define A_LSHLADD(x) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x) : "v"(b));
#define A_MIX_PX(x) asm volatile("v_perm_b32 %0, %0, %1, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b), "v"(c));
#define A_MIX_AX(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));

DEFK(k_xor, A_XOR)
DEFK(k_add3, A_ADD3)
DEFK(k_perm, A_PERM)
DEFK(k_align, A_ALIGN)
DEFK(k_bitop3, A_BITOP3)
DEFK(k_lshlor, A_LSHLOR)
DEFK(k_andor, A_ANDOR)
DEFK(k_add, A_ADD)
DEFK(k_bfe, A_BFE)
DEFK(k_pkadd, A_PKADD)
DEFK(k_lshl, A_LSHL)
DEFK(k_lshr, A_LSHR)
DEFK(k_or, A_OR)
DEFK(k_and, A_AND)
DEFK(k_dpp, A_DPP)
DEFK(k_lshladd, A_LSHLADD)
DEFK(k_mixpx, A_MIX_PX)
DEFK(k_mixax, A_MIX_AX)

// LDS: ds_read_b32 from a 32-replica image (conflict-free random reads)
__global__ void k_lds(uint32_t *out, uint64_t *cyc, uint32_t s)
{
	__shared__ uint32_t t[16384];
	for (int i = threadIdx.x; i < 16384; i += blockDim.x)
		t[i] = i * 2654435761u;
	__syncthreads();
	const uint32_t lo = (threadIdx.x & 31) * 4;
	uint32_t a0 = threadIdx.x * 77 + s, a1 = a0 + 11, a2 = a0 + 23,
		 a3 = a0 + 37;
	uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int i = 0; i < ITERS; i++) {
		uint32_t r0 = *(const uint32_t *)((const char *)t +
			__builtin_amdgcn_perm(a0, lo, 0x0C0C0500u));
		uint32_t r1 = *(const uint32_t *)((const char *)t +
			__builtin_amdgcn_perm(a1, lo, 0x0C0C0500u));
		uint32_t r2 = *(const uint32_t *)((const char *)t +
			__builtin_amdgcn_perm(a2, lo, 0x0C0C0500u));
		uint32_t r3 = *(const uint32_t *)((const char *)t +
			__builtin_amdgcn_perm(a3, lo, 0x0C0C0500u));
		a0 ^= r0 >> 3; a1 ^= r1 >> 5; a2 ^= r2 >> 7; a3 ^= r3 >> 9;
	}
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
	if ((threadIdx.x & 63) == 0)
		cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

typedef void (*kf)(uint32_t *, uint64_t *, uint32_t);

static void run(const char *name, kf f, int wps, double per_iter_instr,
		double lds_per_iter)
{
	// one block per CU up to 4 waves/SIMD, two for 8
	const int cus = 256 * (wps > 4 ? wps / 4 : 1),
		  threads = 64 * 4 * (wps > 4 ? 4 : wps);
	uint32_t *out;
	uint64_t *cyc;
	hipMalloc(&out, (size_t)cus * threads * 4);
	hipMalloc(&cyc, (size_t)cus * threads / 64 * 8);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	f<<<cus, threads>>>(out, cyc, 1);
	hipEventRecord(e0);
	f<<<cus, threads>>>(out, cyc, 2);
	hipEventRecord(e1);
	hipEventSynchronize(e1);
	float ms;
	hipEventElapsedTime(&ms, e0, e1);
	int nw = cus * threads / 64;
	uint64_t *h = (uint64_t *)malloc(nw * 8);
	hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
	double avg = 0;
	for (int i = 0; i < nw; i++)
		avg += h[i];
	avg /= nw;
	double instr = per_iter_instr * ITERS;
	// waves per SIMD run concurrently: SIMD cycles per wave-instruction
	double lane_ops = (double)cus * threads * instr;
	printf("%-8s waves/SIMD=%d  memtime/wave=%.0f  cyc/instr/SIMD=%.3f "
	       "(memtime ticks)  kernel=%.3f ms  %.2f T lane-ops/s%s\n",
	       name, wps, avg, avg / (instr * wps), ms, lane_ops / ms / 1e9,
	       lds_per_iter ? "  [LDS]" : "");
	free(h);
	hipFree(out);
	hipFree(cyc);
}

int main()
{
	int wpss[] = {1, 2, 4, 8};
	for (int w : wpss) {
		run("xor", k_xor, w, 8, 0);
		run("add", k_add, w, 8, 0);
		run("add3", k_add3, w, 8, 0);
		run("perm", k_perm, w, 8, 0);
		run("align", k_align, w, 8, 0);
		run("bitop3", k_bitop3, w, 8, 0);
		run("lshl_or", k_lshlor, w, 8, 0);
		run("and_or", k_andor, w, 8, 0);
		run("bfe", k_bfe, w, 8, 0);
		run("pk_add", k_pkadd, w, 8, 0);
		run("lshl", k_lshl, w, 8, 0);
		run("lshr", k_lshr, w, 8, 0);
		run("or", k_or, w, 8, 0);
		run("and", k_and, w, 8, 0);
		run("dpp_mov", k_dpp, w, 8, 0);
		run("lshl_add", k_lshladd, w, 8, 0);
		run("perm+xor", k_mixpx, w, 16, 0);
		run("align+bitop3", k_mixax, w, 16, 0);
		run("ds_b32", k_lds, w, 4, 4);
	}
	return 0;
}
