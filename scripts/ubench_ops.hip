// ubench_ops.hip -- issue rate of single gfx950 VALU instruction forms
// (operand kinds: v = VGPR, s = SGPR, k = constant), 8 independent
// chains per wave (same harness as ubench_sdwa.hip)
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
		uint32_t sg = __builtin_amdgcn_readfirstlane(s * 0x01030507u);     \
		__syncthreads();                                                   \
		uint64_t t0 = __builtin_amdgcn_s_memtime();                        \
		for (int i = 0; i < ITERS; i++) {                                  \
			CH8(ASM)                                                       \
		}                                                                  \
		uint64_t t1 = __builtin_amdgcn_s_memtime();                        \
		out[blockIdx.x * blockDim.x + threadIdx.x] =                       \
			a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b ^ c;                 \
		if ((threadIdx.x & 63) == 0)                                       \
			cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;  \
	}


#define A_xor_vv(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_xor_vv, A_xor_vv)
#define A_xor_sv(x) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "s"(sg));
DEFK(k_xor_sv, A_xor_sv)
#define A_xor_kv(x) asm volatile("v_xor_b32 %0, 0x12345, %0" : "+v"(x));
DEFK(k_xor_kv, A_xor_kv)
#define A_and_kv(x) asm volatile("v_and_b32 %0, 0xff00, %0" : "+v"(x));
DEFK(k_and_kv, A_and_kv)
#define A_or_sv(x) asm volatile("v_or_b32 %0, %1, %0" : "+v"(x) : "s"(sg));
DEFK(k_or_sv, A_or_sv)
#define A_add_sv(x) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "s"(sg));
DEFK(k_add_sv, A_add_sv)
#define A_add_kv(x) asm volatile("v_add_u32 %0, 0x5a827999, %0" : "+v"(x));
DEFK(k_add_kv, A_add_kv)
#define A_mov_v(x) asm volatile("v_mov_b32 %0, %1" : "+v"(x) : "v"(b));
DEFK(k_mov_v, A_mov_v)
#define A_not_v(x) asm volatile("v_not_b32 %0, %0" : "+v"(x));
DEFK(k_not_v, A_not_v)
#define A_lshr_vv(x) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x) : "v"(b));
DEFK(k_lshr_vv, A_lshr_vv)
#define A_lshl_vv(x) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(b));
DEFK(k_lshl_vv, A_lshl_vv)
#define A_lshl_1(x) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x));
DEFK(k_lshl_1, A_lshl_1)
#define A_lshl_16(x) asm volatile("v_lshlrev_b32 %0, 16, %0" : "+v"(x));
DEFK(k_lshl_16, A_lshl_16)
#define A_ashr_8(x) asm volatile("v_ashrrev_i32 %0, 8, %0" : "+v"(x));
DEFK(k_ashr_8, A_ashr_8)
#define A_lshl_b16(x) asm volatile("v_lshlrev_b16 %0, 8, %0" : "+v"(x));
DEFK(k_lshl_b16, A_lshl_b16)
#define A_lshr_b16(x) asm volatile("v_lshrrev_b16 %0, 8, %0" : "+v"(x));
DEFK(k_lshr_b16, A_lshr_b16)
#define A_add_vv_e64(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_add_vv_e64, A_add_vv_e64)
#define A_xor_vv_e64(x) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_xor_vv_e64, A_xor_vv_e64)
#define A_bitop3_vvv96(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_bitop3_vvv96, A_bitop3_vvv96)
#define A_bitop3_vvvec(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_bitop3_vvvec, A_bitop3_vvvec)
#define A_bitop3_vsv(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "s"(sg), "v"(c));
DEFK(k_bitop3_vsv, A_bitop3_vsv)
#define A_bitop3_vvs(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "s"(sg));
DEFK(k_bitop3_vvs, A_bitop3_vvs)
#define A_align_vvv(x) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(x) : "v"(c));
DEFK(k_align_vvv, A_align_vvv)
#define A_align_vvk(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
DEFK(k_align_vvk, A_align_vvk)
#define A_align_vbk(x) asm volatile("v_alignbit_b32 %0, %0, %1, 2" : "+v"(x) : "v"(b));
DEFK(k_align_vbk, A_align_vbk)
#define A_perm_vvv(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_perm_vvv, A_perm_vvv)
#define A_add3_vvv(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_add3_vvv, A_add3_vvv)
#define A_xad_vvv(x) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_xad_vvv, A_xad_vvv)
#define A_and_or_vvv(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_and_or_vvv, A_and_or_vvv)
#define A_or3_vvv(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_or3_vvv, A_or3_vvv)
#define A_lshl_or_vkv(x) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x) : "v"(b));
DEFK(k_lshl_or_vkv, A_lshl_or_vkv)
#define A_lshl_add_vkv(x) asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(x) : "v"(b));
DEFK(k_lshl_add_vkv, A_lshl_add_vkv)
#define A_add_lshl_vvk(x) asm volatile("v_add_lshl_u32 %0, %0, %1, 8" : "+v"(x) : "v"(b));
DEFK(k_add_lshl_vvk, A_add_lshl_vvk)
#define A_bfe_vkk(x) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x));
DEFK(k_bfe_vkk, A_bfe_vkk)
#define A_bfi_vvv(x) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "v"(b), "v"(c));
DEFK(k_bfi_vvv, A_bfi_vvv)
#define A_mul24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_mul24, A_mul24)
#define A_mullo(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_mullo, A_mullo)
#define A_cndmask(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
DEFK(k_cndmask, A_cndmask)
#define A_max_u32(x) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_max_u32, A_max_u32)
#define A_pk_add_u16(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
DEFK(k_pk_add_u16, A_pk_add_u16)
#define A_dpp_xor(x) asm volatile("v_xor_b32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
DEFK(k_dpp_xor, A_dpp_xor)
typedef void (*kf)(uint32_t *, uint64_t *, uint32_t);

static void run(const char *name, kf f, int wps, double per_iter_instr,
		int lds)
{
	const int cus = 256 * (wps > 4 ? wps / 4 : 1),
		  threads = 64 * 4 * (wps > 4 ? 4 : wps);
	uint32_t *out;
	uint64_t *cyc;
	hipMalloc(&out, (size_t)cus * threads * 4);
	hipMalloc(&cyc, (size_t)cus * threads / 64 * 8);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	float ms = 0;
	for (int rep = 0; rep < 2; rep++) {
		f<<<cus, threads>>>(out, cyc, 1);
		hipEventRecord(e0);
		f<<<cus, threads>>>(out, cyc, 2);
		hipEventRecord(e1);
		hipEventSynchronize(e1);
		hipEventElapsedTime(&ms, e0, e1);
	}
	int nw = cus * threads / 64;
	uint64_t *h = (uint64_t *)malloc(nw * 8);
	hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
	double avg = 0;
	for (int i = 0; i < nw; i++)
		avg += h[i];
	avg /= nw;
	double instr = per_iter_instr * ITERS;
	double lane_ops = (double)cus * threads * instr;
	printf("%-10s waves/SIMD=%d  ticks/instr/SIMD=%.3f  kernel=%.3f ms  "
	       "%.2f T lane-ops/s%s\n", name, wps, avg / (instr * wps), ms,
	       lane_ops / ms / 1e9, lds ? "  [LDS]" : "");
	free(h);
	hipFree(out);
	hipFree(cyc);
}


int main()
{
	int wpss[] = {4, 8};
	for (int w : wpss) {
		run("warm", k_xor_vv, w, 8, 0);
		run("xor_vv", k_xor_vv, w, 8, 0);
		run("xor_sv", k_xor_sv, w, 8, 0);
		run("xor_kv", k_xor_kv, w, 8, 0);
		run("and_kv", k_and_kv, w, 8, 0);
		run("or_sv", k_or_sv, w, 8, 0);
		run("add_sv", k_add_sv, w, 8, 0);
		run("add_kv", k_add_kv, w, 8, 0);
		run("mov_v", k_mov_v, w, 8, 0);
		run("not_v", k_not_v, w, 8, 0);
		run("lshr_vv", k_lshr_vv, w, 8, 0);
		run("lshl_vv", k_lshl_vv, w, 8, 0);
		run("lshl_1", k_lshl_1, w, 8, 0);
		run("lshl_16", k_lshl_16, w, 8, 0);
		run("ashr_8", k_ashr_8, w, 8, 0);
		run("lshl_b16", k_lshl_b16, w, 8, 0);
		run("lshr_b16", k_lshr_b16, w, 8, 0);
		run("add_vv_e64", k_add_vv_e64, w, 8, 0);
		run("xor_vv_e64", k_xor_vv_e64, w, 8, 0);
		run("bitop3_vvv96", k_bitop3_vvv96, w, 8, 0);
		run("bitop3_vvvec", k_bitop3_vvvec, w, 8, 0);
		run("bitop3_vsv", k_bitop3_vsv, w, 8, 0);
		run("bitop3_vvs", k_bitop3_vvs, w, 8, 0);
		run("align_vvv", k_align_vvv, w, 8, 0);
		run("align_vvk", k_align_vvk, w, 8, 0);
		run("align_vbk", k_align_vbk, w, 8, 0);
		run("perm_vvv", k_perm_vvv, w, 8, 0);
		run("add3_vvv", k_add3_vvv, w, 8, 0);
		run("xad_vvv", k_xad_vvv, w, 8, 0);
		run("and_or_vvv", k_and_or_vvv, w, 8, 0);
		run("or3_vvv", k_or3_vvv, w, 8, 0);
		run("lshl_or_vkv", k_lshl_or_vkv, w, 8, 0);
		run("lshl_add_vkv", k_lshl_add_vkv, w, 8, 0);
		run("add_lshl_vvk", k_add_lshl_vvk, w, 8, 0);
		run("bfe_vkk", k_bfe_vkk, w, 8, 0);
		run("bfi_vvv", k_bfi_vvv, w, 8, 0);
		run("mul24", k_mul24, w, 8, 0);
		run("mullo", k_mullo, w, 8, 0);
		run("cndmask", k_cndmask, w, 8, 0);
		run("max_u32", k_max_u32, w, 8, 0);
		run("pk_add_u16", k_pk_add_u16, w, 8, 0);
		run("dpp_xor", k_dpp_xor, w, 8, 0);
	}
	return 0;
}
