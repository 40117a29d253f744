// ubench_sdwa.hip -- issue rates of the byte-select forms an AES T-table
// address can be built with on gfx950 (SDWA byte selects, v_perm with an
// SGPR selector, v_lshl_or), and the ds_read_b32 rate when the address is
// made by full-rate ops only.  Same harness as ubench_valu.hip: each wave
// runs ITERS x 8 independent chains; every line is the second of two runs.
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_sdwa.hip -o /tmp/ubs
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

#define A_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define A_PERMS(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(sg));
#define A_MOVSDWA(x) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(x) : "v"(b));
#define A_ORSDWA(x) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD" : "+v"(x) : "v"(b));
#define A_LSHLSDWA(x) asm volatile("v_lshlrev_b32_sdwa %0, 8, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "+v"(x));
#define A_LSHL8(x) asm volatile("v_lshlrev_b32 %0, 8, %0" : "+v"(x));
#define A_LSHR8(x) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(x));
#define A_LSHLV(x) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(b));
#define A_BITOP3C(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(x) : "v"(b), "s"(sg));
#define A_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x) : "v"(b));
#define A_BFI(x) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "s"(sg), "v"(b));
#define A_ALIGNB(x) asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(x) : "v"(b));
#define A_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define A_XORSDWA(x) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x) : "v"(b));

DEFK(k_xor, A_XOR)
DEFK(k_perms, A_PERMS)
DEFK(k_movsdwa, A_MOVSDWA)
DEFK(k_orsdwa, A_ORSDWA)
DEFK(k_lshlsdwa, A_LSHLSDWA)
DEFK(k_lshl8, A_LSHL8)
DEFK(k_lshr8, A_LSHR8)
DEFK(k_lshlv, A_LSHLV)
DEFK(k_bitop3c, A_BITOP3C)
DEFK(k_lshlor, A_LSHLOR)
DEFK(k_bfi, A_BFI)
DEFK(k_alignb, A_ALIGNB)
DEFK(k_add3, A_ADD3)
DEFK(k_xorsdwa, A_XORSDWA)

// LDS rate with addresses from full-rate ops: a = bitop3(r, mask, lo)
// (byte 1 of the loaded word in place, lane replica in bytes 0/2)
__global__ void k_lds_fast(uint32_t *out, uint64_t *cyc, uint32_t s)
{
	__shared__ uint32_t t[32768];
	for (int i = threadIdx.x; i < 32768; i += blockDim.x)
		t[i] = i * 2654435761u;
	__syncthreads();
	const uint32_t lo = (threadIdx.x & 31) * 4;
	uint32_t a0 = threadIdx.x * 77 + s, a1 = a0 + 11, a2 = a0 + 23,
		 a3 = a0 + 37, a4 = a0 + 41, a5 = a0 + 43, a6 = a0 + 47,
		 a7 = a0 + 53;
	uint64_t t0 = __builtin_amdgcn_s_memtime();
#define LQ(a) \
	a = *(const uint32_t *)((const char *)t + \
		__builtin_amdgcn_bitop3_b32(a, 0xff00u, lo, 0xec));
	for (int i = 0; i < ITERS; i++) {
		LQ(a0) LQ(a1) LQ(a2) LQ(a3) LQ(a4) LQ(a5) LQ(a6) LQ(a7)
	}
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^
						     a5 ^ a6 ^ a7;
	if ((threadIdx.x & 63) == 0)
		cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

// the same with the replica image the kernels use (lane l: replica l & 31,
// entry stride 256 B, two halves at +0/+128): ds_read_b64 of two entries
__global__ void k_lds_b64(uint32_t *out, uint64_t *cyc, uint32_t s)
{
	__shared__ uint32_t t[32768];
	for (int i = threadIdx.x; i < 32768; i += blockDim.x)
		t[i] = i * 2654435761u;
	__syncthreads();
	const uint32_t lo = (threadIdx.x & 31) * 8;
	uint32_t a0 = threadIdx.x * 77 + s, a1 = a0 + 11, a2 = a0 + 23,
		 a3 = a0 + 37, a4 = a0 + 41, a5 = a0 + 43, a6 = a0 + 47,
		 a7 = a0 + 53;
	uint64_t t0 = __builtin_amdgcn_s_memtime();
#define LQ2(a) { const uint2 v = *(const uint2 *)((const char *)t + \
		__builtin_amdgcn_bitop3_b32(a, 0xff00u, lo, 0xec)); a = v.x ^ v.y; }
	for (int i = 0; i < ITERS; i++) {
		LQ2(a0) LQ2(a1) LQ2(a2) LQ2(a3) LQ2(a4) LQ2(a5) LQ2(a6) LQ2(a7)
	}
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^
						     a5 ^ a6 ^ a7;
	if ((threadIdx.x & 63) == 0)
		cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

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
		run("xor", k_xor, w, 8, 0);
		run("perm_sgpr", k_perms, w, 8, 0);
		run("mov_sdwa", k_movsdwa, w, 8, 0);
		run("or_sdwa", k_orsdwa, w, 8, 0);
		run("lshl_sdwa", k_lshlsdwa, w, 8, 0);
		run("xor_sdwa", k_xorsdwa, w, 8, 0);
		run("lshl8", k_lshl8, w, 8, 0);
		run("lshr8", k_lshr8, w, 8, 0);
		run("lshl_v", k_lshlv, w, 8, 0);
		run("bitop3_s", k_bitop3c, w, 8, 0);
		run("lshl_or", k_lshlor, w, 8, 0);
		run("bfi", k_bfi, w, 8, 0);
		run("alignbyte", k_alignb, w, 8, 0);
		run("add3", k_add3, w, 8, 0);
		run("xor", k_xor, w, 8, 0);
		run("lds_fast", k_lds_fast, w, 8, 1);
		run("lds_b64", k_lds_b64, w, 8, 1);
	}
	return 0;
}
