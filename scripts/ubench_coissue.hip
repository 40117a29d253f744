// ubench_coissue.hip -- does gfx950 overlap LDS reads (ds_read_b32 /
// ds_read_b128) with VALU issue from other waves, or does a launch that
// mixes them pay the SUM of the two floors?  (VERDICT r03 "next" 2: the
// headline kernel k_ctr_fast_any runs at ~ the sum of its VALU and LDS
// floors)
//
// Each kernel runs ITERS iterations of a fixed body per wave: R LDS reads
// (conflict-free: lane l reads its own bank, as the kernels' 32-replica
// T-tables do) and V VALU ops over 8 independent chains, then
// s_waitcnt lgkmcnt(0) -- the lookups' results are XORed into the chains
// after the wait, as the AES rounds consume theirs.  Timed with HIP events
// at 4 and 8 waves/SIMD over 256 CUs x 4 SIMDs.  Printed: ns per
// iteration per SIMD-wave slot and, for the mixed bodies, the pure-LDS and
// pure-VALU bodies' times and their max and sum.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 1024

#define V_FULL(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_HALF(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define RD32(r, off) asm volatile("ds_read_b32 %0, %1 offset:" #off : "=v"(r) : "v"(addr));
#define RD128(r, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(r) : "v"(addr4));
#define WAIT() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

#define CH8(M) M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)

// NR LDS reads (b32), NV full-rate (HALF=0) or half-rate (HALF=1) VALU ops
// in groups of 8 chains, interleaved read / 8 ops / read / ...
template <int NR, int NV8, int HALF, int B128>
__global__ void __launch_bounds__(1024)
k_mix(uint32_t *out, uint32_t s)
{
	__shared__ uint32_t lds[16384];
	for (int i = threadIdx.x; i < 16384; i += blockDim.x)
		lds[i] = i * 2654435761u ^ s;
	__syncthreads();
	uint32_t a0 = threadIdx.x ^ s, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,
		 a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
	const uint32_t b = s * 7 + threadIdx.x, c = 0x07060504u ^ s;
	const uint32_t addr = ((threadIdx.x & 31) * 4) |
			      ((threadIdx.x >> 6) << 10);
	const uint32_t addr4 = ((threadIdx.x & 7) * 16) |
			       ((threadIdx.x >> 6) << 10);
	uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
	typedef uint32_t u4 __attribute__((ext_vector_type(4)));
	u4 q0 = 0, q1 = 0;
	for (int it = 0; it < ITERS; it++) {
#define STEP(k, r, off)                                                      \
		if (NR > k) {                                                \
			if (B128) { if (k & 1) RD128(q1, off) else RD128(q0, off) } \
			else RD32(r, off)                                    \
		}                                                            \
		if (NV8 > k) { if (HALF) { CH8(V_HALF) } else { CH8(V_FULL) } }
		STEP(0, r0, 0)
		STEP(1, r1, 128)
		STEP(2, r2, 256)
		STEP(3, r3, 384)
		STEP(4, r4, 512)
		STEP(5, r5, 640)
		STEP(6, r6, 768)
		STEP(7, r7, 896)
		for (int k = 8; k < NV8; k++) {
			if (HALF) { CH8(V_HALF) } else { CH8(V_FULL) }
		}
		WAIT()
		a0 ^= r0 ^ q0.x; a1 ^= r1 ^ q0.y; a2 ^= r2 ^ q1.z;
		a3 ^= r3 ^ q1.w; a4 ^= r4; a5 ^= r5; a6 ^= r6; a7 ^= r7;
#undef STEP
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] =
		a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kf)(uint32_t *, uint32_t);

// ns per iteration per wave-slot: kernel time / (ITERS * waves per SIMD),
// i.e. the SIMD's time to run one iteration of every resident wave
static double run(kf f, int wps)
{
	const int blocks = 256 * 4 * wps / (1024 / 64) > 256 ?
			   256 * 4 * wps * 64 / 1024 : 256;
	uint32_t *out;
	hipMalloc(&out, (size_t)blocks * 1024 * 4);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	float ms = 0;
	for (int rep = 0; rep < 3; rep++) {
		hipEventRecord(e0);
		f<<<blocks, 1024>>>(out, rep);
		hipEventRecord(e1);
		hipEventSynchronize(e1);
		hipEventElapsedTime(&ms, e0, e1);
	}
	hipFree(out);
	hipEventDestroy(e0);
	hipEventDestroy(e1);
	// waves per SIMD actually resident: blocks * 16 waves / 1024 SIMDs
	const double w = (double)blocks * 16 / 1024;
	return ms * 1e6 / ITERS / w;
}

#define K(NR, NV8, H, B) k_mix<NR, NV8, H, B>

int main()
{
	int wpss[] = {4, 8};
	for (int w : wpss) {
		(void)run(K(8, 0, 0, 0), w);           /* warm */
		struct row { const char *name; kf mix, lds, valu; } rows[] = {
			{"8 b32 + 16 full (1:2)", K(8, 2, 0, 0), K(8, 0, 0, 0), K(0, 2, 0, 0)},
			{"8 b32 + 24 full (1:3)", K(8, 3, 0, 0), K(8, 0, 0, 0), K(0, 3, 0, 0)},
			{"8 b32 + 64 full (1:8)", K(8, 8, 0, 0), K(8, 0, 0, 0), K(0, 8, 0, 0)},
			{"8 b32 + 16 half (1:2)", K(8, 2, 1, 0), K(8, 0, 0, 0), K(0, 2, 1, 0)},
			{"8 b32 + 24 half (1:3)", K(8, 3, 1, 0), K(8, 0, 0, 0), K(0, 3, 1, 0)},
			{"4 b32 + 32 full (1:8)", K(4, 4, 0, 0), K(4, 0, 0, 0), K(0, 4, 0, 0)},
			{"2 b128 + 16 full", K(2, 2, 0, 1), K(2, 0, 0, 1), K(0, 2, 0, 0)},
			{"4 b128 + 32 full", K(4, 4, 0, 1), K(4, 0, 0, 1), K(0, 4, 0, 0)},
			{"4 b128 + 32 half", K(4, 4, 1, 1), K(4, 0, 0, 1), K(0, 4, 1, 0)},
		};
		for (auto &r : rows) {
			const double m = run(r.mix, w), l = run(r.lds, w),
				     v = run(r.valu, w);
			const double mx = l > v ? l : v, sm = l + v;
			printf("waves/SIMD=%d %-24s mixed %7.2f ns  lds-only %7.2f  "
			       "valu-only %7.2f  max %7.2f  sum %7.2f  "
			       "(mixed-max)/(sum-max) %.2f\n", w, r.name, m, l, v,
			       mx, sm, (m - mx) / (sm - mx > 1e-9 ? sm - mx : 1));
		}
	}
	return 0;
}
