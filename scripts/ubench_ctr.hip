// ubench_ctr.hip -- where the time of the fused CTR+HMAC kernel goes.
// Runs the kernel's own building blocks (re_amd/csrc/hip: CtrKs T4 cached
// keystream, sha1_compress) per lane over 1M lanes x 19 chunks (a 1200-B
// SRTP packet), without / with the packet memory traffic:
//   aes   : keystream only           sha   : SHA-1 only
//   both  : keystream + SHA-1         mem   : both + 64-B load/store/chunk
//   wave-per-packet: one packet per wavefront (k_wave), the alternative
//                    layout north_star names, for comparison
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Ire_amd/csrc -Iinclude \
//         scripts/ubench_ctr.hip -o /tmp/ubc && /tmp/ubc
#include "hip/kern_common.h"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define NCH 19
#define BLK 1024

enum { M_AES = 1, M_SHA = 2, M_MEM = 4, M_COAL = 8, M_QUAD = 16, M_S16 = 32,
       M_XPQ = 64, M_XP16 = 128 };

/* 4x4 transpose (register r, lane group position) by permlane swaps:
 * group = lanes {i, i+16, i+32, i+48}; stage 1 swaps bit 1, stage 2 bit 0 */
__device__ __forceinline__ void s16_transpose(uint32_t x[4][4])
{
#pragma unroll
	for (int c = 0; c < 4; c++) {
#pragma unroll
		for (int r = 0; r < 2; r++) {
			auto v = __builtin_amdgcn_permlane32_swap(x[r][c], x[r + 2][c],
								  false, false);
			x[r][c] = v[0]; x[r + 2][c] = v[1];
		}
#pragma unroll
		for (int r = 0; r < 4; r += 2) {
			auto v = __builtin_amdgcn_permlane16_swap(x[r][c], x[r + 1][c],
								  false, false);
			x[r][c] = v[0]; x[r + 1][c] = v[1];
		}
	}
}

template <int MODE>
__global__ void __launch_bounds__(BLK) k_ub(const uint32_t *T0g,
					   const uint32_t *rkg, uint8_t *arena,
					   uint32_t *out)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	tt4_fill(smem, T0g);
	__syncthreads();
	const uint32_t t = blockIdx.x * BLK + threadIdx.x;
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	uint32_t rk[44];
#pragma unroll
	for (int k = 0; k < 44; k++)
		rk[k] = __builtin_amdgcn_readfirstlane(rkg[k]);
	uint32_t iv[4] = {t * 0x9e3779b9u, t ^ 0x12345678u, t * 7u, 0};
	CtrKs<10, true, true> C;
	C.init(smem, lo, rk, iv);
	uint32_t h[5] = {t, 1, 2, 3, 4}, carry[4] = {0, 0, 0, 0}, ks[16];
	uint32_t acc = 0;
	uint8_t *pkt = arena + (size_t)t * 1216;
	/* M_COAL: same bytes per wave, lane-contiguous (coalesced) */
	uint8_t *wbase = arena + (size_t)(t & ~63u) * 1216 + (t & 63u) * 16;
	/* M_QUAD: access g, lane 4a+j -> packet 4a+g, quarter j;
	 * M_S16: access g, lane 16q+i -> packet 16g+i, quarter q */
	const uint32_t L = t & 63u, wp = t & ~63u;
	uint8_t *qb[4];
#pragma unroll
	for (int g = 0; g < 4; g++)
		qb[g] = (MODE & M_QUAD) ?
			arena + (size_t)(wp + (L & ~3u) + g) * 1216 + 16 * (L & 3u) :
			arena + (size_t)(wp + 16 * g + (L & 15u)) * 1216 + 16 * (L >> 4);
	for (int k = 0; k < NCH; k++) {
		uint32_t d[16];
		if (MODE & M_MEM) {
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = (MODE & M_COAL) ?
					*(const uint4 *)(wbase + 4096 * k + 1024 * g) :
					(MODE & (M_QUAD | M_S16)) ?
					*(const uint4 *)(qb[g] + 64 * k) :
					*(const uint4 *)(pkt + 64 * k + 16 * g);
				d[4 * g] = v.x; d[4 * g + 1] = v.y;
				d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
			}
			if (MODE & (M_XPQ | M_XP16)) {
				uint32_t x[4][4];
#pragma unroll
				for (int q = 0; q < 16; q++)
					x[q >> 2][q & 3] = d[q];
				if (MODE & M_XPQ)
					quad_transpose(x, L);
				else
					s16_transpose(x);
#pragma unroll
				for (int q = 0; q < 16; q++)
					d[q] = x[q >> 2][q & 3];
			}
		} else {
#pragma unroll
			for (int q = 0; q < 16; q++)
				d[q] = t + k * 16 + q;
		}
		if (MODE & M_AES) {
			chunk_ks<10, 3>(smem, lo, rk, C, 4 * k, carry, ks);
#pragma unroll
			for (int q = 0; q < 16; q++)
				d[q] ^= ks[q];
		}
		if (MODE & M_MEM) {
			if (MODE & (M_XPQ | M_XP16)) {
				uint32_t x[4][4];
#pragma unroll
				for (int q = 0; q < 16; q++)
					x[q >> 2][q & 3] = d[q];
				if (MODE & M_XPQ)
					quad_transpose(x, L);
				else
					s16_transpose(x);
#pragma unroll
				for (int q = 0; q < 16; q++)
					d[q] = x[q >> 2][q & 3];
			}
#pragma unroll
			for (int g = 0; g < 4; g++)
				*(uint4 *)((MODE & M_COAL) ? wbase + 4096 * k + 1024 * g
					   : (MODE & (M_QUAD | M_S16)) ? qb[g] + 64 * k
					   : pkt + 64 * k + 16 * g) =
					make_uint4(d[4 * g], d[4 * g + 1],
						   d[4 * g + 2], d[4 * g + 3]);
		}
		if (MODE & M_SHA) {
			uint32_t w[16];
#pragma unroll
			for (int q = 0; q < 16; q++)
				w[q] = bswap32(d[q]);
			sha1_compress(h, w);
		} else {
#pragma unroll
			for (int q = 0; q < 16; q++)
				acc ^= d[q];
		}
	}
	out[t] = acc ^ h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

/*
 * The north_star's literal layout: one packet per wavefront.  Lane l
 * computes the keystream of 64-byte chunk l (lanes 0..18 of a 1200-B
 * packet; the rest idle) and moves that chunk (coalesced across the wave);
 * then the HMAC's SHA-1 chain runs chunk by chunk with the 16 message
 * words broadcast from the owning lane by wavefront shuffles -- every lane
 * computes the same 80 dependent rounds.  SHA1_ONLY: no keystream.
 */
template <bool SHA1_ONLY>
__global__ void __launch_bounds__(BLK) k_wave(const uint32_t *T0g,
					     const uint32_t *rkg,
					     uint8_t *arena, uint32_t *out)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	tt4_fill(smem, T0g);
	__syncthreads();
	const uint32_t L = threadIdx.x & 63u;
	const uint32_t p = (blockIdx.x * BLK + threadIdx.x) >> 6;  /* packet */
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	uint32_t rk[44];
#pragma unroll
	for (int k = 0; k < 44; k++)
		rk[k] = __builtin_amdgcn_readfirstlane(rkg[k]);
	uint8_t *pkt = arena + (size_t)p * 1216;
	uint32_t d[16];
	if (L < NCH) {
#pragma unroll
		for (int g = 0; g < 4; g++) {
			const uint4 v = *(const uint4 *)(pkt + 64 * L + 16 * g);
			d[4 * g] = v.x; d[4 * g + 1] = v.y;
			d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
		}
		if (!SHA1_ONLY) {
			uint32_t iv[4] = {p * 0x9e3779b9u, p ^ 0x12345678u, p * 7u, 0};
			CtrKs<10, true, true> C;
			C.init(smem, lo, rk, iv);
			uint32_t carry[4] = {0, 0, 0, 0}, ks[16];
			chunk_ks<10, 3>(smem, lo, rk, C, 4 * L, carry, ks);
#pragma unroll
			for (int q = 0; q < 16; q++)
				d[q] ^= ks[q];
		}
#pragma unroll
		for (int g = 0; g < 4; g++)
			*(uint4 *)(pkt + 64 * L + 16 * g) =
				make_uint4(d[4 * g], d[4 * g + 1], d[4 * g + 2],
					   d[4 * g + 3]);
	}
	uint32_t h[5] = {p, 1, 2, 3, 4};
	for (int k = 0; k < NCH; k++) {
		uint32_t w[16];
#pragma unroll
		for (int q = 0; q < 16; q++)
			w[q] = bswap32((uint32_t)__shfl((int)d[q], k));
		sha1_compress(h, w);
	}
	if (L == 0)
		out[p] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

template <bool SHA1_ONLY>
static float run_wave(const uint32_t *T0, const uint32_t *rk, uint8_t *arena,
		      uint32_t *out, int n)
{
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int nb = n / (BLK / 64);
	k_wave<SHA1_ONLY><<<nb, BLK>>>(T0, rk, arena, out);
	hipEventRecord(a);
	for (int i = 0; i < 2; i++)
		k_wave<SHA1_ONLY><<<nb, BLK>>>(T0, rk, arena, out);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms / 2;
}

static uint32_t sbox(int x)
{
	/* AES S-box by inversion + affine map (FIPS-197 5.1.1) */
	uint8_t p = 1, q = 1, s[256];
	s[0] = 0x63;
	do {
		p = p ^ (p << 1) ^ (p & 0x80 ? 0x1B : 0);
		q ^= q << 1; q ^= q << 2; q ^= q << 4;
		q ^= q & 0x80 ? 0x09 : 0;
		uint8_t r = q ^ (q << 1 | q >> 7) ^ (q << 2 | q >> 6) ^
			    (q << 3 | q >> 5) ^ (q << 4 | q >> 4);
		s[p] = r ^ 0x63;
	} while (p != 1);
	return s[x];
}

template <int MODE>
static float run(const uint32_t *T0, const uint32_t *rk, uint8_t *arena,
		 uint32_t *out, int n)
{
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	k_ub<MODE><<<n / BLK, BLK>>>(T0, rk, arena, out);
	hipEventRecord(a);
	for (int i = 0; i < 5; i++)
		k_ub<MODE><<<n / BLK, BLK>>>(T0, rk, arena, out);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms / 5;
}

int main()
{
	const int n = 1 << 20;
	std::vector<uint32_t> T0(256), rk(44);
	for (int x = 0; x < 256; x++) {
		uint32_t s = sbox(x), s2 = (s << 1) ^ (s & 0x80 ? 0x1B : 0);
		s2 &= 0xff;
		T0[x] = s2 | s << 8 | s << 16 | (s2 ^ s) << 24;
	}
	for (int i = 0; i < 44; i++)
		rk[i] = 0x01010101u * i;
	uint32_t *T0d, *rkd, *out;
	uint8_t *arena;
	hipMalloc(&T0d, 1024);
	hipMalloc(&rkd, 176);
	hipMalloc(&out, n * 4);
	hipMalloc(&arena, (size_t)n * 1216);
	hipMemcpy(T0d, T0.data(), 1024, hipMemcpyHostToDevice);
	hipMemcpy(rkd, rk.data(), 176, hipMemcpyHostToDevice);
	hipMemset(arena, 1, (size_t)n * 1216);
	printf("aes  %.3f ms\n", run<M_AES>(T0d, rkd, arena, out, n));
	printf("sha  %.3f ms\n", run<M_SHA>(T0d, rkd, arena, out, n));
	printf("both %.3f ms\n", run<M_AES | M_SHA>(T0d, rkd, arena, out, n));
	printf("mem  %.3f ms\n", run<M_AES | M_SHA | M_MEM>(T0d, rkd, arena,
							     out, n));
	printf("aes+mem %.3f ms\n", run<M_AES | M_MEM>(T0d, rkd, arena, out, n));
	printf("mem-coalesced %.3f ms\n", run<M_AES | M_SHA | M_MEM | M_COAL>(
						   T0d, rkd, arena, out, n));
	const int B = M_AES | M_SHA | M_MEM;
	printf("quad addr %.3f ms\n", run<B | M_QUAD>(T0d, rkd, arena, out, n));
	printf("s16 addr %.3f ms\n", run<B | M_S16>(T0d, rkd, arena, out, n));
	printf("quad+xpose %.3f ms\n", run<B | M_QUAD | M_XPQ>(T0d, rkd, arena, out, n));
	printf("s16+xpose %.3f ms\n", run<B | M_S16 | M_XP16>(T0d, rkd, arena, out, n));
	printf("wave-per-packet sha %.3f ms\n", run_wave<true>(T0d, rkd, arena,
								   out, n));
	printf("wave-per-packet aes+sha+mem %.3f ms\n",
	       run_wave<false>(T0d, rkd, arena, out, n));
	return 0;
}
