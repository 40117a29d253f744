/*
 * dev_common.h -- CDNA4 device primitives for the SRTP kernels.
 *
 * AES (FIPS-197) as a one-T-table cipher whose table lives in LDS:
 *   - T0[x] = (2s, s, s, 3s) and T1 = rotl8(T0), s = S[x], as LE words.
 *   - LDS image: 256 entries x 256 B.  Entry e holds 32 replicas of T0[e]
 *     at bytes [0,128) and 32 replicas of T1[e] at [128,256).  Lane l reads
 *     replica (l & 31): a ds_read_b32 wave-instruction is serviced as two
 *     32-lane groups over 32 banks, so every lane of a group hits its own
 *     bank whatever the table index -> conflict-free random lookups.
 *   - Address generation is one v_perm_b32: ((byte k of x) << 8) | lane*4.
 *   - A middle round column is T0[a]^T1[b]^rotl16(T0[c]^T1[d]^rotl16(rk)),
 *     so round keys for rounds 1..nr-1 are stored pre-rotated (rk16).
 * SHA-1 (FIPS 180-4) with a rolling 16-word schedule, one packet per lane.
 * GHASH (SP 800-38D) with OpenSSL's 4-bit Shoup table (gcm_gmult_4bit
 * layout: i*H table + rem_4bit reduction), table in LDS.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TT_BYTES 65536u

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n)
{
	return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

__device__ __forceinline__ uint32_t rot16(uint32_t x)
{
	return __builtin_amdgcn_alignbit(x, x, 16);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
	return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

/* gfx950 v_bitop3_b32: bit = TT[(a << 2) | (b << 1) | c] */
/*
 * gfx950 VALU issue (scripts/ubench_ops.hip, profiles/r03_ubench_ops.txt):
 * v_xor/or/and/add/mov/lshrrev_b32, v_lshlrev_b16 and v_bitop3_b32 with
 * VGPR (or, VOP2, constant) operands issue at the full rate; any VALU op
 * reading an SGPR, and v_perm, v_alignbit, v_add3, v_lshlrev_b32, v_bfe,
 * DPP, at about 0.6 of it.  vreg() hands a uniform value (a round key, a
 * mask) to its users through a VGPR (a pure asm: copies of one value are
 * merged, loop-invariant ones hoisted), so e.g. the four blocks of a chunk
 * XOR a round key with full-rate v_bitop3 (RK_VCOPY).
 */
#ifndef RK_VCOPY
#define RK_VCOPY 0
#endif
__device__ __forceinline__ uint32_t vreg(uint32_t k)
{
	asm("" : "+v"(k));
	return k;
}

__device__ __forceinline__ uint32_t rkv(uint32_t k)
{
#if RK_VCOPY
	return vreg(k);
#else
	return k;
#endif
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

/* SHA-1 Ch(b,c,d) = b ? c : d, Maj(b,c,d) (FIPS 180-4 4.1.1) */
__device__ __forceinline__ uint32_t sha_ch(uint32_t b, uint32_t c, uint32_t d)
{
	return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);
}

__device__ __forceinline__ uint32_t sha_maj(uint32_t b, uint32_t c, uint32_t d)
{
	return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);
}

/* LDS T-table address of byte k of x for this lane (laneoff = (lane&31)*4):
 * ((byte k of x) << 8) | laneoff, one v_perm_b32 (half rate).  Byte 1 is
 * already in place: TT_B1_BITOP3 makes it one v_bitop3_b32 ((x & 0xff00) |
 * laneoff) -- 1: the mask as a constant (the compiler puts it in an SGPR,
 * which makes the op half rate again: no gain), 2 (default): the mask in
 * a VGPR, full rate.  Same-box A/B (profiles/r03_ab_b1v.txt): config-2
 * unprotect 1.244 -> 1.221 ms; GCM (LDS-bound) unchanged. */
#ifndef TT_B1_BITOP3
#define TT_B1_BITOP3 2
#endif
template <int K>
__device__ __forceinline__ uint32_t tt_addr(uint32_t x, uint32_t laneoff)
{
	if (K == 1 && TT_B1_BITOP3 == 1)
		return __builtin_amdgcn_bitop3_b32(x, 0xff00u, laneoff, 0xEA);
	/* 2: the mask in a VGPR (full-rate v_bitop3, see vreg) */
	if (K == 1 && TT_B1_BITOP3 == 2)
		return __builtin_amdgcn_bitop3_b32(x, vreg(0xff00u), laneoff,
						   0xEA);
	return __builtin_amdgcn_perm(x, laneoff, 0x0C0C0000u | ((4u + K) << 8));
}
#define TT_ADDR(x, k, laneoff) tt_addr<(k)>((x), (laneoff))

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *smem, uint32_t a)
{
	return *(const uint32_t *)(smem + a);
}

/* Fill the replicated T0/T1 image (all threads of the block) */
__device__ __forceinline__ void tt_fill(uint8_t *smem, const uint32_t *T0g)
{
	uint32_t *s = (uint32_t *)smem;
	for (uint32_t i = threadIdx.x; i < TT_BYTES / 4; i += blockDim.x) {
		uint32_t e = i >> 6, r = i & 63;
		uint32_t t = T0g[e];
		s[i] = r < 32 ? t : rotl32(t, 8);
	}
}

/* tt_fill for 1024-thread blocks: thread t's 16 words are entries
 * (t >> 6) + 16 j of T0 (uniform per wave), loads issued together, then
 * the stores (see tt4_fill_b1024) */
__device__ __forceinline__ void tt_fill_b1024(uint8_t *smem,
					      const uint32_t *T0g)
{
	uint32_t *s = (uint32_t *)smem;
	const uint32_t tid = threadIdx.x;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	const bool rot = (tid & 63u) >= 32u;
	uint32_t t[16];
#pragma unroll
	for (int j = 0; j < 16; j++)
		t[j] = T0g[wv + 16u * (uint32_t)j];
#pragma unroll
	for (int j = 0; j < 16; j++)
		s[tid + 1024u * (uint32_t)j] = rot ? rotl32(t[j], 8) : t[j];
}

/* one middle round r (1 <= r < NR) on (s0..s3); k = rk + 4r (rot16'd) */
__device__ __forceinline__ void aes_round(const uint8_t *smem, uint32_t lo,
					  const uint32_t *k, uint32_t &s0,
					  uint32_t &s1, uint32_t &s2,
					  uint32_t &s3)
{
	uint32_t a0 = lds_u32(smem, TT_ADDR(s0, 0, lo));
	uint32_t b1 = lds_u32(smem, TT_ADDR(s1, 1, lo) + 128);
	uint32_t c2 = lds_u32(smem, TT_ADDR(s2, 2, lo));
	uint32_t d3 = lds_u32(smem, TT_ADDR(s3, 3, lo) + 128);
	uint32_t a1 = lds_u32(smem, TT_ADDR(s1, 0, lo));
	uint32_t b2 = lds_u32(smem, TT_ADDR(s2, 1, lo) + 128);
	uint32_t c3 = lds_u32(smem, TT_ADDR(s3, 2, lo));
	uint32_t d0 = lds_u32(smem, TT_ADDR(s0, 3, lo) + 128);
	uint32_t a2 = lds_u32(smem, TT_ADDR(s2, 0, lo));
	uint32_t b3 = lds_u32(smem, TT_ADDR(s3, 1, lo) + 128);
	uint32_t c0 = lds_u32(smem, TT_ADDR(s0, 2, lo));
	uint32_t d1 = lds_u32(smem, TT_ADDR(s1, 3, lo) + 128);
	uint32_t a3 = lds_u32(smem, TT_ADDR(s3, 0, lo));
	uint32_t b0 = lds_u32(smem, TT_ADDR(s0, 1, lo) + 128);
	uint32_t c1 = lds_u32(smem, TT_ADDR(s1, 2, lo));
	uint32_t d2 = lds_u32(smem, TT_ADDR(s2, 3, lo) + 128);
	s0 = xor3(a0, b1, rot16(xor3(c2, d3, rkv(k[0]))));
	s1 = xor3(a1, b2, rot16(xor3(c3, d0, rkv(k[1]))));
	s2 = xor3(a2, b3, rot16(xor3(c0, d1, rkv(k[2]))));
	s3 = xor3(a3, b0, rot16(xor3(c1, d2, rkv(k[3]))));
}

/* final round (SubBytes, ShiftRows, AddRoundKey; k plain) */
__device__ __forceinline__ void aes_final(const uint8_t *smem, uint32_t lo,
					  const uint32_t *k, uint32_t &s0,
					  uint32_t &s1, uint32_t &s2,
					  uint32_t &s3)
{
	/* S[x] = byte1 of T0[x] = byte2 of T0[x] = byte3 of T1[x] */
	uint32_t a0 = lds_u32(smem, TT_ADDR(s0, 0, lo));
	uint32_t b1 = lds_u32(smem, TT_ADDR(s1, 1, lo));
	uint32_t c2 = lds_u32(smem, TT_ADDR(s2, 2, lo));
	uint32_t d3 = lds_u32(smem, TT_ADDR(s3, 3, lo) + 128);
	uint32_t a1 = lds_u32(smem, TT_ADDR(s1, 0, lo));
	uint32_t b2 = lds_u32(smem, TT_ADDR(s2, 1, lo));
	uint32_t c3 = lds_u32(smem, TT_ADDR(s3, 2, lo));
	uint32_t d0 = lds_u32(smem, TT_ADDR(s0, 3, lo) + 128);
	uint32_t a2 = lds_u32(smem, TT_ADDR(s2, 0, lo));
	uint32_t b3 = lds_u32(smem, TT_ADDR(s3, 1, lo));
	uint32_t c0 = lds_u32(smem, TT_ADDR(s0, 2, lo));
	uint32_t d1 = lds_u32(smem, TT_ADDR(s1, 3, lo) + 128);
	uint32_t a3 = lds_u32(smem, TT_ADDR(s3, 0, lo));
	uint32_t b0 = lds_u32(smem, TT_ADDR(s0, 1, lo));
	uint32_t c1 = lds_u32(smem, TT_ADDR(s1, 2, lo));
	uint32_t d2 = lds_u32(smem, TT_ADDR(s2, 3, lo) + 128);
	s0 = xor3(__builtin_amdgcn_perm(a0, b1, 0x0C0C0105u),
		  __builtin_amdgcn_perm(c2, d3, 0x03060C0Cu), rkv(k[0]));
	s1 = xor3(__builtin_amdgcn_perm(a1, b2, 0x0C0C0105u),
		  __builtin_amdgcn_perm(c3, d0, 0x03060C0Cu), rkv(k[1]));
	s2 = xor3(__builtin_amdgcn_perm(a2, b3, 0x0C0C0105u),
		  __builtin_amdgcn_perm(c0, d1, 0x03060C0Cu), rkv(k[2]));
	s3 = xor3(__builtin_amdgcn_perm(a3, b0, 0x0C0C0105u),
		  __builtin_amdgcn_perm(c1, d2, 0x03060C0Cu), rkv(k[3]));
}

/* rounds FIRST .. NR on a state that has been through rounds 0..FIRST-1 */
template <int NR, int FIRST>
__device__ __forceinline__ void aes_rounds(const uint8_t *smem, uint32_t lo,
					   const uint32_t *rk, uint32_t &s0,
					   uint32_t &s1, uint32_t &s2,
					   uint32_t &s3)
{
#pragma unroll
	for (int r = FIRST; r < NR; r++)
		aes_round(smem, lo, rk + 4 * r, s0, s1, s2, s3);
	aes_final(smem, lo, rk + 4 * NR, s0, s1, s2, s3);
}

/*
 * One AES block encryption.  rk: 4*(NR+1) words; words 4..4*NR-1 (rounds
 * 1..NR-1) are rot16'd, round 0 and NR are plain.
 */
template <int NR>
__device__ __forceinline__ void aes_block(const uint8_t *smem, uint32_t lo,
					  const uint32_t *rk, uint32_t &s0,
					  uint32_t &s1, uint32_t &s2,
					  uint32_t &s3)
{
	s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
	aes_rounds<NR, 1>(smem, lo, rk, s0, s1, s2, s3);
}

/*
 * Four-table AES ("T4"): 128 KiB LDS image, no rotations in the rounds.
 *   - half 0 [0, 64 KiB):   T0 at entry*256 + [0,128), T1 at +128
 *   - half 1 [64, 128 KiB): T2 = rotl16(T0) at +0,     T3 = rotl24(T0) at +128
 *   each as 32 lane replicas (conflict-free ds_read_b32 like the T0/T1 image).
 *   Half-1 addresses are one v_perm_b32 as well: the lane offset register
 *   hi = lo | 0x10000 supplies byte 2.
 *   A middle round column is xor3(xor3(T0[a], T1[b], T2[c]), T3[d], rk):
 *   16 lookups + 16 address perms + 8 bitop3, round keys plain (the T0/T1
 *   form needs 4 more half-rate v_alignbit per round).
 * Measured on gfx950 (profiles/r01_ubench_valu_rates.log): v_perm_b32,
 * v_alignbit_b32 and v_add3_u32 issue at half the rate of v_xor_b32 /
 * v_bitop3_b32, so the rotations cost as much as 8 XORs.
 */
#define TT4_BYTES 131072u

/* the same with bytes 0 and 2 of hi kept (hi < 2^24, byte 1 zero) */
__device__ __forceinline__ uint32_t tt_addrh(uint32_t x, uint32_t k,
					     uint32_t hi)
{
	if (k == 1 && TT_B1_BITOP3 == 2)
		return __builtin_amdgcn_bitop3_b32(x, vreg(0xff00u), hi, 0xEA);
	return __builtin_amdgcn_perm(x, hi, 0x0C020000u | ((4u + k) << 8));
}
#define TT_ADDRH(x, k, hi) tt_addrh((x), (k), (hi))

__device__ __forceinline__ void tt4_fill(uint8_t *smem, const uint32_t *T0g)
{
	uint32_t *s = (uint32_t *)smem;
	for (uint32_t i = threadIdx.x; i < TT4_BYTES / 4; i += blockDim.x) {
		const uint32_t e = (i >> 6) & 255u;
		const uint32_t k = ((i >> 13) & 2u) | ((i >> 5) & 1u);
		const uint32_t t = T0g[e];
		s[i] = k ? __builtin_amdgcn_alignbit(t, t, 32 - 8 * k) : t;
	}
}

/* tt4_fill for 1024-thread blocks: thread t's 32 words are entries
 * (t >> 6) + 16 m of T0 (m < 16, each twice: rotations k and k + 2), the
 * same for its whole wave -- 16 uniform loads issued together, then the
 * 32 conflict-free LDS stores, instead of a load and its wait per word
 * (the loop form: ~11 us of the fused kernel's ~15-us plan) */
__device__ __forceinline__ void tt4_fill_b1024(uint8_t *smem,
					       const uint32_t *T0g)
{
	uint32_t *s = (uint32_t *)smem;
	const uint32_t tid = threadIdx.x;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	const uint32_t klo = (tid >> 5) & 1u;
	uint32_t t[16];
#pragma unroll
	for (int m = 0; m < 16; m++)
		t[m] = T0g[wv + 16u * (uint32_t)m];
#pragma unroll
	for (int j = 0; j < 32; j++) {
		const uint32_t k = (((uint32_t)j >> 4) & 1u) << 1 | klo;
		const uint32_t v = t[j & 15];
		s[tid + 1024u * (uint32_t)j] =
			k ? __builtin_amdgcn_alignbit(v, v, 32u - 8u * k) : v;
	}
}

struct Tt4 {
	const uint8_t *smem;
	uint32_t lo, hi;

	__device__ __forceinline__ uint32_t t0(uint32_t x) const
	{
		return lds_u32(smem, TT_ADDR(x, 0, lo));
	}
	__device__ __forceinline__ uint32_t t1(uint32_t x) const
	{
		return lds_u32(smem, TT_ADDR(x, 1, lo) + 128);
	}
	__device__ __forceinline__ uint32_t t2(uint32_t x) const
	{
		return lds_u32(smem, TT_ADDRH(x, 2, hi));
	}
	__device__ __forceinline__ uint32_t t3(uint32_t x) const
	{
		return lds_u32(smem, TT_ADDRH(x, 3, hi) + 128);
	}
};

/* one middle round on (s0..s3), k plain */
__device__ __forceinline__ void aes4_round(const Tt4 &T, const uint32_t *k,
					   uint32_t &s0, uint32_t &s1,
					   uint32_t &s2, uint32_t &s3)
{
	const uint32_t a0 = T.t0(s0), b1 = T.t1(s1), c2 = T.t2(s2), d3 = T.t3(s3);
	const uint32_t a1 = T.t0(s1), b2 = T.t1(s2), c3 = T.t2(s3), d0 = T.t3(s0);
	const uint32_t a2 = T.t0(s2), b3 = T.t1(s3), c0 = T.t2(s0), d1 = T.t3(s1);
	const uint32_t a3 = T.t0(s3), b0 = T.t1(s0), c1 = T.t2(s1), d2 = T.t3(s2);
	s0 = xor3(xor3(a0, b1, c2), d3, rkv(k[0]));
	s1 = xor3(xor3(a1, b2, c3), d0, rkv(k[1]));
	s2 = xor3(xor3(a2, b3, c0), d1, rkv(k[2]));
	s3 = xor3(xor3(a3, b0, c1), d2, rkv(k[3]));
}

template <int NR, int FIRST>
__device__ __forceinline__ void aes4_rounds(const Tt4 &T, const uint32_t *rk,
					    uint32_t &s0, uint32_t &s1,
					    uint32_t &s2, uint32_t &s3)
{
#pragma unroll
	for (int r = FIRST; r < NR; r++)
		aes4_round(T, rk + 4 * r, s0, s1, s2, s3);
	/* the final round reads half 0 only (same as the T0/T1 image) */
	aes_final(T.smem, T.lo, rk + 4 * NR, s0, s1, s2, s3);
}

/* ---- SHA-1 compression, W[] holds the 16 big-endian message words ---- */
/* Round = alignbit + bitop3 + 2 x add3 + alignbit; schedule = bitop3 (xor3)
 * + xor + alignbit (FIPS 180-4 6.1.2, rolling 16-word W). */
__device__ __forceinline__ void sha1_compress(uint32_t h[5], uint32_t w[16])
{
	uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#define SHA_ROUND(i, f, K)                                                   \
	do {                                                                 \
		uint32_t wi;                                                 \
		if ((i) < 16) {                                              \
			wi = w[(i) & 15];                                    \
		} else {                                                     \
			wi = rotl32(xor3(w[((i) + 13) & 15], w[((i) + 8) & 15], \
					 w[((i) + 2) & 15]) ^ w[(i) & 15], 1); \
			w[(i) & 15] = wi;                                    \
		}                                                            \
		uint32_t t = rotl32(a, 5) + (f) + e + (K) + wi;              \
		e = d; d = c; c = rotl32(b, 30); b = a; a = t;               \
	} while (0)
#pragma unroll
	for (int i = 0; i < 20; i++)
		SHA_ROUND(i, sha_ch(b, c, d), 0x5a827999u);
#pragma unroll
	for (int i = 20; i < 40; i++)
		SHA_ROUND(i, xor3(b, c, d), 0x6ed9eba1u);
#pragma unroll
	for (int i = 40; i < 60; i++)
		SHA_ROUND(i, sha_maj(b, c, d), 0x8f1bbcdcu);
#pragma unroll
	for (int i = 60; i < 80; i++)
		SHA_ROUND(i, xor3(b, c, d), 0xca62c1d6u);
#undef SHA_ROUND
	h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

/* ---- GHASH: Z = (X) * H with the 4-bit table at tab (LDS or global) ---- */
/* X given as 4 big-endian words x0..x3 (x0 = bytes 0..3).  rem4 in LDS.
 * Entry i*H lives at tab + i * stride + laneoff: stride 16 / laneoff 0 for
 * a plain table; stride 256 / laneoff (lane & 15) * 16 for the 16x
 * replicated LDS image, where each 16-lane group of a ds_read_b128 hits
 * 16 distinct bank quads whatever the nibbles (conflict-free). */
__device__ __forceinline__ void ghash_mul(uint32_t &x0, uint32_t &x1,
					  uint32_t &x2, uint32_t &x3,
					  const uint8_t *tab, uint32_t stride,
					  uint32_t laneoff,
					  const uint32_t *rem4)
{
	uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
	uint32_t xs[4] = {x0, x1, x2, x3};
#pragma unroll
	for (int wi = 3; wi >= 0; wi--) {
		uint32_t xw = xs[wi];
#pragma unroll
		for (int nb = 0; nb < 8; nb++) {
			/* byte order: word bytes 3..0 are X[4wi+3..4wi] (BE),
			 * low nibble of each byte first */
			uint32_t sh = (uint32_t)((nb >> 1) * 8 + ((nb & 1) ? 4 : 0));
			uint32_t nib = (xw >> sh) & 0xfu;
			uint32_t rem = z3 & 0xfu;
			z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
			z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
			z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
			const uint4 t = *(const uint4 *)(tab + nib * stride +
							 laneoff);
			z0 = xor3(z0 >> 4, rem4[rem], t.x);
			z1 ^= t.y; z2 ^= t.z; z3 ^= t.w;
		}
	}
	x0 = z0; x1 = z1; x2 = z2; x3 = z3;
}
