/*
 * small.hip -- the per-packet path's fused kernel (AES-CM + HMAC-SHA1,
 * AES-GCM).
 *
 * Every unchanged libre caller protects one mbuf per srtp_encrypt() call
 * (reference src/srtp/srtp.c:183-285; unprotect :288-432).  Concurrent
 * calls share a launch (host percall.c one/pc_run) but a launch still carries
 * only a handful of packets, so its cost is latency, not bandwidth.  The
 * general path pays four copies (packets and jobs up, verdicts and packets
 * down), two kernels (k_ctr_coop + the MAC-only k_ctr_hmac) and a sync.
 *
 * k_ctr_small runs one packet per workgroup straight out of the caller's
 * pinned staging memory (mapped: no copies): the workgroup loads the packet
 * into LDS in one coalesced pass, every lane makes one 16-byte keystream
 * block (a 1 KiB T0 table in LDS, rotations in registers: 75 blocks do not
 * amortise the 64 KiB replicated image), lane 0 runs the HMAC-SHA1 chain
 * over LDS -- for unprotect concurrently with the keystream, as the MAC
 * covers the received ciphertext -- and the workgroup writes the packet,
 * verdict and saved tag word back.  Byte-for-byte the job semantics of
 * ctr_hmac_body (k_ctr.h): cipher region, decrypt-if-authentic, the ROC
 * written over the tag (srtp.c:342-344), SRTCP's E||index trailer.
 */
#include "kern_common.h"

#define SMALL_MAX SGPU_SMALL_MAX_BYTES  /* from a packet's start (host-checked) */
#ifndef SMALL_WK
#define SMALL_WK 1      /* inner schedule formed up front (sched_lds) */
#endif

namespace {

/* AES with a plain 1 KiB T0 (LE words: S2 | S << 8 | S << 16 | S3 << 24,
 * srtp_kernels.hip) and plain round keys */
__device__ __forceinline__ void aes_t0(const uint32_t *T, const uint32_t *rk,
				       uint32_t nr, uint32_t &s0, uint32_t &s1,
				       uint32_t &s2, uint32_t &s3)
{
	s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#define TR(a, b, c, d, k)                                                    \
	(T[(a) & 255u] ^ rotl32(T[((b) >> 8) & 255u], 8) ^                   \
	 rotl32(T[((c) >> 16) & 255u], 16) ^ rotl32(T[(d) >> 24], 24) ^ (k))
#pragma unroll 1
	for (uint32_t r = 1; r < nr; r++) {
		const uint32_t *k = rk + 4 * r;
		const uint32_t t0 = TR(s0, s1, s2, s3, k[0]);
		const uint32_t t1 = TR(s1, s2, s3, s0, k[1]);
		const uint32_t t2 = TR(s2, s3, s0, s1, k[2]);
		const uint32_t t3 = TR(s3, s0, s1, s2, k[3]);
		s0 = t0; s1 = t1; s2 = t2; s3 = t3;
	}
#undef TR
	const uint32_t *k = rk + 4 * nr;
#define SB(x) ((T[(x) & 255u] >> 8) & 255u)
#define FR(a, b, c, d, kk)                                                   \
	(SB(a) | SB((b) >> 8) << 8 | SB((c) >> 16) << 16 | SB((d) >> 24) << 24) ^ \
	 (kk)
	const uint32_t t0 = FR(s0, s1, s2, s3, k[0]);
	const uint32_t t1 = FR(s1, s2, s3, s0, k[1]);
	const uint32_t t2 = FR(s2, s3, s0, s1, k[2]);
	const uint32_t t3 = FR(s3, s0, s1, s2, k[3]);
#undef FR
#undef SB
	s0 = t0; s1 = t1; s2 = t2; s3 = t3;
}

/* keystream block b of the packet (ctr_block's counter: IV + b) */
__device__ __forceinline__ void ks_block(const uint32_t *T, const uint32_t *rk,
					 uint32_t nr, const uint32_t iv[4],
					 uint32_t b, uint32_t ks[4])
{
	const uint64_t c = ((uint64_t)bswap32(iv[2]) << 32 | bswap32(iv[3])) +
			   b;
	uint32_t s0 = iv[0], s1 = iv[1];
	uint32_t s2 = bswap32((uint32_t)(c >> 32)), s3 = bswap32((uint32_t)c);
	aes_t0(T, rk, nr, s0, s1, s2, s3);
	ks[0] = s0; ks[1] = s1; ks[2] = s2; ks[3] = s3;
}

/* keystream of the cipher region [c_off, c_end) (c_off 4-aligned) into
 * dst words (XOR into them when XOR, else stored), blocks b0, b0+step.. */
__device__ __forceinline__ void region_ks(const uint32_t *T, const uint32_t *rk,
					  uint32_t nr, const uint32_t iv[4],
					  uint32_t c_off, uint32_t c_end,
					  uint32_t *dst, bool xr, uint32_t b0,
					  uint32_t step, uint32_t *done = nullptr)
{
	for (uint32_t b = b0; c_off + 16u * b < c_end; b += step) {
		uint32_t ks[4];
		ks_block(T, rk, nr, iv, b, ks);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t bp = c_off + 16u * b + 4u * q;
			if (bp >= c_end)
				break;
			const uint32_t n = c_end - bp;
			const uint32_t m = n >= 4 ? 0xffffffffu
						  : (1u << (8 * n)) - 1u;
			uint32_t *p = dst + bp / 4u;
			*p = xr ? *p ^ (ks[q] & m) : (ks[q] & m);
		}
		if (done)
			__hip_atomic_store(done + b, 1u, __ATOMIC_RELEASE,
					   __HIP_MEMORY_SCOPE_WORKGROUP);
	}
}

/* protect: the MAC of chunk k waits until the keystream blocks that
 * overlap [64k, 64k+64) of the cipher region are applied */
struct ks_wait {
	const uint32_t *done;           /* per block, or NULL: nothing */
	uint32_t c_off, c_end;

	__device__ __forceinline__ void operator()(uint32_t k) const
	{
		if (!done)
			return;
		const uint32_t lo = max(64u * k, c_off), hi = min(64u * k + 64u,
								  c_end);
		if (lo >= hi)
			return;
		for (uint32_t b = (lo - c_off) / 16u; b <= (hi - 1u - c_off) / 16u;
		     b++)
			while (!__hip_atomic_load(done + b, __ATOMIC_ACQUIRE,
						  __HIP_MEMORY_SCOPE_WORKGROUP))
				__builtin_amdgcn_s_sleep(1);
	}
};

/* SHA-1 compression for ONE packet's chain (a latency, not a throughput
 * problem): per round only rotl(a, 5) and one v_add3 lie on the serial
 * path -- f(b, c, d) and e + K + w are formed beside it (the plain left-
 * to-right sum puts rotl(a, 5) first and four dependent adds behind it).
 * Measured alternatives: the same chain on the scalar unit (uniform
 * values, shift-pair rotations) ran 77 us per call against 56. */
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c)
{
	uint32_t r;
	asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
	return r;
}

__device__ __forceinline__ void sha1_compress_lat(uint32_t h[5],
						  uint32_t w[16])
{
	uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#define SR(i, f, K)                                                          \
	do {                                                                 \
		uint32_t wi;                                                 \
		if ((i) < 16) {                                              \
			wi = w[(i) & 15];                                    \
		} else {                                                     \
			wi = rotl32(xor3(w[((i) + 13) & 15], w[((i) + 8) & 15], \
					 w[((i) + 2) & 15]) ^ w[(i) & 15], 1); \
			w[(i) & 15] = wi;                                    \
		}                                                            \
		const uint32_t t = add3(rotl32(a, 5), (f), add3(e, (K), wi)); \
		e = d; d = c; c = rotl32(b, 30); b = a; a = t;               \
	} while (0)
#pragma unroll
	for (int i = 0; i < 20; i++)
		SR(i, sha_ch(b, c, d), 0x5a827999u);
#pragma unroll
	for (int i = 20; i < 40; i++)
		SR(i, xor3(b, c, d), 0x6ed9eba1u);
#pragma unroll
	for (int i = 40; i < 60; i++)
		SR(i, sha_maj(b, c, d), 0x8f1bbcdcu);
#pragma unroll
	for (int i = 60; i < 80; i++)
		SR(i, xor3(b, c, d), 0xca62c1d6u);
#undef SR
	h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

/* The inner hash's message schedule depends on the message alone, so the
 * workgroup forms it for every block up front, one block per thread:
 * WK[80 k + i] = W_i + K_i of inner block k (FIPS 180-4 6.1.2; the
 * message buf[0, A) || trailer? || padding || bit length).  The hashing
 * lane then spends five instructions a round (rotl(a, 5), f, e + WK, one
 * v_add3, rotl(b, 30)) instead of eight -- one wave issues one instruction
 * per four cycles whatever its type, so the count is the latency. */
#define SMALL_NB ((SMALL_MAX + 4u + 9u + 63u) / 64u)

__device__ __forceinline__ uint32_t sha_k(int i)
{
	return i < 20 ? 0x5a827999u : i < 40 ? 0x6ed9eba1u
	     : i < 60 ? 0x8f1bbcdcu : 0xca62c1d6u;
}

__device__ __forceinline__ uint32_t mac_blocks(uint32_t A, bool trail)
{
	return (A + (trail ? 4u : 0u) + 9u + 63u) / 64u;
}

__device__ __forceinline__ void sched_lds(const uint32_t *buf, uint32_t A,
					  bool trail, uint32_t trailer,
					  uint32_t *WK, uint32_t t0,
					  uint32_t step)
{
	const uint64_t X = trail ? ((uint64_t)trailer << 32 | 0x80000000u)
				 : 0x8000000000000000ull;
	const uint32_t tl = trail ? 4u : 0u;
	const uint32_t nb = mac_blocks(A, trail);
	const uint64_t bitlen = (uint64_t)(64u + A + tl) * 8u;
	for (uint32_t k = t0; k < nb; k += step) {
		uint32_t w[16], o[80];
#pragma unroll
		for (int g = 0; g < 16; g++) {
			const uint32_t gw = 16u * k + (uint32_t)g;
			const uint32_t v = gw < SMALL_MAX / 4 ? buf[gw] : 0u;
			w[g] = msg_word(gw, bswap32(v), A, X);
		}
		if (k + 1 == nb) {
			w[14] = (uint32_t)(bitlen >> 32);
			w[15] = (uint32_t)bitlen;
		}
#pragma unroll
		for (int i = 0; i < 80; i++) {
			if (i >= 16)
				w[i & 15] = rotl32(xor3(w[(i + 13) & 15],
							w[(i + 8) & 15],
							w[(i + 2) & 15]) ^ w[i & 15], 1);
			o[i] = w[i & 15] + sha_k(i);
		}
		uint4 *dst = (uint4 *)(WK + 80u * k);
#pragma unroll
		for (int g = 0; g < 20; g++)
			dst[g] = make_uint4(o[4 * g], o[4 * g + 1], o[4 * g + 2],
					    o[4 * g + 3]);
	}
}

__device__ __forceinline__ void sha1_compress_wk(uint32_t h[5],
						 const uint32_t *wk)
{
	uint32_t x[80];
#pragma unroll
	for (int g = 0; g < 20; g++) {
		const uint4 v = ((const uint4 *)wk)[g];
		x[4 * g] = v.x; x[4 * g + 1] = v.y;
		x[4 * g + 2] = v.z; x[4 * g + 3] = v.w;
	}
	uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#define SW(i, f)                                                             \
	do {                                                                 \
		const uint32_t t = add3(rotl32(a, 5), (f), e + x[i]);        \
		e = d; d = c; c = rotl32(b, 30); b = a; a = t;               \
	} while (0)
#pragma unroll
	for (int i = 0; i < 20; i++)
		SW(i, sha_ch(b, c, d));
#pragma unroll
	for (int i = 20; i < 40; i++)
		SW(i, xor3(b, c, d));
#pragma unroll
	for (int i = 40; i < 60; i++)
		SW(i, sha_maj(b, c, d));
#pragma unroll
	for (int i = 60; i < 80; i++)
		SW(i, xor3(b, c, d));
#undef SW
	h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

/* HMAC-SHA1 over the scheduled inner blocks, then the outer block */
__device__ __forceinline__ void hmac_wk(const uint32_t *WK, uint32_t nb,
					const struct sgpu_comp *cp,
					uint32_t h[5])
{
	h[0] = cp->ipad[0]; h[1] = cp->ipad[1]; h[2] = cp->ipad[2];
	h[3] = cp->ipad[3]; h[4] = cp->ipad[4];
#pragma unroll 1
	for (uint32_t k = 0; k < nb; k++)
		sha1_compress_wk(h, WK + 80u * k);
	uint32_t w[16];
	w[0] = h[0]; w[1] = h[1]; w[2] = h[2]; w[3] = h[3]; w[4] = h[4];
	w[5] = 0x80000000u;
#pragma unroll
	for (int q = 6; q < 15; q++)
		w[q] = 0;
	w[15] = (64u + 20u) * 8u;
	h[0] = cp->opad[0]; h[1] = cp->opad[1]; h[2] = cp->opad[2];
	h[3] = cp->opad[3]; h[4] = cp->opad[4];
	sha1_compress_lat(h, w);
}

/* HMAC-SHA1 (hmac.c:78-95 via the ipad/opad midstates) of the message
 * buf[0, A) || trailer? -- one lane; digest in h.  Whole 64-byte chunks
 * of [0, A) go straight in, the next chunk's words read from LDS ahead of
 * the compression; the tail chunks take msg_word */
__device__ __forceinline__ void hmac_lds(const uint32_t *buf,
					 const struct sgpu_comp *cp, uint32_t A,
					 bool trail, uint32_t trailer,
					 uint32_t h[5], const ks_wait &wait)
{
	const uint64_t X = trail ? ((uint64_t)trailer << 32 | 0x80000000u)
				 : 0x8000000000000000ull;
	const uint32_t tl = trail ? 4u : 0u;
	const uint32_t nb = (A + tl + 9u + 63u) / 64u;
	const uint64_t bitlen = (uint64_t)(64u + A + tl) * 8u;
	h[0] = cp->ipad[0]; h[1] = cp->ipad[1]; h[2] = cp->ipad[2];
	h[3] = cp->ipad[3]; h[4] = cp->ipad[4];
	const uint32_t kA = A / 64u;
	uint4 nx[4];
	wait(0);
#pragma unroll
	for (int g = 0; g < 4; g++)
		nx[g] = *(const uint4 *)(buf + 4 * g);
#pragma unroll 1
	for (uint32_t k = 0; k < kA; k++) {
		uint32_t w[16];
#pragma unroll
		for (int g = 0; g < 4; g++) {
			w[4 * g] = bswap32(nx[g].x);
			w[4 * g + 1] = bswap32(nx[g].y);
			w[4 * g + 2] = bswap32(nx[g].z);
			w[4 * g + 3] = bswap32(nx[g].w);
		}
		if (16u * (k + 1) < SMALL_MAX / 4) {
			wait(k + 1);
#pragma unroll
			for (int g = 0; g < 4; g++)
				nx[g] = *(const uint4 *)(buf + 16u * (k + 1) +
							  4 * g);
		}
		sha1_compress_lat(h, w);
	}
#pragma unroll 1
	for (uint32_t k = kA; k < nb; k++) {
		uint32_t w[16];
		wait(k);
#pragma unroll
		for (int g = 0; g < 4; g++) {
			const uint32_t gw = 16u * k + 4u * g;
			uint4 v = make_uint4(0, 0, 0, 0);
			if (gw < SMALL_MAX / 4)
				v = *(const uint4 *)(buf + gw);
			w[4 * g] = msg_word(gw, bswap32(v.x), A, X);
			w[4 * g + 1] = msg_word(gw + 1, bswap32(v.y), A, X);
			w[4 * g + 2] = msg_word(gw + 2, bswap32(v.z), A, X);
			w[4 * g + 3] = msg_word(gw + 3, bswap32(v.w), A, X);
		}
		if (k + 1 == nb) {
			w[14] = (uint32_t)(bitlen >> 32);
			w[15] = (uint32_t)bitlen;
		}
		sha1_compress_lat(h, w);
	}
	uint32_t w[16];
	w[0] = h[0]; w[1] = h[1]; w[2] = h[2]; w[3] = h[3]; w[4] = h[4];
	w[5] = 0x80000000u;
#pragma unroll
	for (int q = 6; q < 15; q++)
		w[q] = 0;
	w[15] = (64u + 20u) * 8u;
	h[0] = cp->opad[0]; h[1] = cp->opad[1]; h[2] = cp->opad[2];
	h[3] = cp->opad[3]; h[4] = cp->opad[4];
	sha1_compress_lat(h, w);
}


/* ---- AES-GCM (AEAD_AES_128_GCM / AEAD_AES_256_GCM, aes.c:136-249) ----
 * The workgroup makes the keystream (counter blocks 2.. of J0 = IV || 1,
 * srtp_iv_calc_gcm misc.c:93-105) and wave 0 the GHASH of
 * AAD || C || lengths (SP 800-38D 6.4) in three steps instead of one
 * 77-block chain: lanes 0..m-1 run Horner over m contiguous chunks (the
 * first the short one, the others c blocks each) with the 8-bit table of
 * H, lane m forms H^c meanwhile; the table of H^c is built; lane 0 folds
 * the chunk sums by Horner in H^c.  Results as k_gcmu's: the payload is
 * always transformed, the tag compared (SV_TAG_OK) or written. */

/* M[b] = b * V for all bytes b from the 4-bit table T4 (gh8_fill, one
 * replica: entry b at b) */
__device__ __forceinline__ uint4 m8_entry(const uint4 *T4, uint32_t b)
{
	const uint4 L = T4[b & 15u], H = T4[b >> 4];
	const uint32_t m = L.w & 15u;
	const uint32_t red = (m ^ (m << 5) ^ (m << 6) ^ (m << 7)) << 21;
	return make_uint4((L.x >> 4) ^ red ^ H.x,
			  __builtin_amdgcn_alignbit(L.x, L.y, 4) ^ H.y,
			  __builtin_amdgcn_alignbit(L.y, L.z, 4) ^ H.z,
			  __builtin_amdgcn_alignbit(L.z, L.w, 4) ^ H.w);
}

/* the 4-bit table entry q * V (OpenSSL gcm_init_4bit: V at 8, V x at 4,
 * V x^2 at 2, V x^3 at 1, the rest XORs) */
__device__ __forceinline__ uint4 t4_entry(uint4 v, uint32_t q)
{
	uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
	for (int bit = 8; bit >= 1; bit >>= 1) {
		if (q & (uint32_t)bit) {
			acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
		}
		const uint32_t t = (v.w & 1u) ? 0xe1000000u : 0u;
		v.w = __builtin_amdgcn_alignbit(v.z, v.w, 1);
		v.z = __builtin_amdgcn_alignbit(v.y, v.z, 1);
		v.y = __builtin_amdgcn_alignbit(v.x, v.y, 1);
		v.x = (v.x >> 1) ^ t;
	}
	return acc;
}

/* x = x * V with V's 8-bit table M (ghash8_mul, one replica) */
__device__ __forceinline__ void gmul8(uint32_t x[4], const uint4 *M)
{
	uint32_t R[8];
#pragma unroll
	for (int q = 3; q >= 0; q--) {
		uint4 Mw[4];
#pragma unroll
		for (int w = 0; w < 4; w++)
			Mw[w] = M[(x[w] >> (8 * (3 - q))) & 255u];
		const uint32_t A0 = Mw[0].x;
		const uint32_t A1 = Mw[0].y ^ Mw[1].x;
		const uint32_t A2 = xor3(Mw[0].z, Mw[1].y, Mw[2].x);
		const uint32_t A3 = xor3(Mw[0].w, Mw[1].z, Mw[2].y) ^ Mw[3].x;
		const uint32_t A4 = xor3(Mw[1].w, Mw[2].z, Mw[3].y);
		const uint32_t A5 = Mw[2].w ^ Mw[3].z;
		const uint32_t A6 = Mw[3].w;
		if (q == 3) {
			R[0] = A0; R[1] = A1; R[2] = A2; R[3] = A3;
			R[4] = A4; R[5] = A5; R[6] = A6; R[7] = 0;
		}
		else {
			R[7] = __builtin_amdgcn_alignbit(R[6], R[7], 8);
			R[6] = __builtin_amdgcn_alignbit(R[5], R[6], 8) ^ A6;
			R[5] = __builtin_amdgcn_alignbit(R[4], R[5], 8) ^ A5;
			R[4] = __builtin_amdgcn_alignbit(R[3], R[4], 8) ^ A4;
			R[3] = __builtin_amdgcn_alignbit(R[2], R[3], 8) ^ A3;
			R[2] = __builtin_amdgcn_alignbit(R[1], R[2], 8) ^ A2;
			R[1] = __builtin_amdgcn_alignbit(R[0], R[1], 8) ^ A1;
			R[0] = (R[0] >> 8) ^ A0;
		}
	}
	const uint32_t u0 = R[4], u1 = R[5], u2 = R[6], u3 = R[7];
	x[0] = xor3(xor3(R[0], u0, u0 >> 1), u0 >> 2, u0 >> 7);
	x[1] = xor3(xor3(R[1], u1, __builtin_amdgcn_alignbit(u0, u1, 1)),
		    __builtin_amdgcn_alignbit(u0, u1, 2),
		    __builtin_amdgcn_alignbit(u0, u1, 7));
	x[2] = xor3(xor3(R[2], u2, __builtin_amdgcn_alignbit(u1, u2, 1)),
		    __builtin_amdgcn_alignbit(u1, u2, 2),
		    __builtin_amdgcn_alignbit(u1, u2, 7));
	x[3] = xor3(xor3(R[3], u3, __builtin_amdgcn_alignbit(u2, u3, 1)),
		    __builtin_amdgcn_alignbit(u2, u3, 2),
		    __builtin_amdgcn_alignbit(u2, u3, 7));
}

/* LDS written by some lanes of this wave, read by others next */
__device__ __forceinline__ void wave_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct gcm_in {
	const uint32_t *buf;    /* the packet (LDS) */
	uint32_t A, na, nc, c_off, c_end, c_len, aad_total;
	uint64_t Xtr;           /* trailer word for msg_word (SRTCP) */
};

/* GHASH input block i (BE words): AAD, ciphertext, lengths */
__device__ __forceinline__ void g_block(const gcm_in &g, uint32_t i,
					uint32_t w[4])
{
	if (i < g.na) {
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t gw = 4u * i + (uint32_t)q;
			const uint32_t v = gw < SMALL_MAX / 4 ? g.buf[gw] : 0u;
			w[q] = msg_word(gw, bswap32(v), g.A, g.Xtr);
		}
	}
	else if (i < g.na + g.nc) {
		const uint32_t p = g.c_off + 16u * (i - g.na);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t bp = p + 4u * (uint32_t)q;
			uint32_t v = bp < g.c_end ? bswap32(g.buf[bp / 4u]) : 0u;
			const uint32_t n = bp < g.c_end ? g.c_end - bp : 0u;
			if (n < 4u)
				v &= (uint32_t)(0xFFFFFFFF00000000ull >> (8u * n));
			w[q] = v;
		}
	}
	else {
		const uint64_t al = (uint64_t)g.aad_total * 8u;
		const uint64_t cl = (uint64_t)g.c_len * 8u;
		w[0] = (uint32_t)(al >> 32); w[1] = (uint32_t)al;
		w[2] = (uint32_t)(cl >> 32); w[3] = (uint32_t)cl;
	}
}

/* GHASH by wave 0 (lane < 64); lane 0 returns it in X.  M1: H's table;
 * scratch: Mc (256 entries), Ys (65), T4c (16) */
__device__ __forceinline__ void ghash_wave(const gcm_in &g, const uint4 *M1,
					   uint4 H, uint4 *Mc, uint4 *Ys,
					   uint4 *T4c, uint32_t lane,
					   uint32_t X[4])
{
	const uint32_t n = g.na + g.nc + 1u;
	const uint32_t c = (n + 7u) / 8u;               /* chunk length */
	const uint32_t m = (n + c - 1u) / c;            /* chunks */
	const uint32_t n0 = n - c * (m - 1u);           /* the first's */
	uint32_t x[4] = {0, 0, 0, 0};
	if (lane < m) {
		const uint32_t b0 = lane ? n0 + c * (lane - 1u) : 0u;
		const uint32_t b1 = lane ? b0 + c : n0;
		for (uint32_t b = b0; b < b1; b++) {
			uint32_t w[4];
			g_block(g, b, w);
			x[0] ^= w[0]; x[1] ^= w[1]; x[2] ^= w[2]; x[3] ^= w[3];
			gmul8(x, M1);
		}
	}
	else if (lane == m) {
		x[0] = H.x; x[1] = H.y; x[2] = H.z; x[3] = H.w;
		for (uint32_t k = 1; k < c; k++)
			gmul8(x, M1);
	}
	if (lane <= m)
		Ys[lane] = make_uint4(x[0], x[1], x[2], x[3]);
	wave_sync();
	if (m > 1) {
		if (lane < 16)
			T4c[lane] = t4_entry(Ys[m], lane);
		wave_sync();
		for (uint32_t b = lane; b < 256u; b += 64u)
			Mc[b] = m8_entry(T4c, b);
		wave_sync();
	}
	if (lane == 0) {
		uint4 y = Ys[0];
		x[0] = y.x; x[1] = y.y; x[2] = y.z; x[3] = y.w;
		for (uint32_t k = 1; k < m; k++) {
			gmul8(x, Mc);
			y = Ys[k];
			x[0] ^= y.x; x[1] ^= y.y; x[2] ^= y.z; x[3] ^= y.w;
		}
		X[0] = x[0]; X[1] = x[1]; X[2] = x[2]; X[3] = x[3];
	}
}

/* one GCM job by the workgroup; the packet is in buf (nw_out words,
 * written back by the caller), returns the verdict (thread 0) */
__device__ uint8_t gcm_small(const struct sgpu_job &j,
			     const struct sgpu_comp *cp, bool prot,
			     const uint32_t *T, const uint32_t *rk,
			     uint32_t *buf, uint32_t *ksb, uint4 *gl,
			     uint32_t tid)
{
	/* gl: M1[256] | Mc[256] | Ys[65] | T4c[16] | X | EJ0 */
	uint4 *M1 = gl, *Mc = gl + 256, *Ys = gl + 512, *T4c = gl + 577;
	uint4 *sX = gl + 593, *sE = gl + 594;
	const uint32_t nr = cp->nr;
	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
	gcm_in g;
	g.buf = buf;
	g.A = j.a_len;
	g.aad_total = j.a_len + (trail ? 4u : 0u);
	g.na = (g.aad_total + 15u) / 16u;
	g.c_off = j.c_off;
	g.c_len = do_cipher ? j.c_len : 0u;
	g.c_end = g.c_off + g.c_len;
	g.nc = (g.c_len + 15u) / 16u;
	g.Xtr = trail ? ((uint64_t)j.trailer << 32) : 0ull;
	/* srtp_iv_calc_gcm: IV = k_s ^ (0^16 || SSRC || ROC || SEQ) */
	uint32_t iv[4];
	{
		const uint4 ks = *(const uint4 *)cp->k_s;
		const uint32_t be0 = (j.ssrc >> 16) & 0xffffu;
		const uint32_t be1 = ((j.ssrc & 0xffffu) << 16) | (j.ixhi >> 16);
		const uint32_t be2 = ((j.ixhi & 0xffffu) << 16) |
				     (j.ixlo & 0xffffu);
		iv[0] = ks.x ^ bswap32(be0);
		iv[1] = ks.y ^ bswap32(be1);
		iv[2] = ks.z ^ bswap32(be2);
		iv[3] = 0;
	}
	for (uint32_t b = tid; b < 256u; b += blockDim.x)
		M1[b] = m8_entry((const uint4 *)cp->htab, b);
	const uint4 H = *(const uint4 *)cp->htab[8];
	__syncthreads();
	/* data block b uses counter b + 2: region_ks's block index is the
	 * 64-bit counter offset, so start the region 32 bytes early */
	const uint32_t lane = tid & 63u;
	if (prot) {
		if (do_cipher)
			region_ks(T, rk, nr, iv, g.c_off - 32u, g.c_end, buf,
				  true, tid + 2u, blockDim.x);
		__syncthreads();
		if (tid < 64u)
			ghash_wave(g, M1, H, Mc, Ys, T4c, lane, (uint32_t *)sX);
		else if (tid == 64u) {
			uint32_t e[4];
			ks_block(T, rk, nr, iv, 1u, e);
			*sE = make_uint4(e[0], e[1], e[2], e[3]);
		}
	}
	else {
		if (tid < 64u)
			ghash_wave(g, M1, H, Mc, Ys, T4c, lane, (uint32_t *)sX);
		else {
			if (do_cipher)
				region_ks(T, rk, nr, iv, g.c_off - 32u, g.c_end,
					  ksb, false, tid - 64u + 2u,
					  blockDim.x - 64u);
			if (tid == 64u) {
				uint32_t e[4];
				ks_block(T, rk, nr, iv, 1u, e);
				*sE = make_uint4(e[0], e[1], e[2], e[3]);
			}
		}
	}
	__syncthreads();
	uint8_t vd = do_cipher ? SV_CIPHERED : 0;
	/* tag = GHASH ^ E(K, J0) */
	const uint4 X = *sX, E = *sE;
	const uint32_t t[4] = {X.x ^ bswap32(E.x), X.y ^ bswap32(E.y),
			       X.z ^ bswap32(E.z), X.w ^ bswap32(E.w)};
	uint8_t *tp = (uint8_t *)buf + j.tag_off;
	if (prot) {
		if (tid == 0) {
			for (int q = 0; q < 16; q++)
				tp[q] = (uint8_t)(t[q >> 2] >> (24 - 8 * (q & 3)));
			if (j.flags & SJ_STORE_TRAIL) {
				uint8_t *tr = (uint8_t *)buf + j.t_off;
				tr[0] = (uint8_t)(j.trailer >> 24);
				tr[1] = (uint8_t)(j.trailer >> 16);
				tr[2] = (uint8_t)(j.trailer >> 8);
				tr[3] = (uint8_t)j.trailer;
			}
		}
	}
	else {
		uint32_t diff = 0;
		for (int q = 0; q < 16; q++)
			diff |= tp[q] ^ (uint8_t)(t[q >> 2] >> (24 - 8 * (q & 3)));
		if (diff == 0)
			vd |= SV_TAG_OK;
		__syncthreads();        /* every thread compared the tag */
		if (do_cipher)
			for (uint32_t w = g.c_off / 4u + tid;
			     w < (g.c_end + 3u) / 4u; w += blockDim.x)
				buf[w] ^= ksb[w];
	}
	return vd;
}

/* completion without a stream synchronisation: every wave waits for its
 * stores (s_waitcnt 0: __syncthreads alone does not wait for global
 * stores), the workgroup barrier, one system-scope fence per workgroup
 * (its L2 write-back), then the last workgroup to finish
 * stores the launch's sequence number into the caller's pinned word (the
 * host spins on it).  scripts/ubench_launch.hip: 9.5 us a round trip of
 * 32 such workgroups against 13.0 for launch + hipStreamSynchronize, no
 * stale word in 19.2 M checked (a fence in every thread: 12.7 us) */
__device__ __forceinline__ void small_done(const KArgs &a)
{
	if (!a.done_flag)
		return;
	__builtin_amdgcn_s_waitcnt(0);
	__syncthreads();
	if (threadIdx.x == 0) {
		__threadfence_system();
		if (atomicAdd(a.done_cnt, 1u) + 1u == gridDim.x) {
			*a.done_cnt = 0;
			__hip_atomic_store(a.done_flag, a.done_seq,
					   __ATOMIC_RELEASE,
					   __HIP_MEMORY_SCOPE_SYSTEM);
		}
	}
}

} /* namespace */

/* a workgroup's LDS for one job */
struct SmallLds {
	uint32_t T[256];
	uint32_t rk[60];                /* plain round keys */
	alignas(16) uint32_t buf[SMALL_MAX / 4];
	alignas(16) uint32_t ksb[SMALL_MAX / 4];
	alignas(16) uint32_t WK[SMALL_NB * 80];
	uint32_t s_tag_ok;
};
static_assert(SMALL_NB * 80 * 4 >= 595 * 16, "gcm_small scratch");

/* job i by the calling workgroup.  mode 0 unprotect, 1 protect, 2 per job
 * (SJ_PROTECT): the operations of one shared per-packet launch in one
 * grid (host pc_run_fused) */
__device__ __forceinline__ void small_job(const KArgs &a, uint32_t i,
					  int mode, SmallLds &L)
{
	uint32_t *T = L.T, *rk = L.rk, *buf = L.buf, *ksb = L.ksb, *WK = L.WK;
	uint32_t &s_tag_ok = L.s_tag_ok;
	const uint32_t tid = threadIdx.x;
	const struct sgpu_job j = a.jobs[i];
	const bool PROT = mode == 2 ? (j.flags & SJ_PROTECT) != 0 : mode == 1;
	if (j.flags & SJ_SKIP) {
		if (tid == 0 && a.verdict)
			a.verdict[i] = 0;
		return;
	}
	const struct sgpu_comp *cp = a.comps +
				     __builtin_amdgcn_readfirstlane(j.comp);
	const uint32_t nr = cp->nr;
	T[tid] = a.t0[tid];

	const bool gcm = (j.flags & SJ_GCM) != 0;
	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
	const bool do_hmac = (j.flags & SJ_HMAC) != 0;
	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool cipher_if_ok = !PROT && (j.flags & SJ_CIPHER_IF_OK);
	const bool roc_at_tag = !PROT && (j.flags & SJ_ROC_AT_TAG);
	const uint32_t c_off = j.c_off;
	const uint32_t c_end = do_cipher ? j.c_off + j.c_len : 0u;
	const uint32_t A = (do_hmac || gcm) ? j.a_len : 0u;
	const uint32_t tag_len = do_hmac ? cp->tag_len : gcm ? 16u : 0u;
	const bool store_ct = do_cipher && (PROT || cipher_if_ok || !do_hmac);
	/* bytes read: the MAC input and cipher region, unprotect's tag;
	 * bytes written back: those plus protect's tag and trailer */
	uint32_t in_len = max(c_end, A);
	uint32_t out_len = in_len;
	if (PROT) {
		if (tag_len)
			out_len = max(out_len, j.tag_off + tag_len);
		if (j.flags & SJ_STORE_TRAIL)
			out_len = max(out_len, j.t_off + 4u);
	}
	else {
		if (tag_len)
			in_len = max(in_len, j.tag_off + tag_len);
		if (roc_at_tag)
			in_len = max(in_len, j.tag_off + 4u);
		out_len = in_len;
	}
	const uint32_t nw_in = (in_len + 3u) / 4u, nw_out = (out_len + 3u) / 4u;
	const uint32_t *src = (const uint32_t *)(a.arena + j.off);
	for (uint32_t w = tid; w < nw_out; w += blockDim.x)
		buf[w] = w < nw_in ? src[w] : 0u;

	if (tid < 4 * (nr + 1)) {
		const uint32_t v = cp->rk[tid];
		/* the table stores middle-round keys rot16'd */
		rk[tid] = (tid >= 4 && tid < 4 * nr) ? rot16(v) : v;
	}
	uint32_t iv[4];
	{
		const uint4 ks = *(const uint4 *)cp->k_s;
		iv[0] = ks.x;
		iv[1] = ks.y ^ bswap32(j.ssrc);
		iv[2] = ks.z ^ bswap32(j.ixhi);
		iv[3] = (ks.w ^ (bswap32(j.ixlo) >> 16)) & 0xffffu;
	}
	__syncthreads();

	uint8_t vd = 0;
	uint32_t h[5];
	if (gcm) {
		vd = gcm_small(j, cp, PROT, T, rk, buf, ksb, (uint4 *)WK, tid);
	}
	else if (PROT) {
		/* the MAC covers the ciphertext: keystream first.  (Hashing
		 * each chunk as soon as its blocks are done, the other waves
		 * applying the keystream meanwhile, measured slower: 41.6 vs
		 * 35.9 us per launch -- the per-block flag waits cost more than
		 * the ~3 us keystream pass they hide) */
		if (do_cipher)
			region_ks(T, rk, nr, iv, c_off, c_end, buf, true, tid,
				  blockDim.x);
		__syncthreads();
		if (do_hmac && SMALL_WK) {
			sched_lds(buf, A, trail, j.trailer, WK, tid, blockDim.x);
			__syncthreads();
		}
		if (tid == 0 && do_hmac) {
			if (SMALL_WK) {
				hmac_wk(WK, mac_blocks(A, trail), cp, h);
			}
			else {
				const ks_wait none = {nullptr, 0, 0};
				hmac_lds(buf, cp, A, trail, j.trailer, h, none);
			}
			uint8_t *tp = (uint8_t *)buf + j.tag_off;
			for (uint32_t q = 0; q < tag_len; q++)
				tp[q] = (uint8_t)(h[q >> 2] >> (24 - 8 * (q & 3)));
		}
		if (tid == 0 && (j.flags & SJ_STORE_TRAIL)) {
			uint8_t *tp = (uint8_t *)buf + j.t_off;
			tp[0] = (uint8_t)(j.trailer >> 24);
			tp[1] = (uint8_t)(j.trailer >> 16);
			tp[2] = (uint8_t)(j.trailer >> 8);
			tp[3] = (uint8_t)j.trailer;
		}
	}
	else {
		/* the MAC covers the received ciphertext: lane 0 hashes while
		 * the other waves make the keystream */
		if (do_hmac && SMALL_WK) {
			sched_lds(buf, A, trail, j.trailer, WK, tid, blockDim.x);
			__syncthreads();
		}
		if (tid == 0) {
			uint32_t ok = 1;
			if (do_hmac && SMALL_WK) {
				hmac_wk(WK, mac_blocks(A, trail), cp, h);
			}
			else if (do_hmac) {
				const ks_wait none = {nullptr, 0, 0};
				hmac_lds(buf, cp, A, trail, j.trailer, h, none);
			}
			if (do_hmac) {
				const uint8_t *tp = (const uint8_t *)buf + j.tag_off;
				uint32_t diff = 0;
				for (uint32_t q = 0; q < tag_len; q++)
					diff |= tp[q] ^ (uint8_t)(h[q >> 2] >>
								  (24 - 8 * (q & 3)));
				ok = diff == 0;
			}
			s_tag_ok = ok;
		}
		if (do_cipher && tid >= 64u)
			region_ks(T, rk, nr, iv, c_off, c_end, ksb, false,
				  tid - 64u, blockDim.x - 64u);
		__syncthreads();
		const bool tag_ok = s_tag_ok != 0;
		vd = (do_hmac && tag_ok) ? SV_TAG_OK : 0;
		const bool apply = store_ct && !(cipher_if_ok && !tag_ok);
		if (tid == 0 && roc_at_tag) {
			/* the reference writes the ROC over the tag before
			 * comparing (srtp.c:342-344) */
			uint8_t *tp = (uint8_t *)buf + j.tag_off;
			if (a.save)
				a.save[i] = (uint32_t)tp[0] |
					    (uint32_t)tp[1] << 8 |
					    (uint32_t)tp[2] << 16 |
					    (uint32_t)tp[3] << 24;
			tp[0] = (uint8_t)(j.trailer >> 24);
			tp[1] = (uint8_t)(j.trailer >> 16);
			tp[2] = (uint8_t)(j.trailer >> 8);
			tp[3] = (uint8_t)j.trailer;
		}
		__syncthreads();
		if (apply) {
			for (uint32_t w = c_off / 4u + tid; w < (c_end + 3u) / 4u;
			     w += blockDim.x)
				buf[w] ^= ksb[w];
			vd |= SV_CIPHERED;
		}
	}
	__syncthreads();
	uint32_t *dst = (uint32_t *)(a.arena + j.off);
	for (uint32_t w = tid; w < nw_out; w += blockDim.x)
		dst[w] = buf[w];
	if (tid == 0 && a.verdict)
		a.verdict[i] = vd;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_ctr_small(const KArgs a)
{
	__shared__ SmallLds L;
	/* the last workgroup's count publishes the launch's completion word */
	if (blockIdx.x < a.njobs)
		small_job(a, blockIdx.x, MODE, L);
	small_done(a);
}

/*
 * The lingering form (srtp_gpu_tune pclinger, round 6 A/B): one launch
 * serves a workspace's successive small batches.  Workgroup 0 polls the
 * pinned mailbox (struct sgpu_srv_mb, coherent host memory) and hands each
 * posted batch to the grid through a device word; every workgroup runs its
 * jobs i = blockIdx.x + k * gridDim.x; the last one to finish stores the
 * batch's sequence number into the completion word, as small_done does.
 * Workgroup 0 ends the launch only when the last batch is complete and it
 * has been idle for `linger` ticks of the 100 MHz clock (or the host asked
 * it to stop, or the launch has lived `life` ticks): it tells the grid to
 * exit, then stores `gone` into the mailbox, so the host knows a batch
 * posted after its last look was not taken and launches again.  Every wave
 * reaches that exit: the lifetime bound holds under any traffic.
 */
#define SRV_EXIT 0xffffffffu

__device__ __forceinline__ uint64_t srv_now()
{
	return __builtin_amdgcn_s_memrealtime();
}

__global__ void __launch_bounds__(256)
k_small_srv(const KArgs a0, struct sgpu_srv_mb *mb, struct sgpu_srv_bc *bc,
	    uint32_t linger, uint32_t life)
{
	__shared__ SmallLds L;
	__shared__ uint32_t s_seq;
	const uint32_t tid = threadIdx.x;
	const uint64_t t_start = srv_now();
	uint64_t t_idle = t_start;
	uint32_t cur = 0;               /* the batch last taken (bc zeroed) */
	for (;;) {
		if (tid == 0) {
			uint32_t s;
			for (;;) {
				const uint64_t now = srv_now();
				if (blockIdx.x == 0) {
					/* (relaxed polls: an acquire per poll
					 * would invalidate the caches under
					 * other kernels every few hundred ns) */
					s = __hip_atomic_load(&mb->post,
							      __ATOMIC_RELAXED,
							      __HIP_MEMORY_SCOPE_SYSTEM);
					if (s != cur && s != 0) {
						__builtin_amdgcn_fence(__ATOMIC_ACQUIRE,
								       "");
						/* the batch's arguments to the grid */
						bc->njobs = __hip_atomic_load(&mb->njobs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->mode = __hip_atomic_load(&mb->mode, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->arena = __hip_atomic_load(&mb->arena, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->asz = __hip_atomic_load(&mb->asz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->jobs = __hip_atomic_load(&mb->jobs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->verdict = __hip_atomic_load(&mb->verdict, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->save = __hip_atomic_load(&mb->save, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						bc->comps = __hip_atomic_load(&mb->comps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						__hip_atomic_store(&bc->seq, s,
								   __ATOMIC_RELEASE,
								   __HIP_MEMORY_SCOPE_AGENT);
						break;
					}
					const bool idle =
						__hip_atomic_load(&bc->done,
								  __ATOMIC_RELAXED,
								  __HIP_MEMORY_SCOPE_AGENT) == cur;
					if (!idle)
						t_idle = now;
					else if (now - t_idle > linger ||
						 now - t_start > life ||
						 __hip_atomic_load(&mb->stop,
								   __ATOMIC_RELAXED,
								   __HIP_MEMORY_SCOPE_SYSTEM)) {
						__hip_atomic_store(&bc->seq, SRV_EXIT,
								   __ATOMIC_RELEASE,
								   __HIP_MEMORY_SCOPE_AGENT);
						__hip_atomic_store(&mb->last, cur,
								   __ATOMIC_RELAXED,
								   __HIP_MEMORY_SCOPE_SYSTEM);
						__hip_atomic_store(&mb->gone, 1u,
								   __ATOMIC_RELEASE,
								   __HIP_MEMORY_SCOPE_SYSTEM);
						s = SRV_EXIT;
						break;
					}
					__builtin_amdgcn_s_sleep(2);
				}
				else {
					s = __hip_atomic_load(&bc->seq,
							      __ATOMIC_RELAXED,
							      __HIP_MEMORY_SCOPE_AGENT);
					if (s != cur) {
						__builtin_amdgcn_fence(__ATOMIC_ACQUIRE,
								       "agent");
						break;
					}
					/* (workgroup 0 ends the grid within its
					 * lifetime bound; this one is a backstop) */
					if (now - t_start > 2ull * life + linger) {
						s = SRV_EXIT;
						break;
					}
					__builtin_amdgcn_s_sleep(8);
				}
			}
			s_seq = s;
		}
		__syncthreads();
		const uint32_t s = s_seq;
		if (s == SRV_EXIT)
			return;
		cur = s;
		KArgs a = a0;
		const uint32_t nj = bc->njobs;
		const int mode = (int)bc->mode;
		a.arena = (uint8_t *)bc->arena;
		a.asz = bc->asz;
		a.jobs = (const struct sgpu_job *)bc->jobs;
		a.njobs = nj;
		a.verdict = (uint8_t *)bc->verdict;
		a.save = (uint32_t *)bc->save;
		a.comps = (const struct sgpu_comp *)bc->comps;
		for (uint32_t i = blockIdx.x; i < nj; i += gridDim.x) {
			small_job(a, i, mode, L);
			__syncthreads();
		}
		/* completion (small_done) by the workgroups that had a job
		 * (workgroup 0 alone for an empty batch), and the device copy
		 * of it that workgroup 0's idle test reads */
		const uint32_t parts = nj < gridDim.x ? (nj ? nj : 1u)
						      : gridDim.x;
		__builtin_amdgcn_s_waitcnt(0);
		__syncthreads();
		if (tid == 0 && blockIdx.x < parts) {
			__threadfence_system();
			if (atomicAdd(a0.done_cnt, 1u) + 1u == parts) {
				*a0.done_cnt = 0;
				__hip_atomic_store(a0.done_flag, s, __ATOMIC_RELEASE,
						   __HIP_MEMORY_SCOPE_SYSTEM);
				__hip_atomic_store(&bc->done, s, __ATOMIC_RELEASE,
						   __HIP_MEMORY_SCOPE_AGENT);
			}
		}
		t_idle = srv_now();
		__syncthreads();
	}
}

int small_launch(uint8_t *arena, uint64_t arena_size,
		 const struct sgpu_job *jobs, uint32_t njobs, uint8_t *verdict,
		 uint32_t *save, const struct sgpu_comp *comps,
		 const uint32_t *t0, int prot, uint32_t *done_cnt,
		 uint32_t *done_flag, uint32_t done_seq, void *stream)
{
	if (!njobs)
		return 0;
	KArgs a = {};
	a.arena = arena;
	a.asz = arena_size;
	a.jobs = jobs;
	a.njobs = njobs;
	a.comps = comps;
	a.t0 = t0;
	a.verdict = verdict;
	a.save = save;
	a.done_cnt = done_cnt;
	a.done_flag = done_flag;
	a.done_seq = done_seq;
	hipLaunchKernelGGL(prot == 2 ? k_ctr_small<2>
			   : prot ? k_ctr_small<1> : k_ctr_small<0>,
			   dim3(njobs), dim3(256), 0, (hipStream_t)stream, a);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}

int small_srv_launch(const struct sgpu_comp *comps, const uint32_t *t0,
		     struct sgpu_srv_mb *mb, struct sgpu_srv_bc *bc,
		     uint32_t grid, uint32_t linger_us, uint32_t life_us,
		     uint32_t *done_cnt, uint32_t *done_flag, void *stream)
{
	KArgs a = {};
	a.comps = comps;
	a.t0 = t0;
	a.done_cnt = done_cnt;
	a.done_flag = done_flag;
	hipLaunchKernelGGL(k_small_srv, dim3(grid), dim3(256), 0,
			   (hipStream_t)stream, a, mb, bc, linger_us * 100u,
			   life_us * 100u);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
