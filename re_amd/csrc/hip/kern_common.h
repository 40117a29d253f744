/*
 * kern_common.h -- shared device code of the SRTP crypto kernels: arena
 * access, CTR blocks, the SHA-1 message word of the MAC input, kernel
 * arguments and the two job sources (general sgpu_job / compact
 * descriptor).  Included by ctr10.hip, ctr14.hip and gcm.hip (one
 * translation unit per kernel family, built in parallel).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include "../srtpgpu.h"
#include "dev_common.h"

#define KBLOCK 256
#define CTR_BLOCK 512      /* 8 waves share one 64 KiB T-table image */
#define CTR_BLOCK_MAX 768  /* single-key unprotect: 12 waves, 1 block/CU */

/* ------------------------------------------------------------------ */
/* memory helpers: packet starts are 4-byte aligned (host-checked)     */

__device__ __forceinline__ uint4 ld16(const uint8_t *arena, uint64_t asz,
				      uint64_t a)
{
	if (a + 16 <= asz)
		return *(const uint4 *)(arena + a);
	uint4 r = make_uint4(0, 0, 0, 0);
	if (a + 4 <= asz)  r.x = *(const uint32_t *)(arena + a);
	if (a + 8 <= asz)  r.y = *(const uint32_t *)(arena + a + 4);
	if (a + 12 <= asz) r.z = *(const uint32_t *)(arena + a + 8);
	return r;
}

/* store the low `n` bytes (1..3) of LE word v at p */
__device__ __forceinline__ void st_partial(uint8_t *p, uint32_t v, uint32_t n)
{
	if (n >= 2) {
		*(uint16_t *)p = (uint16_t)v;
		if (n == 3)
			p[2] = (uint8_t)(v >> 16);
	}
	else if (n == 1) {
		p[0] = (uint8_t)v;
	}
}

/* big-endian 32-bit word to 4 byte stores (arbitrary alignment) */
__device__ __forceinline__ void st_be32(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 24);
	p[1] = (uint8_t)(v >> 16);
	p[2] = (uint8_t)(v >> 8);
	p[3] = (uint8_t)v;
}

/* ------------------------------------------------------------------ */
/* CTR keystream block b (IV + b, 128-bit big-endian add, OpenSSL
 * CRYPTO_ctr128_encrypt semantics).  T4: the four-table LDS image
 * (dev_common.h); round keys are then plain for every round. */
template <int NR, bool T4>
__device__ __forceinline__ void ctr_block(const uint8_t *smem, uint32_t lo,
					  const uint32_t *rk, const uint32_t iv[4],
					  int32_t b, uint32_t ks[4])
{
	uint64_t c = ((uint64_t)bswap32(iv[2]) << 32 | bswap32(iv[3])) +
		     (uint64_t)(int64_t)b;
	uint32_t s0 = iv[0], s1 = iv[1];
	uint32_t s2 = bswap32((uint32_t)(c >> 32));
	uint32_t s3 = bswap32((uint32_t)c);
	if (T4) {
		const Tt4 T = {smem, lo, lo | 0x10000u};
		s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
		aes4_rounds<NR, 1>(T, rk, s0, s1, s2, s3);
	}
	else {
		aes_block<NR>(smem, lo, rk, s0, s1, s2, s3);
	}
	ks[0] = s0; ks[1] = s1; ks[2] = s2; ks[3] = s3;
}

/*
 * AES-CTR keystream of one packet with counter-mode caching.  SRTP IVs
 * have bytes 14..15 zero (srtp_iv_calc, misc.c:76-87; the GCM/KDF paths do
 * not use this), so while the block index b < 65536 (payload < 1 MiB) only
 * bytes 14..15 of the counter block change: after round 0 only t3's bytes
 * 2..3 vary, round 1 has two varying lookups (columns 2..3 are constant)
 * and round 2 has eight.  Those constants are computed once per packet.
 * CACHED = false is the plain counter (any packet size).
 *
 * T0/T1 image (T4 = false): middle-round keys rot16'd, constants
 *   A0,P0,A1,P1 (round 1) and R0,C1a,C1b,C2,C3a,C3b (round 2).
 * T4 image: plain keys; round 1 s0 = A0 ^ T3[t3.b3], s1 = A1 ^ T2[t3.b2];
 *   round 2 needs R0 (col 0), C1a (col 1), C2 (col 2), C3a (col 3).
 *   With CTR_B15 s1 is folded into R0/C1a/C2/C3a and A1 holds the LDS
 *   address of the T3 lookup of t3's byte 3 at b = 0.
 */
/* CTR_B15 (T4 image only): packets whose keystream block index stays
 * under 256 (compact launches carry packets under SGPU_CACHED_MAX_CTR
 * bytes), so only IV byte 15 varies: round 1 has one varying lookup,
 * round 2 four (5 instead of 10 per block) */
#ifndef CTR_B15
#define CTR_B15 1
#endif

/* B8 (two-table image only): every block index < 256 -- only the low
 * counter byte varies, so round 1 has one varying lookup and round 2 four
 * (the single-key GCM kernel; SGPU_CACHED_MAX_GCM bounds its packets) */
template <int NR, bool CACHED, bool T4 = false, bool B8 = false>
struct CtrKs {
	uint32_t t0, t1, t2, t3c;       /* IV ^ rk[0..3] (t3c: bytes 14,15 = rk) */
	uint32_t A0, P0, A1, P1;        /* round 1: s0 = A0^rot16(P0^T1[t3.b3]) */
	uint32_t R0, C1a, C1b, C2, C3a, C3b; /* round 2 constants */

	__device__ __forceinline__ void init(const uint8_t *smem, uint32_t lo,
					     const uint32_t *rk,
					     const uint32_t iv[4])
	{
		t0 = iv[0] ^ rk[0];
		t1 = iv[1] ^ rk[1];
		t2 = iv[2] ^ rk[2];
		t3c = iv[3] ^ rk[3];
		if (!CACHED)
			return;
		const uint32_t *k1 = rk + 4, *k2 = rk + 8;
		if (T4) {
			const Tt4 T = {smem, lo, lo | 0x10000u};
			/* round 1 (t3 bytes 0..1 constant) */
			A0 = xor3(T.t0(t0), T.t1(t1), T.t2(t2)) ^ k1[0];
			A1 = xor3(T.t0(t1), T.t1(t2), T.t3(t0)) ^ k1[1];
			const uint32_t S2 = xor3(xor3(T.t0(t2), T.t1(t3c), T.t2(t0)),
						 T.t3(t1), k1[2]);
			const uint32_t S3 = xor3(xor3(T.t0(t3c), T.t1(t0), T.t2(t1)),
						 T.t3(t2), k1[3]);
			/* round 2 constants */
			R0 = xor3(T.t2(S2), T.t3(S3), k2[0]);
			C1a = xor3(T.t1(S2), T.t2(S3), k2[1]);
			C2 = xor3(T.t0(S2), T.t1(S3), k2[2]);
			C3a = xor3(T.t0(S3), T.t3(S2), k2[3]);
#if CTR_B15
			/* b < 256: t3 byte 2 (IV byte 14) is constant too, so
			 * s1 and the four round-2 terms it feeds are constants
			 * and the one varying lookup's address is
			 * AD3 ^ (b << 8) (TT_ADDRH of t3c's byte 3) */
			const uint32_t s1 = A1 ^ T.t2(t3c);
			R0 ^= T.t1(s1);
			C1a ^= T.t0(s1);
			C2 ^= T.t3(s1);
			C3a ^= T.t2(s1);
			A1 = TT_ADDRH(t3c, 3, lo | 0x10000u) + 128u;
#endif
			return;
		}
		A0 = lds_u32(smem, TT_ADDR(t0, 0, lo)) ^
		     lds_u32(smem, TT_ADDR(t1, 1, lo) + 128);
		P0 = lds_u32(smem, TT_ADDR(t2, 2, lo)) ^ k1[0];
		A1 = lds_u32(smem, TT_ADDR(t1, 0, lo)) ^
		     lds_u32(smem, TT_ADDR(t2, 1, lo) + 128);
		P1 = lds_u32(smem, TT_ADDR(t0, 3, lo) + 128) ^ k1[1];
		/* round-1 columns 2 and 3 read t3 bytes 0..1 only: constant */
		const uint32_t S2 = xor3(lds_u32(smem, TT_ADDR(t2, 0, lo)),
					 lds_u32(smem, TT_ADDR(t3c, 1, lo) + 128),
					 rot16(xor3(lds_u32(smem, TT_ADDR(t0, 2, lo)),
						    lds_u32(smem, TT_ADDR(t1, 3, lo) + 128),
						    k1[2])));
		const uint32_t S3 = xor3(lds_u32(smem, TT_ADDR(t3c, 0, lo)),
					 lds_u32(smem, TT_ADDR(t0, 1, lo) + 128),
					 rot16(xor3(lds_u32(smem, TT_ADDR(t1, 2, lo)),
						    lds_u32(smem, TT_ADDR(t2, 3, lo) + 128),
						    k1[3])));
		R0 = rot16(xor3(lds_u32(smem, TT_ADDR(S2, 2, lo)),
				lds_u32(smem, TT_ADDR(S3, 3, lo) + 128), k2[0]));
		C1a = lds_u32(smem, TT_ADDR(S2, 1, lo) + 128);
		C1b = lds_u32(smem, TT_ADDR(S3, 2, lo)) ^ k2[1];
		C2 = lds_u32(smem, TT_ADDR(S2, 0, lo)) ^
		     lds_u32(smem, TT_ADDR(S3, 1, lo) + 128);
		C3a = lds_u32(smem, TT_ADDR(S3, 0, lo));
		C3b = lds_u32(smem, TT_ADDR(S2, 3, lo) + 128) ^ k2[3];
		if (B8) {
			/* t3 byte 2 is constant too: s1 and its four round-2
			 * lookups fold into the constants */
			const uint32_t s1 = A1 ^ rot16(P1 ^ lds_u32(smem,
						TT_ADDR(t3c, 2, lo)));
			R0 ^= lds_u32(smem, TT_ADDR(s1, 1, lo) + 128);
			C1a ^= lds_u32(smem, TT_ADDR(s1, 0, lo));
			C2 ^= rot16(lds_u32(smem, TT_ADDR(s1, 3, lo) + 128) ^
				    k2[2]);
			C3a ^= rot16(lds_u32(smem, TT_ADDR(s1, 2, lo)) ^ C3b);
		}
	}

	/* keystream block b.  CACHED: exact for 0 <= b < 65536, and with
	 * T4 && CTR_B15 for 0 <= b < 256 (SGPU_CACHED_MAX_*: the host and
	 * the device planners send longer packets to the plain general
	 * kernels); b < 0 only ever lands in masked words. */
	__device__ __forceinline__ void block(const uint8_t *smem, uint32_t lo,
					      const uint32_t *rk, int32_t b,
					      uint32_t ks[4]) const
	{
		if (!CACHED) {
			const uint32_t iv[4] = {t0 ^ rk[0], t1 ^ rk[1],
						t2 ^ rk[2], t3c ^ rk[3]};
			ctr_block<NR, T4>(smem, lo, rk, iv, b, ks);
			return;
		}
		if (T4 && CTR_B15) {
			const Tt4 T = {smem, lo, lo | 0x10000u};
			const uint32_t s0 = A0 ^ lds_u32(smem, A1 ^
					(((uint32_t)b & 255u) << 8));
			uint32_t r0 = T.t0(s0) ^ R0;
			uint32_t r1 = T.t3(s0) ^ C1a;
			uint32_t r2 = T.t2(s0) ^ C2;
			uint32_t r3 = T.t1(s0) ^ C3a;
			aes4_rounds<NR, 3>(T, rk, r0, r1, r2, r3);
			ks[0] = r0; ks[1] = r1; ks[2] = r2; ks[3] = r3;
			return;
		}
		const uint32_t t3 = t3c ^ bswap32((uint32_t)b);
		if (T4) {
			const Tt4 T = {smem, lo, lo | 0x10000u};
			const uint32_t s0 = A0 ^ T.t3(t3);
			const uint32_t s1 = A1 ^ T.t2(t3);
			uint32_t r0 = xor3(T.t0(s0), T.t1(s1), R0);
			uint32_t r1 = xor3(T.t0(s1), T.t3(s0), C1a);
			uint32_t r2 = xor3(T.t2(s0), T.t3(s1), C2);
			uint32_t r3 = xor3(T.t1(s0), T.t2(s1), C3a);
			aes4_rounds<NR, 3>(T, rk, r0, r1, r2, r3);
			ks[0] = r0; ks[1] = r1; ks[2] = r2; ks[3] = r3;
			return;
		}
		if (B8) {
			/* b < 256: bswap32(b) = b << 24, one varying byte */
			const uint32_t t3b = t3c ^ ((uint32_t)b << 24);
			const uint32_t s0 = A0 ^ rot16(P0 ^ lds_u32(smem,
						TT_ADDR(t3b, 3, lo) + 128));
			uint32_t r0 = lds_u32(smem, TT_ADDR(s0, 0, lo)) ^ R0;
			uint32_t r1 = C1a ^ rot16(C1b ^ lds_u32(smem,
						TT_ADDR(s0, 3, lo) + 128));
			uint32_t r2 = C2 ^ rot16(lds_u32(smem,
						TT_ADDR(s0, 2, lo)));
			uint32_t r3 = C3a ^ lds_u32(smem,
						   TT_ADDR(s0, 1, lo) + 128);
			aes_rounds<NR, 3>(smem, lo, rk, r0, r1, r2, r3);
			ks[0] = r0; ks[1] = r1; ks[2] = r2; ks[3] = r3;
			return;
		}
		/* round 1: two varying lookups */
		const uint32_t s0 = A0 ^ rot16(P0 ^ lds_u32(smem,
					TT_ADDR(t3, 3, lo) + 128));
		const uint32_t s1 = A1 ^ rot16(P1 ^ lds_u32(smem,
					TT_ADDR(t3, 2, lo)));
		/* round 2: eight varying lookups */
		const uint32_t *k2 = rk + 8;
		uint32_t r0 = xor3(lds_u32(smem, TT_ADDR(s0, 0, lo)),
				   lds_u32(smem, TT_ADDR(s1, 1, lo) + 128), R0);
		uint32_t r1 = xor3(lds_u32(smem, TT_ADDR(s1, 0, lo)), C1a,
				   rot16(C1b ^ lds_u32(smem,
					TT_ADDR(s0, 3, lo) + 128)));
		uint32_t r2 = C2 ^ rot16(xor3(lds_u32(smem, TT_ADDR(s0, 2, lo)),
					      lds_u32(smem, TT_ADDR(s1, 3, lo) + 128),
					      k2[2]));
		uint32_t r3 = xor3(C3a, lds_u32(smem, TT_ADDR(s0, 1, lo) + 128),
				   rot16(lds_u32(smem, TT_ADDR(s1, 2, lo)) ^ C3b));
		aes_rounds<NR, 3>(smem, lo, rk, r0, r1, r2, r3);
		ks[0] = r0; ks[1] = r1; ks[2] = r2; ks[3] = r3;
	}
};

/* the SHA-1 input word at global word index gw of the HMAC message
 * M = data[0,A) ‖ (trailer?) ‖ 0x80 ‖ 0* ‖ len64 -- for non-fast chunks */
__device__ __forceinline__ uint32_t msg_word(uint32_t gw, uint32_t data_be,
					     uint32_t A, uint64_t X)
{
	uint32_t aw = A >> 2, u = A & 3;
	if (gw < aw)
		return data_be;
	if (gw == aw)
		/* 64-bit mask shift: a 32-bit shift by 32 (u = 0) is poison,
		 * which LLVM may propagate past the select guarding it */
		return (data_be & (uint32_t)(0xFFFFFFFF00000000ull >> (8 * u))) |
		       (uint32_t)(X >> (32 + 8 * u));
	if (gw == aw + 1)
		return (uint32_t)(X >> (8 * u));
	return 0;
}

/* ------------------------------------------------------------------ */
/* kernel arguments and job sources                                    */

struct KArgs {
	const uint32_t *t0;             /* AES T0 table (device, 1 KiB) */
	uint8_t *arena;
	uint64_t asz;
	const struct sgpu_job *jobs;    /* general path */
	uint32_t njobs;
	const struct sgpu_comp *comps;
	uint8_t *verdict;
	uint32_t *save;
	struct sgpu_compact c;          /* compact path */
	int nocipher;                   /* general path: the cipher regions are
					   done by k_ctr_coop (small launches) */
	/* k_ctr_small: completion word in pinned host memory (or NULL): the
	 * last workgroup stores done_seq there after every workgroup's
	 * writes, done_cnt (device, 0 between launches) counts them */
	uint32_t *done_cnt;
	uint32_t *done_flag;
	uint32_t done_seq;
	/* srtp_gpu_prof: where the kernel stores the pguard_n guard words it
	 * saw (pinned ring slot, or NULL) -- prof_guard */
	uint32_t *pguard;
	uint32_t pguard_n;
};

/* srtp_gpu_prof: the plan guard words this launch saw, stored by its
 * first thread into the launch's pinned ring slot, so the host can tell a
 * launch that did work from one its rejected plan voided without a copy
 * behind every launch */
__device__ __forceinline__ void prof_guard(const KArgs &a)
{
	if (a.pguard && a.c.guard && blockIdx.x == 0 && threadIdx.x == 0) {
		/* a set second guard word voids every class */
		const bool gf = a.c.gfail && *a.c.gfail;
		for (uint32_t q = 0; q < a.pguard_n; q++)
			a.pguard[q] = gf ? 1u : a.c.guard[q];
	}
}

/*
 * SRTCP job of a device-planned packet, exactly as plan_rtcp_enc /
 * plan_rtcp_dec (re_amd/csrc/host/srtp.c) build it (srtcp.c:31-140,
 * 143-287 of the reference): cipher region from byte 8, E || index
 * trailer, HMAC over the packet with the trailer (protect) or up to the
 * tag (unprotect), GCM with the AAD forms of srtcp.c:82-102 / 239-262.
 */
template <int MODE, bool PROT>
__device__ __forceinline__ bool rtcp_job(const KArgs &a,
					 const struct sgpu_compact &c,
					 uint32_t p, uint64_t d, uint8_t vd,
					 struct sgpu_job &j)
{
	const uint32_t comp = c.compmap[0];
	const struct sgpu_comp *cp = a.comps + comp;
	const uint32_t off = c.pos[p];
	const uint32_t L = c.end[p] - off;
	const uint32_t ix = (uint32_t)d & 0x7fffffffu;
	const uint32_t E = ((uint32_t)d >> 31) & 1u;
	const uint32_t T = cp->tag_len;
	const bool hmac = (cp->flags & 2u) != 0;
	j.off = off;
	j.comp = comp;
	j.ssrc = ((const uint32_t *)(c.hdr + p))[0];
	j.ixhi = ix >> 16;
	j.ixlo = ix & 0xffffu;
	j.trailer = E << 31 | ix;
	j.c_off = 8;
	j.t_off = 0;
	if (PROT) {
		if (MODE == SGPU_MODE_CTR) {
			j.flags = SJ_PROTECT | SJ_STORE_TRAIL |
				  (E ? SJ_CIPHER : 0u) |
				  (hmac ? (SJ_HMAC | SJ_TRAILER) : 0u);
			j.c_len = L - 8u;
			j.t_off = L;
			j.a_len = L;
			j.tag_off = L + 4u;
		}
		else {
			j.flags = SJ_PROTECT | SJ_GCM | SJ_TRAILER |
				  SJ_STORE_TRAIL | (E ? SJ_CIPHER : 0u);
			j.a_len = E ? 8u : L;
			j.c_len = E ? L - 8u : 0u;
			j.tag_off = L;
			j.t_off = L + 16u;
		}
		return true;
	}
	if (MODE == SGPU_MODE_CTR) {
		const uint32_t tag_start = L - T, eix_start = L - T - 4u;
		j.c_len = eix_start - 8u;
		j.a_len = tag_start;
		j.tag_off = tag_start;
		if (c.undo)
			j.flags = (vd & SV_CIPHERED) ? SJ_CIPHER : 0u;
		else
			j.flags = SJ_HMAC | ((E && (cp->flags & 1u)) ?
					     (SJ_CIPHER | SJ_CIPHER_IF_OK) : 0u);
	}
	else {
		const uint32_t tag_start = L - 4u - 16u;
		j.tag_off = tag_start;
		j.a_len = E ? 8u : tag_start;
		j.c_len = E ? tag_start - 8u : 0u;
		j.flags = c.undo ? (SJ_GCM | SJ_CIPHER | SJ_UNDO)
				 : (SJ_GCM | SJ_TRAILER | (E ? SJ_CIPHER : 0u));
	}
	return true;
}

/*
 * Job of thread t.  General path: jobs[t], results at slot t.  Compact
 * path: packet p = idx[base+t] (or base+t); the job is derived exactly as
 * plan_rtp_enc / plan_rtp_dec (re_amd/csrc/host/srtp.c) build it, from the
 * packet window, the parsed header and the 8-byte descriptor
 * (srtp.c:215-277, 325-382, 383-424 of the reference).
 */
template <bool COMPACT, int MODE, bool PROT>
__device__ __forceinline__ bool get_job(const KArgs &a, uint32_t t,
					struct sgpu_job &j, uint32_t &slot)
{
	if (!COMPACT) {
		if (t >= a.njobs)
			return false;
		j = a.jobs[t];
		slot = t;
		return true;
	}
	const struct sgpu_compact &c = a.c;
	if (t >= c.n)
		return false;
	if (c.guard && *c.guard)        /* the device plan was rejected */
		return false;
	const uint32_t p = c.idx ? c.idx[c.base + t] : c.base + t;
	slot = p;
	const uint64_t d = c.desc[p];
	const uint32_t fl = (uint32_t)(d >> 48);
	j.flags = SJ_SKIP;
	j.comp = 0;
	if (!(fl & SD_RUN))
		return true;
	uint8_t vd = 0;
	if (c.undo) {
		vd = a.verdict[p];
		if (MODE == SGPU_MODE_GCM && !(vd & SV_CIPHERED))
			return true;
	}
	if (c.rtcp)
		return rtcp_job<MODE, PROT>(a, c, p, d, vd, j);
	const uint32_t comp = c.compmap[c.sess ? c.sess[p] : 0u];
	const uint32_t off = c.pos[p];
	const uint32_t L = c.end[p] - off;
	const uint32_t *hw = (const uint32_t *)(c.hdr + p);
	const uint32_t ssrc = hw[0], hl = hw[2];
	const uint32_t ixhi = (uint32_t)(d >> 16);
	j.off = off;
	j.comp = comp;
	j.ssrc = ssrc;
	j.ixhi = ixhi;
	j.ixlo = (uint32_t)(d & 0xffffu);
	j.trailer = ixhi + ((fl & SD_ROC_P1) ? 1u : 0u) -
		    ((fl & SD_ROC_M1) ? 1u : 0u);
	j.t_off = 0;
	j.c_off = hl;
	if (MODE == SGPU_MODE_CTR) {
		if (PROT) {
			j.flags = SJ_PROTECT | SJ_CIPHER | SJ_HMAC | SJ_TRAILER;
			j.a_len = L;
			j.c_len = L - hl;
			j.tag_off = L;
		}
		else {
			const uint32_t T = a.comps[comp].tag_len;
			j.a_len = L - T;
			j.tag_off = L - T;
			j.c_len = L - T - hl;
			if (c.undo)
				j.flags = (vd & SV_CIPHERED) ? SJ_CIPHER : 0u;
			else
				j.flags = SJ_HMAC | SJ_TRAILER | SJ_ROC_AT_TAG |
					  ((fl & SD_CIPHER) ?
					   (SJ_CIPHER | SJ_CIPHER_IF_OK) : 0u);
		}
	}
	else {
		j.a_len = hl;
		if (PROT) {
			j.flags = SJ_PROTECT | SJ_CIPHER | SJ_GCM;
			j.c_len = L - hl;
			j.tag_off = L;
		}
		else {
			j.flags = c.undo ? (SJ_GCM | SJ_CIPHER | SJ_UNDO)
					 : (SJ_GCM | SJ_CIPHER);
			j.c_len = L - 16u - hl;
			j.tag_off = L - 16u;
		}
	}
	return true;
}

/* byte mask of chunk word bpos..bpos+3 inside the cipher region
 * [c_off, c_end) (c_off is a multiple of 4) */
__device__ __forceinline__ uint32_t region_mask(uint32_t bpos, uint32_t c_off,
						uint32_t c_end)
{
	const uint32_t nbytes = (bpos >= c_off && bpos < c_end) ?
				min(c_end - bpos, 4u) : 0u;
	/* no 32-bit shift by 32 (poison, which LLVM may carry past a select:
	 * observed as whole-word tail stores, ROCm 7.2 -O3) */
	return (uint32_t)((1ull << (8 * nbytes)) - 1ull);
}

/*
 * XOR the keystream into the 16 words d[] of chunk k as each AES block is
 * produced (no 16-word keystream buffer).  Word jj of the chunk takes
 * keystream word jj - SHIFT of block blk0 = 4k - cw4; the first SHIFT words
 * take the tail of the previous chunk's last block (carry).  MASKED: only
 * the bytes inside the cipher region [c_off, c_end) change (chunk starts
 * at byte c0); the mask is computed per word, not held in an array.
 */
template <int NR, int SHIFT, bool MASKED, bool CACHED, bool T4>
__device__ __forceinline__ void ks_xor(const uint8_t *smem, uint32_t lo,
				       const uint32_t *rk,
				       const CtrKs<NR, CACHED, T4> &C,
				       int32_t blk0, uint32_t carry[4],
				       uint32_t d[16], uint32_t c0 = 0,
				       uint32_t c_off = 0, uint32_t c_end = 0)
{
#define KS_MASK(jj) (MASKED ? region_mask(c0 + 4u * (jj), c_off, c_end) \
			    : 0xffffffffu)
#pragma unroll
	for (int q = 0; q < SHIFT; q++)
		d[q] ^= carry[4 - SHIFT + q] & KS_MASK(q);
#pragma unroll
	for (int m = 0; m < 4; m++) {
		uint32_t B[4];
		C.block(smem, lo, rk, blk0 + m, B);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const int jj = SHIFT + 4 * m + q;
			if (jj < 16)
				d[jj] ^= B[q] & KS_MASK(jj);
			else
				carry[q] = B[q];
		}
		if (m == 3 && SHIFT == 0) {
#pragma unroll
			for (int q = 0; q < 4; q++)
				carry[q] = B[q];
		}
	}
#undef KS_MASK
}

/* ks_xor (unmasked) with a per-lane keystream mask: d ^= ks & km, one
 * v_bitop3 per word (a ^ (b & c): table 0x78) */
template <int NR, int SHIFT, bool CACHED, bool T4>
__device__ __forceinline__ void ks_xor_km(const uint8_t *smem, uint32_t lo,
					  const uint32_t *rk,
					  const CtrKs<NR, CACHED, T4> &C,
					  int32_t blk0, uint32_t carry[4],
					  uint32_t d[16], uint32_t km)
{
#pragma unroll
	for (int q = 0; q < SHIFT; q++)
		d[q] = __builtin_amdgcn_bitop3_b32(d[q], carry[4 - SHIFT + q], km,
						   0x78);
#pragma unroll
	for (int m = 0; m < 4; m++) {
		uint32_t B[4];
		C.block(smem, lo, rk, blk0 + m, B);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const int jj = SHIFT + 4 * m + q;
			if (jj < 16)
				d[jj] = __builtin_amdgcn_bitop3_b32(d[jj], B[q], km,
								   0x78);
			else
				carry[q] = B[q];
		}
		if (m == 3 && SHIFT == 0) {
#pragma unroll
			for (int q = 0; q < 4; q++)
				carry[q] = B[q];
		}
	}
}

/*
 * The 16 keystream words of chunk k (blk0 = 4k - cw4) into ks[], carry as
 * in ks_xor.  Used one chunk ahead of the MAC: the AES lookups of chunk
 * k+1 (LDS-latency bound) have no dependence on the SHA-1 rounds of chunk
 * k (VALU-chain bound), so one basic block holds both and the scheduler
 * fills each lookup's latency with SHA-1 work.
 */
template <int NR, int SHIFT, bool CACHED, bool T4>
__device__ __forceinline__ void chunk_ks(const uint8_t *smem, uint32_t lo,
					 const uint32_t *rk,
					 const CtrKs<NR, CACHED, T4> &C,
					 int32_t blk0, uint32_t carry[4],
					 uint32_t ks[16])
{
#pragma unroll
	for (int q = 0; q < SHIFT; q++)
		ks[q] = carry[4 - SHIFT + q];
#pragma unroll
	for (int m = 0; m < 4; m++) {
		uint32_t B[4];
		C.block(smem, lo, rk, blk0 + m, B);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const int jj = SHIFT + 4 * m + q;
			if (jj < 16)
				ks[jj] = B[q];
			else
				carry[q] = B[q];
		}
	}
}

/* ------------------------------------------------------------------ */
/*
 * Quad-coalesced chunk access.  With one packet per lane, a wave64 load of
 * 16 B per lane touches 64 cache lines (one per packet).  Instead the four
 * lanes of a quad move one packet's 64-byte chunk together: in access g,
 * lane j of the quad reads/writes bytes [16j, 16j+16) of the chunk of quad
 * lane g, so one instruction touches 16 lines, 64 contiguous bytes each.
 * A 4x4 transpose across the quad (two DPP quad_perm + select stages)
 * turns "quarter j of packet g" into "quarter g of my packet" and back.
 * scripts/ubench_ctr.hip: the per-lane pattern costs the fused CTR+HMAC
 * loop ~30 % over its compute time, the coalesced one ~1 %.
 */
#define DPP_QXOR1 0xB1   /* quad_perm [1,0,3,2] */
#define DPP_QXOR2 0x4E   /* quad_perm [2,3,0,1] */

template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t v)
{
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

/* x[r][c] = word c of register r; transposes (register, quad lane).  The
 * selects are v_bitop3 with lane masks (a ?: on many values can become a
 * divergent branch, which would split the loop body). */
__device__ __forceinline__ void quad_transpose(uint32_t x[4][4], uint32_t lane)
{
	const uint32_t m0 = 0u - (lane & 1u), m1 = 0u - ((lane >> 1) & 1u);
#pragma unroll
	for (int c = 0; c < 4; c++) {
#pragma unroll
		for (int r = 0; r < 4; r += 2) {
			const uint32_t t0 = qdpp<DPP_QXOR1>(x[r][c]);
			const uint32_t t1 = qdpp<DPP_QXOR1>(x[r + 1][c]);
			x[r + 1][c] = sha_ch(m0, x[r + 1][c], t0);
			x[r][c] = sha_ch(m0, t1, x[r][c]);
		}
#pragma unroll
		for (int r = 0; r < 2; r++) {
			const uint32_t t0 = qdpp<DPP_QXOR2>(x[r][c]);
			const uint32_t t2 = qdpp<DPP_QXOR2>(x[r + 2][c]);
			x[r + 2][c] = sha_ch(m1, x[r + 2][c], t0);
			x[r][c] = sha_ch(m1, t2, x[r][c]);
		}
	}
}

/* qb[g] = arena offset of the packet of quad lane g + 16 * (my quad index)
 * (offsets, not pointers: the arena pointer keeps the accesses global) */
__device__ __forceinline__ void quad_offsets(uint64_t off, uint32_t lane,
					     uint64_t qb[4])
{
	const uint32_t lo = (uint32_t)off, hi = (uint32_t)(off >> 32);
	const uint32_t l4[4] = {qdpp<0x00>(lo), qdpp<0x55>(lo),
				qdpp<0xAA>(lo), qdpp<0xFF>(lo)};
	const uint32_t h4[4] = {qdpp<0x00>(hi), qdpp<0x55>(hi),
				qdpp<0xAA>(hi), qdpp<0xFF>(hi)};
#pragma unroll
	for (int g = 0; g < 4; g++)
		qb[g] = ((uint64_t)h4[g] << 32 | l4[g]) + 16u * (lane & 3u);
}

/* own 16 words of chunk c0 (every lane of the quad takes part) */
__device__ __forceinline__ void quad_load(const uint8_t *arena,
					  const uint64_t qb[4], uint32_t c0,
					  uint32_t lane, uint32_t d[16])
{
	uint32_t x[4][4];
#pragma unroll
	for (int g = 0; g < 4; g++) {
		const uint4 v = *(const uint4 *)(arena + qb[g] + c0);
		x[g][0] = v.x; x[g][1] = v.y; x[g][2] = v.z; x[g][3] = v.w;
	}
	quad_transpose(x, lane);
#pragma unroll
	for (int q = 0; q < 4; q++)
#pragma unroll
		for (int c = 0; c < 4; c++)
			d[4 * q + c] = x[q][c];
}

__device__ __forceinline__ void quad_store(uint8_t *arena, const uint64_t qb[4],
					   uint32_t c0, uint32_t lane,
					   const uint32_t s[16])
{
	uint32_t x[4][4];
#pragma unroll
	for (int q = 0; q < 4; q++)
#pragma unroll
		for (int c = 0; c < 4; c++)
			x[q][c] = s[4 * q + c];
	quad_transpose(x, lane);
#pragma unroll
	for (int g = 0; g < 4; g++)
		*(uint4 *)(arena + qb[g] + c0) =
			make_uint4(x[g][0], x[g][1], x[g][2], x[g][3]);
}

/* store_region with volatile stores: exactly the bytes of the region,
 * never widened to the whole word (see gcm.hip k_gcmu) */
__device__ __forceinline__ void store_region_exact(uint8_t *pkt, uint32_t c0,
						   const uint32_t d[16],
						   uint32_t c_off, uint32_t c_end)
{
	volatile uint8_t *vp = pkt;
#pragma unroll
	for (int jj = 0; jj < 16; jj++) {
		const uint32_t bpos = c0 + 4u * jj;
		if (bpos >= c_off && bpos < c_end) {
			const uint32_t nbytes = min(c_end - bpos, 4u);
			if (nbytes == 4)
				*(volatile uint32_t *)(vp + bpos) = d[jj];
			else
				for (uint32_t z = 0; z < nbytes; z++)
					vp[bpos + z] = (uint8_t)(d[jj] >> (8 * z));
		}
	}
}

/* store the words of chunk c0 that lie in the cipher region */
__device__ __forceinline__ void store_region(uint8_t *pkt, uint32_t c0,
					     const uint32_t d[16],
					     uint32_t c_off, uint32_t c_end)
{
#pragma unroll
	for (int jj = 0; jj < 16; jj++) {
		const uint32_t bpos = c0 + 4u * jj;
		if (bpos >= c_off && bpos < c_end) {
			const uint32_t nbytes = min(c_end - bpos, 4u);
			if (nbytes == 4)
				*(uint32_t *)(pkt + bpos) = d[jj];
			else
				st_partial(pkt + bpos, d[jj], nbytes);
		}
	}
}

typedef void (*kfn_t)(const KArgs);

/* small.hip: the per-packet path's fused kernel over (mapped) memory */
#define SGPU_SMALL_MAX_BYTES 2048
int small_launch(uint8_t *arena, uint64_t arena_size,
		 const struct sgpu_job *jobs, uint32_t njobs, uint8_t *verdict,
		 uint32_t *save, const struct sgpu_comp *comps,
		 const uint32_t *t0, int prot, uint32_t *done_cnt,
		 uint32_t *done_flag, uint32_t done_seq, void *stream);

int small_srv_launch(const struct sgpu_comp *comps, const uint32_t *t0,
		     struct sgpu_srv_mb *mb, struct sgpu_srv_bc *bc,
		     uint32_t grid, uint32_t linger_us, uint32_t life_us,
		     uint32_t *done_cnt, uint32_t *done_flag, void *stream);

/* kernel pickers, one per translation unit */
unsigned sgpu_ctr_block(bool uni, int prot);
kfn_t sgpu_pick_ctr10(bool compact, bool uni, int shift, int prot);
kfn_t sgpu_pick_ctr10_coop(int prot);
kfn_t sgpu_pick_gcm_coop(int nr);
kfn_t sgpu_pick_ctr14_coop(int prot);
kfn_t sgpu_pick_ctr14(bool compact, bool uni, int shift, int prot);
kfn_t sgpu_pick_ctr10_any(bool uni, int prot);
kfn_t sgpu_pick_ctr14_any(bool uni, int prot);
kfn_t sgpu_pick_gcm(bool compact, bool uni, int nr, int prot);
/* refix: 0 the kernel, 1 full-grid restore, 2 list restore (c.flist) */
kfn_t sgpu_pick_ctr10_fast(int prot, int refix);
kfn_t sgpu_pick_ctr14_fast(int prot, int refix);
unsigned sgpu_ctr_fast_block(int prot);
kfn_t sgpu_pick_ctr10_fast_mk(int prot);
kfn_t sgpu_pick_ctr14_fast_mk(int prot);
kfn_t sgpu_pick_ctr10_fast_rtcp(int prot);
kfn_t sgpu_pick_ctr14_fast_rtcp(int prot);
unsigned sgpu_ctr_fast_mk_block(void);
unsigned sgpu_gcm_block(bool uni);
