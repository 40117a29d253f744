/*
 * k_ctr_fast.h -- lean AES-CM + HMAC-SHA1 kernel for device-planned,
 * single-key RTP batches (BASELINE configs 2 and 5: srtp_encrypt
 * srtp.c:183-285 / srtp_decrypt srtp.c:288-432 of one stream, every packet
 * planned by k_plan_* with SD_RUN | SD_CIPHER).
 *
 * k_ctr_hmac (k_ctr.h) serves every job shape of the general engine and the
 * host-scanned batches: skips, undo passes, SRTCP trailers, decrypt-if-
 * authentic with an in-kernel restore, per-lane keys.  Carried through one
 * register allocation that generality spills at 4 waves/SIMD.  This kernel
 * knows the shape the device planner guarantees:
 *   - one session key: round keys and HMAC midstates in SGPRs;
 *   - cipher region [hl, A) and MAC input [0, A) || BE32(ROC), A = L
 *     (protect) or L - tag (unprotect);
 *   - unprotect decrypts speculatively; a forged packet is restored to its
 *     ciphertext by k_ctr_fast_refix (launched behind, exits at once when
 *     the miss counter is zero), so this kernel holds no restore state;
 *   - arena offsets are 32-bit (host-checked), quad-coalesced steady
 *     chunks in both directions.
 * 1024-thread blocks, 4 waves/SIMD, one 128 KiB T4 image per CU.
 */
#pragma once
#include "kern_common.h"

#ifndef CTRF_BLOCK
#define CTRF_BLOCK 1024
#endif
#ifndef CTRF_BLOCK_U        /* unprotect block (its register budget) */
#define CTRF_BLOCK_U CTRF_BLOCK
#endif
#define CTRF_BLK(PROT) ((PROT) ? CTRF_BLOCK : CTRF_BLOCK_U)
#ifndef CTRF_COAL_P         /* quad-coalesced steady chunks, protect */
#define CTRF_COAL_P 1
#endif
#ifndef CTRF_COAL_U         /* ... unprotect */
#define CTRF_COAL_U 1
#endif
#ifndef CTRF_COAL_MK        /* ... per-lane-key (multi-session) kernel */
#define CTRF_COAL_MK 1
#endif
#ifndef CTRF_SB_ST          /* per-lane steady chunks: stores together --
			       off: unlike GCM's, config 4 moved the same
			       bytes either way (3.28 GB, 1.05 ms per launch,
			       same-box A/B) and the unprotect body spilled
			       147 VGPRs instead of 110 */
#define CTRF_SB_ST 0
#endif
#ifndef CTRF_PRIO           /* steady chunks lower the wave's issue priority
				   as it advances (s_setprio 3..0 by quarter of
				   the packet): the SIMD's oldest-first
				   arbitration otherwise finishes its 4 waves at
				   51/68/84/100 % of a workgroup's lifetime
				   (profiles/r05/fused_waves.txt) */
#define CTRF_PRIO 0
#endif
#ifndef CTRF_SHAFIRST_U     /* unprotect steady chunk: MAC, then decrypt */
#define CTRF_SHAFIRST_U 1
#endif
#ifndef CTRF_SB_BLOCKS      /* scheduling barrier every N AES blocks of a
			       steady chunk (0: none) -- bounds the AES ILP
			       the scheduler builds, i.e. the VGPRs */
#define CTRF_SB_BLOCKS 0
#endif
#ifndef CTRF_SB_SHA         /* scheduling barrier between MAC and cipher */
#define CTRF_SB_SHA 0
#endif

/* ks_xor (unmasked, kern_common.h) with scheduling barriers between the
 * four keystream blocks of a chunk */
template <int NR, int SHIFT>
__device__ __forceinline__ void fast_ks_xor(const uint8_t *smem, uint32_t lo,
					    const uint32_t *rk,
					    const CtrKs<NR, true, true> &C,
					    int32_t blk0, uint32_t carry[4],
					    uint32_t d[16])
{
#pragma unroll
	for (int q = 0; q < SHIFT; q++)
		d[q] ^= carry[4 - SHIFT + q];
#pragma unroll
	for (int m = 0; m < 4; m++) {
		uint32_t B[4];
		C.block(smem, lo, rk, blk0 + m, B);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const int jj = SHIFT + 4 * m + q;
			if (jj < 16)
				d[jj] ^= B[q];
			else
				carry[q] = B[q];
		}
		if (m == 3 && SHIFT == 0) {
#pragma unroll
			for (int q = 0; q < 4; q++)
				carry[q] = B[q];
		}
		if (CTRF_SB_BLOCKS && (m + 1) % (CTRF_SB_BLOCKS > 0 ?
						 CTRF_SB_BLOCKS : 1) == 0 &&
		    m < 3)
			__builtin_amdgcn_sched_barrier(0);
	}
}

/* the planned packet of thread t: window, header length, index, ROC */
struct FastPkt {
	uint32_t p, off, L, hl, ssrc, ixhi, ixlo, roc;
};

template <bool RTCP = false>
__device__ __forceinline__ bool fast_pkt(const struct sgpu_compact &c,
					 uint32_t t, FastPkt &f)
{
	if (t >= c.n)
		return false;
	f.p = c.idx ? c.idx[c.base + t] : c.base + t;
	const uint64_t d = c.desc[f.p];
	const uint32_t fl = (uint32_t)(d >> 48);
	if (!(fl & SD_RUN))
		return false;
	f.off = c.pos[f.p];
	f.L = c.end[f.p] - f.off;
	const uint32_t *hw = (const uint32_t *)(c.hdr + f.p);
	f.ssrc = hw[0];
	f.hl = hw[2];
	if (RTCP) {
		/* SRTCP (sgpu_rdesc): E || index is both the IV's index
		 * (srtcp.c srtp_iv_calc) and the MAC trailer word */
		const uint32_t w = (uint32_t)d;
		f.ixhi = (w & 0x7fffffffu) >> 16;
		f.ixlo = w & 0xffffu;
		f.roc = w;
		return true;
	}
	f.ixhi = (uint32_t)(d >> 16);
	f.ixlo = (uint32_t)(d & 0xffffu);
	f.roc = f.ixhi + ((fl & SD_ROC_P1) ? 1u : 0u) -
		((fl & SD_ROC_M1) ? 1u : 0u);
	return true;
}

/* round keys of context ci (uniform) in SGPRs, plain (T4 rounds) */
template <int NR>
__device__ __forceinline__ const struct sgpu_comp *
fast_keys_at(const KArgs &a, uint32_t ci, uint32_t rk[4 * (NR + 1)])
{
	const struct sgpu_comp *cp = a.comps + ci;
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		const uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}
#pragma unroll
	for (int k = 4; k < 4 * NR; k++)
		rk[k] = rot16(rk[k]);
#pragma unroll
	for (int k = 0; k < 4 * (NR + 1); k++)
		rk[k] = __builtin_amdgcn_readfirstlane(rk[k]);
	return cp;
}

/* ... of the launch's one context (c.compmap[0]) */
template <int NR>
__device__ __forceinline__ const struct sgpu_comp *
fast_keys(const KArgs &a, uint32_t rk[4 * (NR + 1)])
{
	return fast_keys_at<NR>(
		a, __builtin_amdgcn_readfirstlane(a.c.compmap[0]), rk);
}

/* round keys of packet f's own context in VGPRs (multi-session batches:
 * one context per lane, c.compmap[c.sess[p]]), same layout as fast_keys */
template <int NR>
__device__ __forceinline__ const struct sgpu_comp *
lane_keys(const KArgs &a, const FastPkt &f, uint32_t rk[4 * (NR + 1)])
{
	const struct sgpu_comp *cp = a.comps + a.c.compmap[a.c.sess[f.p]];
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		const uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}
#pragma unroll
	for (int k = 4; k < 4 * NR; k++)
		rk[k] = rot16(rk[k]);
	return cp;
}

/* srtp_iv_calc (misc.c:76-87): k_s ^ (0, ssrc, ix >> 16, ix << 16) */
__device__ __forceinline__ void fast_iv(const struct sgpu_comp *cp,
					const FastPkt &f, uint32_t iv[4])
{
	const uint4 ks = *(const uint4 *)cp->k_s;
	iv[0] = ks.x;
	iv[1] = ks.y ^ bswap32(f.ssrc);
	iv[2] = ks.z ^ bswap32(f.ixhi);
	iv[3] = (ks.w ^ (bswap32(f.ixlo) >> 16)) & 0xffffu;
}

/*
 * Keystream over the cipher region [c_off, c_end) of a head/tail chunk
 * and write-back of every word it touches.  Each word's byte mask passes
 * an optimisation barrier and the store is always the whole word (loaded
 * bytes outside the region go back unchanged): hipcc (ROCm 7.2, -O3)
 * compiled the masked partial-word form (region_mask + store_region) into
 * whole-word stores of unmasked keystream at some region ends, over the
 * tag.
 */
template <int NR, int SHIFT>
__device__ __forceinline__ void tail_xor_store(const uint8_t *smem,
					       uint32_t lo, const uint32_t *rk,
					       const CtrKs<NR, true, true> &C,
					       int32_t blk0, uint32_t carry[4],
					       uint32_t d[16], uint8_t *pkt,
					       uint32_t c0, uint32_t c_off,
					       uint32_t c_end)
{
	uint32_t ks[16];
	chunk_ks<NR, SHIFT>(smem, lo, rk, C, blk0, carry, ks);
#pragma unroll
	for (int jj = 0; jj < 16; jj++) {
		const uint32_t bpos = c0 + 4u * jj;
		uint32_t m = region_mask(bpos, c_off, c_end);
		asm volatile("" : "+v"(m));
		d[jj] = __builtin_amdgcn_bitop3_b32(d[jj], ks[jj], m, 0x78);
		if (bpos + 4u > c_off && bpos < c_end)
			*(uint32_t *)(pkt + bpos) = d[jj];
	}
}

/*
 * RTCP: single-key SRTCP batches planned by k_plan_rtcp (srtcp_encrypt
 * srtcp.c:31-140, srtcp_decrypt srtcp.c:143-287): header class 2 (hl =
 * 8), the MAC trailer word is E || index (protect: stored at L in front
 * of the tag; unprotect: the 4 bytes in front of the tag, so A = L - T -
 * 4), no ROC written over the tag, E = 0: no cipher region.
 */
/* one planned packet f (T4 image already in smem); ci: the launch's one
 * context (uniform), unused with MK */
template <int NR, int SHIFT, bool PROT, bool MK = false, bool RTCP = false>
__device__ __forceinline__ void ctr_fast_pkt(const KArgs &a, uint8_t *smem,
					     const FastPkt &f, uint32_t ci)
{
	uint32_t rk[4 * (NR + 1)];
	/* MK: every lane its own session context (keys in VGPRs); all of
	 * them one suite, so the tag length stays uniform */
	const struct sgpu_comp *cp = MK ? lane_keys<NR>(a, f, rk)
					: fast_keys_at<NR>(a, ci, rk);
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	const uint32_t lane = threadIdx.x & 63u;
	uint8_t *const arena = a.arena;
	uint8_t *const pkt = arena + f.off;
	const uint64_t pasz = a.asz - f.off;
	const uint32_t T = PROT ? 0u : __builtin_amdgcn_readfirstlane(cp->tag_len);
	/* MAC data / cipher end */
	const uint32_t A = f.L - T - (RTCP && !PROT ? 4u : 0u);
	/* unencrypted SRTCP (E = 0): an empty cipher region */
	const uint32_t hl = RTCP && !(f.roc >> 31) ? A : f.hl;

	uint32_t iv[4];
	fast_iv(cp, f, iv);
	CtrKs<NR, true, true> C;
	C.init(smem, lo, rk, iv);
	uint32_t h[5] = {cp->ipad[0], cp->ipad[1], cp->ipad[2], cp->ipad[3],
			 cp->ipad[4]};
	const uint64_t X = (uint64_t)f.roc << 32 | 0x80000000u;
	const uint32_t nb = (A + 4u + 9u + 63u) / 64u;   /* SHA-1 blocks */
	const uint64_t bitlen = (uint64_t)(64u + A + 4u) * 8u;
	const int32_t cw4 = (int32_t)(hl >> 4);
	/* steady chunks: wholly inside [0, A), cipher from word SHIFT of
	 * the first 16 bytes on (the zero carry leaves words < hl as is) */
	const uint32_t kf0 = hl < 16u ? 0u : min((hl + 63u) / 64u, nb);
	const uint32_t kf1 = max(A / 64u, kf0);
	uint32_t carry[4] = {0, 0, 0, 0};

	/* header / tail chunk: byte-exact region, trailer and padding */
	auto general = [&](uint32_t k) {
		const uint32_t c0 = 64u * k;
		uint32_t d[16], w[16];
#pragma unroll
		for (int g = 0; g < 4; g++) {
			uint4 v = make_uint4(0, 0, 0, 0);
			if (c0 + 16u * g < A)
				v = ld16(pkt, pasz, c0 + 16u * g);
			d[4 * g] = v.x; d[4 * g + 1] = v.y;
			d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
		}
		if (!PROT) {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = msg_word(16u * k + jj, bswap32(d[jj]), A, X);
		}
		if (c0 + 64u > hl && c0 < A)
			tail_xor_store<NR, SHIFT>(smem, lo, rk, C,
						  (int32_t)(4 * k) - cw4, carry,
						  d, pkt, c0, hl, A);
		if (PROT) {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = msg_word(16u * k + jj, bswap32(d[jj]), A, X);
		}
		if (k + 1 == nb) {
			w[14] = (uint32_t)(bitlen >> 32);
			w[15] = (uint32_t)bitlen;
		}
		sha1_compress(h, w);
	};

	uint32_t k = 0;
	for (; k < kf0; k++)
		general(k);

	constexpr bool COAL = MK ? CTRF_COAL_MK :
			      PROT ? CTRF_COAL_P : CTRF_COAL_U;
	uint32_t K0 = kf1, K1 = kf1;
	uint32_t qo[4];                         /* 32-bit quad offsets */
	if constexpr (COAL) {
		qo[0] = qdpp<0x00>(f.off) + 16u * (lane & 3u);
		qo[1] = qdpp<0x55>(f.off) + 16u * (lane & 3u);
		qo[2] = qdpp<0xAA>(f.off) + 16u * (lane & 3u);
		qo[3] = qdpp<0xFF>(f.off) + 16u * (lane & 3u);
		const uint64_t act = __ballot(1);
		uint32_t a0 = max(kf0, qdpp<DPP_QXOR1>(kf0));
		a0 = max(a0, qdpp<DPP_QXOR2>(a0));
		uint32_t a1 = min(kf1, qdpp<DPP_QXOR1>(kf1));
		a1 = min(a1, qdpp<DPP_QXOR2>(a1));
		if (((act >> (lane & ~3u)) & 0xfull) == 0xfull && a0 < a1) {
			K0 = a0;
			K1 = a1;
		}
	}
	auto steady = [&](uint32_t k, auto coal) {
		constexpr bool CO = decltype(coal)::value;
		const uint32_t c0 = 64u * k;
		if (CTRF_PRIO) {
			/* wave-uniform progress quarter -> priority 3..0 */
			const uint32_t q4 =
				(uint32_t)__builtin_amdgcn_readfirstlane(4u * k) /
				(uint32_t)__builtin_amdgcn_readfirstlane(nb);
			if (q4 == 0)
				__builtin_amdgcn_s_setprio(3);
			else if (q4 == 1)
				__builtin_amdgcn_s_setprio(2);
			else if (q4 == 2)
				__builtin_amdgcn_s_setprio(1);
			else
				__builtin_amdgcn_s_setprio(0);
		}
		uint32_t d[16], w[16];
		if constexpr (CO) {
			uint32_t x[4][4];
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = *(const uint4 *)(arena + (qo[g] + c0));
				x[g][0] = v.x; x[g][1] = v.y; x[g][2] = v.z;
				x[g][3] = v.w;
			}
			quad_transpose(x, lane);
#pragma unroll
			for (int q = 0; q < 4; q++)
#pragma unroll
				for (int cc = 0; cc < 4; cc++)
					d[4 * q + cc] = x[q][cc];
		}
		else {
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = *(const uint4 *)(pkt + c0 + 16u * g);
				d[4 * g] = v.x; d[4 * g + 1] = v.y;
				d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
			}
		}
		if (!PROT && CTRF_SHAFIRST_U) {
			/* the MAC covers the received ciphertext */
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = bswap32(d[jj]);
			sha1_compress(h, w);
			if (CTRF_SB_SHA)
				__builtin_amdgcn_sched_barrier(0);
		}
		fast_ks_xor<NR, SHIFT>(smem, lo, rk, C, (int32_t)(4 * k) - cw4,
				       carry, d);
		if constexpr (CO) {
			uint32_t x[4][4];
#pragma unroll
			for (int q = 0; q < 4; q++)
#pragma unroll
				for (int cc = 0; cc < 4; cc++)
					x[q][cc] = d[4 * q + cc];
			quad_transpose(x, lane);
#pragma unroll
			for (int g = 0; g < 4; g++)
				*(uint4 *)(arena + (qo[g] + c0)) =
					make_uint4(x[g][0], x[g][1], x[g][2],
						   x[g][3]);
		}
		else {
			/* CTRF_SB_ST: a lane's four 16-B stores of its 64-B
			 * line back to back (gcm.hip gcma_packet) */
			if (CTRF_SB_ST)
				__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int g = 0; g < 4; g++)
				*(uint4 *)(pkt + c0 + 16u * g) =
					make_uint4(d[4 * g], d[4 * g + 1],
						   d[4 * g + 2], d[4 * g + 3]);
		}
		if (PROT) {
			/* the MAC covers the ciphertext just produced */
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = bswap32(d[jj]);
			sha1_compress(h, w);
		}
		else if (!CTRF_SHAFIRST_U) {
			/* d is plaintext now: the MAC needs the ciphertext
			 * back (CTR: d ^ ks) -- not this form's default */
		}
	};
	static_assert(PROT || CTRF_SHAFIRST_U,
		      "unprotect steady chunks MAC the ciphertext first");
	for (; k < K0; k++)
		steady(k, std::false_type());
	if constexpr (COAL) {
		for (; k < K1; k++)
			steady(k, std::true_type());
		for (; k < kf1; k++)
			steady(k, std::false_type());
	}
	for (; k < nb; k++)
		general(k);

	/* outer hash: opad midstate + 20-byte inner digest */
	{
		uint32_t w[16];
		w[0] = h[0]; w[1] = h[1]; w[2] = h[2]; w[3] = h[3]; w[4] = h[4];
		w[5] = 0x80000000u;
#pragma unroll
		for (int q = 6; q < 15; q++)
			w[q] = 0;
		w[15] = (64u + 20u) * 8u;
		h[0] = cp->opad[0]; h[1] = cp->opad[1]; h[2] = cp->opad[2];
		h[3] = cp->opad[3]; h[4] = cp->opad[4];
		sha1_compress(h, w);
	}
	const uint32_t tag_len = __builtin_amdgcn_readfirstlane(cp->tag_len);
	uint8_t *tp = pkt + A;
	if (PROT) {
		if (RTCP) {
			st_be32(tp, f.roc);     /* E || index (srtcp.c:115) */
			tp += 4;
		}
		for (uint32_t q = 0; q < tag_len; q++)
			tp[q] = (uint8_t)(h[q >> 2] >> (24 - 8 * (q & 3)));
		return;
	}
	if (RTCP) {
		/* tp = the tag: no ROC written over it */
		tp += 4;
		uint32_t diff = 0;
		for (uint32_t q = 0; q < tag_len; q++)
			diff |= tp[q] ^ (uint8_t)(h[q >> 2] >> (24 - 8 * (q & 3)));
		const uint8_t vd = (diff == 0 ? SV_TAG_OK : 0) | SV_CIPHERED;
		if (!(vd & SV_TAG_OK))
			atomicAdd(a.c.nfail, 1u);
		if (a.verdict)
			a.verdict[f.p] = vd;
		return;
	}
	uint32_t diff = 0;
	for (uint32_t q = 0; q < tag_len; q++)
		diff |= tp[q] ^ (uint8_t)(h[q >> 2] >> (24 - 8 * (q & 3)));
	/* the reference writes the ROC over the tag before comparing
	 * (srtp.c:342-344); the original word is kept for an undo */
	if (a.c.save)
		a.c.save[f.p] = (uint32_t)tp[0] | (uint32_t)tp[1] << 8 |
				(uint32_t)tp[2] << 16 | (uint32_t)tp[3] << 24;
	st_be32(tp, f.roc);
	const uint8_t vd = (diff == 0 ? SV_TAG_OK : 0) | SV_CIPHERED;
	if (!(vd & SV_TAG_OK)) {
		const uint32_t q = atomicAdd(a.c.nfail, 1u);
		if (a.c.flist)
			a.c.flist[q] = f.p;
	}
	if (a.verdict)
		a.verdict[f.p] = vd;
}

#ifndef CTRF_FILL_LOOP
#define CTRF_FILL_LOOP 0
#endif
template <int NR, int SHIFT, bool PROT, bool MK = false, bool RTCP = false>
__device__ __forceinline__ void ctr_fast_body(const KArgs &a, uint8_t *smem)
{
	if (CTRF_FILL_LOOP || blockDim.x != 1024u)
		tt4_fill(smem, a.t0);
	else
		tt4_fill_b1024(smem, a.t0);
	__syncthreads();
	FastPkt f;
	if (!fast_pkt<RTCP>(a.c, blockIdx.x * blockDim.x + threadIdx.x, f))
		return;
	ctr_fast_pkt<NR, SHIFT, PROT, MK, RTCP>(
		a, smem, f,
		MK ? 0u : __builtin_amdgcn_readfirstlane(a.c.compmap[0]));
}

/*
 * The same restore from the list of forged packets (a.c.flist, filled by
 * the fast kernel): one packet per workgroup, one 16-byte keystream block
 * per thread, so a few forged packets cost a few short blocks instead of
 * a full-grid pass where each forged packet runs its whole keystream on
 * one lane.  Bytes [hl, A) only: the ROC at A stays (srtp.c:342-344).
 */
template <int NR, bool MK = false>
__global__ void __launch_bounds__(256)
k_ctr_refix_list(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	const uint32_t nf = *(volatile const uint32_t *)a.c.nfail;
	if (blockIdx.x >= nf)
		return;
	tt4_fill(smem, a.t0);
	__syncthreads();
	uint32_t rk[4 * (NR + 1)];
	/* MK (multi-session batches): the forged packet's own session
	 * context, uniform over the workgroup, loaded per packet below */
	const struct sgpu_comp *cp = MK ? a.comps : fast_keys<NR>(a, rk);
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	for (uint32_t q = blockIdx.x; q < nf; q += gridDim.x) {
		const uint32_t p = a.c.flist[q];
		FastPkt f;
		if (!MK && !fast_pkt(a.c, p - a.c.base, f))
			continue;
		if (MK) {
			/* the fast kernel walked c.idx (launch order): the
			 * listed p is a packet index, so read it directly */
			const uint64_t d = a.c.desc[p];
			const uint32_t fl = (uint32_t)(d >> 48);
			if (!(fl & SD_RUN))
				continue;
			f.p = p;
			f.off = a.c.pos[p];
			f.L = a.c.end[p] - f.off;
			const uint32_t *hw = (const uint32_t *)(a.c.hdr + p);
			f.ssrc = hw[0];
			f.hl = hw[2];
			f.ixhi = (uint32_t)(d >> 16);
			f.ixlo = (uint32_t)(d & 0xffffu);
			f.roc = f.ixhi + ((fl & SD_ROC_P1) ? 1u : 0u) -
				((fl & SD_ROC_M1) ? 1u : 0u);
			const uint32_t ci = __builtin_amdgcn_readfirstlane(
				a.c.compmap[a.c.sess[p]]);
			cp = a.comps + ci;
#pragma unroll
			for (int k = 0; k < NR + 1; k++) {
				const uint4 v = *(const uint4 *)&cp->rk[4 * k];
				rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
				rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
			}
#pragma unroll
			for (int k = 4; k < 4 * NR; k++)
				rk[k] = rot16(rk[k]);
#pragma unroll
			for (int k = 0; k < 4 * (NR + 1); k++)
				rk[k] = __builtin_amdgcn_readfirstlane(rk[k]);
		}
		const uint32_t T = __builtin_amdgcn_readfirstlane(cp->tag_len);
		uint8_t *pkt = a.arena + f.off;
		const uint32_t A = f.L - T;
		uint32_t iv[4];
		fast_iv(cp, f, iv);
		CtrKs<NR, true, true> C;
		C.init(smem, lo, rk, iv);
		for (uint32_t b = threadIdx.x; f.hl + 16u * b < A;
		     b += blockDim.x) {
			uint32_t ks[4];
			C.block(smem, lo, rk, (int32_t)b, ks);
			const uint32_t p0 = f.hl + 16u * b;
#pragma unroll
			for (int w = 0; w < 4; w++) {
				const uint32_t bp = p0 + 4u * w;
				if (bp >= A)
					break;
				if (A - bp >= 4u) {
					uint32_t *wp = (uint32_t *)(pkt + bp);
					*wp = *wp ^ ks[w];
				}
				else {
					for (uint32_t k = 0; k < A - bp; k++)
						pkt[bp + k] ^= (uint8_t)(ks[w] >>
									 (8 * k));
				}
			}
		}
		if (threadIdx.x == 0)
			a.verdict[p] &= (uint8_t)~SV_CIPHERED;
	}
}

/*
 * Unprotect of a forged packet (srtp.c:342-359: EAUTH leaves the
 * ciphertext, with the ROC over the tag): re-apply the keystream the fast
 * kernel applied speculatively.  Exits at once when no tag failed.
 */
template <int NR, int SHIFT>
__device__ __forceinline__ void ctr_refix_body(const KArgs &a, uint8_t *smem)
{
	if (*(volatile const uint32_t *)a.c.nfail == 0)
		return;
	FastPkt f;
	const bool live = fast_pkt(a.c, blockIdx.x * blockDim.x + threadIdx.x,
				   f);
	const uint8_t vd = live ? a.verdict[f.p] : (uint8_t)SV_TAG_OK;
	const bool need = !(vd & SV_TAG_OK) && (vd & SV_CIPHERED);
	/* only blocks holding a forged packet fill the 128 KiB table */
	if (!__syncthreads_or(need))
		return;
	tt4_fill(smem, a.t0);
	__syncthreads();
	if (!need)
		return;
	uint32_t rk[4 * (NR + 1)];
	const struct sgpu_comp *cp = fast_keys<NR>(a, rk);
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	uint8_t *pkt = a.arena + f.off;
	const uint64_t pasz = a.asz - f.off;
	const uint32_t A = f.L - cp->tag_len;
	const int32_t cw4 = (int32_t)(f.hl >> 4);
	uint32_t iv[4];
	fast_iv(cp, f, iv);
	CtrKs<NR, true, true> C;
	C.init(smem, lo, rk, iv);
	uint32_t carry[4] = {0, 0, 0, 0};
	for (uint32_t k = 0; 64u * k < A; k++) {
		const uint32_t c0 = 64u * k;
		if (c0 + 64u <= f.hl)
			continue;
		uint32_t d[16];
#pragma unroll
		for (int g = 0; g < 4; g++) {
			uint4 v = make_uint4(0, 0, 0, 0);
			if (c0 + 16u * g < A)
				v = ld16(pkt, pasz, c0 + 16u * g);
			d[4 * g] = v.x; d[4 * g + 1] = v.y;
			d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
		}
		/* the ROC already sits at A: loaded, written back as is */
		tail_xor_store<NR, SHIFT>(smem, lo, rk, C,
					  (int32_t)(4 * k) - cw4, carry, d, pkt,
					  c0, f.hl, A);
	}
	a.verdict[f.p] = vd & (uint8_t)~SV_CIPHERED;
}

/* the header class of a device plan is known only on the device: the
 * plan's skip[0..3] names it (k_plan_final), as for k_ctr_hmac_any */
__device__ __forceinline__ int fast_class(const KArgs &a)
{
	prof_guard(a);
	if (a.c.gfail && *a.c.gfail)
		return -1;              /* the bucket planner's plan failed */
	const uint32_t *g = a.c.guard;
	return !g[3] ? 3 : !g[0] ? 0 : !g[1] ? 1 : !g[2] ? 2 : -1;
}

template <int NR, bool PROT>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, CTRF_BLK(PROT))))
__attribute__((amdgpu_waves_per_eu(CTRF_BLK(PROT) / 256, 8)))
k_ctr_fast_any(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	switch (fast_class(a)) {
	case 0: ctr_fast_body<NR, 0, PROT>(a, smem); break;
	case 1: ctr_fast_body<NR, 1, PROT>(a, smem); break;
	case 2: ctr_fast_body<NR, 2, PROT>(a, smem); break;
	case 3: ctr_fast_body<NR, 3, PROT>(a, smem); break;
	default: break;                 /* rejected plan */
	}
}

/*
 * The lean kernel for multi-session batches (the multi-session device
 * planner's shape: every packet planned, one suite, per-lane keys, packets
 * taken in the planner's launch order c.idx).  A forged packet is listed
 * in c.flist and left decrypted with SV_CIPHERED; the pass behind this
 * launch (k_ctr_refix_list<NR, true>, one workgroup per listed packet with
 * its own session's keys) puts it back to its ciphertext, and the device
 * verdict fold (sgpu_mfold_rtp) writes the EAUTH results and states --
 * only a fold the device cannot settle undoes the batch for the host.
 */
#ifndef CTRF_MK_BLOCK
#define CTRF_MK_BLOCK 768
#endif
template <int NR, bool PROT>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, CTRF_MK_BLOCK)))
__attribute__((amdgpu_waves_per_eu(CTRF_MK_BLOCK / 256, 8)))
k_ctr_fast_mk(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	switch (fast_class(a)) {
	case 0: ctr_fast_body<NR, 0, PROT, true>(a, smem); break;
	case 1: ctr_fast_body<NR, 1, PROT, true>(a, smem); break;
	case 2: ctr_fast_body<NR, 2, PROT, true>(a, smem); break;
	case 3: ctr_fast_body<NR, 3, PROT, true>(a, smem); break;
	default: break;                 /* rejected plan */
	}
}

/* single-key SRTCP batches (header class 2); a.c.guard: the plan's skip
 * word of class 2 */
template <int NR, bool PROT>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, CTRF_BLK(PROT))))
__attribute__((amdgpu_waves_per_eu(CTRF_BLK(PROT) / 256, 8)))
k_ctr_fast_rtcp(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	prof_guard(a);
	if (*a.c.guard)
		return;                 /* rejected plan */
	ctr_fast_body<NR, 2, PROT, false, true>(a, smem);
}

template <int NR>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, CTRF_BLOCK)))
__attribute__((amdgpu_waves_per_eu(CTRF_BLOCK / 256, 8)))
k_ctr_fast_refix(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	switch (fast_class(a)) {
	case 0: ctr_refix_body<NR, 0>(a, smem); break;
	case 1: ctr_refix_body<NR, 1>(a, smem); break;
	case 2: ctr_refix_body<NR, 2>(a, smem); break;
	case 3: ctr_refix_body<NR, 3>(a, smem); break;
	default: break;
	}
}
