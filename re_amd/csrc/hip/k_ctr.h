/*
 * k_ctr.h -- fused AES-CM + HMAC-SHA1 kernel template (SRTP/SRTCP with the
 * AES_CM_* suites).  Instantiated by ctr10.hip (AES-128) and ctr14.hip
 * (AES-256).
 */
#pragma once
#include <type_traits>
#include "kern_common.h"

/*
 * Occupancy.  The 128 KiB four-table image (dev_common.h, T4) allows one
 * block per CU.  Single-key launches (round keys and HMAC midstates in
 * SGPRs) keep the pipelined chunk (ciphertext, plaintext, next keystream,
 * quad-transpose temporaries) in ~170 VGPRs: 768-thread blocks = 3
 * waves/SIMD, no scratch.  Per-lane keys need ~190 VGPRs: 512-thread
 * blocks = 2 waves/SIMD.
 */
/* build knobs (kernel-variant experiments, scripts/build_variants.sh) */
/* _P: protect, _U: unprotect */
#ifndef CTR_COAL_P          /* quad-coalesced steady-state chunk access */
#define CTR_COAL_P 1
#endif
#ifndef CTR_COAL_U
#define CTR_COAL_U 0
#endif
#ifndef CTR_PIPE_P          /* keystream one chunk ahead of the MAC */
#define CTR_PIPE_P 0
#endif
#ifndef CTR_PIPE_U
#define CTR_PIPE_U 1
#endif
#ifndef CTR_SHAFIRST_U      /* unprotect steady chunk: MAC of the received
			       ciphertext, then the keystream in place */
#define CTR_SHAFIRST_U 0
#endif
#ifndef CTR_SCHED_BARRIER_U /* ... with a scheduling barrier between them */
#define CTR_SCHED_BARRIER_U 0
#endif
#ifndef CTR_UNI_PROT_BLOCK  /* single-key protect block size */
#define CTR_UNI_PROT_BLOCK 1024
#endif
#ifndef CTR_UNI_UNP_BLOCK   /* single-key unprotect block size */
#define CTR_UNI_UNP_BLOCK 768
#endif

#ifndef CTR_MULTI_BLOCK     /* per-lane keys (multi-session batches) */
#define CTR_MULTI_BLOCK 512u
#endif

__host__ __device__ constexpr unsigned ctr_block(bool prot, bool uni)
{
	return uni ? (prot ? CTR_UNI_PROT_BLOCK : CTR_UNI_UNP_BLOCK)
		   : CTR_MULTI_BLOCK;
}

__host__ __device__ constexpr int ctr_waves(bool prot, bool uni)
{
	return uni || CTR_MULTI_BLOCK > 512u ?
		(int)(ctr_block(prot, uni) / 256u) : 1;
}

/*
 * Fused AES-CM + HMAC-SHA1, one packet per lane.
 *   SHIFT = (c_off / 4) & 3: the cipher region starts SHIFT words into a
 *   16-byte packet granule (3 for a 12-byte RTP header, 2 for SRTCP).
 *   UNI: every packet of the launch uses one session context, so round
 *   keys and HMAC midstates live in SGPRs (fewer VGPRs, more waves).
 * Chunks wholly inside both the cipher region and the MAC input run a
 * branch-free steady-state body; the header / tail chunks take the
 * general byte-exact path.
 */
template <int NR, int SHIFT, bool PROT, bool COMPACT, bool UNI>
__device__ __forceinline__ void ctr_hmac_body(const KArgs &a, uint8_t *smem)
{
	if (COMPACT)
		prof_guard(a);
	if (COMPACT && a.c.guard && *a.c.guard)  /* rejected plan / class */
		return;
	if (COMPACT || !a.nocipher)     /* MAC only: no AES */
		tt4_fill(smem, a.t0);
	__syncthreads();

	uint8_t *const arena = a.arena;
	const uint64_t asz = a.asz;
	uint8_t *__restrict__ verdict = a.verdict;
	uint32_t *__restrict__ save = a.save;
	const bool undo = COMPACT && a.c.undo;
	struct sgpu_job j;
	uint32_t i;
	if (!get_job<COMPACT, SGPU_MODE_CTR, PROT>(
		    a, blockIdx.x * blockDim.x + threadIdx.x, j, i))
		return;
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	if (j.flags & SJ_SKIP) {
		if (verdict && !undo)
			verdict[i] = 0;
		return;
	}
	const uint32_t ci = UNI ? __builtin_amdgcn_readfirstlane(j.comp)
				: j.comp;
	const struct sgpu_comp *cp = a.comps + ci;

	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}
	/* the table stores middle-round keys rot16'd for the T0/T1 image;
	 * the four-table rounds take them plain */
#pragma unroll
	for (int k = 4; k < 4 * NR; k++)
		rk[k] = rot16(rk[k]);
	if (UNI) {
#pragma unroll
		for (int k = 0; k < 4 * (NR + 1); k++)
			rk[k] = __builtin_amdgcn_readfirstlane(rk[k]);
	}

	const bool do_cipher = (j.flags & SJ_CIPHER) != 0 &&
			       (COMPACT || !a.nocipher);
	const bool do_hmac = (j.flags & SJ_HMAC) != 0;
	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool cipher_if_ok = !PROT && (j.flags & SJ_CIPHER_IF_OK);
	const uint32_t c_off = j.c_off, c_end = j.c_off + j.c_len;
	const uint32_t A = do_hmac ? j.a_len : 0;
	const uint32_t data_end = max(c_end, A);
	uint8_t *pkt = arena + j.off;
	const uint64_t pasz = asz - j.off;   /* bytes addressable from pkt */

	/* srtp_iv_calc (misc.c:76-87): k_s ^ (0, ssrc, ix>>16, ix<<16) */
	uint32_t iv[4];
	{
		uint4 ks = *(const uint4 *)cp->k_s;
		iv[0] = ks.x;
		iv[1] = ks.y ^ bswap32(j.ssrc);
		iv[2] = ks.z ^ bswap32(j.ixhi);
		iv[3] = (ks.w ^ (bswap32(j.ixlo) >> 16)) & 0xffffu;
	}

	/* compact launches never carry packets of 1 MiB or more (host) */
	CtrKs<NR, COMPACT, true> C;
	C.init(smem, lo, rk, iv);

	uint32_t h[5];
	if (do_hmac) {
		h[0] = cp->ipad[0]; h[1] = cp->ipad[1]; h[2] = cp->ipad[2];
		h[3] = cp->ipad[3]; h[4] = cp->ipad[4];
	}
	const uint64_t X = trail ? ((uint64_t)j.trailer << 32 | 0x80000000u)
				 : 0x8000000000000000ull;
	const uint32_t tl = trail ? 4u : 0u;
	const uint32_t nb = do_hmac ? (A + tl + 9u + 63u) / 64u : 0u;
	const uint64_t bitlen = (uint64_t)(64u + A + tl) * 8u;
	const uint32_t nck = do_cipher ? (c_end + 63u) / 64u : 0u;
	const uint32_t nchunk = max(nb, nck);
	const int32_t cw4 = (int32_t)(c_off >> 4);   /* (c_off/4) >> 2 */
	const bool store_ct = do_cipher && (PROT || cipher_if_ok ||
					    !do_hmac);
	/* chunks [kf0, kf1) lie wholly inside the cipher region and the MAC
	 * input: steady-state body */
	uint32_t kf0 = nchunk, kf1 = nchunk;
	if (do_cipher && do_hmac) {
		/* a cipher region starting in the first 16 bytes (RTP without
		 * CSRC/extension, SRTCP) lets chunk 0 run the steady body: its
		 * words before c_off take the zero carry and stay unchanged */
		kf0 = c_off < 16u ? 0u : min((c_off + 63u) / 64u, nchunk);
		kf1 = max(min(c_end, A) / 64u, kf0);
	}

	uint32_t carry[4] = {0, 0, 0, 0};
	uint32_t ks[16];     /* keystream of the next chunk (pipelined loop) */

	/* general chunk: any mix of header, cipher, MAC and padding;
	 * have_ks: ks[] already holds this chunk's keystream */
	auto chunk_general = [&](uint32_t k, bool have_ks) {
		const uint32_t c0 = 64u * k;
		uint32_t d[16], w[16];
#pragma unroll
		for (int g = 0; g < 4; g++) {
			uint4 v = make_uint4(0, 0, 0, 0);
			if (c0 + 16u * g < data_end)
				v = ld16(pkt, pasz, c0 + 16u * g);
			d[4 * g] = v.x; d[4 * g + 1] = v.y;
			d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
		}
		const bool mac = do_hmac && k < nb;
		/* unprotect: the MAC covers the received ciphertext */
		if (!PROT && mac) {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = msg_word(16u * k + jj, bswap32(d[jj]), A,
						 X);
			if (k + 1 == nb) {
				w[14] = (uint32_t)(bitlen >> 32);
				w[15] = (uint32_t)bitlen;
			}
			sha1_compress(h, w);
		}
		const bool need_ks = do_cipher && (c0 + 64u > c_off) &&
				     (c0 < c_end);
		if (need_ks) {
			if (have_ks) {
#pragma unroll
				for (int jj = 0; jj < 16; jj++)
					d[jj] ^= ks[jj] & region_mask(c0 + 4u * jj,
								      c_off, c_end);
			}
			else {
				ks_xor<NR, SHIFT, true, COMPACT>(smem, lo, rk, C,
						(int32_t)(4 * k) - cw4, carry, d,
						c0, c_off, c_end);
			}
			if (store_ct)
				store_region(pkt, c0, d, c_off, c_end);
		}
		/* protect: the MAC covers the ciphertext just produced */
		if (PROT && mac) {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = msg_word(16u * k + jj, bswap32(d[jj]), A,
						 X);
			if (k + 1 == nb) {
				w[14] = (uint32_t)(bitlen >> 32);
				w[15] = (uint32_t)bitlen;
			}
			sha1_compress(h, w);
		}
	};

	uint32_t k = 0;
	if (!COMPACT && !do_cipher && do_hmac) {
		/* MAC only (KArgs.nocipher: the small-launch split, or a job
		 * without a cipher region): whole 64-byte chunks of [0, A)
		 * straight into SHA-1, the rest by the general chunk */
		const uint32_t kA = A / 64u;
		for (; k < kA; k++) {
			uint32_t w[16];
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = ld16(pkt, pasz, 64u * k + 16u * g);
				w[4 * g] = bswap32(v.x);
				w[4 * g + 1] = bswap32(v.y);
				w[4 * g + 2] = bswap32(v.z);
				w[4 * g + 3] = bswap32(v.w);
			}
			sha1_compress(h, w);
		}
	}
	for (; k < kf0; k++)
		chunk_general(k, false);
	/*
	 * Steady state, software-pipelined: the keystream of chunk k+1 is
	 * generated in the same basic block as the MAC of chunk k (no
	 * dependence between them).  The last iteration's keystream is that
	 * of chunk kf1, which the general tail chunk uses (have_ks).
	 * Chunk bytes move quad-coalesced (quad_load/quad_store) over the
	 * part [K0, K1) of the range that all four lanes of a quad share.
	 */
	constexpr bool PIPE = PROT ? CTR_PIPE_P : CTR_PIPE_U;
	constexpr bool COAL = PROT ? CTR_COAL_P : CTR_COAL_U;
	const bool piped = PIPE && kf0 < kf1;
	if (piped)
		chunk_ks<NR, SHIFT>(smem, lo, rk, C, (int32_t)(4 * kf0) - cw4,
				    carry, ks);
	const uint32_t lane = threadIdx.x & 63u;
	uint32_t K0 = kf1, K1 = kf1;
	uint64_t qb[4];
	if constexpr (COMPACT && COAL) {
		quad_offsets(j.off, lane, qb);
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
	/* unprotect, SHA-first form: the keystream applied to bytes that
	 * must stay ciphertext (no decryption) is masked to zero */
	const uint32_t km = store_ct ? 0xffffffffu : 0u;
	auto steady = [&](uint32_t k, auto coal) {
		constexpr bool CO = decltype(coal)::value;
		const uint32_t c0 = 64u * k;
		uint32_t d[16], o[16], w[16];
		if constexpr (CO) {
			quad_load(arena, qb, c0, lane, d);
		}
		else {
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = *(const uint4 *)(pkt + c0 + 16u * g);
				d[4 * g] = v.x; d[4 * g + 1] = v.y;
				d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
			}
		}
		if constexpr (!PROT && CTR_SHAFIRST_U && !PIPE) {
			/* the MAC covers the received ciphertext: run it first,
			 * then decrypt d in place -- only d, the schedule and
			 * the SHA-1 state live at once */
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = bswap32(d[jj]);
			sha1_compress(h, w);
			if (CTR_SCHED_BARRIER_U)
				__builtin_amdgcn_sched_barrier(0);
			ks_xor_km<NR, SHIFT>(smem, lo, rk, C,
					     (int32_t)(4 * k) - cw4, carry, d, km);
			if constexpr (CO) {
				quad_store(arena, qb, c0, lane, d);
			}
			else {
#pragma unroll
				for (int g = 0; g < 4; g++)
					*(uint4 *)(pkt + c0 + 16u * g) =
						make_uint4(d[4 * g], d[4 * g + 1],
							   d[4 * g + 2], d[4 * g + 3]);
			}
			return;
		}
		if constexpr (PIPE) {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				o[jj] = d[jj] ^ ks[jj];
			chunk_ks<NR, SHIFT>(smem, lo, rk, C,
					    (int32_t)(4 * (k + 1)) - cw4, carry,
					    ks);
		}
		else {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				o[jj] = d[jj];
			ks_xor<NR, SHIFT, false, COMPACT>(smem, lo, rk, C,
							  (int32_t)(4 * k) - cw4,
							  carry, o);
		}
		/* branch-free: protect always stores here (do_cipher),
		 * unprotect writes the received bytes back when it must not
		 * decrypt */
		uint32_t s[16];
#pragma unroll
		for (int jj = 0; jj < 16; jj++)
			s[jj] = (PROT || store_ct) ? o[jj] : d[jj];
		if constexpr (CO) {
			quad_store(arena, qb, c0, lane, s);
		}
		else {
#pragma unroll
			for (int g = 0; g < 4; g++)
				*(uint4 *)(pkt + c0 + 16u * g) =
					make_uint4(s[4 * g], s[4 * g + 1],
						   s[4 * g + 2], s[4 * g + 3]);
		}
		/* the MAC covers the ciphertext: produced (protect) or
		 * received (unprotect) */
#pragma unroll
		for (int jj = 0; jj < 16; jj++)
			w[jj] = bswap32(PROT ? o[jj] : d[jj]);
		sha1_compress(h, w);
	};
	for (; k < K0; k++)
		steady(k, std::false_type());
	if constexpr (COMPACT && COAL) {
		for (; k < K1; k++)
			steady(k, std::true_type());
		for (; k < kf1; k++)
			steady(k, std::false_type());
	}
	for (; k < nchunk; k++)
		chunk_general(k, piped && k == kf1);

	uint8_t vd = 0;
	if (do_hmac) {
		/* outer hash: opad midstate + 20-byte inner digest */
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

		const uint32_t tag_len = cp->tag_len;
		uint8_t *tp = pkt + j.tag_off;
		if (PROT) {
			for (uint32_t q = 0; q < tag_len; q++)
				tp[q] = (uint8_t)(h[q >> 2] >> (24 - 8 * (q & 3)));
		}
		else {
			uint32_t diff = 0;
			for (uint32_t q = 0; q < tag_len; q++)
				diff |= tp[q] ^ (uint8_t)(h[q >> 2] >>
							  (24 - 8 * (q & 3)));
			vd = diff == 0 ? SV_TAG_OK : 0;
			if (j.flags & SJ_ROC_AT_TAG) {
				/* the reference writes the ROC over the tag
				 * before comparing (srtp.c:342-344); keep the
				 * original bytes for a possible re-run */
				if (save)
					save[i] = (uint32_t)tp[0] |
						  (uint32_t)tp[1] << 8 |
						  (uint32_t)tp[2] << 16 |
						  (uint32_t)tp[3] << 24;
				st_be32(tp, j.trailer);
			}
		}
	}
	if (PROT && (j.flags & SJ_STORE_TRAIL))
		st_be32(pkt + j.t_off, j.trailer);

	if (store_ct && !PROT)
		vd |= SV_CIPHERED;

	/* unprotect with decrypt-if-authentic: the plaintext was written
	 * speculatively during the single pass; a forged packet is restored
	 * by re-applying the keystream (rare path) */
	if (cipher_if_ok && !(vd & SV_TAG_OK)) {
#pragma unroll
		for (int q = 0; q < 4; q++)
			carry[q] = 0;
		for (uint32_t kk = 0; kk < nck; kk++) {
			const uint32_t c0 = 64u * kk;
			if (!(c0 + 64u > c_off && c0 < c_end))
				continue;
			uint32_t d[16];
#pragma unroll
			for (int g = 0; g < 4; g++) {
				uint4 v = make_uint4(0, 0, 0, 0);
				if (c0 + 16u * g < c_end)
					v = ld16(pkt, pasz, c0 + 16u * g);
				d[4 * g] = v.x; d[4 * g + 1] = v.y;
				d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
			}
			ks_xor<NR, SHIFT, true, COMPACT>(smem, lo, rk, C,
						 (int32_t)(4 * kk) - cw4, carry, d,
						 c0, c_off, c_end);
			/* exact byte stores: this pass runs after the ROC word
			 * was written at c_end (hipcc widened the partial last
			 * word of store_region here, as in gcm.hip k_gcmu) */
			store_region_exact(pkt, c0, d, c_off, c_end);
		}
		vd &= (uint8_t)~SV_CIPHERED;
	}
	if (undo && a.c.rtcp)
		return;
	if (undo) {
		/* compact undo: the word under the ROC back (srtp.c:342-344) */
		uint8_t *tp = pkt + j.tag_off;
		const uint32_t v = save[i];
		tp[0] = (uint8_t)v; tp[1] = (uint8_t)(v >> 8);
		tp[2] = (uint8_t)(v >> 16); tp[3] = (uint8_t)(v >> 24);
		return;
	}
	if (COMPACT && !PROT && !(vd & SV_TAG_OK))
		atomicAdd(a.c.nfail, 1u);
	if (verdict)
		verdict[i] = vd;
}

/*
 * Small general launches (the per-packet API's one mbuf per call, a few
 * concurrent callers): one packet per lane leaves a 1200-B packet's 75
 * AES blocks and 21 SHA-1 compressions as one serial chain (~110 us).
 * k_ctr_coop takes the cipher regions instead, one packet per workgroup
 * and one 16-byte keystream block per lane, and k_ctr_hmac runs with
 * KArgs.nocipher (MAC only): protect encrypts first (the MAC covers the
 * ciphertext), unprotect runs after the MAC and applies the keystream
 * where the general kernel would have stored plaintext (store_ct: no MAC,
 * or decrypt-if-authentic with the tag ok) -- the same bytes and verdicts
 * (SV_CIPHERED) as the fused kernel.  Byte-exact stores at the region
 * end: the ROC may already sit right behind it (srtp.c:342-344).
 */
template <int NR, bool PROT>
__global__ void __launch_bounds__(256)
k_ctr_coop(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT_BYTES];
	const uint32_t i = blockIdx.x;
	if (i >= a.njobs)
		return;
	const struct sgpu_job j = a.jobs[i];
	if ((j.flags & SJ_SKIP) || !(j.flags & SJ_CIPHER))
		return;
	if (!PROT) {
		const bool do_hmac = (j.flags & SJ_HMAC) != 0;
		const bool if_ok = (j.flags & SJ_CIPHER_IF_OK) != 0;
		if (!(if_ok || !do_hmac))
			return;                 /* no plaintext stored */
		if (if_ok && !(a.verdict[i] & SV_TAG_OK))
			return;                 /* forged: ciphertext stays */
	}
	tt_fill(smem, a.t0);
	__syncthreads();
	const struct sgpu_comp *cp = a.comps +
				     __builtin_amdgcn_readfirstlane(j.comp);
	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < 4 * (NR + 1); k++)
		rk[k] = __builtin_amdgcn_readfirstlane(cp->rk[k]);
	uint32_t iv[4];
	{
		const uint4 ks = *(const uint4 *)cp->k_s;
		iv[0] = ks.x;
		iv[1] = ks.y ^ bswap32(j.ssrc);
		iv[2] = ks.z ^ bswap32(j.ixhi);
		iv[3] = (ks.w ^ (bswap32(j.ixlo) >> 16)) & 0xffffu;
	}
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	uint8_t *pkt = a.arena + j.off;
	const uint32_t c_end = j.c_off + j.c_len;
	for (uint32_t b = threadIdx.x; j.c_off + 16u * b < c_end;
	     b += blockDim.x) {
		uint32_t ks[4];
		ctr_block<NR, false>(smem, lo, rk, iv, (int32_t)b, ks);
		const uint32_t p0 = j.c_off + 16u * b;
#pragma unroll
		for (int w = 0; w < 4; w++) {
			const uint32_t bp = p0 + 4u * w;
			if (bp >= c_end)
				break;
			if (c_end - bp >= 4u) {
				uint32_t *wp = (uint32_t *)(pkt + bp);
				*wp = *wp ^ ks[w];
			}
			else {
				for (uint32_t k = 0; k < c_end - bp; k++)
					pkt[bp + k] ^= (uint8_t)(ks[w] >> (8 * k));
			}
		}
	}
	if (!PROT && threadIdx.x == 0 && a.verdict)
		a.verdict[i] |= SV_CIPHERED;
}

template <int NR, int SHIFT, bool PROT, bool COMPACT, bool UNI>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, ctr_block(PROT, UNI))))
__attribute__((amdgpu_waves_per_eu(ctr_waves(PROT, UNI), 8)))
k_ctr_hmac(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	ctr_hmac_body<NR, SHIFT, PROT, COMPACT, UNI>(a, smem);
}

/*
 * One launch for a device-planned batch whose header class (SHIFT) is
 * known only on the device: a.c.guard points at the plan's skip[0..3]
 * (k_plan_final: skip[s] = fail || class != s), at most one of which is
 * zero.  Saves the three empty class launches of the per-class scheme.
 */
template <int NR, bool PROT, bool UNI>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, ctr_block(PROT, UNI))))
__attribute__((amdgpu_waves_per_eu(ctr_waves(PROT, UNI), 8)))
k_ctr_hmac_any(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	prof_guard(a);
	const uint32_t *g = a.c.guard;
	const uint32_t q = !g[3] ? 3u : !g[0] ? 0u : !g[1] ? 1u : !g[2] ? 2u
								    : 4u;
	if (q > 3u)
		return;                 /* rejected plan */
	KArgs b = a;
	b.c.guard = NULL;
	switch (q) {
	case 0: ctr_hmac_body<NR, 0, PROT, true, UNI>(b, smem); break;
	case 1: ctr_hmac_body<NR, 1, PROT, true, UNI>(b, smem); break;
	case 2: ctr_hmac_body<NR, 2, PROT, true, UNI>(b, smem); break;
	default: ctr_hmac_body<NR, 3, PROT, true, UNI>(b, smem); break;
	}
}
