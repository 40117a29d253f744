/*
 * gcm.hip -- AES-GCM (AEAD_AES_128_GCM / AEAD_AES_256_GCM) kernels.
 */
#include "kern_common.h"

/* OpenSSL gcm_gmult_4bit rem_4bit (values << 16 into the top word) */
__constant__ uint32_t c_rem4[16] = {
	0x0000u << 16, 0x1C20u << 16, 0x3840u << 16, 0x2460u << 16,
	0x7080u << 16, 0x6CA0u << 16, 0x48C0u << 16, 0x54E0u << 16,
	0xE100u << 16, 0xFD20u << 16, 0xD940u << 16, 0xC560u << 16,
	0x9180u << 16, 0x8DA0u << 16, 0xA9C0u << 16, 0xB5E0u << 16,
};

/* ------------------------------------------------------------------ */
/* AES-GCM, one packet per lane.                                        */

/* bytes [p, p+16) of the GCM AAD stream  AAD = pkt[0,A) ‖ trailer? ,
 * as 4 big-endian words, zero padded */
__device__ __forceinline__ void aad_block(const uint8_t *pkt, uint64_t pasz,
					  uint32_t p, uint32_t A, bool trail,
					  uint32_t trailer, uint32_t w[4])
{
	uint4 v = make_uint4(0, 0, 0, 0);
	if (p < A)
		v = ld16(pkt, pasz, p);
	uint32_t d[4] = {v.x, v.y, v.z, v.w};
	const uint64_t X = trail ? ((uint64_t)trailer << 32) : 0ull;
#pragma unroll
	for (int q = 0; q < 4; q++)
		w[q] = msg_word((p >> 2) + q, bswap32(d[q]), A, X);
}

template <int NR, bool PROT, bool COMPACT>
__global__ void __launch_bounds__(KBLOCK)
k_gcm(const KArgs a)
{
	uint8_t *const arena = a.arena;
	const uint64_t asz = a.asz;
	const struct sgpu_comp *__restrict__ comps = a.comps;
	uint8_t *__restrict__ verdict = a.verdict;
	const bool undo = COMPACT && a.c.undo;
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT_BYTES + 4096 + 64];
	uint8_t *htab_lds = smem + TT_BYTES;                  /* 16 waves x 256 */
	uint32_t *rem4 = (uint32_t *)(smem + TT_BYTES + 4096);
	if (COMPACT && a.c.guard && *a.c.guard)  /* rejected plan / class */
		return;
	tt_fill(smem, a.t0);
	if (threadIdx.x < 16)
		rem4[threadIdx.x] = c_rem4[threadIdx.x];
	__syncthreads();

	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	struct sgpu_job j;
	uint32_t i = 0;
	const bool live = get_job<COMPACT, SGPU_MODE_GCM, PROT>(
		a, blockIdx.x * blockDim.x + threadIdx.x, j, i);
	if (!live)
		j.flags = SJ_SKIP, j.comp = 0;
	/* stage the GHASH table: per wave, in LDS if the wave's packets
	 * share one context, else per-lane reads from global memory */
	uint32_t c_first = __builtin_amdgcn_readfirstlane(j.comp);
	const bool uniform = __all(j.comp == c_first || (j.flags & SJ_SKIP));
	const uint8_t *tab;
	if (uniform) {
		uint8_t *wt = htab_lds + wv * 256u;
		if (lane < 16)
			*(uint4 *)(wt + lane * 16) =
				*(const uint4 *)comps[c_first].htab[lane];
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		tab = wt;
	}
	else {
		tab = (const uint8_t *)comps[j.comp].htab;
	}
	if (!live)
		return;
	if (j.flags & SJ_SKIP) {
		if (verdict && !undo)
			verdict[i] = 0;
		return;
	}
	const struct sgpu_comp *cp = comps + j.comp;
	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}
	uint8_t *pkt = arena + j.off;
	const uint64_t pasz = asz - j.off;

	/* srtp_iv_calc_gcm (misc.c:93-105); J0 = IV ‖ 0^31 ‖ 1 */
	uint32_t iv[3];
	{
		uint4 ks = *(const uint4 *)cp->k_s;
		uint32_t ixhi = j.ixhi, ixlo = j.ixlo;
		/* BE16 words: w1=ssrc>>16 w2=ssrc w3=ix>>32 w4=ix>>16 w5=ix */
		uint32_t be0 = (j.ssrc >> 16) & 0xffffu;            /* bytes 2,3 */
		uint32_t be1 = ((j.ssrc & 0xffffu) << 16) | (ixhi >> 16);
		uint32_t be2 = ((ixhi & 0xffffu) << 16) | (ixlo & 0xffffu);
		iv[0] = ks.x ^ bswap32(be0);
		iv[1] = ks.y ^ bswap32(be1);
		iv[2] = ks.z ^ bswap32(be2);
	}

	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
	if (j.flags & SJ_UNDO) {
		/* re-apply the GCM keystream (restores a speculatively
		 * decrypted payload before a re-run) */
		const uint32_t nb = (j.c_len + 15u) / 16u;
		for (uint32_t b = 0; b < nb; b++) {
			const uint32_t p = j.c_off + 16u * b;
			uint32_t s0 = iv[0], s1 = iv[1], s2 = iv[2];
			uint32_t s3 = bswap32(b + 2u);
			aes_block<NR>(smem, lo, rk, s0, s1, s2, s3);
			uint32_t ks[4] = {s0, s1, s2, s3};
			const uint32_t rem = j.c_off + j.c_len - p;
			for (int q = 0; q < 4; q++) {
				uint32_t bp = 4u * q;
				uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
				if (nbytes == 4) {
					uint32_t *w = (uint32_t *)(pkt + p + bp);
					*w = *w ^ ks[q];
				}
				else if (nbytes) {
					uint32_t v = 0;
					for (uint32_t z = 0; z < nbytes; z++)
						v |= (uint32_t)pkt[p + bp + z] << (8 * z);
					st_partial(pkt + p + bp, v ^ ks[q], nbytes);
				}
			}
		}
		if (verdict && !undo)
			verdict[i] = 0;
		return;
	}
	const uint32_t A = j.a_len;
	const uint32_t aad_total = A + (trail ? 4u : 0u);
	const uint32_t c_off = j.c_off, c_len = do_cipher ? j.c_len : 0u;
	const uint32_t c_end = c_off + c_len;

	uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
	/* GHASH over AAD */
	for (uint32_t p = 0; p < aad_total; p += 16) {
		uint32_t w[4];
		aad_block(pkt, pasz, p, A, trail, j.trailer, w);
		/* msg_word adds the SHA 0x80 marker only when X has it; for
		 * GCM X carries no marker, zero padding is implied */
		x0 ^= w[0]; x1 ^= w[1]; x2 ^= w[2]; x3 ^= w[3];
		ghash_mul(x0, x1, x2, x3, tab, rem4);
	}
	/* CTR + GHASH over the cipher region, in 16-B payload blocks */
	const uint32_t nblk = (c_len + 15u) / 16u;
	for (uint32_t b = 0; b < nblk; b++) {
		const uint32_t p = c_off + 16u * b;
		uint4 v = ld16(pkt, pasz, p);
		uint32_t d[4] = {v.x, v.y, v.z, v.w};
		uint32_t s0 = iv[0], s1 = iv[1], s2 = iv[2];
		uint32_t s3 = bswap32(b + 2u);          /* inc32(J0) + b */
		aes_block<NR>(smem, lo, rk, s0, s1, s2, s3);
		uint32_t ks[4] = {s0, s1, s2, s3};
		uint32_t o[4], ct[4];
		const uint32_t rem = c_end - p;
		if (rem >= 16) {
#pragma unroll
			for (int q = 0; q < 4; q++) {
				o[q] = d[q] ^ ks[q];
				ct[q] = PROT ? o[q] : d[q];
			}
			*(uint4 *)(pkt + p) = make_uint4(o[0], o[1], o[2], o[3]);
		}
		else {
#pragma unroll
			for (int q = 0; q < 4; q++) {
				uint32_t bp = 4u * q;
				uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
				uint32_t m = nbytes >= 4 ? 0xffffffffu
					   : ((1u << (8 * nbytes)) - 1u);
				o[q] = (d[q] ^ ks[q]) & m;
				ct[q] = PROT ? o[q] : (d[q] & m);
				if (nbytes == 4)
					*(uint32_t *)(pkt + p + bp) = o[q];
				else if (nbytes)
					st_partial(pkt + p + bp, o[q], nbytes);
			}
		}
		x0 ^= bswap32(ct[0]); x1 ^= bswap32(ct[1]);
		x2 ^= bswap32(ct[2]); x3 ^= bswap32(ct[3]);
		ghash_mul(x0, x1, x2, x3, tab, rem4);
	}
	/* length block: bitlen(AAD) ‖ bitlen(C) */
	{
		uint64_t al = (uint64_t)aad_total * 8u, cl = (uint64_t)c_len * 8u;
		x0 ^= (uint32_t)(al >> 32); x1 ^= (uint32_t)al;
		x2 ^= (uint32_t)(cl >> 32); x3 ^= (uint32_t)cl;
		ghash_mul(x0, x1, x2, x3, tab, rem4);
	}
	/* tag = GHASH ^ E(K, J0) */
	uint32_t s0 = iv[0], s1 = iv[1], s2 = iv[2], s3 = bswap32(1u);
	aes_block<NR>(smem, lo, rk, s0, s1, s2, s3);
	uint32_t t[4] = {x0 ^ bswap32(s0), x1 ^ bswap32(s1), x2 ^ bswap32(s2),
			 x3 ^ bswap32(s3)};
	uint8_t *tp = pkt + j.tag_off;
	uint8_t vd = do_cipher ? SV_CIPHERED : 0;
	if (PROT) {
#pragma unroll
		for (int q = 0; q < 4; q++)
			st_be32(tp + 4 * q, t[q]);
		if (j.flags & SJ_STORE_TRAIL)
			st_be32(pkt + j.t_off, j.trailer);
	}
	else {
		uint32_t diff = 0;
#pragma unroll
		for (int q = 0; q < 16; q++)
			diff |= tp[q] ^ (uint8_t)(t[q >> 2] >> (24 - 8 * (q & 3)));
		if (diff == 0)
			vd |= SV_TAG_OK;
		if (COMPACT && !(vd & SV_TAG_OK))
			atomicAdd(a.c.nfail, 1u);
	}
	if (verdict)
		verdict[i] = vd;
}


kfn_t sgpu_pick_gcm(bool compact, int nr, int prot)
{
	if (compact) {
		if (nr == 10)
			return prot ? k_gcm<10, true, true> : k_gcm<10, false, true>;
		if (nr == 14)
			return prot ? k_gcm<14, true, true> : k_gcm<14, false, true>;
	}
	else {
		if (nr == 10)
			return prot ? k_gcm<10, true, false> : k_gcm<10, false, false>;
		if (nr == 14)
			return prot ? k_gcm<14, true, false> : k_gcm<14, false, false>;
	}
	return NULL;
}
