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

/* GHASH table image in LDS: 16 entries x 16 replicas x 16 B */
#define HT_BYTES 4096u
/* single-key GCM fits 64 VGPRs: 16 waves share one T-table + GHASH image,
 * two blocks per CU = 8 waves/SIMD */
#define GCM_UNI_BLOCK 1024u

/*
 * AES-GCM with a 96-bit IV, one packet per lane (aes.c:136-249 semantics:
 * J0 = IV || 0^31 || 1, inc32 counter, tag = GHASH ^ E(K, J0)).
 *   UNI: every packet of the launch uses one session context: round keys
 *   in SGPRs, one GHASH image per block (1024 threads, 8 waves/SIMD).
 *   Otherwise 256-thread blocks with one GHASH image per wave when the
 *   wave's packets share a context, per-lane global reads if not.
 * The CTR part uses the cached counter block (CtrKs) in compact launches:
 * the GCM counter is bytes 12..15 of IV || ctr and stays below 2^16.
 */
template <int NR, bool PROT, bool COMPACT, bool UNI>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, UNI ? GCM_UNI_BLOCK : KBLOCK)))
__attribute__((amdgpu_waves_per_eu(UNI ? 8 : 1, 8)))
k_gcm(const KArgs a)
{
	uint8_t *const arena = a.arena;
	const uint64_t asz = a.asz;
	const struct sgpu_comp *__restrict__ comps = a.comps;
	uint8_t *__restrict__ verdict = a.verdict;
	const bool undo = COMPACT && a.c.undo;
	__shared__ __attribute__((aligned(16)))
	uint8_t smem[TT_BYTES + (UNI ? 1u : KBLOCK / 64u) * HT_BYTES + 64];
	uint8_t *ht = smem + TT_BYTES;
	uint32_t *rem4 = (uint32_t *)(smem + TT_BYTES +
				      (UNI ? 1u : KBLOCK / 64u) * HT_BYTES);
	if (COMPACT && a.c.guard && *a.c.guard)  /* rejected plan / class */
		return;
	tt_fill(smem, a.t0);
	if (threadIdx.x < 16)
		rem4[threadIdx.x] = c_rem4[threadIdx.x];

	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	struct sgpu_job j;
	uint32_t i = 0;
	const bool live = get_job<COMPACT, SGPU_MODE_GCM, PROT>(
		a, blockIdx.x * blockDim.x + threadIdx.x, j, i);
	if (!live)
		j.flags = SJ_SKIP, j.comp = 0;

	/* GHASH table image (replicated 16x, conflict-free) */
	const uint8_t *tab;
	uint32_t stride = 256u, laneoff = (lane & 15u) * 16u;
	if (UNI) {
		/* the block's first live packet names the context (every
		 * packet of a UNI launch shares it) */
		__shared__ uint32_t blk_comp;
		if (threadIdx.x == 0)
			blk_comp = 0xffffffffu;
		__syncthreads();
		if (live && !(j.flags & SJ_SKIP))
			atomicMin(&blk_comp, j.comp);
		__syncthreads();
		const uint32_t bc = blk_comp;
		if (bc != 0xffffffffu)
			for (uint32_t q = threadIdx.x; q < 256u; q += blockDim.x)
				*(uint4 *)(ht + (q >> 4) * 256u + (q & 15u) * 16u) =
					*(const uint4 *)comps[bc].htab[q >> 4];
		__syncthreads();
		tab = ht;
	}
	else {
		__syncthreads();
		const uint32_t c_first = __builtin_amdgcn_readfirstlane(j.comp);
		const bool uniform = __all(j.comp == c_first ||
					   (j.flags & SJ_SKIP));
		if (uniform) {
			uint8_t *wt = ht + wv * HT_BYTES;
#pragma unroll
			for (uint32_t q = lane; q < 256u; q += 64u)
				*(uint4 *)(wt + (q >> 4) * 256u + (q & 15u) * 16u) =
					*(const uint4 *)comps[c_first].htab[q >> 4];
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			tab = wt;
		}
		else {
			tab = (const uint8_t *)comps[j.comp].htab;
			stride = 16u;
			laneoff = 0;
		}
	}
	if (!live)
		return;
	if (j.flags & SJ_SKIP) {
		if (verdict && !undo)
			verdict[i] = 0;
		return;
	}
	const uint32_t ci = UNI ? __builtin_amdgcn_readfirstlane(j.comp)
				: j.comp;
	const struct sgpu_comp *cp = comps + ci;
	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}
	if (UNI) {
#pragma unroll
		for (int k = 0; k < 4 * (NR + 1); k++)
			rk[k] = __builtin_amdgcn_readfirstlane(rk[k]);
	}
	uint8_t *pkt = arena + j.off;
	const uint64_t pasz = asz - j.off;

	/* srtp_iv_calc_gcm (misc.c:93-105); J0 = IV || 0^31 || 1 */
	uint32_t iv[4];
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
		iv[3] = 0;              /* counter word (big-endian) */
	}
	/* keystream block b = E(K, IV || BE32(b)): b = 2.. payload, 1 tag */
	CtrKs<NR, COMPACT> C;
	C.init(smem, lo, rk, iv);

	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
	if (j.flags & SJ_UNDO) {
		/* re-apply the GCM keystream (restores a speculatively
		 * decrypted payload before a re-run) */
		const uint32_t nb = (j.c_len + 15u) / 16u;
		for (uint32_t b = 0; b < nb; b++) {
			const uint32_t p = j.c_off + 16u * b;
			uint32_t ks[4];
			C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
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
		ghash_mul(x0, x1, x2, x3, tab, stride, laneoff, rem4);
	}
	/* CTR + GHASH over the cipher region, in 16-B payload blocks */
	const uint32_t nblk = (c_len + 15u) / 16u;
	const uint32_t nfull = c_len / 16u;
	for (uint32_t b = 0; b < nfull; b++) {
		const uint32_t p = c_off + 16u * b;
		uint4 v = ld16(pkt, pasz, p);
		uint32_t ks[4];
		C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
		const uint32_t o0 = v.x ^ ks[0], o1 = v.y ^ ks[1];
		const uint32_t o2 = v.z ^ ks[2], o3 = v.w ^ ks[3];
		*(uint4 *)(pkt + p) = make_uint4(o0, o1, o2, o3);
		x0 ^= bswap32(PROT ? o0 : v.x); x1 ^= bswap32(PROT ? o1 : v.y);
		x2 ^= bswap32(PROT ? o2 : v.z); x3 ^= bswap32(PROT ? o3 : v.w);
		ghash_mul(x0, x1, x2, x3, tab, stride, laneoff, rem4);
	}
	if (nblk > nfull) {
		const uint32_t b = nfull, p = c_off + 16u * b;
		uint4 v = ld16(pkt, pasz, p);
		uint32_t d[4] = {v.x, v.y, v.z, v.w};
		uint32_t ks[4], ct[4];
		C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
		const uint32_t rem = c_end - p;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			uint32_t bp = 4u * q;
			uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
			uint32_t m = nbytes >= 4 ? 0xffffffffu
				   : ((1u << (8 * nbytes)) - 1u);
			const uint32_t o = (d[q] ^ ks[q]) & m;
			ct[q] = PROT ? o : (d[q] & m);
			if (nbytes == 4)
				*(uint32_t *)(pkt + p + bp) = o;
			else if (nbytes)
				st_partial(pkt + p + bp, o, nbytes);
		}
		x0 ^= bswap32(ct[0]); x1 ^= bswap32(ct[1]);
		x2 ^= bswap32(ct[2]); x3 ^= bswap32(ct[3]);
		ghash_mul(x0, x1, x2, x3, tab, stride, laneoff, rem4);
	}
	/* length block: bitlen(AAD) || bitlen(C) */
	{
		uint64_t al = (uint64_t)aad_total * 8u, cl = (uint64_t)c_len * 8u;
		x0 ^= (uint32_t)(al >> 32); x1 ^= (uint32_t)al;
		x2 ^= (uint32_t)(cl >> 32); x3 ^= (uint32_t)cl;
		ghash_mul(x0, x1, x2, x3, tab, stride, laneoff, rem4);
	}
	/* tag = GHASH ^ E(K, J0) */
	uint32_t e0[4];
	C.block(smem, lo, rk, 1, e0);
	uint32_t t[4] = {x0 ^ bswap32(e0[0]), x1 ^ bswap32(e0[1]),
			 x2 ^ bswap32(e0[2]), x3 ^ bswap32(e0[3])};
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

kfn_t sgpu_pick_gcm(bool compact, bool uni, int nr, int prot)
{
#define PICKG(C, U)                                                            \
	if (compact == C && uni == U) {                                        \
		if (nr == 10)                                                  \
			return prot ? k_gcm<10, true, C, U>                    \
				    : k_gcm<10, false, C, U>;                  \
		if (nr == 14)                                                  \
			return prot ? k_gcm<14, true, C, U>                    \
				    : k_gcm<14, false, C, U>;                  \
	}
	PICKG(false, false)
	PICKG(true, false)
	PICKG(true, true)
#undef PICKG
	return NULL;
}

unsigned sgpu_gcm_block(bool uni)
{
	return uni ? GCM_UNI_BLOCK : KBLOCK;
}
