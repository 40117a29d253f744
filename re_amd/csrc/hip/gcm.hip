/*
 * gcm.hip -- AES-GCM (AEAD_AES_128_GCM / AEAD_AES_256_GCM) kernels.
 */
#include <type_traits>
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
	if (COMPACT)
		prof_guard(a);
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
	/* small general launches: k_gcm_coop applies the keystream (before
	 * this kernel on protect, after it on unprotect); here GHASH reads
	 * the ciphertext as it lies */
	const bool ks_here = COMPACT || !a.nocipher;

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
		if (!ks_here) {
			x0 ^= bswap32(v.x); x1 ^= bswap32(v.y);
			x2 ^= bswap32(v.z); x3 ^= bswap32(v.w);
			ghash_mul(x0, x1, x2, x3, tab, stride, laneoff, rem4);
			continue;
		}
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
		uint32_t ks[4] = {0, 0, 0, 0}, ct[4];
		if (ks_here)
			C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
		const uint32_t rem = c_end - p;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			uint32_t bp = 4u * q;
			uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
			uint32_t m = (uint32_t)((1ull << (8 * nbytes)) - 1ull);
			const uint32_t o = (d[q] ^ ks[q]) & m;
			ct[q] = PROT && ks_here ? o : (d[q] & m);
			if (!ks_here)
				continue;
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

/*
 * Small general launches (k_ctr_coop's GCM form): the keystream of one
 * packet's cipher region across a workgroup, one 16-byte block (counter
 * b + 2) per lane; k_gcm runs with KArgs.nocipher and only GHASHes.
 * Protect: this kernel first (GHASH covers the ciphertext); unprotect:
 * after k_gcm (which read the received ciphertext), decrypting in place
 * whatever the tag (aes.c:136-249: the EVP decrypt writes before the
 * final tag check), like the fused kernel.  Undo jobs stay in k_gcm.
 */
template <int NR>
__global__ void __launch_bounds__(256)
k_gcm_coop(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT_BYTES];
	const uint32_t i = blockIdx.x;
	if (i >= a.njobs)
		return;
	const struct sgpu_job j = a.jobs[i];
	if ((j.flags & (SJ_SKIP | SJ_UNDO)) || !(j.flags & SJ_CIPHER))
		return;
	tt_fill(smem, a.t0);
	__syncthreads();
	const struct sgpu_comp *cp = a.comps +
				     __builtin_amdgcn_readfirstlane(j.comp);
	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < 4 * (NR + 1); k++)
		rk[k] = __builtin_amdgcn_readfirstlane(cp->rk[k]);
	/* srtp_iv_calc_gcm (misc.c:93-105), as k_gcm */
	uint32_t iv[3];
	{
		const uint4 ks = *(const uint4 *)cp->k_s;
		const uint32_t be0 = (j.ssrc >> 16) & 0xffffu;
		const uint32_t be1 = ((j.ssrc & 0xffffu) << 16) | (j.ixhi >> 16);
		const uint32_t be2 = ((j.ixhi & 0xffffu) << 16) | (j.ixlo & 0xffffu);
		iv[0] = ks.x ^ bswap32(be0);
		iv[1] = ks.y ^ bswap32(be1);
		iv[2] = ks.z ^ bswap32(be2);
	}
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	uint8_t *pkt = a.arena + j.off;
	const uint32_t c_end = j.c_off + j.c_len;
	for (uint32_t b = threadIdx.x; j.c_off + 16u * b < c_end;
	     b += blockDim.x) {
		uint32_t s0 = iv[0], s1 = iv[1], s2 = iv[2], s3 = bswap32(b + 2u);
		aes_block<NR>(smem, lo, rk, s0, s1, s2, s3);
		const uint32_t ks[4] = {s0, s1, s2, s3};
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
}

kfn_t sgpu_pick_gcm_coop(int nr)
{
	return nr == 10 ? k_gcm_coop<10> : k_gcm_coop<14>;
}

/* ------------------------------------------------------------------ */
/*
 * Single-key AES-GCM (compact launches whose packets share one session
 * context -- the BASELINE config-3 path).  Same structure as the CTR
 * kernel (k_ctr.h): 64-byte chunks aligned to the packet, a branch-free
 * steady-state body with quad-coalesced chunk access, general byte-exact
 * chunks at the head/tail.  GHASH uses an 8-bit table (ghash8_mul).
 *
 * LDS: T0/T1 image [0, 64 KiB) + GHASH M8 image [64, 128 KiB).
 */
#define GH8_OFF TT_BYTES
#define GH8_BYTES 65536u
#ifndef GCMU_BLOCK
#define GCMU_BLOCK 1024u    /* 4 waves/SIMD at <= 128 VGPRs (protect spills
				   32 to scratch): 1.93 -> 1.69 ms per 1M
				   packets against 768 threads (3 waves/SIMD,
				   no spills) -- the LDS latency wants waves */
#endif
#ifndef GCMU_COAL           /* quad-coalesced 64-byte chunks: off since the
			       1024-thread blocks -- the quad offsets and
			       transposes cost registers (protect spilled),
			       and per-lane chunks measured faster (protect
			       1.64 -> 1.57 ms, unprotect 1.64 -> 1.62) */
#define GCMU_COAL 0
#endif
#ifndef GCMU_B8             /* counters < 256 (packets < SGPU_CACHED_MAX_GCM
			       = 4032 B): 5 fewer T-table lookups per block */
#define GCMU_B8 1
#endif
#ifndef GCMU_ALIGNED        /* packet-aligned 64-byte chunks (gcma_packet) */
#define GCMU_ALIGNED 1
#endif

/*
 * M8[b] = b * H for all bytes b (OpenSSL Htable convention, BE words),
 * from the 4-bit table: M8[b] = T4[b >> 4] ^ T4[b & 15] * x^4 (one 4-bit
 * Shoup shift step, reduction rem_4bit[r] = clmul(r, 0xE1) << 21 in the
 * top word).  Image: entry b at b * 256 + (lane & 15) * 16, 16 replicas:
 * a ds_read_b128 serves 16 lanes per LDS cycle, each from its own 16-byte
 * bank group whatever the entries (conflict-free).
 */
__device__ __forceinline__ void gh8_fill(uint8_t *img, const uint32_t (*ht)[4])
{
	for (uint32_t i = threadIdx.x; i < 256u * 16u; i += blockDim.x) {
		const uint32_t b = i >> 4, r = i & 15u;
		const uint4 L = *(const uint4 *)ht[b & 15u];
		const uint4 H = *(const uint4 *)ht[b >> 4];
		const uint32_t m = L.w & 15u;
		const uint32_t red = (m ^ (m << 5) ^ (m << 6) ^ (m << 7)) << 21;
		*(uint4 *)(img + b * 256u + r * 16u) = make_uint4(
			(L.x >> 4) ^ red ^ H.x,
			__builtin_amdgcn_alignbit(L.x, L.y, 4) ^ H.y,
			__builtin_amdgcn_alignbit(L.y, L.z, 4) ^ H.z,
			__builtin_amdgcn_alignbit(L.z, L.w, 4) ^ H.w);
	}
}

/* gh8_fill for 1024-thread blocks: thread t's 4 entries b = (t >> 4) +
 * 64 j share L = ht[(t >> 4) & 15]; the 5 table loads issued together */
__device__ __forceinline__ void gh8_fill_b1024(uint8_t *img,
					       const uint32_t (*ht)[4])
{
	const uint32_t tid = threadIdx.x, r = tid & 15u;
	const uint4 L = *(const uint4 *)ht[(tid >> 4) & 15u];
	uint4 H[4];
#pragma unroll
	for (int j = 0; j < 4; j++)
		H[j] = *(const uint4 *)ht[(tid >> 8) + 4u * (uint32_t)j];
	const uint32_t m = L.w & 15u;
	const uint32_t red = (m ^ (m << 5) ^ (m << 6) ^ (m << 7)) << 21;
	const uint32_t lx = (L.x >> 4) ^ red;
	const uint32_t ly = __builtin_amdgcn_alignbit(L.x, L.y, 4);
	const uint32_t lz = __builtin_amdgcn_alignbit(L.y, L.z, 4);
	const uint32_t lw = __builtin_amdgcn_alignbit(L.z, L.w, 4);
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint32_t b = (tid >> 4) + 64u * (uint32_t)j;
		*(uint4 *)(img + b * 256u + r * 16u) = make_uint4(
			lx ^ H[j].x, ly ^ H[j].y, lz ^ H[j].z, lw ^ H[j].w);
	}
}

#ifndef GCM_FILL_LOOP
#define GCM_FILL_LOOP 0
#endif

/*
 * X = X * H (SP 800-38D 6.3) with the 8-bit table and one deferred
 * reduction.  With X_i the byte i of X and i = 4w + q:
 *   X * H = sum_i M8[X_i] x^(8i) = sum_q x^(8q) A_q,
 *   A_q   = sum_w M8[X_(4w+q)] x^(32w)        (word shifts: free)
 * evaluated by Horner in q on an 8-word accumulator (x^8 = an 8-bit right
 * shift of BE words), then the degrees 128..247 are folded back with
 * x^128 = 1 + x + x^2 + x^7.  16 ds_read_b128 + ~110 VALU per block, no
 * per-byte reduction table (OpenSSL's gcm_gmult_4bit: 32 lookups + 32
 * reduction lookups).  hi16 = (lane & 15) * 16 | 0x10000 (image base).
 */
__device__ __forceinline__ void ghash8_mul(uint32_t x[4], const uint8_t *smem,
					   uint32_t hi16)
{
	uint32_t R[8];
#pragma unroll
	for (int q = 3; q >= 0; q--) {
		uint4 M[4];
#pragma unroll
		for (int w = 0; w < 4; w++)
			M[w] = *(const uint4 *)(smem + TT_ADDRH(x[w], 3 - q, hi16));
		const uint32_t A0 = M[0].x;
		const uint32_t A1 = M[0].y ^ M[1].x;
		const uint32_t A2 = xor3(M[0].z, M[1].y, M[2].x);
		const uint32_t A3 = xor3(M[0].w, M[1].z, M[2].y) ^ M[3].x;
		const uint32_t A4 = xor3(M[1].w, M[2].z, M[3].y);
		const uint32_t A5 = M[2].w ^ M[3].z;
		const uint32_t A6 = M[3].w;
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

/*
 * One packet.  The cipher region is walked in 64-byte units aligned to its
 * start c_off (four GHASH blocks each, so no block straddles two units):
 * full units run a branch-free body (quad-coalesced when the four lanes of
 * a quad all have one), the remainder (< 64 bytes) takes the byte-exact
 * per-block path of the general kernel (k_gcm).  Returns the SV_* verdict.
 */
template <int NR, bool PROT>
__device__ __forceinline__ uint8_t gcmu_packet(const uint8_t *smem, uint32_t lo,
					       uint32_t hi16, const uint32_t *rk,
					       const CtrKs<NR, true, false, GCMU_B8> &C,
					       uint8_t *arena, uint64_t asz,
					       const struct sgpu_job &j,
					       uint32_t lane)
{
	uint8_t *pkt = arena + j.off;
	const uint64_t pasz = asz - j.off;
	const uint32_t A = j.a_len;
	const uint32_t c_off = j.c_off, c_len = j.c_len;
	const uint32_t c_end = c_off + c_len;
	uint32_t X[4] = {0, 0, 0, 0};
	for (uint32_t p = 0; p < A; p += 16) {
		uint32_t w[4];
		aad_block(pkt, pasz, p, A, false, 0u, w);
		X[0] ^= w[0]; X[1] ^= w[1]; X[2] ^= w[2]; X[3] ^= w[3];
		ghash8_mul(X, smem, hi16);
	}

	const uint32_t nunit = c_len / 64u;
	uint32_t M1 = 0;
	uint64_t qb[4];
	if (GCMU_COAL) {
		quad_offsets((uint64_t)j.off + c_off, lane, qb);
		const uint64_t act = __ballot(1);
		uint32_t a1 = min(nunit, qdpp<DPP_QXOR1>(nunit));
		a1 = min(a1, qdpp<DPP_QXOR2>(a1));
		if (((act >> (lane & ~3u)) & 0xfull) == 0xfull)
			M1 = a1;
	}
	auto unit = [&](uint32_t m, auto coal) {
		constexpr bool CO = decltype(coal)::value;
		const uint32_t p0 = c_off + 64u * m;
		uint32_t d[16], o[16];
		if constexpr (CO) {
			quad_load(arena, qb, 64u * m, lane, d);
		}
		else {
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = *(const uint4 *)(pkt + p0 + 16u * g);
				d[4 * g] = v.x; d[4 * g + 1] = v.y;
				d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
			}
		}
#pragma unroll
		for (int b = 0; b < 4; b++) {
			uint32_t ks[4];
			C.block(smem, lo, rk, (int32_t)(4u * m + b + 2u), ks);
#pragma unroll
			for (int q = 0; q < 4; q++)
				o[4 * b + q] = d[4 * b + q] ^ ks[q];
		}
		if constexpr (CO) {
			quad_store(arena, qb, 64u * m, lane, o);
		}
		else {
#pragma unroll
			for (int g = 0; g < 4; g++)
				*(uint4 *)(pkt + p0 + 16u * g) =
					make_uint4(o[4 * g], o[4 * g + 1],
						   o[4 * g + 2], o[4 * g + 3]);
		}
#pragma unroll
		for (int b = 0; b < 4; b++) {
			const uint32_t *c = PROT ? o + 4 * b : d + 4 * b;
			X[0] ^= bswap32(c[0]); X[1] ^= bswap32(c[1]);
			X[2] ^= bswap32(c[2]); X[3] ^= bswap32(c[3]);
			ghash8_mul(X, smem, hi16);
		}
	};
	uint32_t m = 0;
	if (GCMU_COAL)
		for (; m < M1; m++)
			unit(m, std::true_type());
	for (; m < nunit; m++)
		unit(m, std::false_type());

	/* remainder: whole 16-byte blocks, then the partial one (k_gcm) */
	const uint32_t nfull = c_len / 16u;
	for (uint32_t b = 4u * nunit; b < nfull; b++) {
		const uint32_t p = c_off + 16u * b;
		const uint4 v = ld16(pkt, pasz, p);
		uint32_t ks[4];
		C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
		const uint32_t o0 = v.x ^ ks[0], o1 = v.y ^ ks[1];
		const uint32_t o2 = v.z ^ ks[2], o3 = v.w ^ ks[3];
		*(uint4 *)(pkt + p) = make_uint4(o0, o1, o2, o3);
		X[0] ^= bswap32(PROT ? o0 : v.x); X[1] ^= bswap32(PROT ? o1 : v.y);
		X[2] ^= bswap32(PROT ? o2 : v.z); X[3] ^= bswap32(PROT ? o3 : v.w);
		ghash8_mul(X, smem, hi16);
	}
	if (c_len > 16u * nfull) {
		const uint32_t b = nfull, p = c_off + 16u * b;
		const uint4 v = ld16(pkt, pasz, p);
		const uint32_t d[4] = {v.x, v.y, v.z, v.w};
		uint32_t ks[4], ct[4];
		C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
		const uint32_t rem = c_end - p;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t bp = 4u * q;
			const uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
			const uint32_t mk = (uint32_t)((1ull << (8 * nbytes)) - 1ull);
			const uint32_t o = (d[q] ^ ks[q]) & mk;
			ct[q] = PROT ? o : (d[q] & mk);
			if (nbytes == 4)
				*(uint32_t *)(pkt + p + bp) = o;
			else if (nbytes)
				st_partial(pkt + p + bp, o, nbytes);
		}
		X[0] ^= bswap32(ct[0]); X[1] ^= bswap32(ct[1]);
		X[2] ^= bswap32(ct[2]); X[3] ^= bswap32(ct[3]);
		ghash8_mul(X, smem, hi16);
	}

	/* length block: bitlen(AAD) || bitlen(C) */
	{
		const uint64_t al = (uint64_t)A * 8u, cl = (uint64_t)c_len * 8u;
		X[0] ^= (uint32_t)(al >> 32); X[1] ^= (uint32_t)al;
		X[2] ^= (uint32_t)(cl >> 32); X[3] ^= (uint32_t)cl;
		ghash8_mul(X, smem, hi16);
	}
	/* tag = GHASH ^ E(K, J0) */
	uint32_t e0[4];
	C.block(smem, lo, rk, 1, e0);
	const uint32_t t[4] = {X[0] ^ bswap32(e0[0]), X[1] ^ bswap32(e0[1]),
			       X[2] ^ bswap32(e0[2]), X[3] ^ bswap32(e0[3])};
	uint8_t *tp = pkt + j.tag_off;
	uint8_t vd = SV_CIPHERED;
	if (PROT) {
#pragma unroll
		for (int q = 0; q < 4; q++)
			st_be32(tp + 4 * q, t[q]);
	}
	else {
		uint32_t diff = 0;
#pragma unroll
		for (int q = 0; q < 16; q++)
			diff |= tp[q] ^ (uint8_t)(t[q >> 2] >> (24 - 8 * (q & 3)));
		if (diff == 0)
			vd |= SV_TAG_OK;
	}
	return vd;
}

/* one whole cipher block b of the per-block path (c_off-aligned, 16 B) */
template <int NR, bool PROT>
__device__ __forceinline__ void gcm_block16(const uint8_t *smem, uint32_t lo,
					   uint32_t hi16, const uint32_t *rk,
					   const CtrKs<NR, true, false, GCMU_B8> &C, uint8_t *pkt,
					   uint64_t pasz, uint32_t c_off,
					   uint32_t b, uint32_t X[4])
{
	const uint32_t p = c_off + 16u * b;
	const uint4 v = ld16(pkt, pasz, p);
	uint32_t ks[4];
	C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
	const uint32_t o0 = v.x ^ ks[0], o1 = v.y ^ ks[1];
	const uint32_t o2 = v.z ^ ks[2], o3 = v.w ^ ks[3];
	*(uint4 *)(pkt + p) = make_uint4(o0, o1, o2, o3);
	X[0] ^= bswap32(PROT ? o0 : v.x); X[1] ^= bswap32(PROT ? o1 : v.y);
	X[2] ^= bswap32(PROT ? o2 : v.z); X[3] ^= bswap32(PROT ? o3 : v.w);
	ghash8_mul(X, smem, hi16);
}

/*
 * gcmu_packet with packet-aligned memory traffic.  The GHASH / counter
 * blocks start at c_off = 16 t + 4 S, so a 64-byte chunk k of the packet
 * (bytes [64k, 64k + 64), the arena's own line grid when slots are
 * 64-byte multiples) holds, for S > 0: the last S words of block
 * beta - 1 (beta = 4k - t), blocks beta .. beta + 2 whole, and the first
 * 4 - S words of block beta + 3, whose remaining keystream and ciphertext
 * words are carried in registers to chunk k + 1 (S = 0: four whole
 * blocks).  Chunks whose words all lie in whole cipher blocks run that
 * branch-free body with aligned (quad-coalesced) 64-byte loads and stores;
 * the blocks before them and after them take the per-block path, and the
 * straddling block at either end is finished word by word.  Same
 * results as gcmu_packet (SP 800-38D GCTR + GHASH, aes.c:136-249).
 */
template <int NR, bool PROT, int S>
__device__ __forceinline__ uint8_t gcma_packet(const uint8_t *smem, uint32_t lo,
					       uint32_t hi16, const uint32_t *rk,
					       const CtrKs<NR, true, false, GCMU_B8> &C,
					       uint8_t *arena, uint64_t asz,
					       const struct sgpu_job &j,
					       uint32_t lane)
{
	uint8_t *pkt = arena + j.off;
	const uint64_t pasz = asz - j.off;
	const uint32_t A = j.a_len;
	/* SRTCP: E || index closes the AAD (srtcp.c:82-102, 239-262); an
	 * unencrypted SRTCP packet has no cipher region */
	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
	const uint32_t aad_total = A + (trail ? 4u : 0u);
	const uint32_t c_off = j.c_off, c_len = do_cipher ? j.c_len : 0u;
	const uint32_t c_end = c_off + c_len;
	const uint32_t t = c_off >> 4;
	const uint32_t nfull = c_len / 16u;
	uint32_t X[4] = {0, 0, 0, 0};
	for (uint32_t p = 0; p < aad_total; p += 16) {
		uint32_t w[4];
		aad_block(pkt, pasz, p, A, trail, j.trailer, w);
		X[0] ^= w[0]; X[1] ^= w[1]; X[2] ^= w[2]; X[3] ^= w[3];
		ghash8_mul(X, smem, hi16);
	}

	/* steady chunks [k0, k1): block beta - 1 >= 0 (S > 0), the last
	 * block touched (beta + 3) whole */
	const uint32_t k0 = S ? (t + 4u) / 4u : (t + 3u) / 4u;
	uint32_t k1 = (nfull + t) / 4u;
	if (k1 < k0)
		k1 = k0;
	const uint32_t nst = k1 - k0;
	/* per-block prologue: blocks [0, P) */
	const uint32_t P = nst ? 4u * k0 - t - (S ? 1u : 0u) : nfull;
	for (uint32_t b = 0; b < P; b++)
		gcm_block16<NR, PROT>(smem, lo, hi16, rk, C, pkt, pasz, c_off, b,
				      X);
	uint32_t cks[4] = {0, 0, 0, 0};  /* keystream words S.. of the block */
	uint32_t chd[4] = {0, 0, 0, 0};  /* its ciphertext words 0..3-S */
	if (S && nst) {
		/* head of block P: the last 4 - S words of chunk k0 - 1 */
		uint32_t ks[4];
		C.block(smem, lo, rk, (int32_t)(P + 2u), ks);
		const uint32_t hp = 64u * k0 - 4u * (4 - S);
#pragma unroll
		for (int q = 0; q < 4 - S; q++) {
			uint32_t *wp = (uint32_t *)(pkt + hp + 4u * q);
			const uint32_t v = *wp, o = v ^ ks[q];
			*wp = o;
			chd[q] = PROT ? o : v;
		}
#pragma unroll
		for (int q = 0; q < S; q++)
			cks[q] = ks[4 - S + q];
	}

	uint32_t M1 = 0;
	uint64_t qb[4];
	if (GCMU_COAL) {
		quad_offsets((uint64_t)j.off + 64u * k0, lane, qb);
		const uint64_t act = __ballot(1);
		uint32_t a1 = min(nst, qdpp<DPP_QXOR1>(nst));
		a1 = min(a1, qdpp<DPP_QXOR2>(a1));
		if (((act >> (lane & ~3u)) & 0xfull) == 0xfull)
			M1 = a1;
	}
	auto chunk = [&](uint32_t m, auto coal) {
		constexpr bool CO = decltype(coal)::value;
		const uint32_t k = k0 + m;
		const uint32_t beta = 4u * k - t;
		uint32_t d[16], o[16];
		if constexpr (CO) {
			quad_load(arena, qb, 64u * m, lane, d);
		}
		else {
#pragma unroll
			for (int g = 0; g < 4; g++) {
				const uint4 v = *(const uint4 *)(pkt + 64u * k +
								 16u * g);
				d[4 * g] = v.x; d[4 * g + 1] = v.y;
				d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
			}
		}
		uint32_t hb[4];         /* block beta - 1 (S > 0) */
		if (S) {
#pragma unroll
			for (int q = 0; q < S; q++)
				o[q] = d[q] ^ cks[q];
#pragma unroll
			for (int q = 0; q < 4 - S; q++)
				hb[q] = chd[q];
#pragma unroll
			for (int q = 0; q < S; q++)
				hb[4 - S + q] = PROT ? o[q] : d[q];
		}
#pragma unroll
		for (int mm = 0; mm < (S ? 3 : 4); mm++) {
			uint32_t ks[4];
			C.block(smem, lo, rk, (int32_t)(beta + mm + 2u), ks);
#pragma unroll
			for (int q = 0; q < 4; q++)
				o[S + 4 * mm + q] = d[S + 4 * mm + q] ^ ks[q];
		}
		if (S) {
			uint32_t ks[4];
			C.block(smem, lo, rk, (int32_t)(beta + 5u), ks);
#pragma unroll
			for (int q = 0; q < 4 - S; q++) {
				o[12 + S + q] = d[12 + S + q] ^ ks[q];
				chd[q] = PROT ? o[12 + S + q] : d[12 + S + q];
			}
#pragma unroll
			for (int q = 0; q < S; q++)
				cks[q] = ks[4 - S + q];
		}
		if constexpr (CO) {
			quad_store(arena, qb, 64u * m, lane, o);
		}
		else {
			/* the chunk's four 16-B stores back to back: scheduled
			 * as each block is ready (the unprotect S = 2 body put
			 * ~1000 instructions between them), a lane's 64-B line
			 * was evicted half written and written back twice --
			 * SRTCP-GCM unprotect moved 2.6 GB of writes against
			 * 1.7 for the same bytes (TCC_NORMAL_WRITEBACK x2) */
			__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int g = 0; g < 4; g++)
				*(uint4 *)(pkt + 64u * k + 16u * g) =
					make_uint4(o[4 * g], o[4 * g + 1],
						   o[4 * g + 2], o[4 * g + 3]);
		}
		if (S) {
			X[0] ^= bswap32(hb[0]); X[1] ^= bswap32(hb[1]);
			X[2] ^= bswap32(hb[2]); X[3] ^= bswap32(hb[3]);
			ghash8_mul(X, smem, hi16);
		}
#pragma unroll
		for (int mm = 0; mm < (S ? 3 : 4); mm++) {
			const uint32_t *c = (PROT ? o : d) + S + 4 * mm;
			X[0] ^= bswap32(c[0]); X[1] ^= bswap32(c[1]);
			X[2] ^= bswap32(c[2]); X[3] ^= bswap32(c[3]);
			ghash8_mul(X, smem, hi16);
		}
	};
	uint32_t m = 0;
	if (GCMU_COAL)
		for (; m < M1; m++)
			chunk(m, std::true_type());
	for (; m < nst; m++)
		chunk(m, std::false_type());

	uint32_t b = P;
	if (nst) {
		b = 4u * k1 - t;
		if (S) {
			/* tail of block b - 1: the first S words of chunk k1 */
			uint32_t hb[4];
#pragma unroll
			for (int q = 0; q < 4 - S; q++)
				hb[q] = chd[q];
#pragma unroll
			for (int q = 0; q < S; q++) {
				uint32_t *wp = (uint32_t *)(pkt + 64u * k1 + 4u * q);
				const uint32_t v = *wp, o = v ^ cks[q];
				*wp = o;
				hb[4 - S + q] = PROT ? o : v;
			}
			X[0] ^= bswap32(hb[0]); X[1] ^= bswap32(hb[1]);
			X[2] ^= bswap32(hb[2]); X[3] ^= bswap32(hb[3]);
			ghash8_mul(X, smem, hi16);
		}
	}
	for (; b < nfull; b++)
		gcm_block16<NR, PROT>(smem, lo, hi16, rk, C, pkt, pasz, c_off, b,
				      X);
	if (c_len > 16u * nfull) {
		const uint32_t bb = nfull, p = c_off + 16u * bb;
		const uint4 v = ld16(pkt, pasz, p);
		const uint32_t d[4] = {v.x, v.y, v.z, v.w};
		uint32_t ks[4], ct[4];
		C.block(smem, lo, rk, (int32_t)(bb + 2u), ks);
		const uint32_t rem = c_end - p;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t bp = 4u * q;
			const uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
			const uint32_t mk = (uint32_t)((1ull << (8 * nbytes)) - 1ull);
			const uint32_t o = (d[q] ^ ks[q]) & mk;
			ct[q] = PROT ? o : (d[q] & mk);
			if (nbytes == 4)
				*(uint32_t *)(pkt + p + bp) = o;
			else if (nbytes)
				st_partial(pkt + p + bp, o, nbytes);
		}
		X[0] ^= bswap32(ct[0]); X[1] ^= bswap32(ct[1]);
		X[2] ^= bswap32(ct[2]); X[3] ^= bswap32(ct[3]);
		ghash8_mul(X, smem, hi16);
	}

	/* length block: bitlen(AAD) || bitlen(C) */
	{
		const uint64_t al = (uint64_t)aad_total * 8u;
		const uint64_t cl = (uint64_t)c_len * 8u;
		X[0] ^= (uint32_t)(al >> 32); X[1] ^= (uint32_t)al;
		X[2] ^= (uint32_t)(cl >> 32); X[3] ^= (uint32_t)cl;
		ghash8_mul(X, smem, hi16);
	}
	/* tag = GHASH ^ E(K, J0) */
	uint32_t e0[4];
	C.block(smem, lo, rk, 1, e0);
	const uint32_t tg[4] = {X[0] ^ bswap32(e0[0]), X[1] ^ bswap32(e0[1]),
				X[2] ^ bswap32(e0[2]), X[3] ^ bswap32(e0[3])};
	uint8_t *tp = pkt + j.tag_off;
	uint8_t vd = do_cipher ? SV_CIPHERED : 0;
	if (PROT) {
#pragma unroll
		for (int q = 0; q < 4; q++)
			st_be32(tp + 4 * q, tg[q]);
		if (j.flags & SJ_STORE_TRAIL)
			st_be32(pkt + j.t_off, j.trailer);
	}
	else {
		uint32_t diff = 0;
#pragma unroll
		for (int q = 0; q < 16; q++)
			diff |= tp[q] ^ (uint8_t)(tg[q >> 2] >> (24 - 8 * (q & 3)));
		if (diff == 0)
			vd |= SV_TAG_OK;
	}
	return vd;
}

template <int NR, bool PROT>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, GCMU_BLOCK)))
__attribute__((amdgpu_waves_per_eu(GCMU_BLOCK / 256u, 8)))
k_gcmu(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT_BYTES + GH8_BYTES];
	__shared__ uint32_t blk_comp;
	prof_guard(a);
	if (a.c.guard && *a.c.guard)          /* rejected plan */
		return;
	static_assert(GCMU_BLOCK == 1024u, "tt_fill_b1024 / gh8_fill_b1024");
	if (GCM_FILL_LOOP || blockDim.x != 1024u)
		tt_fill(smem, a.t0);
	else
		tt_fill_b1024(smem, a.t0);
	uint8_t *__restrict__ verdict = a.verdict;
	const bool undo = a.c.undo;
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	struct sgpu_job j;
	uint32_t i = 0;
	const bool live = get_job<true, SGPU_MODE_GCM, PROT>(
		a, blockIdx.x * blockDim.x + threadIdx.x, j, i);
	if (!live)
		j.flags = SJ_SKIP, j.comp = 0;
	/* the block's first live packet names the context (every packet of
	 * a single-key launch shares it) */
	if (threadIdx.x == 0)
		blk_comp = 0xffffffffu;
	__syncthreads();
	if (live && !(j.flags & SJ_SKIP))
		atomicMin(&blk_comp, j.comp);
	__syncthreads();
	const uint32_t bc = blk_comp;
	if (bc != 0xffffffffu) {
		if (GCM_FILL_LOOP || blockDim.x != 1024u)
			gh8_fill(smem + GH8_OFF, a.comps[bc].htab);
		else
			gh8_fill_b1024(smem + GH8_OFF, a.comps[bc].htab);
	}
	__syncthreads();
	if (!live)
		return;
	if (j.flags & SJ_SKIP) {
		if (verdict && !undo)
			verdict[i] = 0;
		return;
	}
	const uint32_t ci = __builtin_amdgcn_readfirstlane(j.comp);
	const struct sgpu_comp *cp = a.comps + ci;
	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}
#pragma unroll
	for (int k = 0; k < 4 * (NR + 1); k++)
		rk[k] = __builtin_amdgcn_readfirstlane(rk[k]);
	uint8_t *pkt = a.arena + j.off;

	/* srtp_iv_calc_gcm (misc.c:93-105); J0 = IV || 0^31 || 1 */
	uint32_t iv[4];
	{
		uint4 ks = *(const uint4 *)cp->k_s;
		const uint32_t ixhi = j.ixhi, ixlo = j.ixlo;
		const uint32_t be0 = (j.ssrc >> 16) & 0xffffu;
		const uint32_t be1 = ((j.ssrc & 0xffffu) << 16) | (ixhi >> 16);
		const uint32_t be2 = ((ixhi & 0xffffu) << 16) | (ixlo & 0xffffu);
		iv[0] = ks.x ^ bswap32(be0);
		iv[1] = ks.y ^ bswap32(be1);
		iv[2] = ks.z ^ bswap32(be2);
		iv[3] = 0;
	}
	CtrKs<NR, true, false, GCMU_B8> C;
	C.init(smem, lo, rk, iv);

	if (j.flags & SJ_UNDO) {
		/* re-apply the keystream: restores a speculatively decrypted
		 * payload before the exact re-run (counter b + 2) */
		const uint32_t nb = (j.c_len + 15u) / 16u;
		for (uint32_t b = 0; b < nb; b++) {
			const uint32_t p = j.c_off + 16u * b;
			uint32_t ks[4];
			C.block(smem, lo, rk, (int32_t)(b + 2u), ks);
			const uint32_t rem = j.c_off + j.c_len - p;
			for (int q = 0; q < 4; q++) {
				const uint32_t bp = 4u * q;
				const uint32_t nbytes = bp < rem ? min(rem - bp, 4u) : 0u;
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
		return;
	}
	const uint32_t hi16 = ((lane & 15u) << 4) | 0x10000u;
	uint8_t vd;
	if (GCMU_ALIGNED) {
		switch ((j.c_off >> 2) & 3u) {
		case 0:
			vd = gcma_packet<NR, PROT, 0>(smem, lo, hi16, rk, C,
						      a.arena, a.asz, j, lane);
			break;
		case 1:
			vd = gcma_packet<NR, PROT, 1>(smem, lo, hi16, rk, C,
						      a.arena, a.asz, j, lane);
			break;
		case 2:
			vd = gcma_packet<NR, PROT, 2>(smem, lo, hi16, rk, C,
						      a.arena, a.asz, j, lane);
			break;
		default:
			vd = gcma_packet<NR, PROT, 3>(smem, lo, hi16, rk, C,
						      a.arena, a.asz, j, lane);
			break;
		}
	}
	else {
		vd = gcmu_packet<NR, PROT>(smem, lo, hi16, rk, C, a.arena,
					   a.asz, j, lane);
	}
	if (!PROT && !(vd & SV_TAG_OK))
		atomicAdd(a.c.nfail, 1u);
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
#undef PICKG
	if (compact && uni) {
		if (nr == 10)
			return prot ? k_gcmu<10, true> : k_gcmu<10, false>;
		if (nr == 14)
			return prot ? k_gcmu<14, true> : k_gcmu<14, false>;
	}
	return NULL;
}

unsigned sgpu_gcm_block(bool uni)
{
	return uni ? GCMU_BLOCK : KBLOCK;
}
