/*
 * srtp_kernels.hip -- MI355X (gfx950) kernels for SRTP/SRTCP protect and
 * unprotect, plus the thin C-ABI shim declared in ../srtpgpu.h.
 *
 * Work decomposition: ONE PACKET PER LANE.  SHA-1 is a serial chain of
 * 80-round compressions per packet (20 of them for a 1200-B RTP packet), so
 * giving each packet its own lane keeps all 64 lanes of a wave busy; a
 * packet-per-workgroup split would leave 63/64 lanes idle during SHA-1
 * ("Hard parts").  AES-CTR for the same packet runs in the same
 * lane, fused with the MAC: the payload is read once and written once.
 *
 *   k_ctr_hmac<NR,SHIFT,PROT>  AES-CM (src/aes/openssl/aes.c:136-171) fused
 *                              with HMAC-SHA1 (src/hmac/openssl/hmac.c:87):
 *                              srtp_encrypt srtp.c:215-277, srtp_decrypt
 *                              srtp.c:325-382, srtcp.c:56-135, 180-227.
 *   k_gcm<NR,PROT>             AES-GCM with 96-bit IV (aes.c:136-249):
 *                              srtp.c:226-253, 383-424; srtcp.c:69-112,228-282
 *   k_setup                    srtp_alloc/comp_init KDF (srtp.c:33-72,
 *                              misc.c:44-73), key schedule, HMAC midstates,
 *                              GHASH table.
 *   k_parse_rtp / k_parse_rtcp rtp_hdr_decode (src/rtp/rtp.c:88-137),
 *                              get_rtcp_ssrc (srtcp.c:19-28) for
 *                              device-resident batches.
 *
 * No MFMA: this is byte/word integer work (VALU + LDS).
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include "../srtpgpu.h"
#include "dev_common.h"

#define KBLOCK 256

__device__ uint32_t g_T0[256];          /* T0 table (source of LDS image) */
__device__ uint8_t g_sbox[256];

/* OpenSSL gcm_gmult_4bit rem_4bit (values << 16 into the top word) */
__constant__ uint32_t c_rem4[16] = {
	0x0000u << 16, 0x1C20u << 16, 0x3840u << 16, 0x2460u << 16,
	0x7080u << 16, 0x6CA0u << 16, 0x48C0u << 16, 0x54E0u << 16,
	0xE100u << 16, 0xFD20u << 16, 0xD940u << 16, 0xC560u << 16,
	0x9180u << 16, 0x8DA0u << 16, 0xA9C0u << 16, 0xB5E0u << 16,
};

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
 * CRYPTO_ctr128_encrypt semantics) */
template <int NR>
__device__ __forceinline__ void ctr_block(const uint8_t *smem, uint32_t lo,
					  const uint32_t *rk, const uint32_t iv[4],
					  int32_t b, uint32_t ks[4])
{
	uint64_t c = ((uint64_t)bswap32(iv[2]) << 32 | bswap32(iv[3])) +
		     (uint64_t)(int64_t)b;
	uint32_t s0 = iv[0], s1 = iv[1];
	uint32_t s2 = bswap32((uint32_t)(c >> 32));
	uint32_t s3 = bswap32((uint32_t)c);
	aes_block<NR>(smem, lo, rk, s0, s1, s2, s3);
	ks[0] = s0; ks[1] = s1; ks[2] = s2; ks[3] = s3;
}

/* the SHA-1 input word at global word index gw of the HMAC message
 * M = data[0,A) ‖ (trailer?) ‖ 0x80 ‖ 0* ‖ len64 -- for non-fast chunks */
__device__ __forceinline__ uint32_t msg_word(uint32_t gw, uint32_t data_be,
					     uint32_t A, uint64_t X)
{
	uint32_t aw = A >> 2, u = A & 3;
	if (gw < aw)
		return data_be;
	if (gw == aw)
		return (u ? (data_be & (0xFFFFFFFFu << (32 - 8 * u))) : 0u) |
		       (uint32_t)(X >> (32 + 8 * u));
	if (gw == aw + 1)
		return (uint32_t)(X >> (8 * u));
	return 0;
}

/* ------------------------------------------------------------------ */
/* kernel arguments and job sources                                    */

struct KArgs {
	uint8_t *arena;
	uint64_t asz;
	const struct sgpu_job *jobs;    /* general path */
	uint32_t njobs;
	const struct sgpu_comp *comps;
	uint8_t *verdict;
	uint32_t *save;
	struct sgpu_compact c;          /* compact path */
};

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

/*
 * Fused AES-CM + HMAC-SHA1, one packet per lane.
 *   SHIFT = (c_off / 4) & 3: the cipher region starts SHIFT words into a
 *   16-byte packet granule (3 for a 12-byte RTP header, 2 for SRTCP).
 */
template <int NR, int SHIFT, bool PROT, bool COMPACT>
__global__ void __launch_bounds__(KBLOCK)
k_ctr_hmac(const KArgs a)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT_BYTES];
	tt_fill(smem, g_T0);
	__syncthreads();

	uint8_t *const arena = a.arena;
	const uint64_t asz = a.asz;
	const struct sgpu_comp *__restrict__ comps = a.comps;
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
	const struct sgpu_comp *cp = comps + j.comp;

	uint32_t rk[4 * (NR + 1)];
#pragma unroll
	for (int k = 0; k < NR + 1; k++) {
		uint4 v = *(const uint4 *)&cp->rk[4 * k];
		rk[4 * k] = v.x; rk[4 * k + 1] = v.y;
		rk[4 * k + 2] = v.z; rk[4 * k + 3] = v.w;
	}

	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
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

	uint32_t carry[4] = {0, 0, 0, 0};

	for (uint32_t k = 0; k < nchunk; k++) {
		const uint32_t c0 = 64u * k;
		uint32_t d[16];
		/* ---- load ---- */
#pragma unroll
		for (int g = 0; g < 4; g++) {
			uint4 v = make_uint4(0, 0, 0, 0);
			if (c0 + 16u * g < data_end)
				v = ld16(pkt, pasz, c0 + 16u * g);
			d[4 * g] = v.x; d[4 * g + 1] = v.y;
			d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
		}
		/* ---- keystream ---- */
		uint32_t ksw[16];
		const bool need_ks = do_cipher && (c0 + 64u > c_off) &&
				     (c0 < c_end);
		if (need_ks) {
			uint32_t B[4][4];
#pragma unroll
			for (int m = 0; m < 4; m++)
				ctr_block<NR>(smem, lo, rk, iv,
					      (int32_t)(4 * k) - cw4 + m, B[m]);
#pragma unroll
			for (int jj = 0; jj < 16; jj++) {
				if (SHIFT == 0)
					ksw[jj] = B[jj >> 2][jj & 3];
				else if (jj < SHIFT)
					ksw[jj] = carry[jj + 4 - SHIFT];
				else
					ksw[jj] = B[(jj - SHIFT) >> 2][(jj - SHIFT) & 3];
			}
#pragma unroll
			for (int q = 0; q < 4; q++)
				carry[q] = B[3][q];
		}
		else {
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				ksw[jj] = 0;
		}

		const bool fast = (c0 + 64u <= data_end) &&
				  (!do_cipher || (c0 >= c_off && c0 + 64u <= c_end)) &&
				  (!do_hmac || c0 + 64u <= A);
		uint32_t w[16];
		if (fast) {
			uint32_t o[16];
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				o[jj] = d[jj] ^ ksw[jj];
			if (store_ct) {
#pragma unroll
				for (int g = 0; g < 4; g++)
					*(uint4 *)(pkt + c0 + 16u * g) =
						make_uint4(o[4 * g], o[4 * g + 1],
							   o[4 * g + 2], o[4 * g + 3]);
			}
			/* MAC input is always the ciphertext */
#pragma unroll
			for (int jj = 0; jj < 16; jj++)
				w[jj] = bswap32(PROT ? o[jj] : d[jj]);
		}
		else {
#pragma unroll
			for (int jj = 0; jj < 16; jj++) {
				const uint32_t bpos = c0 + 4u * jj;
				uint32_t o = d[jj];
				if (do_cipher && bpos >= c_off && bpos < c_end) {
					uint32_t nbytes = min(c_end - bpos, 4u);
					uint32_t m = nbytes == 4 ? 0xffffffffu
						   : ((1u << (8 * nbytes)) - 1u);
					o = d[jj] ^ (ksw[jj] & m);
					if (store_ct) {
						if (nbytes == 4)
							*(uint32_t *)(pkt + bpos) = o;
						else
							st_partial(pkt + bpos, o, nbytes);
					}
				}
				w[jj] = msg_word(16u * k + jj,
						 bswap32(PROT ? o : d[jj]), A, X);
			}
			if (k + 1 == nb) {
				w[14] = (uint32_t)(bitlen >> 32);
				w[15] = (uint32_t)bitlen;
			}
		}
		if (do_hmac && k < nb)
			sha1_compress(h, w);
	}

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
		for (uint32_t k = 0; k < nck; k++) {
			const uint32_t c0 = 64u * k;
			if (!(c0 + 64u > c_off && c0 < c_end))
				continue;
			uint32_t B[4][4];
#pragma unroll
			for (int m = 0; m < 4; m++)
				ctr_block<NR>(smem, lo, rk, iv,
					      (int32_t)(4 * k) - cw4 + m, B[m]);
			uint32_t ksw[16];
#pragma unroll
			for (int jj = 0; jj < 16; jj++) {
				if (SHIFT == 0)
					ksw[jj] = B[jj >> 2][jj & 3];
				else if (jj < SHIFT)
					ksw[jj] = carry[jj + 4 - SHIFT];
				else
					ksw[jj] = B[(jj - SHIFT) >> 2][(jj - SHIFT) & 3];
			}
#pragma unroll
			for (int q = 0; q < 4; q++)
				carry[q] = B[3][q];
#pragma unroll
			for (int jj = 0; jj < 16; jj++) {
				const uint32_t bpos = c0 + 4u * jj;
				if (bpos >= c_off && bpos < c_end) {
					uint32_t nbytes = min(c_end - bpos, 4u);
					if (nbytes == 4) {
						uint32_t *p = (uint32_t *)(pkt + bpos);
						*p = *p ^ ksw[jj];
					}
					else {
						uint32_t v = 0;
						for (uint32_t q = 0; q < nbytes; q++)
							v |= (uint32_t)pkt[bpos + q] << (8 * q);
						st_partial(pkt + bpos, v ^ ksw[jj], nbytes);
					}
				}
			}
		}
		vd &= (uint8_t)~SV_CIPHERED;
	}
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
	tt_fill(smem, g_T0);
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

/* ------------------------------------------------------------------ */
/* Session setup: KDF + key schedule + HMAC midstates + GHASH table.   */
/* One thread per (session, comp).  Cold path: byte-oriented AES.      */

__device__ uint8_t d_xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

__device__ void d_aes_expand(const uint8_t *key, uint32_t nk, uint8_t *rkb)
{
	uint32_t nr = nk + 6, i;
	uint8_t rcon = 1;
	for (i = 0; i < 4 * nk; i++)
		rkb[i] = key[i];
	for (i = nk; i < 4 * (nr + 1); i++) {
		uint8_t t[4];
		for (int r = 0; r < 4; r++)
			t[r] = rkb[4 * (i - 1) + r];
		if (i % nk == 0) {
			uint8_t u = t[0];
			t[0] = (uint8_t)(g_sbox[t[1]] ^ rcon);
			t[1] = g_sbox[t[2]];
			t[2] = g_sbox[t[3]];
			t[3] = g_sbox[u];
			rcon = d_xt(rcon);
		}
		else if (nk > 6 && i % nk == 4) {
			for (int r = 0; r < 4; r++)
				t[r] = g_sbox[t[r]];
		}
		for (int r = 0; r < 4; r++)
			rkb[4 * i + r] = (uint8_t)(rkb[4 * (i - nk) + r] ^ t[r]);
	}
}

__device__ void d_aes_block(const uint8_t *rkb, uint32_t nr,
			    const uint8_t in[16], uint8_t out[16])
{
	uint8_t s[16], t[16];
	for (int q = 0; q < 16; q++)
		s[q] = in[q] ^ rkb[q];
	for (uint32_t r = 1; r <= nr; r++) {
		for (int c = 0; c < 4; c++)
			for (int q = 0; q < 4; q++)
				t[4 * c + q] = g_sbox[s[4 * ((c + q) % 4) + q]];
		if (r != nr) {
			for (int c = 0; c < 4; c++) {
				uint8_t a0 = t[4 * c], a1 = t[4 * c + 1];
				uint8_t a2 = t[4 * c + 2], a3 = t[4 * c + 3];
				s[4 * c + 0] = (uint8_t)(d_xt(a0) ^ d_xt(a1) ^ a1 ^ a2 ^ a3);
				s[4 * c + 1] = (uint8_t)(a0 ^ d_xt(a1) ^ d_xt(a2) ^ a2 ^ a3);
				s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ d_xt(a2) ^ d_xt(a3) ^ a3);
				s[4 * c + 3] = (uint8_t)(d_xt(a0) ^ a0 ^ a1 ^ a2 ^ d_xt(a3));
			}
		}
		else {
			for (int q = 0; q < 16; q++)
				s[q] = t[q];
		}
		for (int q = 0; q < 16; q++)
			s[q] ^= rkb[16 * r + q];
	}
	for (int q = 0; q < 16; q++)
		out[q] = s[q];
}

/* srtp_derive (misc.c:44-73): AES-CTR(master, IV = salt‖0 ^ label@7) */
__device__ void d_derive(uint8_t *out, uint32_t out_len, uint8_t label,
			 const uint8_t *mrk, uint32_t mnr, const uint8_t *salt,
			 uint32_t salt_bytes)
{
	uint8_t x[16];
	for (int q = 0; q < 16; q++)
		x[q] = (uint32_t)q < salt_bytes ? salt[q] : 0;
	x[7] ^= label;
	for (uint32_t o = 0; o < out_len; o += 16) {
		uint8_t ks[16];
		d_aes_block(mrk, mnr, x, ks);
		for (uint32_t q = 0; q < 16 && o + q < out_len; q++)
			out[o + q] = ks[q];
		for (int q = 15; q >= 0; q--)
			if (++x[q])
				break;
	}
}

__device__ void d_sha1_block(uint32_t h[5], const uint8_t blk[64])
{
	uint32_t w[16];
	for (int q = 0; q < 16; q++)
		w[q] = (uint32_t)blk[4 * q] << 24 | (uint32_t)blk[4 * q + 1] << 16 |
		       (uint32_t)blk[4 * q + 2] << 8 | blk[4 * q + 3];
	sha1_compress(h, w);
}

__global__ void k_setup(const struct sgpu_keyreq *__restrict__ req,
			const uint32_t *__restrict__ slot, uint32_t n,
			struct sgpu_session *__restrict__ table)
{
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= 2 * n)
		return;
	const uint32_t si = t >> 1, which = t & 1;   /* 0 rtp, 1 rtcp */
	const struct sgpu_keyreq r = req[si];
	struct sgpu_comp *c = &table[slot[si]].comp[which];
	const uint32_t offs = which ? 3u : 0u;       /* srtp.c:164-169 */
	const uint32_t kb = r.cipher_bytes;
	uint8_t mrk[240], k_e[32], k_a[20], k_s[16];

	d_aes_expand(r.master, kb / 4, mrk);
	d_derive(k_e, kb, (uint8_t)(0x00 + offs), mrk, kb / 4 + 6,
		 r.master + kb, r.salt_bytes);
	d_derive(k_a, 20, (uint8_t)(0x01 + offs), mrk, kb / 4 + 6,
		 r.master + kb, r.salt_bytes);
	d_derive(k_s, 14, (uint8_t)(0x02 + offs), mrk, kb / 4 + 6,
		 r.master + kb, r.salt_bytes);
	k_s[14] = k_s[15] = 0;

	const uint32_t nr = kb / 4 + 6;
	const bool enc = which ? (r.rtcp_encrypted != 0) : true;
	const bool has_aes = enc || r.mode == SGPU_MODE_GCM;   /* srtp.c:59 */
	uint8_t rkb[240];
	d_aes_expand(k_e, kb / 4, rkb);
	for (uint32_t q = 0; q < 4 * (nr + 1); q++) {
		uint32_t wv = (uint32_t)rkb[4 * q] | (uint32_t)rkb[4 * q + 1] << 8 |
			      (uint32_t)rkb[4 * q + 2] << 16 |
			      (uint32_t)rkb[4 * q + 3] << 24;
		if (q >= 4 && q < 4 * nr)
			wv = (wv >> 16) | (wv << 16);
		c->rk[q] = wv;
	}
	for (uint32_t q = 4 * (nr + 1); q < 60; q++)
		c->rk[q] = 0;
	c->nr = nr;
	c->mode = r.mode;
	c->tag_len = r.tag_len;
	c->flags = (has_aes ? 1u : 0u) | (r.hash ? 2u : 0u);
	for (int q = 0; q < 4; q++)
		c->k_s[q] = (uint32_t)k_s[4 * q] | (uint32_t)k_s[4 * q + 1] << 8 |
			    (uint32_t)k_s[4 * q + 2] << 16 |
			    (uint32_t)k_s[4 * q + 3] << 24;

	/* HMAC-SHA1 midstates over (k_a ‖ 0^44) ^ ipad/opad (RFC 2104) */
	uint8_t blk[64];
	uint32_t h[5];
	for (int pass = 0; pass < 2; pass++) {
		uint8_t pv = pass ? 0x5c : 0x36;
		for (int q = 0; q < 64; q++)
			blk[q] = (uint8_t)((q < 20 ? k_a[q] : 0) ^ pv);
		h[0] = 0x67452301u; h[1] = 0xefcdab89u; h[2] = 0x98badcfeu;
		h[3] = 0x10325476u; h[4] = 0xc3d2e1f0u;
		d_sha1_block(h, blk);
		for (int q = 0; q < 5; q++) {
			if (pass)
				c->opad[q] = h[q];
			else
				c->ipad[q] = h[q];
		}
	}
	c->pad0[0] = c->pad0[1] = 0;

	/* GHASH H = E(k_e, 0^128); Htable per OpenSSL gcm_init_4bit */
	uint8_t zero[16] = {0}, H[16];
	d_aes_block(rkb, nr, zero, H);
	uint64_t vh = 0, vl = 0;
	for (int q = 0; q < 8; q++) {
		vh = vh << 8 | H[q];
		vl = vl << 8 | H[8 + q];
	}
	uint64_t th[16], tlo[16];
	th[0] = tlo[0] = 0;
	th[8] = vh; tlo[8] = vl;
	for (int s = 4; s >= 1; s >>= 1) {
		uint64_t T = 0xe100000000000000ull & (0ull - (vl & 1));
		vl = (vh << 63) | (vl >> 1);
		vh = (vh >> 1) ^ T;
		th[s] = vh; tlo[s] = vl;
	}
	for (int q = 1; q < 16; q++) {
		if (q == 1 || q == 2 || q == 4 || q == 8)
			continue;
		uint64_t a = 0, b = 0;
		for (int bit = 1; bit < 16; bit <<= 1)
			if (q & bit) {
				a ^= th[bit];
				b ^= tlo[bit];
			}
		th[q] = a; tlo[q] = b;
	}
	for (int q = 0; q < 16; q++) {
		c->htab[q][0] = (uint32_t)(th[q] >> 32);
		c->htab[q][1] = (uint32_t)th[q];
		c->htab[q][2] = (uint32_t)(tlo[q] >> 32);
		c->htab[q][3] = (uint32_t)tlo[q];
	}
}

/* ------------------------------------------------------------------ */
/* rtp_hdr_decode (src/rtp/rtp.c:88-137), including the position at
 * which each EBADMSG is raised.  get_rtcp_ssrc (srtcp.c:19-28).        */

__global__ void k_parse(const uint8_t *__restrict__ arena,
			const uint32_t *__restrict__ pos,
			const uint32_t *__restrict__ end,
			struct sgpu_hdr *__restrict__ out,
			uint32_t *__restrict__ eix, uint32_t n, int rtcp)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t p = pos[i], e = end[i];
	const uint32_t left = e > p ? e - p : 0;
	const uint8_t *b = arena + p;
	struct sgpu_hdr h;
	h.ssrc = 0; h.seq = 0; h.err_pos = 0; h.hdr_len = 0xffffffffu;
	if (rtcp) {
		if (left >= 8) {
			h.ssrc = (uint32_t)b[4] << 24 | (uint32_t)b[5] << 16 |
				 (uint32_t)b[6] << 8 | b[7];
			h.hdr_len = 8;
		}
		if (eix) {
			const uint32_t tl[3] = {0, 4, 10};
			for (int k = 0; k < 3; k++) {
				uint32_t v = 0;
				if (left >= 12 + tl[k]) {
					const uint8_t *q = arena + e - 4 - tl[k];
					v = (uint32_t)q[0] << 24 |
					    (uint32_t)q[1] << 16 |
					    (uint32_t)q[2] << 8 | q[3];
				}
				eix[3 * i + k] = v;
			}
		}
		out[i] = h;
		return;
	}
	if (left < 12) {
		out[i] = h;
		return;
	}
	const uint32_t cc = b[0] & 0x0fu, x = (b[0] >> 4) & 1u;
	h.seq = (uint16_t)(b[2] << 8 | b[3]);
	h.ssrc = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 |
		 (uint32_t)b[10] << 8 | b[11];
	uint32_t hl = 12;
	if (left - hl < 4 * cc) {
		h.err_pos = (uint16_t)hl;
		out[i] = h;
		return;
	}
	hl += 4 * cc;
	if (x) {
		if (left - hl < 4) {
			h.err_pos = (uint16_t)hl;
			out[i] = h;
			return;
		}
		const uint32_t xl = (uint32_t)b[hl + 2] << 8 | b[hl + 3];
		hl += 4;
		if (left - hl < 4 * xl) {
			h.err_pos = (uint16_t)hl;
			out[i] = h;
			return;
		}
		hl += 4 * xl;
	}
	h.hdr_len = hl;
	out[i] = h;
}

/* ------------------------------------------------------------------ */
/* Device-side planning of a single-stream RTP batch (srtpgpu.h).      */

#define PLAN_BLOCK 256

/* sgpu_desc() (srtpgpu.h) on the device */
__device__ __forceinline__ uint64_t d_desc(uint64_t ix, uint32_t flags)
{
	return (ix & 0xffffull) | ((uint64_t)(uint32_t)(ix >> 16) << 16) |
	       ((uint64_t)flags << 48);
}

/* srtp_get_index (misc.c:22-41), including the int wrap of roc +- 1 */
__device__ __forceinline__ int32_t plan_v(uint32_t roc, uint32_t s_l,
					  uint32_t seq)
{
	if (s_l < 32768)
		return ((int)seq - (int)s_l > 32768) ? (int32_t)(roc - 1)
						     : (int32_t)roc;
	return ((int)s_l - 32768 > (int)seq) ? (int32_t)(roc + 1)
					     : (int32_t)roc;
}

/* speculated s_l seen by packet i: the previous packet's seq */
__device__ __forceinline__ uint32_t plan_sb(const struct sgpu_plan_in &in,
					    const struct sgpu_hdr *hdr,
					    uint32_t i)
{
	if (i == 0)
		return in.fresh ? hdr[0].seq : in.s_l;
	return hdr[i - 1].seq;
}

/* ROC rollover seen by a packet (srtp.c:208-213, 318-321) */
__device__ __forceinline__ bool plan_wrap(uint32_t seq, uint32_t sb)
{
	return (int)seq - (int)sb <= -32768;
}

__global__ void __launch_bounds__(PLAN_BLOCK)
k_plan_count(const struct sgpu_plan_in in, const struct sgpu_hdr *hdr,
	     const uint32_t *pos, const uint32_t *end, uint32_t *bcnt,
	     struct sgpu_plan_out *out)
{
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	bool wrap = false;
	uint32_t f = 0;
	if (i < in.n) {
		const struct sgpu_hdr h = hdr[i];
		const uint32_t hl0 = hdr[0].hdr_len;
		const uint32_t ssrc0 = in.ssrc_any ? hdr[0].ssrc : in.ssrc;
		const uint32_t seq = h.seq, sb = plan_sb(in, hdr, i);
		if (h.hdr_len == 0xffffffffu || hl0 == 0xffffffffu)
			f |= SPF_PARSE;
		else if (((h.hdr_len ^ hl0) >> 2) & 3u)
			f |= SPF_CLASS;
		if (h.ssrc != ssrc0)
			f |= SPF_SSRC;
		if (!in.prot && h.hdr_len != 0xffffffffu &&
		    end[i] - pos[i] - h.hdr_len < in.tag)
			f |= SPF_PARSE;
		if (!in.prot && (int)seq - (int)sb > 32768)
			f |= SPF_TIMEOUT;
		wrap = plan_wrap(seq, sb);
		/* the next packet sees s_l = seq only if this one left it so */
		if (i + 1 < in.n && !wrap && seq < sb)
			f |= SPF_ORDER;
		if (i == 0) {
			out->ssrc0 = h.ssrc;
			out->hl0 = h.hdr_len;
		}
		if (f)
			atomicOr(&out->fail, f);
	}
	const int c = __syncthreads_count(wrap);
	if (threadIdx.x == 0)
		bcnt[blockIdx.x] = (uint32_t)c;
}

/* exclusive scan of the per-block wrap counts (one workgroup) */
__global__ void __launch_bounds__(1024)
k_plan_scan(uint32_t *bcnt, uint32_t nb, struct sgpu_plan_out *out)
{
	__shared__ uint32_t part[1024];
	const uint32_t per = (nb + 1023u) / 1024u;
	const uint32_t a = threadIdx.x * per;
	uint32_t sum = 0;
	for (uint32_t k = a; k < a + per && k < nb; k++)
		sum += bcnt[k];
	part[threadIdx.x] = sum;
	__syncthreads();
	for (uint32_t d = 1; d < 1024; d <<= 1) {
		uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
		__syncthreads();
		part[threadIdx.x] += v;
		__syncthreads();
	}
	uint32_t run = part[threadIdx.x] - sum;
	for (uint32_t k = a; k < a + per && k < nb; k++) {
		const uint32_t v = bcnt[k];
		bcnt[k] = run;
		run += v;
	}
	if (threadIdx.x == 1023)
		out->wraps = part[1023];
}

__global__ void __launch_bounds__(PLAN_BLOCK)
k_plan_desc(const struct sgpu_plan_in in, const struct sgpu_hdr *hdr,
	    const uint32_t *bpre, uint64_t *desc, struct sgpu_plan_out *out)
{
	__shared__ uint32_t wsum[PLAN_BLOCK / 64];
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	uint32_t seq = 0, sb = 0;
	bool wrap = false;
	if (i < in.n) {
		seq = hdr[i].seq;
		sb = plan_sb(in, hdr, i);
		wrap = plan_wrap(seq, sb);
	}
	const uint64_t m = __ballot(wrap);
	if (lane == 0)
		wsum[wv] = (uint32_t)__popcll(m);
	__syncthreads();
	uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
	for (uint32_t k = 0; k < wv; k++)
		pre += wsum[k];
	if (i >= in.n)
		return;
	/* ROC after this packet's own rollover */
	const uint32_t roc = in.roc + bpre[blockIdx.x] + pre + (wrap ? 1u : 0u);
	uint64_t ix;
	uint32_t fl = SD_RUN | SD_CIPHER;
	if (in.prot) {
		ix = 65536ull * roc + seq;              /* srtp.c:215 */
	}
	else {
		const int32_t v = plan_v(roc, wrap ? 0u : sb, seq);
		ix = seq + (uint64_t)(int64_t)v * 65536ull;
		if ((uint32_t)v != roc)
			fl |= (uint32_t)v + 1u == roc ? SD_ROC_P1 : SD_ROC_M1;
		/* replay: every packet must be new (replay.c:32-62) */
		bool ok;
		if (i == 0) {
			if (ix > in.lix)
				ok = true;
			else {
				const uint64_t d = in.lix - ix;
				ok = d < 64 && !(in.bitmap & (1ull << d));
			}
		}
		else {
			const uint32_t pseq = hdr[i - 1].seq;
			const uint32_t psb = plan_sb(in, hdr, i - 1);
			const bool pw = plan_wrap(pseq, psb);
			const uint32_t proc = roc - (wrap ? 1u : 0u);
			const int32_t pv = plan_v(proc, pw ? 0u : psb, pseq);
			const uint64_t pix = pseq +
					     (uint64_t)(int64_t)pv * 65536ull;
			ok = ix > pix;
		}
		if (!ok)
			atomicOr(&out->fail, (uint32_t)SPF_REPLAY);
	}
	desc[i] = d_desc(ix, fl);
	const uint32_t t0 = in.n > SGPU_PLAN_TAIL ? in.n - SGPU_PLAN_TAIL : 0u;
	if (i >= t0)
		out->tail_ix[i - t0] = ix;
	if (i + 1 == in.n)
		out->s_l_last = wrap ? seq : (seq > sb ? seq : sb);
}

/* ================================================================== */
/* C-ABI shim                                                          */

static char g_err[256];
static int g_inited;
static struct sgpu_session *g_table;
static uint32_t g_table_cap;
static struct sgpu_keyreq *g_req_dev;
static uint32_t *g_slot_dev;
static uint32_t g_req_cap;

static int herr(hipError_t e, const char *what)
{
	if (e == hipSuccess)
		return 0;
	snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
	return EIO;
}

extern "C" const char *sgpu_last_error(void) { return g_err; }

static uint8_t h_xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

extern "C" int sgpu_init(void)
{
	int n = 0;
	if (g_inited)
		return 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
		snprintf(g_err, sizeof(g_err), "no HIP device visible");
		return ENODEV;
	}
	/* S-box (FIPS-197 5.1.1) and T0 on the host, uploaded once */
	uint8_t sbox[256];
	uint32_t T0[256];
	for (int x = 0; x < 256; x++) {
		uint8_t inv = 0;
		for (int y = 1; x && y < 256; y++) {
			uint8_t a = (uint8_t)x, b = (uint8_t)y, r = 0;
			while (b) {
				if (b & 1)
					r ^= a;
				a = h_xt(a);
				b >>= 1;
			}
			if (r == 1) {
				inv = (uint8_t)y;
				break;
			}
		}
		uint8_t s = inv;
		s = (uint8_t)(inv ^ (uint8_t)((inv << 1) | (inv >> 7)) ^
			      (uint8_t)((inv << 2) | (inv >> 6)) ^
			      (uint8_t)((inv << 3) | (inv >> 5)) ^
			      (uint8_t)((inv << 4) | (inv >> 4)) ^ 0x63);
		sbox[x] = s;
	}
	for (int x = 0; x < 256; x++) {
		uint8_t s = sbox[x], s2 = h_xt(s), s3 = (uint8_t)(s2 ^ s);
		T0[x] = (uint32_t)s2 | (uint32_t)s << 8 | (uint32_t)s << 16 |
			(uint32_t)s3 << 24;
	}
	int e = herr(hipMemcpyToSymbol(HIP_SYMBOL(g_sbox), sbox, 256), "sbox");
	if (!e)
		e = herr(hipMemcpyToSymbol(HIP_SYMBOL(g_T0), T0, 1024), "T0");
	if (e)
		return e;
	g_inited = 1;
	return 0;
}

extern "C" int sgpu_table_reserve(uint32_t nsessions)
{
	if (nsessions <= g_table_cap)
		return 0;
	uint32_t cap = g_table_cap ? g_table_cap : 1024;
	while (cap < nsessions)
		cap *= 2;
	struct sgpu_session *nt = NULL;
	int e = herr(hipMalloc(&nt, (size_t)cap * sizeof(*nt)), "table alloc");
	if (e)
		return e;
	if (g_table) {
		e = herr(hipMemcpy(nt, g_table,
				   (size_t)g_table_cap * sizeof(*nt),
				   hipMemcpyDeviceToDevice), "table grow");
		(void)hipDeviceSynchronize();
		(void)hipFree(g_table);
	}
	g_table = nt;
	g_table_cap = cap;
	return e;
}

extern "C" uint64_t sgpu_table_device_ptr(void) { return (uint64_t)(uintptr_t)g_table; }

extern "C" int sgpu_setup_sessions(const struct sgpu_keyreq *req,
				   const uint32_t *slot, uint32_t n)
{
	int e;
	if (!n)
		return 0;
	if (n > g_req_cap) {
		if (g_req_dev) {
			(void)hipFree(g_req_dev);
			(void)hipFree(g_slot_dev);
		}
		g_req_cap = n < 256 ? 256 : n;
		e = herr(hipMalloc(&g_req_dev, g_req_cap * sizeof(*req)), "req");
		if (!e)
			e = herr(hipMalloc(&g_slot_dev, g_req_cap * 4u), "slot");
		if (e)
			return e;
	}
	e = herr(hipMemcpy(g_req_dev, req, n * sizeof(*req),
			   hipMemcpyHostToDevice), "req h2d");
	if (!e)
		e = herr(hipMemcpy(g_slot_dev, slot, n * 4u,
				   hipMemcpyHostToDevice), "slot h2d");
	if (e)
		return e;
	const uint32_t thr = 64, nthreads = 2 * n;
	hipLaunchKernelGGL(k_setup, dim3((nthreads + thr - 1) / thr), dim3(thr),
			   0, 0, g_req_dev, g_slot_dev, n, g_table);
	e = herr(hipGetLastError(), "k_setup launch");
	if (!e)
		e = herr(hipDeviceSynchronize(), "k_setup");
	return e;
}

/* ---- kernel timing with HIP events on the launch stream (bench.py) ---- */
#include <pthread.h>
static pthread_mutex_t g_prof_lock = PTHREAD_MUTEX_INITIALIZER;
static int g_prof_on;
struct prof_ev { hipEvent_t a, b; int slot; uint32_t jobs; };
static struct prof_ev *g_pev;
static size_t g_npev, g_pev_cap;
static double g_prof_ms[32];
static uint64_t g_prof_launch[32], g_prof_jobs[32];

extern "C" void sgpu_prof_enable(int on)
{
	pthread_mutex_lock(&g_prof_lock);
	g_prof_on = on;
	pthread_mutex_unlock(&g_prof_lock);
}

static void prof_drain_locked(void)
{
	for (size_t k = 0; k < g_npev; k++) {
		float ms = 0;
		(void)hipEventSynchronize(g_pev[k].b);
		(void)hipEventElapsedTime(&ms, g_pev[k].a, g_pev[k].b);
		g_prof_ms[g_pev[k].slot] += ms;
		g_prof_launch[g_pev[k].slot]++;
		g_prof_jobs[g_pev[k].slot] += g_pev[k].jobs;
		(void)hipEventDestroy(g_pev[k].a);
		(void)hipEventDestroy(g_pev[k].b);
	}
	g_npev = 0;
}

/* slot = prot*16 + mode*8 + (nr==14)*4 + shift; reading resets */
extern "C" void sgpu_prof_read(double *ms, uint64_t *launches, uint64_t *jobs)
{
	pthread_mutex_lock(&g_prof_lock);
	prof_drain_locked();
	for (int k = 0; k < 32; k++) {
		if (ms) ms[k] = g_prof_ms[k];
		if (launches) launches[k] = g_prof_launch[k];
		if (jobs) jobs[k] = g_prof_jobs[k];
		g_prof_ms[k] = 0;
		g_prof_launch[k] = g_prof_jobs[k] = 0;
	}
	pthread_mutex_unlock(&g_prof_lock);
}

typedef void (*kfn_t)(const KArgs);

template <bool COMPACT>
static kfn_t pick_ctr(int nr, int shift, int prot)
{
#define PICK(NR, S)                                                            \
	if (nr == NR && shift == S)                                            \
		return prot ? k_ctr_hmac<NR, S, true, COMPACT>                 \
			    : k_ctr_hmac<NR, S, false, COMPACT>;
	PICK(10, 0) PICK(10, 1) PICK(10, 2) PICK(10, 3)
	PICK(14, 0) PICK(14, 1) PICK(14, 2) PICK(14, 3)
#undef PICK
	return NULL;
}

template <bool COMPACT>
static kfn_t pick_gcm(int nr, int prot)
{
	if (nr == 10)
		return prot ? k_gcm<10, true, COMPACT> : k_gcm<10, false, COMPACT>;
	if (nr == 14)
		return prot ? k_gcm<14, true, COMPACT> : k_gcm<14, false, COMPACT>;
	return NULL;
}

static int launch(kfn_t f, const KArgs &a, uint32_t n, int slot,
		  hipStream_t stream)
{
	struct prof_ev pe;
	int prof = 0;
	if (g_prof_on && slot >= 0) {
		prof = hipEventCreate(&pe.a) == hipSuccess &&
		       hipEventCreate(&pe.b) == hipSuccess;
		if (prof)
			(void)hipEventRecord(pe.a, stream);
	}
	hipLaunchKernelGGL(f, dim3((n + KBLOCK - 1) / KBLOCK), dim3(KBLOCK), 0,
			   stream, a);
	int e = herr(hipGetLastError(), "kernel launch");
	if (prof) {
		(void)hipEventRecord(pe.b, stream);
		pe.slot = slot;
		pe.jobs = n;
		pthread_mutex_lock(&g_prof_lock);
		if (g_npev == g_pev_cap) {
			size_t nc = g_pev_cap ? 2 * g_pev_cap : 64;
			struct prof_ev *np = (struct prof_ev *)realloc(
				g_pev, nc * sizeof(*np));
			if (np) {
				g_pev = np;
				g_pev_cap = nc;
			}
		}
		if (g_npev < g_pev_cap)
			g_pev[g_npev++] = pe;
		pthread_mutex_unlock(&g_prof_lock);
	}
	return e;
}

static int prof_slot(int mode, int nr, int shift, int prot)
{
	return (prot ? 16 : 0) + (mode ? 8 : 0) + (nr == 14 ? 4 : 0) +
	       (mode ? 0 : shift);
}

/*
 * Launch one kernel over jobs[0..njobs).  The caller (host C) groups jobs
 * so that one launch shares (mode, key size, shift class, direction).
 */
extern "C" int sgpu_run_class(uint8_t *arena, uint64_t arena_size,
			      const struct sgpu_job *jobs, uint32_t njobs,
			      uint8_t *verdict, uint32_t *save, int mode,
			      int nr, int shift, int prot, void *stream)
{
	if (!njobs)
		return 0;
	kfn_t f = mode == SGPU_MODE_GCM ? pick_gcm<false>(nr, prot)
					: pick_ctr<false>(nr, shift, prot);
	if (!f) {
		snprintf(g_err, sizeof(g_err), "no kernel for mode %d nr %d",
			 mode, nr);
		return EINVAL;
	}
	KArgs a;
	memset(&a, 0, sizeof(a));
	a.arena = arena;
	a.asz = arena_size;
	a.jobs = jobs;
	a.njobs = njobs;
	a.comps = (const struct sgpu_comp *)g_table;
	a.verdict = verdict;
	a.save = save;
	return launch(f, a, njobs, prof_slot(mode, nr, shift, prot),
		      (hipStream_t)stream);
}

extern "C" int sgpu_run_compact(uint8_t *arena, uint64_t arena_size,
				const struct sgpu_compact *c, int mode, int nr,
				int shift, int prot, void *stream)
{
	if (!c->n)
		return 0;
	kfn_t f = mode == SGPU_MODE_GCM ? pick_gcm<true>(nr, prot)
					: pick_ctr<true>(nr, shift, prot);
	if (!f) {
		snprintf(g_err, sizeof(g_err), "no kernel for mode %d nr %d",
			 mode, nr);
		return EINVAL;
	}
	KArgs a;
	memset(&a, 0, sizeof(a));
	a.arena = arena;
	a.asz = arena_size;
	a.comps = (const struct sgpu_comp *)g_table;
	a.verdict = c->verdict;
	a.save = c->save;
	a.c = *c;
	return launch(f, a, c->n,
		      c->undo ? -1 : prof_slot(mode, nr, shift, prot),
		      (hipStream_t)stream);
}

extern "C" int sgpu_parse_headers(const uint8_t *arena, const uint32_t *pos,
				  const uint32_t *end, struct sgpu_hdr *out,
				  uint32_t *eix, uint32_t n, int rtcp,
				  void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_parse, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, arena, pos, end, out, eix, n,
			   rtcp);
	return herr(hipGetLastError(), "k_parse launch");
}

__global__ void k_store_words(uint8_t *__restrict__ arena,
			      const uint32_t *__restrict__ offs,
			      const uint32_t *__restrict__ vals, uint32_t n)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	uint8_t *p = arena + offs[i];
	const uint32_t v = vals[i];
	p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8);
	p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

extern "C" int sgpu_store_words(uint8_t *arena, const uint32_t *offs,
				const uint32_t *vals, uint32_t n, void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_store_words, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, arena, offs, vals, n);
	return herr(hipGetLastError(), "k_store_words launch");
}

extern "C" void *sgpu_malloc(size_t n)
{
	void *p = NULL;
	if (herr(hipMalloc(&p, n ? n : 1), "hipMalloc"))
		return NULL;
	return p;
}

extern "C" void sgpu_free(void *p) { if (p) (void)hipFree(p); }

extern "C" void *sgpu_host_alloc(size_t n)
{
	void *p = NULL;
	if (herr(hipHostMalloc(&p, n ? n : 1, hipHostMallocDefault),
		 "hipHostMalloc"))
		return NULL;
	return p;
}

extern "C" void sgpu_host_free(void *p) { if (p) (void)hipHostFree(p); }

extern "C" int sgpu_memcpy_h2d(void *dst, const void *src, size_t n,
			       void *stream)
{
	if (!n)
		return 0;
	return herr(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice,
				   (hipStream_t)stream), "h2d");
}

extern "C" int sgpu_memcpy_d2h(void *dst, const void *src, size_t n,
			       void *stream)
{
	if (!n)
		return 0;
	return herr(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost,
				   (hipStream_t)stream), "d2h");
}

extern "C" int sgpu_memset(void *dst, int v, size_t n, void *stream)
{
	return herr(hipMemsetAsync(dst, v, n, (hipStream_t)stream), "memset");
}

extern "C" int sgpu_stream_sync(void *stream)
{
	return herr(hipStreamSynchronize((hipStream_t)stream), "stream sync");
}

extern "C" int sgpu_device_sync(void)
{
	return herr(hipDeviceSynchronize(), "device sync");
}

extern "C" void *sgpu_stream_create(void)
{
	hipStream_t s = NULL;
	if (herr(hipStreamCreateWithFlags(&s, hipStreamNonBlocking),
		 "stream create"))
		return NULL;
	return (void *)s;
}

extern "C" void sgpu_stream_destroy(void *s)
{
	if (s)
		(void)hipStreamDestroy((hipStream_t)s);
}

extern "C" int sgpu_set_device(int dev)
{
	return herr(hipSetDevice(dev), "hipSetDevice");
}

extern "C" int sgpu_get_device(void)
{
	int d = -1;
	(void)hipGetDevice(&d);
	return d;
}

extern "C" void *sgpu_event_create(void)
{
	hipEvent_t e = NULL;
	if (herr(hipEventCreateWithFlags(&e, hipEventDisableTiming),
		 "event create"))
		return NULL;
	return (void *)e;
}

extern "C" void sgpu_event_destroy(void *ev)
{
	if (ev)
		(void)hipEventDestroy((hipEvent_t)ev);
}

extern "C" int sgpu_event_record(void *ev, void *stream)
{
	return herr(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream),
		    "event record");
}

extern "C" int sgpu_event_sync(void *ev)
{
	return herr(hipEventSynchronize((hipEvent_t)ev), "event sync");
}

extern "C" int sgpu_stream_wait(void *stream, void *ev)
{
	return herr(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0),
		    "stream wait");
}

extern "C" int sgpu_plan_rtp(const struct sgpu_plan_in *in,
			     const struct sgpu_hdr *hdr, const uint32_t *pos,
			     const uint32_t *end, uint64_t *desc,
			     uint32_t *scratch, struct sgpu_plan_out *out,
			     void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t nb = (in->n + PLAN_BLOCK - 1) / PLAN_BLOCK;
	if (!in->n)
		return EINVAL;
	int e = herr(hipMemsetAsync(out, 0, sizeof(*out), st), "plan memset");
	if (e)
		return e;
	hipLaunchKernelGGL(k_plan_count, dim3(nb), dim3(PLAN_BLOCK), 0, st,
			   *in, hdr, pos, end, scratch, out);
	hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, st, scratch,
			   nb, out);
	hipLaunchKernelGGL(k_plan_desc, dim3(nb), dim3(PLAN_BLOCK), 0, st,
			   *in, hdr, (const uint32_t *)scratch, desc, out);
	return herr(hipGetLastError(), "plan launch");
}
