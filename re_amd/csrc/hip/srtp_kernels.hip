/*
 * srtp_kernels.hip -- MI355X (gfx950) session setup, header parse and
 * device planner kernels, plus the thin C-ABI shim declared in ../srtpgpu.h.
 * The crypto kernels live in ctr10.hip, ctr14.hip and gcm.hip.
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
#include <stddef.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include "../srtpgpu.h"
#include "kern_common.h"
#include "plan_common.h"
#include "k_ctr_fused.h"

#ifndef EAUTH
#define EAUTH 217               /* include/re_types.h:215-217 */
#endif


__device__ uint32_t g_T0[256];          /* T0 table (source of LDS image) */
__device__ uint8_t g_sbox[256];

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

/*
 * k_parse for an RTP batch of a device planner, with the planner's
 * per-packet window checks (k_plan_count / k_mp_count) made here, where
 * pos / end / cap are read coalesced: the OR of a 256-packet block goes
 * to wchk[block] (plain stores, read by the planner's scan -- no zeroed
 * word needed).  Block size 256 (= the planners' blocks).
 */
__device__ __forceinline__ void k_parse_rtp_checked(
	const uint8_t *__restrict__ arena, uint64_t asz,
	const uint32_t *__restrict__ pos, const uint32_t *__restrict__ end,
	struct sgpu_hdr *__restrict__ out, uint32_t n,
	const struct sgpu_prologue &pro)
{
	__shared__ uint32_t bf;
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (threadIdx.x == 0)
		bf = 0;
	__syncthreads();
	if (i < n) {
		const uint32_t p = pos[i], e = end[i];
		if (pro.end_copy)
			pro.end_copy[i] = e;
		const uint32_t left = (e > p && e <= asz) ? e - p : 0;
		const struct sgpu_hdr h = parse_rtp_hdr(arena + p, p, left);
		out[i] = h;
		uint32_t f = 0;
		if (h.hdr_len == 0xffffffffu)
			f |= SPF_PARSE;
		else if (!pro.prot && e - p - h.hdr_len < pro.tag)
			f |= SPF_PARSE;
		if (e - p >= pro.maxlen)
			f |= SPF_SIZE;
		const uint32_t c = pro.cap ? pro.cap[i] : 0u;
		if ((p & 3u) || p > e || e > asz ||
		    (pro.cap && (e > c || c > asz)))
			f |= SPF_BAD;
		if (pro.prot && pro.cap &&
		    (uint64_t)e + pro.need > (uint64_t)c)
			f |= SPF_CAP;
		if (f)
			atomicOr(&bf, f);
	}
	__syncthreads();
	if (threadIdx.x == 0)
		pro.wchk[blockIdx.x] = bf;
}

__global__ void k_parse(const uint8_t *__restrict__ arena, uint64_t asz,
			const uint32_t *__restrict__ pos,
			const uint32_t *__restrict__ end,
			struct sgpu_hdr *__restrict__ out,
			uint32_t *__restrict__ eix, uint32_t n, int rtcp,
			struct sgpu_prologue pro)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (blockIdx.x == 0) {
		/* the batch prologue folded into the parse launch */
		for (uint32_t k = threadIdx.x; k < pro.nz0; k += blockDim.x)
			pro.z0[k] = 0;
		for (uint32_t k = threadIdx.x; k < pro.nz1; k += blockDim.x)
			pro.z1[k] = 0;
		if (pro.cm_out && threadIdx.x == 0)
			*pro.cm_out = pro.cm;
	}
	for (uint32_t k = i; k < pro.nz2; k += gridDim.x * blockDim.x)
		pro.z2[k] = 0;
	if (pro.wchk) {
		k_parse_rtp_checked(arena, asz, pos, end, out, n, pro);
		return;
	}
	if (i >= n)
		return;
	const uint32_t p = pos[i], e = end[i];
	if (pro.end_copy)
		pro.end_copy[i] = e;
	/* a window outside the arena is never read (the planner rejects it) */
	const uint32_t left = (e > p && e <= asz) ? e - p : 0;
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
	uint32_t b0;
	if (!(p & 3u)) {
		/* the batch APIs' 4-byte aligned windows: two dword loads
		 * (words 0 and 2 of the header) instead of seven byte loads */
		const uint32_t w0 = *(const uint32_t *)b;
		const uint32_t w2 = *(const uint32_t *)(b + 8);
		b0 = w0 & 0xffu;
		h.seq = (uint16_t)((w0 >> 8 & 0xff00u) | (w0 >> 24));
		h.ssrc = __builtin_bswap32(w2);
	}
	else {
		b0 = b[0];
		h.seq = (uint16_t)(b[2] << 8 | b[3]);
		h.ssrc = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 |
			 (uint32_t)b[10] << 8 | b[11];
	}
	const uint32_t cc = b0 & 0x0fu, x = (b0 >> 4) & 1u;
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

/* speculated s_l seen by packet i: the previous packet's seq */
__device__ __forceinline__ uint32_t plan_sb(const struct sgpu_plan_in &in,
					    const struct sgpu_hdr *hdr,
					    uint32_t i)
{
	if (i == 0)
		return in.fresh ? hdr[0].seq : in.s_l;
	return hdr[i - 1].seq;
}

__global__ void __launch_bounds__(PLAN_BLOCK)
k_plan_count(const struct sgpu_plan_in in, const struct sgpu_hdr *hdr,
	     const uint32_t *pos, const uint32_t *end, const uint32_t *cap,
	     uint64_t asz, uint32_t *bcnt, struct sgpu_plan_out *out)
{
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	bool wrap = false;
	uint32_t f = 0;
	if (i == 0 && in.pred && *in.pred)     /* sgpu_gate_pred */
		atomicOr(&out->fail, (uint32_t)SPF_PRED);
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
		if (end[i] - pos[i] >= in.maxlen)
			f |= SPF_SIZE;
		if ((pos[i] & 3u) || pos[i] > end[i] || end[i] > asz ||
		    (cap && (end[i] > cap[i] || cap[i] > asz)))
			f |= SPF_BAD;
		if (in.prot && cap &&
		    (uint64_t)end[i] + in.need > (uint64_t)cap[i])
			f |= SPF_CAP;
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
			/* above the pre-batch window too: a packet 0 below
			 * lix leaves the window's bits in play (replay.c:53-61)
			 * and the tail-based final window (plan_replay) holds
			 * only for indices above it */
			ok = ix > pix && ix > in.lix;
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

/* ------------------------------------------------------------------ */
/* Device-side planning of a single-stream SRTCP batch (srtpgpu.h).    */

__device__ __forceinline__ uint32_t rplan_eix(const struct sgpu_rplan_in &in,
					      const uint32_t *eix, uint32_t i)
{
	/* the E || index word at end - 4 - tag (k_parse, tl = 0, 4, 10) */
	return eix[3 * i + (in.tag == 0 ? 0 : in.tag == 4 ? 1 : 2)];
}

__global__ void __launch_bounds__(PLAN_BLOCK)
k_plan_rtcp(const struct sgpu_rplan_in in, const struct sgpu_hdr *hdr,
	    const uint32_t *eix, const uint32_t *pos, const uint32_t *end,
	    const uint32_t *cap, uint64_t asz, uint64_t *desc,
	    struct sgpu_plan_out *out)
{
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	if (i >= in.n)
		return;
	const struct sgpu_hdr h = hdr[i];
	const uint32_t ssrc0 = in.ssrc_any ? hdr[0].ssrc : in.ssrc;
	const uint32_t L = end[i] - pos[i];
	uint32_t f = 0;
	if (h.hdr_len == 0xffffffffu)
		f |= SPF_PARSE;                 /* < 8 bytes: EBADMSG */
	else if (h.ssrc != ssrc0)
		f |= SPF_SSRC;
	if ((pos[i] & 3u) || pos[i] > end[i] || end[i] > asz ||
	    (cap && (end[i] > cap[i] || cap[i] > asz)))
		f |= SPF_BAD;
	if (L >= in.maxlen)
		f |= SPF_SIZE;
	uint32_t ix, E;
	if (in.prot) {
		if (cap && (uint64_t)end[i] + in.need > (uint64_t)cap[i])
			f |= SPF_CAP;           /* ENOMEM (cap_short) */
		ix = (in.rtcp_index + i + 1u) & 0x7fffffffu;    /* srtcp.c:54 */
		E = in.encrypted;
	}
	else {
		/* srtcp.c:166-172 (and 239-241 for GCM): room for E || index,
		 * the tag, and the GCM tag before them */
		if (L < 8u + 4u + in.tag + (in.gcm ? 16u : 0u))
			f |= SPF_PARSE;
		const uint32_t v = rplan_eix(in, eix, i);
		ix = v & 0x7fffffffu;
		E = v >> 31;
		if (in.hmac) {
			/* replay (srtcp.c:208-209), speculated: every index new
			 * and increasing */
			bool ok;
			if (i == 0) {
				if (ix > in.lix) {
					ok = true;
				}
				else {
					const uint64_t dl = in.lix - ix;
					ok = dl < 64 && !(in.bitmap & (1ull << dl));
				}
			}
			else {
				ok = ix > (rplan_eix(in, eix, i - 1) & 0x7fffffffu);
			}
			if (!ok)
				f |= SPF_REPLAY;
		}
	}
	desc[i] = ((uint64_t)(ix & 0x7fffffffu)) | ((uint64_t)E << 31) |
		  ((uint64_t)SD_RUN << 48);
	const uint32_t t0 = in.n > SGPU_PLAN_TAIL ? in.n - SGPU_PLAN_TAIL : 0u;
	if (i >= t0)
		out->tail_ix[i - t0] = ix;
	if (i == 0) {
		out->ssrc0 = h.ssrc;
		out->hl0 = 8;
	}
	if (f)
		atomicOr(&out->fail, f);
}

extern "C" int sgpu_plan_rtcp(const struct sgpu_rplan_in *in,
			      const struct sgpu_hdr *hdr, const uint32_t *eix,
			      const uint32_t *pos, const uint32_t *end,
			      const uint32_t *cap, uint64_t arena_size,
			      uint64_t *desc, struct sgpu_plan_out *out,
			      void *stream);

/* the E || index word of SRTCP packet i (k_parse's eix word for the
 * stream's tag length) */
__device__ __forceinline__ uint32_t rp_word(const uint8_t *arena, uint64_t asz,
					    uint32_t p, uint32_t e,
					    uint32_t tag)
{
	const uint32_t left = (e > p && e <= asz) ? e - p : 0u;
	if (left < 12u + tag)
		return 0;
	const uint8_t *q = arena + e - 4u - tag;
	return (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 |
	       (uint32_t)q[2] << 8 | q[3];
}

/* k_parse (SRTCP form) + k_plan_rtcp in one launch (srtpgpu.h struct
 * sgpu_rfused; srtcp.c:31-140, 143-287) */
__global__ void __launch_bounds__(PLAN_BLOCK)
k_rp_plan(const uint8_t *__restrict__ arena, uint64_t asz,
	  const struct sgpu_rfused R)
{
	__shared__ uint32_t ssrc0s, vw[PLAN_BLOCK + 1];
	const struct sgpu_rplan_in &in = R.in;
	const uint32_t tid = threadIdx.x;
	const uint32_t i = blockIdx.x * PLAN_BLOCK + tid;
	if (tid == 0) {
		/* packet 0's SSRC (get_rtcp_ssrc, srtcp.c:19-29) */
		const uint32_t q = R.pos[0], qe = R.end[0];
		const uint32_t left = (qe > q && qe <= asz) ? qe - q : 0u;
		ssrc0s = left >= 8 ? (uint32_t)arena[q + 4] << 24 |
				     (uint32_t)arena[q + 5] << 16 |
				     (uint32_t)arena[q + 6] << 8 | arena[q + 7]
				   : 0u;
		if (blockIdx.x == 0) {
			/* the next launch's counters; the context index */
			R.out_next->fail = 0;
			R.out_next->nfail = 0;
			if (R.cm_out)
				*R.cm_out = R.comp;
		}
		/* the packet before the workgroup's first (the replay order) */
		vw[0] = (!in.prot && i > 0 && i - 1 < in.n) ?
			rp_word(arena, asz, R.pos[i - 1], R.end[i - 1], in.tag)
			: 0u;
	}
	const bool live = i < in.n;
	uint32_t p = 0, e = 0, c = 0, v = 0;
	struct sgpu_hdr h;
	h.ssrc = 0; h.seq = 0; h.err_pos = 0; h.hdr_len = 0xffffffffu;
	if (live) {
		p = R.pos[i];
		e = R.end[i];
		c = R.cap ? R.cap[i] : 0u;
		const uint32_t left = (e > p && e <= asz) ? e - p : 0u;
		if (left >= 8) {
			const uint8_t *b = arena + p;
			h.ssrc = (uint32_t)b[4] << 24 | (uint32_t)b[5] << 16 |
				 (uint32_t)b[6] << 8 | b[7];
			h.hdr_len = 8;
		}
		if (!in.prot)
			v = rp_word(arena, asz, p, e, in.tag);
		R.hdr[i] = h;
		R.es[i] = e;
	}
	vw[tid + 1] = v;
	__syncthreads();
	if (!live)
		return;
	const uint32_t ssrc0 = in.ssrc_any ? ssrc0s : in.ssrc;
	const uint32_t L = e - p;
	uint32_t f = 0;
	if (h.hdr_len == 0xffffffffu)
		f |= SPF_PARSE;                 /* < 8 bytes: EBADMSG */
	else if (h.ssrc != ssrc0)
		f |= SPF_SSRC;
	if ((p & 3u) || p > e || e > asz || (R.cap && (e > c || c > asz)))
		f |= SPF_BAD;
	if (L >= in.maxlen)
		f |= SPF_SIZE;
	uint32_t ix, E;
	if (in.prot) {
		if (R.cap && (uint64_t)e + in.need > (uint64_t)c)
			f |= SPF_CAP;           /* ENOMEM (cap_short) */
		ix = (in.rtcp_index + i + 1u) & 0x7fffffffu;    /* srtcp.c:54 */
		E = in.encrypted;
	}
	else {
		/* srtcp.c:166-172 (and 239-241 for GCM) */
		if (L < 8u + 4u + in.tag + (in.gcm ? 16u : 0u))
			f |= SPF_PARSE;
		ix = v & 0x7fffffffu;
		E = v >> 31;
		if (in.hmac) {
			/* replay (srtcp.c:208-209), speculated: every index new
			 * and increasing */
			bool ok;
			if (i == 0) {
				if (ix > in.lix) {
					ok = true;
				}
				else {
					const uint64_t dl = in.lix - ix;
					ok = dl < 64 && !(in.bitmap & (1ull << dl));
				}
			}
			else {
				ok = ix > (vw[tid] & 0x7fffffffu);
			}
			if (!ok)
				f |= SPF_REPLAY;
		}
	}
	R.desc[i] = ((uint64_t)(ix & 0x7fffffffu)) | ((uint64_t)E << 31) |
		    ((uint64_t)SD_RUN << 48);
	const uint32_t t0 = in.n > SGPU_PLAN_TAIL ? in.n - SGPU_PLAN_TAIL : 0u;
	if (i >= t0)
		R.out->tail_ix[i - t0] = ix;
	if (i == 0) {
		R.out->ssrc0 = h.ssrc;
		R.out->hl0 = 8;
	}
	/* (no results here: the workgroup after this one reads this
	 * packet's end for its replay order) */
	if (f)
		atomicOr(&R.out->fail, f);
}

/* ================================================================== */
/* C-ABI shim                                                          */

static char g_err[256];
static int g_inited;
static struct sgpu_session *g_table;
static struct sgpu_sstate *g_sst;       /* per slot: RTP stream 0 state of
					   resident multi-session batches */
static uint32_t g_table_cap;
static struct sgpu_keyreq *g_req_dev;

extern "C" struct sgpu_sstate *sgpu_sst_table(void)
{
	return g_sst;
}
static uint32_t *g_slot_dev;
static uint32_t g_req_cap;

static const uint32_t *g_T0_dev;

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
	if (!e)
		e = herr(hipGetSymbolAddress((void **)&g_T0_dev, HIP_SYMBOL(g_T0)),
			 "T0 address");
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
	struct sgpu_sstate *ns = NULL;
	int e = herr(hipMalloc(&nt, (size_t)cap * sizeof(*nt)), "table alloc");
	if (!e)
		e = herr(hipMalloc(&ns, (size_t)cap * sizeof(*ns)),
			 "state table alloc");
	if (e) {
		(void)hipFree(nt);
		return e;
	}
	if (g_table) {
		e = herr(hipMemcpy(nt, g_table,
				   (size_t)g_table_cap * sizeof(*nt),
				   hipMemcpyDeviceToDevice), "table grow");
		if (!e)
			e = herr(hipMemcpy(ns, g_sst,
					   (size_t)g_table_cap * sizeof(*ns),
					   hipMemcpyDeviceToDevice),
				 "state table grow");
		(void)hipDeviceSynchronize();
		(void)hipFree(g_table);
		(void)hipFree(g_sst);
	}
	g_table = nt;
	g_sst = ns;
	g_table_cap = cap;
	return e;
}

/* ---- asynchronous batch chains (srtpgpu.h sgpu_gate_*) --------------- */

__global__ void k_gate_pred(const uint32_t *pred, uint32_t *fail)
{
	if (*pred)
		atomicOr(fail, (uint32_t)SPF_PRED);
}

__global__ void k_gate_set(const uint32_t *fail, const uint32_t *nfail,
			   uint32_t *gate)
{
	*gate = (*fail || (nfail && *nfail)) ? 1u : 0u;
}

extern "C" int sgpu_gate_pred(const uint32_t *pred, uint32_t *fail,
			      void *stream)
{
	hipLaunchKernelGGL(k_gate_pred, dim3(1), dim3(1), 0,
			   (hipStream_t)stream, pred, fail);
	return herr(hipGetLastError(), "k_gate_pred launch");
}

extern "C" int sgpu_gate_set(const uint32_t *fail, const uint32_t *nfail,
			     uint32_t *gate, void *stream)
{
	hipLaunchKernelGGL(k_gate_set, dim3(1), dim3(1), 0,
			   (hipStream_t)stream, fail, nfail, gate);
	return herr(hipGetLastError(), "k_gate_set launch");
}

/* ---- resident RTP stream states (srtpgpu.h sgpu_sst_*) ---------------- */

__global__ void k_sst_zero(const uint32_t *slot, uint32_t n,
			   struct sgpu_sstate *sst)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n)
		sst[slot[i]] = sgpu_sstate{};
}

/* the 32-byte state as two 16-byte words (table and arrays are 32-byte
 * strided from 256-byte aligned bases): plain vector loads and stores --
 * a struct copy here was promoted through LDS (32 KiB per block) */
static_assert(sizeof(struct sgpu_sstate) == 32 &&
	      offsetof(struct sgpu_sstate, flags) == 12,
	      "sst_ld/sst_st move the state as two 16-byte words");

__device__ __forceinline__ void sst_ld(const struct sgpu_sstate *p, uint4 &a,
				       uint4 &b)
{
	a = ((const uint4 *)p)[0];
	b = ((const uint4 *)p)[1];
}

__device__ __forceinline__ void sst_st(struct sgpu_sstate *p, uint4 a, uint4 b)
{
	((uint4 *)p)[0] = a;
	((uint4 *)p)[1] = b;
}

__global__ void k_sst_load(const uint32_t *cm, const uint8_t *need,
			   const struct sgpu_sstate *up, uint32_t nsess,
			   struct sgpu_sstate *sst, struct sgpu_sstate *st_in)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= nsess)
		return;
	const uint32_t slot = cm[k] >> 1;
	uint4 a, b;
	if (need && need[k]) {
		sst_ld(up + k, a, b);
		sst_st(sst + slot, a, b);
	}
	else {
		sst_ld(sst + slot, a, b);
	}
	sst_st(st_in + k, a, b);
}

__global__ void k_sst_commit(const uint32_t *cm,
			     const struct sgpu_sstate *st_out, uint32_t nsess,
			     const uint32_t *fail, const uint32_t *nfail,
			     struct sgpu_sstate *sst)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= nsess || *fail || *nfail)
		return;
	uint4 a, b;
	sst_ld(st_out + k, a, b);
	if (!(a.w & SST_TOUCHED))       /* flags: the fourth word */
		return;
	a.w &= ~(uint32_t)SST_TOUCHED;
	sst_st(sst + (cm[k] >> 1), a, b);
}

__global__ void k_sst_read(const uint32_t *slot, uint32_t n,
			   const struct sgpu_sstate *sst,
			   struct sgpu_sstate *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n)
		out[i] = sst[slot[i]];
}

extern "C" int sgpu_sst_load(const uint32_t *cm, const uint8_t *need,
			     const struct sgpu_sstate *up, uint32_t nsess,
			     struct sgpu_sstate *st_in, void *stream)
{
	if (!nsess)
		return 0;
	hipLaunchKernelGGL(k_sst_load, dim3((nsess + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, cm, need, up, nsess, g_sst,
			   st_in);
	return herr(hipGetLastError(), "k_sst_load launch");
}

extern "C" int sgpu_sst_commit(const uint32_t *cm,
			       const struct sgpu_sstate *st_out, uint32_t nsess,
			       const uint32_t *fail, const uint32_t *nfail,
			       void *stream)
{
	if (!nsess)
		return 0;
	hipLaunchKernelGGL(k_sst_commit, dim3((nsess + 255) / 256), dim3(256),
			   0, (hipStream_t)stream, cm, st_out, nsess, fail, nfail,
			   g_sst);
	return herr(hipGetLastError(), "k_sst_commit launch");
}

extern "C" int sgpu_sst_read(const uint32_t *slot, uint32_t n,
			     struct sgpu_sstate *out)
{
	uint32_t *sd = NULL;
	struct sgpu_sstate *od = NULL;
	int e;
	if (!n)
		return 0;
	e = herr(hipMalloc(&sd, (size_t)n * 4), "sst read alloc");
	if (!e)
		e = herr(hipMalloc(&od, (size_t)n * sizeof(*od)),
			 "sst read alloc");
	if (!e)
		e = herr(hipMemcpy(sd, slot, (size_t)n * 4,
				   hipMemcpyHostToDevice), "sst read h2d");
	if (!e) {
		hipLaunchKernelGGL(k_sst_read, dim3((n + 255) / 256), dim3(256),
				   0, 0, sd, n, g_sst, od);
		e = herr(hipGetLastError(), "k_sst_read launch");
	}
	if (!e)
		e = herr(hipMemcpy(out, od, (size_t)n * sizeof(*od),
				   hipMemcpyDeviceToHost), "sst read d2h");
	(void)hipFree(sd);
	(void)hipFree(od);
	return e;
}

extern "C" uint32_t sgpu_table_capacity(void) { return g_table_cap; }

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
	if (!e) {
		/* a new session has no stream yet (resident state table) */
		hipLaunchKernelGGL(k_sst_zero, dim3((n + 255) / 256), dim3(256),
				   0, 0, g_slot_dev, n, g_sst);
		e = herr(hipGetLastError(), "k_sst_zero launch");
	}
	if (!e)
		e = herr(hipDeviceSynchronize(), "k_setup");
	return e;
}

/* ---- kernel timing with HIP events on the launch stream (bench.py) ---- */
#include <pthread.h>
static pthread_mutex_t g_prof_lock = PTHREAD_MUTEX_INITIALIZER;
static int g_prof_on;
struct prof_ev { hipEvent_t a, b; int slot; uint32_t jobs;
		  const char *name; int nr, prot; int gw; int gslot; };
static struct prof_ev *g_pev;
static size_t g_npev, g_pev_cap;
static uint32_t g_prof_gen;             /* + 1 per drain of g_pev */
/* a launch behind a device plan does nothing when the plan was rejected
 * (its guard words, k_ctr_fast.h fast_class, k_ctr.h k_ctr_hmac_any, the
 * single-word guards): the kernel itself stores the words it saw into a
 * pinned ring slot (KArgs.pguard, kern_common.h prof_guard) and such a
 * launch is not counted as work (sgpu_prof_voided) */
#define PROF_GRING 65536
static uint32_t *g_pguard;              /* pinned, 4 words per slot */
static size_t g_ngslot;                 /* ring slots handed out */
static uint64_t g_prof_voided;
static double g_prof_ms[32];
static uint64_t g_prof_launch[32], g_prof_jobs[32];
/* the kernel a slot's launches ran ("<name><nr,prot>"; "+" appended when
 * launches of different kernels shared the slot since the last read) */
static char g_prof_name[32][SGPU_PROF_NAME];
static int g_prof_mixed[32];

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
		if (g_pev[k].gw) {
			/* gw < 0: voided by the host (sgpu_prof_void) */
			const volatile uint32_t *w = g_pev[k].gw < 0 ? NULL :
				g_pguard + 4 * g_pev[k].gslot;
			const bool work = !w ? false : g_pev[k].gw == 4 ?
				(!w[0] || !w[1] || !w[2] || !w[3]) : !w[0];
			if (!work) {
				g_prof_voided++;
				(void)hipEventDestroy(g_pev[k].a);
				(void)hipEventDestroy(g_pev[k].b);
				continue;
			}
		}
		const int sl = g_pev[k].slot;
		char nm[SGPU_PROF_NAME];
		snprintf(nm, sizeof(nm), "%s<%d,%d>", g_pev[k].name,
			 g_pev[k].nr, g_pev[k].prot);
		if (!g_prof_name[sl][0])
			snprintf(g_prof_name[sl], SGPU_PROF_NAME, "%s", nm);
		else if (strcmp(g_prof_name[sl], nm))
			g_prof_mixed[sl] = 1;
		g_prof_ms[sl] += ms;
		g_prof_launch[sl]++;
		g_prof_jobs[sl] += g_pev[k].jobs;
		(void)hipEventDestroy(g_pev[k].a);
		(void)hipEventDestroy(g_pev[k].b);
	}
	g_npev = 0;
	g_prof_gen++;
	g_ngslot = 0;
}

/* slot = prot*16 + mode*8 + (nr==14)*4 + shift; reading resets */
extern "C" void sgpu_prof_read(double *ms, uint64_t *launches, uint64_t *jobs,
			       char (*names)[SGPU_PROF_NAME])
{
	pthread_mutex_lock(&g_prof_lock);
	prof_drain_locked();
	for (int k = 0; k < 32; k++) {
		if (ms) ms[k] = g_prof_ms[k];
		if (launches) launches[k] = g_prof_launch[k];
		if (jobs) jobs[k] = g_prof_jobs[k];
		if (names)
			snprintf(names[k], SGPU_PROF_NAME, "%s%s",
				 g_prof_name[k], g_prof_mixed[k] ? "+" : "");
		g_prof_mixed[k] = 0;
		g_prof_ms[k] = 0;
		g_prof_launch[k] = g_prof_jobs[k] = 0;
		g_prof_name[k][0] = 0;
	}
	pthread_mutex_unlock(&g_prof_lock);
}

extern "C" uint64_t sgpu_prof_voided(void)
{
	pthread_mutex_lock(&g_prof_lock);
	prof_drain_locked();
	const uint64_t v = g_prof_voided;
	pthread_mutex_unlock(&g_prof_lock);
	return v;
}

/* gw: the launch's guard (a.c.guard) is 4 class words, work iff one is 0
 * (the any-class kernels), or 1 word, work iff 0 */
static int launch(kfn_t f, const KArgs &a, uint32_t n, int slot,
		  hipStream_t stream, uint32_t block, const char *name,
		  int nr, int prot, int gw = 1)
{
	struct prof_ev pe;
	KArgs b = a;
	int prof = 0, gslot = -1;
	if (g_prof_on && slot >= 0) {
		prof = hipEventCreate(&pe.a) == hipSuccess &&
		       hipEventCreate(&pe.b) == hipSuccess;
		if (prof && a.c.guard) {
			/* a ring slot for the guard words the kernel sees */
			pthread_mutex_lock(&g_prof_lock);
			if (!g_pguard &&
			    hipHostMalloc((void **)&g_pguard, PROF_GRING * 16,
					  hipHostMallocDefault) != hipSuccess)
				g_pguard = NULL;
			if (g_pguard && g_ngslot < PROF_GRING)
				gslot = (int)g_ngslot++;
			pthread_mutex_unlock(&g_prof_lock);
		}
		if (gslot >= 0) {
			/* 0 = work, for a kernel that does not store its
			 * guard; the launch below orders these writes */
			for (int q = 0; q < 4; q++)
				g_pguard[4 * gslot + q] = 0;
			b.pguard = g_pguard + 4 * gslot;
			b.pguard_n = gw == 4 ? 4u : 1u;
		}
		if (prof)
			(void)hipEventRecord(pe.a, stream);
	}
	hipLaunchKernelGGL(f, dim3((n + block - 1) / block), dim3(block), 0,
			   stream, b);
	int e = herr(hipGetLastError(), "kernel launch");
	if (prof) {
		(void)hipEventRecord(pe.b, stream);
		pe.slot = slot;
		pe.jobs = n;
		pe.name = name;
		pe.nr = nr;
		pe.prot = prot;
		pe.gw = gslot >= 0 ? (int)b.pguard_n : 0;
		pe.gslot = gslot;
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

/* the same profiling bracket around a fused plan + crypto launch
 * (k_ctr_fused.h): never voided as a whole (each workgroup plans itself) */
typedef void (*kfn_f)(const FArgs);
kfn_f sgpu_pick_fused(int nr, int prot, int undo);      /* fused.hip */
kfn_f sgpu_pick_fzplan(int prot);                       /* fused.hip */
unsigned sgpu_lp_wg(void);                              /* fused.hip */

/* grid = n / block; jobs: the packets it processes (srtp_gpu_prof);
 * *pid: the profiling record of the launch (sgpu_prof_void), or 0 */
static int launch_fused(kfn_f f, const FArgs &a, uint32_t n, uint32_t jobs,
			int slot, hipStream_t stream, uint32_t block,
			const char *name, int nr, int prot, uint64_t *pid)
{
	*pid = 0;
	struct prof_ev pe;
	int prof = 0;
	if (g_prof_on && slot >= 0) {
		prof = hipEventCreate(&pe.a) == hipSuccess &&
		       hipEventCreate(&pe.b) == hipSuccess;
		if (prof)
			(void)hipEventRecord(pe.a, stream);
	}
	hipLaunchKernelGGL(f, dim3((n + block - 1) / block), dim3(block), 0,
			   stream, a);
	int e = herr(hipGetLastError(), "fused launch");
	if (prof) {
		(void)hipEventRecord(pe.b, stream);
		pe.slot = slot;
		pe.jobs = jobs;
		pe.name = name;
		pe.nr = nr;
		pe.prot = prot;
		pe.gw = 0;
		pe.gslot = -1;
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
		if (g_npev < g_pev_cap) {
			*pid = (uint64_t)g_prof_gen << 32 | (g_npev + 1);
			g_pev[g_npev++] = pe;
		}
		pthread_mutex_unlock(&g_prof_lock);
	}
	return e;
}

/* a fused launch whose plan the host found rejected did no work that
 * counts (it was undone): leave it out of the kernel profile */
extern "C" void sgpu_prof_void(uint64_t id)
{
	if (!id)
		return;
	pthread_mutex_lock(&g_prof_lock);
	const uint32_t k = (uint32_t)id - 1;
	if ((uint32_t)(id >> 32) == g_prof_gen && k < g_npev)
		g_pev[k].gw = -1;
	pthread_mutex_unlock(&g_prof_lock);
}

static int prof_slot(int mode, int nr, int shift, int prot)
{
	return (prot ? 16 : 0) + (mode ? 8 : 0) + (nr == 14 ? 4 : 0) +
	       (mode ? 0 : shift);
}

static int g_coop = 1;

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
	kfn_t f = mode == SGPU_MODE_GCM ? sgpu_pick_gcm(false, false, nr, prot)
		  : nr == 10 ? sgpu_pick_ctr10(false, false, shift, prot)
			     : sgpu_pick_ctr14(false, false, shift, prot);
	/* small CTR launches: cipher regions by k_ctr_coop (k_ctr.h) */
	const bool coop = njobs <= SGPU_COOP_MAX && g_coop &&
			  (mode == SGPU_MODE_GCM || prot || verdict);
			  /* CTR unprotect: the MAC's verdict gates it */
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
	a.t0 = g_T0_dev;
	a.verdict = verdict;
	a.save = save;
	if (!coop)
		return launch(f, a, njobs, prof_slot(mode, nr, shift, prot),
			      (hipStream_t)stream,
			      mode == SGPU_MODE_GCM ? KBLOCK : CTR_BLOCK,
			      mode == SGPU_MODE_GCM ? "k_gcm" : "k_ctr_hmac", nr,
			      prot);
	a.nocipher = 1;
	kfn_t fc = mode == SGPU_MODE_GCM ? sgpu_pick_gcm_coop(nr)
		   : nr == 10 ? sgpu_pick_ctr10_coop(prot)
			      : sgpu_pick_ctr14_coop(prot);
	int e = 0;
	if (prot) {
		hipLaunchKernelGGL(fc, dim3(njobs), dim3(256), 0,
				   (hipStream_t)stream, a);
		e = herr(hipGetLastError(), "coop launch");
	}
	if (!e)
		e = launch(f, a, njobs, prof_slot(mode, nr, shift, prot),
			   (hipStream_t)stream,
			   mode == SGPU_MODE_GCM ? KBLOCK : CTR_BLOCK,
			   mode == SGPU_MODE_GCM ? "k_gcm" : "k_ctr_hmac", nr, prot);
	if (!e && !prot) {
		hipLaunchKernelGGL(fc, dim3(njobs), dim3(256), 0,
				   (hipStream_t)stream, a);
		e = herr(hipGetLastError(), "coop launch");
	}
	return e;
}

/* the per-packet path's fused kernel over pinned host memory (small.hip) */
extern "C" int sgpu_run_small(uint8_t *arena, uint64_t arena_size,
			      const struct sgpu_job *jobs, uint32_t njobs,
			      uint8_t *verdict, uint32_t *save, int prot,
			      uint32_t *done_cnt, uint32_t *done_flag,
			      uint32_t done_seq, void *stream)
{
	return small_launch(arena, arena_size, jobs, njobs, verdict, save,
			    (const struct sgpu_comp *)g_table, g_T0_dev, prot,
			    done_cnt, done_flag, done_seq, stream);
}

/* the lingering small kernel (small.hip k_small_srv) on a workspace's
 * stream */
extern "C" int sgpu_run_small_srv(struct sgpu_srv_mb *mb,
				  struct sgpu_srv_bc *bc, uint32_t grid,
				  uint32_t linger_us, uint32_t life_us,
				  uint32_t *done_cnt, uint32_t *done_flag,
				  void *stream)
{
	return small_srv_launch((const struct sgpu_comp *)g_table, g_T0_dev,
				mb, bc, grid, linger_us, life_us, done_cnt,
				done_flag, stream);
}

/* the session table's device address now (a lingering small kernel's
 * batches carry it: the table moves when it grows) */
extern "C" const void *sgpu_table_ptr(void)
{
	return g_table;
}

/* srtp_gpu_tune nocoop (A/B): small general launches fused as usual */
extern "C" void sgpu_set_coop(int on)
{
	g_coop = on;
}

extern "C" int sgpu_run_compact(uint8_t *arena, uint64_t arena_size,
				const struct sgpu_compact *c, int mode, int nr,
				int shift, int prot, void *stream)
{
	if (!c->n)
		return 0;
	if (mode == SGPU_MODE_CTR && shift < 0 && c->uniform == 2 &&
	    !c->undo && !c->idx) {
		/* device-planned single-key batch: lean kernel (k_ctr_fast.h),
		 * then the forged-packet restore behind it (unprotect) */
		KArgs a;
		memset(&a, 0, sizeof(a));
		a.arena = arena;
		a.asz = arena_size;
		a.comps = (const struct sgpu_comp *)g_table;
		a.t0 = g_T0_dev;
		a.verdict = c->verdict;
		a.save = c->save;
		a.c = *c;
		kfn_t ff = nr == 10 ? sgpu_pick_ctr10_fast(prot, 0)
				    : sgpu_pick_ctr14_fast(prot, 0);
		int e = launch(ff, a, c->n, prof_slot(mode, nr, 3, prot),
			       (hipStream_t)stream, sgpu_ctr_fast_block(prot),
			       "k_ctr_fast_any", nr, prot, 4);
		if (!e && !prot && c->flist && !c->gfail) {
			/* one workgroup per listed forged packet (grid-
			 * strided past 1024); all exit at once if none.
			 * (Behind the one-launch planner -- gfail set -- the
			 * caller launches it only when there are misses.) */
			const uint32_t g = c->n < 1024u ? c->n : 1024u;
			hipLaunchKernelGGL(nr == 10 ? sgpu_pick_ctr10_fast(0, 2)
						    : sgpu_pick_ctr14_fast(0, 2),
					   dim3(g), dim3(256), 0,
					   (hipStream_t)stream, a);
			e = herr(hipGetLastError(), "refix launch");
		}
		else if (!e && !prot && !c->flist)
			/* no list: a full-grid pass finds the forged packets */
			e = launch(nr == 10 ? sgpu_pick_ctr10_fast(0, 1)
					    : sgpu_pick_ctr14_fast(0, 1),
				   a, c->n, -1, (hipStream_t)stream,
				   sgpu_ctr_fast_block(1), "k_ctr_fast_restore", nr,
				   0);
		return e;
	}
	if (mode == SGPU_MODE_CTR && shift == 2 && c->rtcp &&
	    c->uniform == 4 && !c->undo && !c->idx && !c->sess) {
		/* device-planned single-key SRTCP batch: the lean kernel's
		 * SRTCP form (a forged packet is undone with the whole batch
		 * by the caller, as for the general kernel) */
		KArgs a;
		memset(&a, 0, sizeof(a));
		a.arena = arena;
		a.asz = arena_size;
		a.comps = (const struct sgpu_comp *)g_table;
		a.t0 = g_T0_dev;
		a.verdict = c->verdict;
		a.save = c->save;
		a.c = *c;
		return launch(nr == 10 ? sgpu_pick_ctr10_fast_rtcp(prot)
				       : sgpu_pick_ctr14_fast_rtcp(prot),
			      a, c->n, prof_slot(mode, nr, 2, prot),
			      (hipStream_t)stream, sgpu_ctr_fast_block(prot),
			      "k_ctr_fast_rtcp", nr, prot);
	}
	if (mode == SGPU_MODE_CTR && shift < 0 && c->uniform == 3 &&
	    !c->undo && c->sess) {
		/* multi-session device plan: the lean kernel with per-lane
		 * keys, in the planner's launch order */
		KArgs a;
		memset(&a, 0, sizeof(a));
		a.arena = arena;
		a.asz = arena_size;
		a.comps = (const struct sgpu_comp *)g_table;
		a.t0 = g_T0_dev;
		a.verdict = c->verdict;
		a.save = c->save;
		a.c = *c;
		a.c.uniform = 0;
		int e = launch(nr == 10 ? sgpu_pick_ctr10_fast_mk(prot)
				       : sgpu_pick_ctr14_fast_mk(prot),
			      a, c->n, prof_slot(mode, nr, 3, prot),
			      (hipStream_t)stream, sgpu_ctr_fast_mk_block(),
			      "k_ctr_fast_mk", nr, prot, 4);
		if (!e && !prot && c->flist) {
			/* forged packets back to their ciphertext, each with
			 * its own session's keys (the device verdict fold of
			 * multi-session batches); exits at once if none */
			const uint32_t g = c->n < 1024u ? c->n : 1024u;
			hipLaunchKernelGGL(nr == 10 ? sgpu_pick_ctr10_fast(0, 3)
						    : sgpu_pick_ctr14_fast(0, 3),
					   dim3(g), dim3(256), 0,
					   (hipStream_t)stream, a);
			e = herr(hipGetLastError(), "refix mk launch");
		}
		return e;
	}
	kfn_t f = mode == SGPU_MODE_GCM ?
			  sgpu_pick_gcm(true, c->uniform != 0, nr, prot)
		  : nr == 10 ? sgpu_pick_ctr10(true, c->uniform != 0, shift, prot)
			     : sgpu_pick_ctr14(true, c->uniform != 0, shift, prot);
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
	a.t0 = g_T0_dev;
	a.verdict = c->verdict;
	a.save = c->save;
	a.c = *c;
	return launch(f, a, c->n,
		      c->undo ? -1 : prof_slot(mode, nr, shift < 0 ? 3 : shift,
					       prot),
		      (hipStream_t)stream,
		      mode == SGPU_MODE_GCM ? sgpu_gcm_block(c->uniform != 0)
					    : sgpu_ctr_block(c->uniform != 0, prot),
		      mode == SGPU_MODE_GCM ?
			      (c->uniform ? "k_gcmu" : "k_gcm_compact") :
		      shift < 0 ? (c->uniform ? "k_ctr_hmac_any_uni"
					      : "k_ctr_hmac_any") :
				  (c->uniform ? "k_ctr_hmac_uni"
					      : "k_ctr_hmac_compact"),
		      nr, prot, mode == SGPU_MODE_CTR && shift < 0 ? 4 : 1);
}

/* ---- single-stream batches planned inside the crypto launch ---------- */

static void fz_args(FArgs &fa, uint8_t *arena, uint64_t asz,
		   const struct sgpu_fused *f)
{
	memset(&fa, 0, sizeof(fa));
	KArgs &a = fa.a;
	a.arena = arena;
	a.asz = asz;
	a.comps = (const struct sgpu_comp *)g_table;
	a.t0 = g_T0_dev;
	a.verdict = f->verdict;
	a.save = f->save;
	/* what the launches behind it (k_ctr_refix_list, the undo) read as a
	 * compact batch: windows with the original ends, the parsed headers,
	 * the descriptors, the context index the launch stored */
	a.c.pos = f->pos;
	a.c.end = f->es;
	a.c.hdr = f->hdr;
	a.c.desc = f->desc;
	a.c.compmap = f->cm_out;
	a.c.n = f->in.n;
	a.c.verdict = f->verdict;
	a.c.save = f->save;
	a.c.nfail = &f->out->nfail;
	a.c.flist = f->flist;
	a.c.uniform = 2;
	fa.p = *f;
}

extern "C" unsigned sgpu_fused_block(void)
{
	return FZ_BLOCK;
}

extern "C" int sgpu_run_fused(uint8_t *arena, uint64_t arena_size,
			      struct sgpu_fused *f, int nr, void *stream)
{
	FArgs fa;
	if (!f->in.n || (nr != 10 && nr != 14))
		return EINVAL;
	const int prot = f->in.prot != 0;
	const uint32_t nwg = (f->in.n + FZ_BLOCK - 1) / FZ_BLOCK;
	f->ntickets = nwg;
	fz_args(fa, arena, arena_size, f);
	return launch_fused(sgpu_pick_fused(nr, prot, 0), fa, nwg * FZ_BLOCK,
			    f->in.n, prof_slot(SGPU_MODE_CTR, nr, 3, prot),
			    (hipStream_t)stream, FZ_BLOCK, "k_ctr_fused", nr,
			    prot, &f->prof_id);
}

extern "C" int sgpu_run_fzplan(uint8_t *arena, uint64_t arena_size,
			       struct sgpu_fused *f, void *stream)
{
	FArgs fa;
	if (!f->in.n)
		return EINVAL;
	const uint32_t wg = sgpu_lp_wg();      /* packets per workgroup */
	const uint32_t nwg = (f->in.n + wg - 1) / wg;
	f->ntickets = nwg;
	f->prof_id = 0;
	fz_args(fa, arena, arena_size, f);
	hipLaunchKernelGGL(sgpu_pick_fzplan(f->in.prot != 0), dim3(nwg),
			   dim3(FZ_BLOCK), 0, (hipStream_t)stream, fa);
	return herr(hipGetLastError(), "plan launch");
}

extern "C" int sgpu_fused_undo(uint8_t *arena, uint64_t arena_size,
			       const struct sgpu_fused *f, int nr, int prot,
			       void *stream)
{
	FArgs fa;
	if (!f->in.n || (nr != 10 && nr != 14) || f->shift > 3)
		return EINVAL;
	fz_args(fa, arena, arena_size, f);
	hipLaunchKernelGGL(sgpu_pick_fused(nr, prot, 1),
			   dim3((f->in.n + FZ_BLOCK - 1) / FZ_BLOCK),
			   dim3(FZ_BLOCK), 0, (hipStream_t)stream, fa);
	return herr(hipGetLastError(), "fused undo launch");
}

extern "C" int sgpu_fused_refix(uint8_t *arena, uint64_t arena_size,
				const struct sgpu_fused *f, int nr,
				void *stream)
{
	FArgs fa;
	if (!f->in.n || (nr != 10 && nr != 14))
		return EINVAL;
	fz_args(fa, arena, arena_size, f);
	/* one workgroup per listed forged packet, grid-strided past 1024 */
	const uint32_t g = f->in.n < 1024u ? f->in.n : 1024u;
	hipLaunchKernelGGL(nr == 10 ? sgpu_pick_ctr10_fast(0, 2)
				    : sgpu_pick_ctr14_fast(0, 2),
			   dim3(g), dim3(256), 0, (hipStream_t)stream, fa.a);
	return herr(hipGetLastError(), "fused refix launch");
}

extern "C" int sgpu_parse_headers(const uint8_t *arena, uint64_t arena_size,
				  const uint32_t *pos, const uint32_t *end,
				  struct sgpu_hdr *out, uint32_t *eix, uint32_t n,
				  int rtcp, void *stream)
{
	if (!n)
		return 0;
	struct sgpu_prologue pro;
	memset(&pro, 0, sizeof(pro));
	return sgpu_parse_prologue(arena, arena_size, pos, end, out, eix, n,
				   rtcp, &pro, stream);
}

extern "C" int sgpu_parse_prologue(const uint8_t *arena, uint64_t arena_size,
				   const uint32_t *pos, const uint32_t *end,
				   struct sgpu_hdr *out, uint32_t *eix,
				   uint32_t n, int rtcp,
				   const struct sgpu_prologue *pro,
				   void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_parse, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, arena, arena_size, pos, end, out,
			   eix, n, rtcp, *pro);
	return herr(hipGetLastError(), "k_parse launch");
}

/* srtp_rx_index_dev: one word per parsed packet for the host's receiver
 * walk -- seq | ok << 16 | (ssrc != ssrc0) << 17 | wide << 23 |
 * (res & 255) << 24 (wide: res outside 0..255, sent separately) */
__global__ void k_rx_pack(const struct sgpu_hdr *__restrict__ hd,
			  const int32_t *__restrict__ res, uint32_t ssrc0,
			  uint32_t *__restrict__ out, uint32_t n)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const struct sgpu_hdr h = hd[i];
	const int32_t r = res[i];
	const bool ok = h.hdr_len != 0xffffffffu;
	uint32_t v = ok ? (uint32_t)h.seq | 1u << 16 : 0u;
	if (ok && h.ssrc != ssrc0)
		v |= 1u << 17;
	if (r < 0 || r > 255)
		v |= 1u << 23;
	else
		v |= (uint32_t)r << 24;
	out[i] = v;
}

extern "C" int sgpu_rx_pack(const struct sgpu_hdr *hd, const int32_t *res,
			    uint32_t ssrc0, uint32_t *out, uint32_t n,
			    void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_rx_pack, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, hd, res, ssrc0, out, n);
	return herr(hipGetLastError(), "k_rx_pack launch");
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

/* pinned host memory the device reads while a kernel runs (the lingering
 * small kernel's mailbox): coherent, not cached on the device */
extern "C" void *sgpu_host_alloc_coherent(size_t n)
{
	void *p = NULL;
	if (herr(hipHostMalloc(&p, n ? n : 1, hipHostMallocCoherent),
		 "hipHostMalloc coherent"))
		return NULL;
	return p;
}

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

/* 0: the stream's work is done, EAGAIN: not yet, else EIO */
extern "C" int sgpu_stream_query(void *stream)
{
	const hipError_t e = hipStreamQuery((hipStream_t)stream);
	if (e == hipErrorNotReady)
		return EAGAIN;
	return herr(e, "stream query");
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

/* per-class launch guards, once every planning block has finished */
__global__ void k_plan_final(struct sgpu_plan_out *out)
{
	if (threadIdx.x < 4)
		out->skip[threadIdx.x] =
			out->fail || (((out->hl0 >> 2) & 3u) != threadIdx.x);
}

extern "C" int sgpu_plan_rtp(const struct sgpu_plan_in *in,
			     const struct sgpu_hdr *hdr, const uint32_t *pos,
			     const uint32_t *end, const uint32_t *cap,
			     uint64_t arena_size, uint64_t *desc,
			     uint32_t *scratch, struct sgpu_plan_out *out,
			     void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t nb = (in->n + PLAN_BLOCK - 1) / PLAN_BLOCK;
	if (!in->n)
		return EINVAL;
	int e = in->zeroed ? 0 : herr(hipMemsetAsync(out, 0, sizeof(*out), st),
				      "plan memset");
	if (e)
		return e;
	hipLaunchKernelGGL(k_plan_count, dim3(nb), dim3(PLAN_BLOCK), 0, st,
			   *in, hdr, pos, end, cap, arena_size, scratch, out);
	hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, st, scratch,
			   nb, out);
	hipLaunchKernelGGL(k_plan_desc, dim3(nb), dim3(PLAN_BLOCK), 0, st,
			   *in, hdr, (const uint32_t *)scratch, desc, out);
	hipLaunchKernelGGL(k_plan_final, dim3(1), dim3(64), 0, st, out);
	return herr(hipGetLastError(), "plan launch");
}

/* ------------------------------------------------------------------ */
/* Verdict fold of a device-planned unprotect (srtpgpu.h sgpu_fold_rtp) */

/* packet k changes s_l for the packets after it: authentic (s_l = seq)
 * or a rollover (s_l = 0 when forged) -- srtp.c:318-321, 426-427 */
__device__ __forceinline__ bool fold_event(const struct sgpu_plan_in &in,
					   const struct sgpu_hdr *hdr,
					   const uint8_t *vd, uint32_t k)
{
	return (vd[k] & SV_TAG_OK) ||
	       plan_wrap(hdr[k].seq, plan_sb(in, hdr, k));
}

__global__ void __launch_bounds__(PLAN_BLOCK)
k_fold_count(const struct sgpu_plan_in in, const struct sgpu_hdr *hdr,
	     const uint8_t *vd, int32_t *blast, int32_t *bred,
	     const uint32_t *nfail, struct sgpu_fold_out *out)
{
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	if (i == 0) {
		/* the verdict starts held (also when there is nothing to
		 * fold: nfail, queued behind the kernels, is 0) */
		out->fail = 0;
		out->nok = 0;
		out->first_ok = 0xffffffffu;
		out->last_ok = 0xffffffffu;
		out->s_l = 0;
		out->pad = 0;
		out->lix = 0;
		out->bitmap = 0;
	}
	if (nfail && *nfail == 0u)
		return;
	int32_t last = -1, fok = 0x7fffffff, lok = -1;
	bool ok = false;
	if (i < in.n) {
		if (fold_event(in, hdr, vd, i))
			last = (int32_t)i;
		ok = (vd[i] & SV_TAG_OK) != 0;
		if (ok)
			fok = lok = (int32_t)i;
	}
	/* block reductions (k_fold_scan folds the blocks: no same-address
	 * atomics, which serialise at L2) */
	const uint32_t cnt = (uint32_t)__popcll(__ballot(ok));
	for (int o = 32; o > 0; o >>= 1) {
		last = max(last, __shfl_xor(last, o));
		fok = min(fok, __shfl_xor(fok, o));
		lok = max(lok, __shfl_xor(lok, o));
	}
	__shared__ int32_t wl[PLAN_BLOCK / 64][4];
	if ((threadIdx.x & 63u) == 0) {
		wl[threadIdx.x >> 6][0] = last;
		wl[threadIdx.x >> 6][1] = fok;
		wl[threadIdx.x >> 6][2] = lok;
		wl[threadIdx.x >> 6][3] = (int32_t)cnt;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		int32_t m = -1, f = 0x7fffffff, l = -1, c = 0;
		for (int w = 0; w < PLAN_BLOCK / 64; w++) {
			m = max(m, wl[w][0]);
			f = min(f, wl[w][1]);
			l = max(l, wl[w][2]);
			c += wl[w][3];
		}
		blast[blockIdx.x] = m;
		bred[3 * blockIdx.x] = f;
		bred[3 * blockIdx.x + 1] = l;
		bred[3 * blockIdx.x + 2] = c;
	}
}

/* exclusive prefix maximum of the block maxima (one workgroup) */
__global__ void __launch_bounds__(1024)
k_fold_scan(const int32_t *blast, const int32_t *bred, int32_t *bprev,
	    uint32_t nb, struct sgpu_fold_out *out, const uint32_t *nfail)
{
	__shared__ int32_t part[1024];
	__shared__ int32_t red[3];
	if (nfail && *nfail == 0u)
		return;
	const uint32_t per = (nb + 1023u) / 1024u;
	const uint32_t a = threadIdx.x * per;
	int32_t m = -1, f = 0x7fffffff, l = -1, c = 0;
	if (threadIdx.x == 0) {
		red[0] = 0x7fffffff;
		red[1] = -1;
		red[2] = 0;
	}
	for (uint32_t k = a; k < a + per && k < nb; k++) {
		m = max(m, blast[k]);
		f = min(f, bred[3 * k]);
		l = max(l, bred[3 * k + 1]);
		c += bred[3 * k + 2];
	}
	__syncthreads();
	/* authentic-packet count and first / last (LDS atomics) */
	if (c) {
		atomicMin(&red[0], f);
		atomicMax(&red[1], l);
		atomicAdd(&red[2], c);
	}
	part[threadIdx.x] = m;
	__syncthreads();
	for (uint32_t d = 1; d < 1024; d <<= 1) {
		int32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : -1;
		__syncthreads();
		part[threadIdx.x] = max(part[threadIdx.x], v);
		__syncthreads();
	}
	int32_t run = threadIdx.x ? part[threadIdx.x - 1] : -1;
	for (uint32_t k = a; k < a + per && k < nb; k++) {
		bprev[k] = run;
		run = max(run, blast[k]);
	}
	if (threadIdx.x == 0) {
		out->nok = (uint32_t)red[2];
		out->first_ok = red[2] ? (uint32_t)red[0] : 0xffffffffu;
		out->last_ok = red[2] ? (uint32_t)red[1] : 0xffffffffu;
	}
}

/* s_l packet i really sees: after the last event before it */
__device__ __forceinline__ uint32_t fold_sl(const struct sgpu_plan_in &in,
					    const struct sgpu_hdr *hdr,
					    const uint8_t *vd, int32_t k)
{
	if (k < 0)
		return in.fresh ? hdr[0].seq : in.s_l;
	return (vd[k] & SV_TAG_OK) ? hdr[k].seq : 0u;
}

__global__ void __launch_bounds__(PLAN_BLOCK)
k_fold_check(const struct sgpu_plan_in in, const struct sgpu_hdr *hdr,
	     const uint8_t *vd, const int32_t *bprev,
	     struct sgpu_fold_out *out, const uint32_t *nfail)
{
	__shared__ int32_t sc[PLAN_BLOCK];
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	if (nfail && *nfail == 0u)
		return;
	const bool ev = i < in.n && fold_event(in, hdr, vd, i);
	/* inclusive prefix max of event indices inside the block */
	sc[threadIdx.x] = ev ? (int32_t)i : -1;
	__syncthreads();
	for (uint32_t d = 1; d < PLAN_BLOCK; d <<= 1) {
		int32_t v = threadIdx.x >= d ? sc[threadIdx.x - d] : -1;
		__syncthreads();
		sc[threadIdx.x] = max(sc[threadIdx.x], v);
		__syncthreads();
	}
	if (i >= in.n)
		return;
	const int32_t k = max(bprev[blockIdx.x],
			      threadIdx.x ? sc[threadIdx.x - 1] : -1);
	const uint32_t seq = hdr[i].seq;
	const uint32_t sb = plan_sb(in, hdr, i);        /* speculated */
	const uint32_t sl = fold_sl(in, hdr, vd, k);    /* true */
	const bool wrap = plan_wrap(seq, sb);
	bool bad = plan_wrap(seq, sl) != wrap ||
		   (int)seq - (int)sl > 32768;          /* ETIMEDOUT */
	if (!bad && !wrap) {
		/* same index estimate (misc.c:22-41): roc is the same */
		bad = plan_v(in.roc, sl, seq) != plan_v(in.roc, sb, seq);
		/* an authentic packet sets s_l = seq only if seq > s_l
		 * (srtp.c:426-427); fold_sl assumes it does */
		if ((vd[i] & SV_TAG_OK) && seq < sl)
			bad = true;
	}
	if (bad)
		atomicOr(&out->fail, 1u);
}

/* forged packets' results; the final s_l and replay window (one wave) */
__global__ void k_fold_results(const struct sgpu_plan_in in,
			       const struct sgpu_hdr *hdr, const uint8_t *vd,
			       const uint64_t *desc, const uint32_t *end0,
			       const int32_t *blast, const int32_t *bprev,
			       uint32_t nb, uint32_t *pos, uint32_t *end,
			       int32_t *err, int gcm, struct sgpu_fold_out *out,
			       const uint32_t *nfail)
{
	const uint32_t i = blockIdx.x * PLAN_BLOCK + threadIdx.x;
	if ((nfail && *nfail == 0u) || out->fail)
		return;
	if (i < in.n && !(vd[i] & SV_TAG_OK)) {
		err[i] = EAUTH;
		pos[i] += hdr[i].hdr_len;
		if (gcm)
			end[i] = end0[i];
	}
	if (blockIdx.x != 0 || threadIdx.x != 0)
		return;
	/* s_l after the last packet: the last event's value */
	out->s_l = fold_sl(in, hdr, vd, max(bprev[nb - 1], blast[nb - 1]));
	/* replay (replay.c:32-62) over the authentic packets: every index is
	 * new and increasing, so the window after the last authentic packet
	 * j holds the authentic packets j-63 .. j (and, if j < 64, the window
	 * before the batch) */
	uint64_t lix = in.lix, bm = in.bitmap;
	if (out->last_ok != 0xffffffffu) {
		const uint32_t j = out->last_ok;
		uint32_t q = 0;
		if (j >= 64) {
			q = j - 63;
			lix = (desc[j - 64] & 0xffffull) |
			      ((desc[j - 64] >> 16) & 0xffffffffull) << 16;
			bm = 0;
		}
		for (; q <= j; q++) {
			if (!(vd[q] & SV_TAG_OK))
				continue;
			const uint64_t ix = (desc[q] & 0xffffull) |
					    ((desc[q] >> 16) & 0xffffffffull) << 16;
			if (ix > lix) {
				const uint64_t dl = ix - lix;
				bm = dl < 64 ? (bm << dl) | 1ull : 1ull;
				lix = ix;
			}
			else {
				bm |= 1ull << (lix - ix);
			}
		}
	}
	out->lix = lix;
	out->bitmap = bm;
}

/* the first authentic packet against the window before the batch (the
 * plan checked packet 0; a forged packet 0 leaves it to the next) */
__global__ void k_fold_first(const struct sgpu_plan_in in,
			     const uint64_t *desc, struct sgpu_fold_out *out)
{
	const uint32_t f = out->first_ok;
	if (f == 0xffffffffu || f == 0)
		return;
	const uint64_t ix = (desc[f] & 0xffffull) |
			    ((desc[f] >> 16) & 0xffffffffull) << 16;
	bool ok;
	if (ix > in.lix) {
		ok = true;
	}
	else {
		const uint64_t dl = in.lix - ix;
		ok = dl < 64 && !(in.bitmap & (1ull << dl));
	}
	if (!ok)
		atomicOr(&out->fail, 2u);
}

extern "C" int sgpu_fold_rtp(int phase, const uint32_t *nfail,
			     const struct sgpu_plan_in *in,
			     const struct sgpu_hdr *hdr, const uint64_t *desc,
			     const uint8_t *verdict, const uint32_t *end0,
			     uint32_t *pos, uint32_t *end, int32_t *err,
			     int gcm, uint32_t *scratch,
			     struct sgpu_fold_out *out, void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t nb = (in->n + PLAN_BLOCK - 1) / PLAN_BLOCK;
	int32_t *blast = (int32_t *)scratch, *bprev = blast + nb + 2;
	int32_t *bred = bprev + nb + 2;
	if (!in->n)
		return EINVAL;
	if (phase != 2) {
		hipLaunchKernelGGL(k_fold_count, dim3(nb), dim3(PLAN_BLOCK), 0,
				   st, *in, hdr, verdict, blast, bred, nfail, out);
		hipLaunchKernelGGL(k_fold_scan, dim3(1), dim3(1024), 0, st,
				   blast, (const int32_t *)bred, bprev, nb, out,
				   nfail);
		hipLaunchKernelGGL(k_fold_check, dim3(nb), dim3(PLAN_BLOCK), 0,
				   st, *in, hdr, verdict, (const int32_t *)bprev,
				   out, nfail);
		hipLaunchKernelGGL(k_fold_first, dim3(1), dim3(1), 0, st, *in,
				   desc, out);
	}
	if (phase != 1)
		hipLaunchKernelGGL(k_fold_results, dim3(nb), dim3(PLAN_BLOCK), 0,
				   st, *in, hdr, verdict, desc, end0,
				   (const int32_t *)blast, (const int32_t *)bprev,
				   nb, pos, end, err, gcm, out, nfail);
	return herr(hipGetLastError(), "fold launch");
}

extern "C" int sgpu_plan_rtcp(const struct sgpu_rplan_in *in,
			      const struct sgpu_hdr *hdr, const uint32_t *eix,
			      const uint32_t *pos, const uint32_t *end,
			      const uint32_t *cap, uint64_t arena_size,
			      uint64_t *desc, struct sgpu_plan_out *out,
			      void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	if (!in->n)
		return EINVAL;
	hipLaunchKernelGGL(k_plan_rtcp, dim3((in->n + PLAN_BLOCK - 1) /
					     PLAN_BLOCK), dim3(PLAN_BLOCK), 0,
			   st, *in, hdr, eix, pos, end, cap, arena_size, desc,
			   out);
	/* guards: the SRTCP cipher region starts at byte 8 (class 2) */
	hipLaunchKernelGGL(k_plan_final, dim3(1), dim3(64), 0, st, out);
	return herr(hipGetLastError(), "rtcp plan launch");
}

__global__ void __launch_bounds__(256)
k_plan_results(const uint32_t *__restrict__ guard,
	       const uint32_t *__restrict__ end0, uint32_t *__restrict__ end,
	       int32_t *__restrict__ err, uint32_t n, int32_t delta)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n || *guard)
		return;
	end[i] = end0[i] + (uint32_t)delta;
	err[i] = 0;
}

__global__ void __launch_bounds__(256)
k_plan_finish(const uint32_t *__restrict__ guard,
	      const uint32_t *__restrict__ end0, uint32_t *__restrict__ end,
	      int32_t *__restrict__ err, uint32_t n, int32_t delta,
	      const uint32_t *nfail, uint32_t *gate, uint32_t *nfail_out,
	      const uint32_t *ffail)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	const uint32_t g = *guard;
	if (i == 0) {
		const uint32_t nf = nfail ? *nfail : 0u;
		if (gate)
			*gate = g || (nf && (!ffail || *ffail));
		if (nfail_out)
			*nfail_out = nf;
	}
	if (i >= n || g)
		return;
	end[i] = end0[i] + (uint32_t)delta;
	err[i] = 0;
}

extern "C" int sgpu_plan_finish(const uint32_t *guard, const uint32_t *end0,
				uint32_t *end, int32_t *err, uint32_t n,
				int32_t delta, const uint32_t *nfail,
				uint32_t *gate, uint32_t *nfail_out,
				const uint32_t *ffail, void *stream)
{
	const uint32_t nb = n ? (n + 255) / 256 : 1;
	hipLaunchKernelGGL(k_plan_finish, dim3(nb), dim3(256), 0,
			   (hipStream_t)stream, guard, end0, end, err, n, delta,
			   nfail, gate, nfail_out, ffail);
	return herr(hipGetLastError(), "finish launch");
}

/* the plan out to the caller's pinned mirror with vector stores, and the
 * chained call's gate word (k_plan_finish's rule): one launch in place of
 * the gate launch + the blit copy behind every single-stream call (the
 * copy's completion cost ~10 us before the next launch could start,
 * profiles/r06 config2a timeline) */
__global__ void __launch_bounds__(256)
k_plan_post(const uint32_t *__restrict__ src, uint32_t *__restrict__ host,
	    uint32_t nwords, uint32_t *gate, uint32_t *done, uint32_t seq)
{
	const uint32_t i = threadIdx.x;
	for (uint32_t w = i; w < nwords; w += blockDim.x)
		host[w] = src[w];
	if (i == 0 && gate) {
		const struct sgpu_plan_out *o = (const struct sgpu_plan_out *)src;
		*gate = o->fail || o->nfail;
	}
	if (done) {
		/* the completion word (small_done's pattern): after every
		 * thread's stores */
		__builtin_amdgcn_s_waitcnt(0);
		__syncthreads();
		if (i == 0) {
			__threadfence_system();
			__hip_atomic_store(done, seq, __ATOMIC_RELEASE,
					   __HIP_MEMORY_SCOPE_SYSTEM);
		}
	}
}

extern "C" int sgpu_plan_post(const void *out, void *host, uint32_t bytes,
			      uint32_t *gate, uint32_t *done, uint32_t seq,
			      void *stream)
{
	hipLaunchKernelGGL(k_plan_post, dim3(1), dim3(256), 0,
			   (hipStream_t)stream, (const uint32_t *)out,
			   (uint32_t *)host, (bytes + 3u) / 4u, gate, done, seq);
	return herr(hipGetLastError(), "post launch");
}

extern "C" int sgpu_plan_results(const uint32_t *guard, const uint32_t *end0,
				 uint32_t *end, int32_t *err, uint32_t n,
				 int32_t delta, void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_plan_results, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, guard, end0, end, err, n, delta);
	return herr(hipGetLastError(), "results launch");
}

extern "C" int sgpu_run_rpplan(const uint8_t *arena, uint64_t arena_size,
			       const struct sgpu_rfused *r, void *stream)
{
	if (!r->in.n)
		return EINVAL;
	hipLaunchKernelGGL(k_rp_plan, dim3((r->in.n + PLAN_BLOCK - 1) /
					   PLAN_BLOCK),
			   dim3(PLAN_BLOCK), 0, (hipStream_t)stream, arena,
			   arena_size, *r);
	return herr(hipGetLastError(), "rtcp plan launch");
}

extern "C" int sgpu_memcpy_d2d(void *dst, const void *src, size_t n,
			       void *stream)
{
	if (!n)
		return 0;
	return herr(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice,
				   (hipStream_t)stream), "d2d");
}
