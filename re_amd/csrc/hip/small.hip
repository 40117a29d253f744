/*
 * small.hip -- the per-packet path's fused kernel (AES-CM + HMAC-SHA1).
 *
 * Every unchanged libre caller protects one mbuf per srtp_encrypt() call
 * (reference src/srtp/srtp.c:183-285; unprotect :288-432).  Concurrent
 * calls share a launch (host srtp.c one/pc_run) but a launch still carries
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

} /* namespace */

/* MODE 0 unprotect, 1 protect, 2 per job (SJ_PROTECT): the operations of
 * one shared per-packet launch in one grid (host pc_run_fused) */
template <int MODE>
__global__ void __launch_bounds__(256) k_ctr_small(const KArgs a)
{
	__shared__ uint32_t T[256];
	__shared__ uint32_t rk[60];     /* plain round keys */
	__shared__ __attribute__((aligned(16))) uint32_t buf[SMALL_MAX / 4];
	__shared__ __attribute__((aligned(16))) uint32_t ksb[SMALL_MAX / 4];
	__shared__ uint32_t s_tag_ok;
	const uint32_t i = blockIdx.x, tid = threadIdx.x;
	if (i >= a.njobs)
		return;
	const struct sgpu_job j = a.jobs[i];
	const bool PROT = MODE == 2 ? (j.flags & SJ_PROTECT) != 0 : MODE == 1;
	if (j.flags & SJ_SKIP) {
		if (tid == 0 && a.verdict)
			a.verdict[i] = 0;
		return;
	}
	const struct sgpu_comp *cp = a.comps +
				     __builtin_amdgcn_readfirstlane(j.comp);
	const uint32_t nr = cp->nr;
	T[tid] = a.t0[tid];

	const bool do_cipher = (j.flags & SJ_CIPHER) != 0;
	const bool do_hmac = (j.flags & SJ_HMAC) != 0;
	const bool trail = (j.flags & SJ_TRAILER) != 0;
	const bool cipher_if_ok = !PROT && (j.flags & SJ_CIPHER_IF_OK);
	const bool roc_at_tag = !PROT && (j.flags & SJ_ROC_AT_TAG);
	const uint32_t c_off = j.c_off;
	const uint32_t c_end = do_cipher ? j.c_off + j.c_len : 0u;
	const uint32_t A = do_hmac ? j.a_len : 0u;
	const uint32_t tag_len = do_hmac ? cp->tag_len : 0u;
	const bool store_ct = do_cipher && (PROT || cipher_if_ok || !do_hmac);
	/* bytes read: the MAC input and cipher region, unprotect's tag;
	 * bytes written back: those plus protect's tag and trailer */
	uint32_t in_len = max(c_end, A);
	uint32_t out_len = in_len;
	if (PROT) {
		if (do_hmac)
			out_len = max(out_len, j.tag_off + tag_len);
		if (j.flags & SJ_STORE_TRAIL)
			out_len = max(out_len, j.t_off + 4u);
	}
	else {
		if (do_hmac)
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
	if (PROT) {
		/* the MAC covers the ciphertext: keystream first.  (Hashing
		 * each chunk as soon as its blocks are done, the other waves
		 * applying the keystream meanwhile, measured slower: 41.6 vs
		 * 35.9 us per launch -- the per-block flag waits cost more than
		 * the ~3 us keystream pass they hide) */
		if (do_cipher)
			region_ks(T, rk, nr, iv, c_off, c_end, buf, true, tid,
				  blockDim.x);
		__syncthreads();
		if (tid == 0 && do_hmac) {
			const ks_wait none = {nullptr, 0, 0};
			hmac_lds(buf, cp, A, trail, j.trailer, h, none);
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
		if (tid == 0) {
			uint32_t ok = 1;
			if (do_hmac) {
				const ks_wait none = {nullptr, 0, 0};
				hmac_lds(buf, cp, A, trail, j.trailer, h, none);
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

int small_launch(uint8_t *arena, uint64_t arena_size,
		 const struct sgpu_job *jobs, uint32_t njobs, uint8_t *verdict,
		 uint32_t *save, const struct sgpu_comp *comps,
		 const uint32_t *t0, int prot, void *stream)
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
	hipLaunchKernelGGL(prot == 2 ? k_ctr_small<2>
			   : prot ? k_ctr_small<1> : k_ctr_small<0>,
			   dim3(njobs), dim3(256), 0, (hipStream_t)stream, a);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
