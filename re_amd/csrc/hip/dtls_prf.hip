/*
 * dtls_prf.hip -- batched DTLS-SRTP keying export on the GPU.
 *
 * libre's tls_srtp_keyinfo() (src/tls/openssl/tls.c:1083-1157) obtains
 * 2 * (key + salt) bytes with SSL_export_keying_material(...,
 * "EXTRACTOR-dtls_srtp", no context); for (D)TLS 1.2 that is the RFC 5705
 * exporter: the TLS 1.2 PRF (RFC 5246 section 5) of the master secret with
 * seed = label || client_random || server_random, P_<hash> with the
 * handshake hash of the negotiated cipher suite: P_SHA256, or P_SHA384 for
 * the *_SHA384 suites (RFC 5289 3).  This kernel evaluates it for many
 * sessions at once, one thread per session (a cold path: ~20 SHA-256 or
 * ~12 SHA-512 compressions per session), so that a burst of new calls gets
 * its SRTP contexts from two launches (this one and k_setup).
 * SHA-256 / SHA-384: FIPS 180-4; HMAC: RFC 2104 with the 48-byte master
 * secret.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include "../srtpgpu.h"

__constant__ uint32_t c_k256[64] = {
	0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu,
	0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u, 0xd807aa98u, 0x12835b01u,
	0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u,
	0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu,
	0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u,
	0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
	0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
	0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
	0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u,
	0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u, 0x1e376c08u,
	0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu,
	0x682e6ff3u, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u,
	0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};

/* FIPS 180-4 4.2.3: first 64 bits of the fractional parts of the cube
 * roots of the first 80 primes */
__constant__ uint64_t c_k512[80] = {
	0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full,
	0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull, 0x59f111f1b605d019ull,
	0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull,
	0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
	0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
	0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull,
	0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull, 0x2de92c6f592b0275ull,
	0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
	0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full,
	0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
	0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull,
	0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
	0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull,
	0x92722c851482353bull, 0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull,
	0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
	0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
	0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull,
	0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull,
	0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull,
	0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
	0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull,
	0xc67178f2e372532bull, 0xca273eceea26619cull, 0xd186b8c721c0c207ull,
	0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull,
	0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
	0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
	0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull,
	0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull,
};

__device__ __forceinline__ uint32_t ror(uint32_t x, int n)
{
	return __builtin_amdgcn_alignbit(x, x, n);
}

/* one SHA-256 compression of the 64-byte block b (FIPS 180-4 6.2.2) */
__device__ void sha256_block(uint32_t h[8], const uint8_t *b)
{
	uint32_t w[64];
	for (int i = 0; i < 16; i++)
		w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 |
		       (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
	for (int i = 16; i < 64; i++) {
		const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^
				    (w[i - 15] >> 3);
		const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^
				    (w[i - 2] >> 10);
		w[i] = w[i - 16] + s0 + w[i - 7] + s1;
	}
	uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5],
		 g = h[6], hh = h[7];
	for (int i = 0; i < 64; i++) {
		const uint32_t S1 = ror(e, 6) ^ ror(e, 11) ^ ror(e, 25);
		const uint32_t ch = (e & f) ^ (~e & g);
		const uint32_t t1 = hh + S1 + ch + c_k256[i] + w[i];
		const uint32_t S0 = ror(a, 2) ^ ror(a, 13) ^ ror(a, 22);
		const uint32_t mj = (a & bb) ^ (a & c) ^ (bb & c);
		const uint32_t t2 = S0 + mj;
		hh = g; g = f; f = e; e = d + t1;
		d = c; c = bb; bb = a; a = t1 + t2;
	}
	h[0] += a; h[1] += bb; h[2] += c; h[3] += d;
	h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

__device__ void sha256_init(uint32_t h[8])
{
	h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u;
	h[3] = 0xa54ff53au; h[4] = 0x510e527fu; h[5] = 0x9b05688cu;
	h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

/* SHA-256 of (64-byte prefix already in h) || m[0, len), digest to out */
__device__ void sha256_finish(uint32_t h[8], const uint8_t *m, uint32_t len,
			      uint8_t out[32])
{
	uint8_t blk[64];
	uint32_t done = 0;
	while (len - done >= 64) {
		sha256_block(h, m + done);
		done += 64;
	}
	const uint32_t r = len - done;
	for (uint32_t i = 0; i < 64; i++)
		blk[i] = i < r ? m[done + i] : 0;
	blk[r] = 0x80;
	if (r >= 56) {
		sha256_block(h, blk);
		for (int i = 0; i < 64; i++)
			blk[i] = 0;
	}
	const uint64_t bits = (uint64_t)(64u + len) * 8u;
	for (int i = 0; i < 8; i++)
		blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
	sha256_block(h, blk);
	for (int i = 0; i < 8; i++) {
		out[4 * i] = (uint8_t)(h[i] >> 24);
		out[4 * i + 1] = (uint8_t)(h[i] >> 16);
		out[4 * i + 2] = (uint8_t)(h[i] >> 8);
		out[4 * i + 3] = (uint8_t)h[i];
	}
}

/* HMAC-SHA256 with precomputed ipad / opad midstates */
__device__ void hmac256(const uint32_t ih[8], const uint32_t oh[8],
			const uint8_t *m, uint32_t len, uint8_t out[32])
{
	uint32_t h[8];
	uint8_t inner[32];
	for (int i = 0; i < 8; i++)
		h[i] = ih[i];
	sha256_finish(h, m, len, inner);
	for (int i = 0; i < 8; i++)
		h[i] = oh[i];
	sha256_finish(h, inner, 32, out);
}

__device__ __forceinline__ uint64_t ror64(uint64_t x, int n)
{
	return (x >> n) | (x << (64 - n));
}

/* one SHA-512 compression of the 128-byte block b (FIPS 180-4 6.4.2) */
__device__ void sha512_block(uint64_t h[8], const uint8_t *b)
{
	uint64_t w[80];
	for (int i = 0; i < 16; i++) {
		uint64_t v = 0;
		for (int k = 0; k < 8; k++)
			v = v << 8 | b[8 * i + k];
		w[i] = v;
	}
	for (int i = 16; i < 80; i++) {
		const uint64_t s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^
				    (w[i - 15] >> 7);
		const uint64_t s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^
				    (w[i - 2] >> 6);
		w[i] = w[i - 16] + s0 + w[i - 7] + s1;
	}
	uint64_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5],
		 g = h[6], hh = h[7];
	for (int i = 0; i < 80; i++) {
		const uint64_t S1 = ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41);
		const uint64_t ch = (e & f) ^ (~e & g);
		const uint64_t t1 = hh + S1 + ch + c_k512[i] + w[i];
		const uint64_t S0 = ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
		const uint64_t mj = (a & bb) ^ (a & c) ^ (bb & c);
		const uint64_t t2 = S0 + mj;
		hh = g; g = f; f = e; e = d + t1;
		d = c; c = bb; bb = a; a = t1 + t2;
	}
	h[0] += a; h[1] += bb; h[2] += c; h[3] += d;
	h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* SHA-384 initial hash value (FIPS 180-4 5.3.4) */
__device__ void sha384_init(uint64_t h[8])
{
	h[0] = 0xcbbb9d5dc1059ed8ull; h[1] = 0x629a292a367cd507ull;
	h[2] = 0x9159015a3070dd17ull; h[3] = 0x152fecd8f70e5939ull;
	h[4] = 0x67332667ffc00b31ull; h[5] = 0x8eb44a8768581511ull;
	h[6] = 0xdb0c2e0d64f98fa7ull; h[7] = 0x47b5481dbefa4fa4ull;
}

/* SHA-384 of (128-byte prefix already in h) || m[0, len), 48-byte digest */
__device__ void sha384_finish(uint64_t h[8], const uint8_t *m, uint32_t len,
			      uint8_t out[48])
{
	uint8_t blk[128];
	uint32_t done = 0;
	while (len - done >= 128) {
		sha512_block(h, m + done);
		done += 128;
	}
	const uint32_t r = len - done;
	for (uint32_t i = 0; i < 128; i++)
		blk[i] = i < r ? m[done + i] : 0;
	blk[r] = 0x80;
	if (r >= 112) {
		sha512_block(h, blk);
		for (int i = 0; i < 128; i++)
			blk[i] = 0;
	}
	/* 128-bit big-endian bit length; the high 64 bits are zero here */
	const uint64_t bits = (uint64_t)(128u + len) * 8u;
	for (int i = 0; i < 8; i++)
		blk[120 + i] = (uint8_t)(bits >> (56 - 8 * i));
	sha512_block(h, blk);
	for (int i = 0; i < 6; i++)
		for (int k = 0; k < 8; k++)
			out[8 * i + k] = (uint8_t)(h[i] >> (56 - 8 * k));
}

/* HMAC-SHA384 with precomputed ipad / opad midstates */
__device__ void hmac384(const uint64_t ih[8], const uint64_t oh[8],
			const uint8_t *m, uint32_t len, uint8_t out[48])
{
	uint64_t h[8];
	uint8_t inner[48];
	for (int i = 0; i < 8; i++)
		h[i] = ih[i];
	sha384_finish(h, m, len, inner);
	for (int i = 0; i < 8; i++)
		h[i] = oh[i];
	sha384_finish(h, inner, 48, out);
}

#define KEYING_LABEL "EXTRACTOR-dtls_srtp"
#define KEYING_LABEL_LEN 19u
#define KEYING_SEED_LEN (KEYING_LABEL_LEN + 64u)

/* P_SHA256(secret, seed) -> o[0, outlen) */
__device__ void p_sha256(const uint8_t *ms, const uint8_t *seed, uint8_t *o,
			 uint32_t outlen)
{
	/* HMAC key block: the 48-byte secret, zero padded (RFC 2104) */
	uint32_t ih[8], oh[8];
	uint8_t blk[64];
	for (int pass = 0; pass < 2; pass++) {
		const uint8_t pad = pass ? 0x5c : 0x36;
		for (int i = 0; i < 64; i++)
			blk[i] = (uint8_t)((i < 48 ? ms[i] : 0) ^ pad);
		uint32_t *h = pass ? oh : ih;
		sha256_init(h);
		sha256_block(h, blk);
	}
	/* buf = A(i) (32) || seed */
	uint8_t buf[32 + KEYING_SEED_LEN], a[32], r[32];
	for (uint32_t i = 0; i < KEYING_SEED_LEN; i++)
		buf[32 + i] = seed[i];
	hmac256(ih, oh, buf + 32, KEYING_SEED_LEN, a);          /* A(1) */
	for (uint32_t done = 0; done < outlen; done += 32) {
		for (int i = 0; i < 32; i++)
			buf[i] = a[i];
		hmac256(ih, oh, buf, 32 + KEYING_SEED_LEN, r);
		for (uint32_t i = 0; i < 32 && done + i < outlen; i++)
			o[done + i] = r[i];
		hmac256(ih, oh, a, 32, a);                      /* A(i+1) */
	}
}

/* P_SHA384(secret, seed) -> o[0, outlen) */
__device__ void p_sha384(const uint8_t *ms, const uint8_t *seed, uint8_t *o,
			 uint32_t outlen)
{
	uint64_t ih[8], oh[8];
	uint8_t blk[128];
	for (int pass = 0; pass < 2; pass++) {
		const uint8_t pad = pass ? 0x5c : 0x36;
		for (int i = 0; i < 128; i++)
			blk[i] = (uint8_t)((i < 48 ? ms[i] : 0) ^ pad);
		uint64_t *h = pass ? oh : ih;
		sha384_init(h);
		sha512_block(h, blk);
	}
	uint8_t buf[48 + KEYING_SEED_LEN], a[48], r[48];
	for (uint32_t i = 0; i < KEYING_SEED_LEN; i++)
		buf[48 + i] = seed[i];
	hmac384(ih, oh, buf + 48, KEYING_SEED_LEN, a);          /* A(1) */
	for (uint32_t done = 0; done < outlen; done += 48) {
		for (int i = 0; i < 48; i++)
			buf[i] = a[i];
		hmac384(ih, oh, buf, 48 + KEYING_SEED_LEN, r);
		for (uint32_t i = 0; i < 48 && done + i < outlen; i++)
			o[done + i] = r[i];
		hmac384(ih, oh, a, 48, a);                      /* A(i+1) */
	}
}

/* in: n records of `stride` bytes (struct srtp_dtls_secret: master 48 |
 * client_random 32 | server_random 32 | prf u32 LE at 112);
 * out: n x outlen bytes of P_<hash>(master, seed) */
__global__ void k_dtls_prf(const uint8_t *__restrict__ in, uint32_t n,
			   uint32_t stride, uint32_t outlen,
			   uint8_t *__restrict__ out)
{
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n)
		return;
	const uint8_t *ms = in + (size_t)stride * t;
	uint8_t *o = out + (size_t)outlen * t;
	/* seed = label || client_random || server_random */
	uint8_t seed[KEYING_SEED_LEN];
	const char *label = KEYING_LABEL;
	for (uint32_t i = 0; i < KEYING_LABEL_LEN; i++)
		seed[i] = (uint8_t)label[i];
	for (uint32_t i = 0; i < 64; i++)
		seed[KEYING_LABEL_LEN + i] = ms[48 + i];
	if (ms[112] == 1)       /* SRTP_DTLS_PRF_SHA384 (the host checked) */
		p_sha384(ms, seed, o, outlen);
	else
		p_sha256(ms, seed, o, outlen);
}

extern "C" int sgpu_dtls_prf(const uint8_t *in, uint32_t n, uint32_t stride,
			     uint32_t outlen, uint8_t *out)
{
	uint8_t *din = NULL, *dout = NULL;
	hipError_t e;
	if (!n)
		return 0;
	if (!in || !out || !outlen || outlen > 256 || stride < 116)
		return EINVAL;
	e = hipMalloc(&din, (size_t)n * stride);
	if (e == hipSuccess)
		e = hipMalloc(&dout, (size_t)n * outlen);
	if (e == hipSuccess)
		e = hipMemcpy(din, in, (size_t)n * stride, hipMemcpyHostToDevice);
	if (e == hipSuccess) {
		hipLaunchKernelGGL(k_dtls_prf, dim3((n + 63) / 64), dim3(64), 0,
				   0, din, n, stride, outlen, dout);
		e = hipGetLastError();
	}
	if (e == hipSuccess)
		e = hipMemcpy(out, dout, (size_t)n * outlen,
			      hipMemcpyDeviceToHost);
	/* scrub the secrets and the exported keys before the memory goes
	 * back to the allocator (mem_secclean, tls.c:1156) */
	if (din)
		(void)hipMemset(din, 0, (size_t)n * stride);
	if (dout)
		(void)hipMemset(dout, 0, (size_t)n * outlen);
	(void)hipDeviceSynchronize();
	(void)hipFree(din);
	(void)hipFree(dout);
	return e == hipSuccess ? 0 : EIO;
}
