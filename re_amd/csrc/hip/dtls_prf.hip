/*
 * dtls_prf.hip -- batched DTLS-SRTP keying export on the GPU.
 *
 * libre's tls_srtp_keyinfo() (src/tls/openssl/tls.c:1083-1157) obtains
 * 2 * (key + salt) bytes with SSL_export_keying_material(...,
 * "EXTRACTOR-dtls_srtp", no context); for (D)TLS 1.2 that is the RFC 5705
 * exporter: the TLS 1.2 PRF (RFC 5246 section 5, P_SHA256) of the master
 * secret with seed = label || client_random || server_random.  This kernel
 * evaluates it for many sessions at once, one thread per session (a cold
 * path: ~20 SHA-256 compressions per session), so that a burst of new
 * calls gets its SRTP contexts from two launches (this one and k_setup).
 * SHA-256: FIPS 180-4; HMAC: RFC 2104 with the 48-byte master secret.
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

#define KEYING_LABEL "EXTRACTOR-dtls_srtp"
#define KEYING_LABEL_LEN 19u
#define KEYING_SEED_LEN (KEYING_LABEL_LEN + 64u)

/* in: n x (master 48 | client_random 32 | server_random 32);
 * out: n x outlen bytes of P_SHA256(master, seed) */
__global__ void k_dtls_prf(const uint8_t *__restrict__ in, uint32_t n,
			   uint32_t outlen, uint8_t *__restrict__ out)
{
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n)
		return;
	const uint8_t *ms = in + 112u * t;
	uint8_t *o = out + (size_t)outlen * t;
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
	/* buf = A(i) (32) || seed (label || client_random || server_random) */
	uint8_t buf[32 + KEYING_SEED_LEN], a[32], r[32];
	const char *label = KEYING_LABEL;
	for (uint32_t i = 0; i < KEYING_LABEL_LEN; i++)
		buf[32 + i] = (uint8_t)label[i];
	for (uint32_t i = 0; i < 64; i++)
		buf[32 + KEYING_LABEL_LEN + i] = ms[48 + i];
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

extern "C" int sgpu_dtls_prf(const uint8_t *in, uint32_t n, uint32_t outlen,
			     uint8_t *out)
{
	uint8_t *din = NULL, *dout = NULL;
	hipError_t e;
	if (!n)
		return 0;
	if (!in || !out || !outlen || outlen > 256)
		return EINVAL;
	e = hipMalloc(&din, (size_t)n * 112u);
	if (e == hipSuccess)
		e = hipMalloc(&dout, (size_t)n * outlen);
	if (e == hipSuccess)
		e = hipMemcpy(din, in, (size_t)n * 112u, hipMemcpyHostToDevice);
	if (e == hipSuccess) {
		hipLaunchKernelGGL(k_dtls_prf, dim3((n + 63) / 64), dim3(64), 0,
				   0, din, n, outlen, dout);
		e = hipGetLastError();
	}
	if (e == hipSuccess)
		e = hipMemcpy(out, dout, (size_t)n * outlen,
			      hipMemcpyDeviceToHost);
	(void)hipFree(din);
	(void)hipFree(dout);
	return e == hipSuccess ? 0 : EIO;
}
