/*
 * srtp_oracle.c -- CPU restatement of libre's SRTP/SRTCP hot path.
 *
 * TEST INFRASTRUCTURE ONLY: this file is the parity oracle.  It is never
 * linked into or called by the product (re_amd/).  It restates, function by
 * function, /root/reference (baresip/re v4.10.0):
 *
 *   src/srtp/srtp.c    srtp_alloc/comp_init/srtp_encrypt/srtp_decrypt
 *   src/srtp/srtcp.c   srtcp_encrypt/srtcp_decrypt
 *   src/srtp/misc.c    srtp_get_index/srtp_derive/srtp_iv_calc(_gcm)
 *   src/srtp/replay.c  srtp_replay_check
 *   src/srtp/stream.c  stream_get/stream_get_seq (8-stream cap)
 *   src/rtp/rtp.c      rtp_hdr_decode (header parse, error positions)
 *   src/mbuf/mbuf.c    mbuf_write_mem growth policy, mbuf_read_mem
 *
 * The cipher/MAC arithmetic the reference delegates to OpenSSL 3.0.2
 * (EVP_aes_{128,256}_{ctr,gcm}, HMAC(EVP_sha1)) is restated from FIPS-197,
 * NIST SP 800-38A/38D, FIPS 180-4 and RFC 2104 in portable byte-oriented C.
 * Deliberately simple (no tables beyond the S-box, bitwise GF(2^128)).
 */
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include "srtp_oracle.h"

#ifndef EAUTH
#define EAUTH 217            /* include/re_types.h:215-217 */
#endif

enum { MODE_CTR = 0, MODE_GCM = 1 };

/* ------------------------------------------------------------------ AES */

static uint8_t sbox[256];
static int sbox_ready;

static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

static uint8_t gmul(uint8_t a, uint8_t b)
{
	uint8_t r = 0;
	while (b) {
		if (b & 1)
			r ^= a;
		a = xt(a);
		b >>= 1;
	}
	return r;
}

/* FIPS-197 5.1.1: S-box = affine(inverse in GF(2^8)) */
static void sbox_init(void)
{
	int x;
	if (sbox_ready)
		return;
	for (x = 0; x < 256; x++) {
		uint8_t inv = 0, b, s;
		int y;
		if (x) {
			for (y = 1; y < 256; y++)
				if (gmul((uint8_t)x, (uint8_t)y) == 1) {
					inv = (uint8_t)y;
					break;
				}
		}
		b = inv;
		s = (uint8_t)(b ^ (uint8_t)((b << 1) | (b >> 7)) ^
			      (uint8_t)((b << 2) | (b >> 6)) ^
			      (uint8_t)((b << 3) | (b >> 5)) ^
			      (uint8_t)((b << 4) | (b >> 4)) ^ 0x63);
		sbox[x] = s;
	}
	sbox_ready = 1;
}

struct oaes {
	uint8_t rk[15][16];
	int nr;
};

/* FIPS-197 5.2 key expansion, byte oriented */
static void aes_setkey(struct oaes *a, const uint8_t *key, size_t key_bits)
{
	uint8_t w[60][4];
	int nk = (int)(key_bits / 32), i, r;
	uint8_t rcon = 1;

	sbox_init();
	a->nr = nk + 6;
	for (i = 0; i < nk; i++)
		memcpy(w[i], key + 4 * i, 4);
	for (i = nk; i < 4 * (a->nr + 1); i++) {
		uint8_t t[4];
		memcpy(t, w[i - 1], 4);
		if (i % nk == 0) {
			uint8_t u = t[0];
			t[0] = (uint8_t)(sbox[t[1]] ^ rcon);
			t[1] = sbox[t[2]];
			t[2] = sbox[t[3]];
			t[3] = sbox[u];
			rcon = xt(rcon);
		}
		else if (nk > 6 && i % nk == 4) {
			for (r = 0; r < 4; r++)
				t[r] = sbox[t[r]];
		}
		for (r = 0; r < 4; r++)
			w[i][r] = (uint8_t)(w[i - nk][r] ^ t[r]);
	}
	for (r = 0; r <= a->nr; r++)
		for (i = 0; i < 4; i++)
			memcpy(&a->rk[r][4 * i], w[4 * r + i], 4);
}

static void aes_block(const struct oaes *a, const uint8_t in[16],
		      uint8_t out[16])
{
	uint8_t s[16], t[16];
	int r, c, i;

	for (i = 0; i < 16; i++)
		s[i] = in[i] ^ a->rk[0][i];
	for (r = 1; r <= a->nr; r++) {
		/* SubBytes + ShiftRows: state byte (row, col) = s[4*col+row] */
		for (c = 0; c < 4; c++)
			for (i = 0; i < 4; i++)
				t[4 * c + i] = sbox[s[4 * ((c + i) % 4) + i]];
		if (r != a->nr) {        /* MixColumns */
			for (c = 0; c < 4; c++) {
				uint8_t *p = &t[4 * c];
				uint8_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
				s[4 * c + 0] = (uint8_t)(xt(a0) ^ xt(a1) ^ a1 ^ a2 ^ a3);
				s[4 * c + 1] = (uint8_t)(a0 ^ xt(a1) ^ xt(a2) ^ a2 ^ a3);
				s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xt(a2) ^ xt(a3) ^ a3);
				s[4 * c + 3] = (uint8_t)(xt(a0) ^ a0 ^ a1 ^ a2 ^ xt(a3));
			}
		}
		else
			memcpy(s, t, 16);
		for (i = 0; i < 16; i++)
			s[i] ^= a->rk[r][i];
	}
	memcpy(out, s, 16);
}

/* 128-bit big-endian counter increment (OpenSSL CRYPTO_ctr128_encrypt) */
static void ctr_inc128(uint8_t c[16])
{
	int i;
	for (i = 15; i >= 0; i--)
		if (++c[i])
			break;
}

/* 32-bit increment of the last word (SP 800-38D inc32) */
static void ctr_inc32(uint8_t c[16])
{
	int i;
	for (i = 15; i >= 12; i--)
		if (++c[i])
			break;
}

/* Streaming cipher context: the restatement of struct aes
 * (src/aes/openssl/aes.c:16-20) with the EVP state it relies on. */
struct ocipher {
	struct oaes k;
	int mode;
	uint8_t ctr[16];
	uint8_t ks[16];
	unsigned num;          /* bytes of ks already used */
	/* GCM */
	uint8_t h[16], j0[16];
	uint8_t *aad;
	size_t aad_len, aad_cap;
	uint8_t *ct;
	size_t ct_len, ct_cap;
};

static void cipher_init(struct ocipher *c, int mode, const uint8_t *key,
			size_t key_bits)
{
	static const uint8_t zero[16];
	memset(c, 0, sizeof(*c));
	aes_setkey(&c->k, key, key_bits);
	c->mode = mode;
	aes_block(&c->k, zero, c->h);
}

/* aes_set_iv (aes.c:123-133): CTR takes 16 B, GCM a 96-bit IV */
static void cipher_set_iv(struct ocipher *c, const uint8_t *iv)
{
	c->num = 0;
	c->aad_len = 0;
	c->ct_len = 0;
	if (c->mode == MODE_CTR) {
		memcpy(c->ctr, iv, 16);
	}
	else {
		memcpy(c->j0, iv, 12);
		c->j0[12] = 0; c->j0[13] = 0; c->j0[14] = 0; c->j0[15] = 1;
		memcpy(c->ctr, c->j0, 16);
		ctr_inc32(c->ctr);
	}
}

static void append(uint8_t **b, size_t *len, size_t *cap, const uint8_t *p,
		   size_t n)
{
	if (*len + n > *cap) {
		*cap = (*len + n) * 2 + 64;
		*b = realloc(*b, *cap);
	}
	memcpy(*b + *len, p, n);
	*len += n;
}

/* aes_encr / aes_decr (aes.c:136-171): out == NULL feeds GCM AAD */
static void cipher_update(struct ocipher *c, uint8_t *out, const uint8_t *in,
			  size_t len, int encrypt)
{
	size_t i;

	if (!out) {
		append(&c->aad, &c->aad_len, &c->aad_cap, in, len);
		return;
	}
	if (c->mode == MODE_GCM && !encrypt)
		append(&c->ct, &c->ct_len, &c->ct_cap, in, len);
	for (i = 0; i < len; i++) {
		if (c->num == 0) {
			aes_block(&c->k, c->ctr, c->ks);
			if (c->mode == MODE_CTR)
				ctr_inc128(c->ctr);
			else
				ctr_inc32(c->ctr);
		}
		out[i] = in[i] ^ c->ks[c->num];
		c->num = (c->num + 1) & 15;
	}
	if (c->mode == MODE_GCM && encrypt)
		append(&c->ct, &c->ct_len, &c->ct_cap, out, len);
}

/* GF(2^128) multiply, SP 800-38D Algorithm 1 (bitwise) */
static void gf_mul(uint8_t x[16], const uint8_t y[16])
{
	uint8_t z[16] = {0}, v[16];
	int i, j;
	memcpy(v, y, 16);
	for (i = 0; i < 128; i++) {
		int lsb;
		if (x[i / 8] & (0x80 >> (i % 8)))
			for (j = 0; j < 16; j++)
				z[j] ^= v[j];
		lsb = v[15] & 1;
		for (j = 15; j > 0; j--)
			v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
		v[0] >>= 1;
		if (lsb)
			v[0] ^= 0xe1;
	}
	memcpy(x, z, 16);
}

static void ghash_feed(uint8_t x[16], const uint8_t h[16], const uint8_t *p,
		       size_t n)
{
	size_t i, j;
	for (i = 0; i < n; i += 16) {
		for (j = 0; j < 16 && i + j < n; j++)
			x[j] ^= p[i + j];
		gf_mul(x, h);
	}
}

/* EVP_EncryptFinal_ex + GCM_GET_TAG (aes.c:183-209) */
static void gcm_tag(struct ocipher *c, uint8_t tag[16])
{
	uint8_t x[16] = {0}, lb[16], ej0[16];
	uint64_t al = (uint64_t)c->aad_len * 8, cl = (uint64_t)c->ct_len * 8;
	int i;

	ghash_feed(x, c->h, c->aad, c->aad_len);
	ghash_feed(x, c->h, c->ct, c->ct_len);
	for (i = 0; i < 8; i++) {
		lb[i] = (uint8_t)(al >> (56 - 8 * i));
		lb[8 + i] = (uint8_t)(cl >> (56 - 8 * i));
	}
	ghash_feed(x, c->h, lb, 16);
	aes_block(&c->k, c->j0, ej0);
	for (i = 0; i < 16; i++)
		tag[i] = x[i] ^ ej0[i];
}

static void cipher_free(struct ocipher *c)
{
	free(c->aad);
	free(c->ct);
	c->aad = c->ct = NULL;
}

/* ---------------------------------------------------------------- SHA-1 */

static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void sha1_compress(uint32_t h[5], const uint8_t blk[64])
{
	uint32_t w[80], a, b, c, d, e, t;
	int i;
	for (i = 0; i < 16; i++)
		w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 |
		       (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
	for (i = 16; i < 80; i++)
		w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
	a = h[0]; b = h[1]; c = h[2]; d = h[3]; e = h[4];
	for (i = 0; i < 80; i++) {
		uint32_t f, k;
		if (i < 20)      { f = (b & c) | (~b & d);          k = 0x5a827999; }
		else if (i < 40) { f = b ^ c ^ d;                   k = 0x6ed9eba1; }
		else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdc; }
		else             { f = b ^ c ^ d;                   k = 0xca62c1d6; }
		t = rol(a, 5) + f + e + k + w[i];
		e = d; d = c; c = rol(b, 30); b = a; a = t;
	}
	h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

struct osha1 {
	uint32_t h[5];
	uint8_t buf[64];
	size_t n;
	uint64_t total;
};

static void sha1_init(struct osha1 *s)
{
	s->h[0] = 0x67452301; s->h[1] = 0xefcdab89; s->h[2] = 0x98badcfe;
	s->h[3] = 0x10325476; s->h[4] = 0xc3d2e1f0;
	s->n = 0;
	s->total = 0;
}

static void sha1_update(struct osha1 *s, const uint8_t *p, size_t len)
{
	s->total += len;
	while (len) {
		size_t k = 64 - s->n < len ? 64 - s->n : len;
		memcpy(s->buf + s->n, p, k);
		s->n += k; p += k; len -= k;
		if (s->n == 64) {
			sha1_compress(s->h, s->buf);
			s->n = 0;
		}
	}
}

static void sha1_final(struct osha1 *s, uint8_t md[20])
{
	uint64_t bits = s->total * 8;
	uint8_t pad = 0x80, z = 0, lb[8];
	int i;
	sha1_update(s, &pad, 1);
	while (s->n != 56)
		sha1_update(s, &z, 1);
	for (i = 0; i < 8; i++)
		lb[i] = (uint8_t)(bits >> (56 - 8 * i));
	sha1_update(s, lb, 8);
	for (i = 0; i < 5; i++) {
		md[4 * i] = (uint8_t)(s->h[i] >> 24);
		md[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
		md[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
		md[4 * i + 3] = (uint8_t)s->h[i];
	}
}

void oracle_sha1(const uint8_t *data, size_t len, uint8_t md[20])
{
	struct osha1 s;
	sha1_init(&s);
	sha1_update(&s, data, len);
	sha1_final(&s, md);
}

/* RFC 2104 HMAC (what HMAC(EVP_sha1()) computes, hmac.c:87) */
void oracle_hmac_sha1(const uint8_t *key, size_t key_len, const uint8_t *data,
		      size_t len, uint8_t md[20])
{
	uint8_t k[64] = {0}, pad[64], inner[20];
	struct osha1 s;
	int i;

	if (key_len > 64)
		oracle_sha1(key, key_len, k);
	else
		memcpy(k, key, key_len);
	for (i = 0; i < 64; i++)
		pad[i] = k[i] ^ 0x36;
	sha1_init(&s);
	sha1_update(&s, pad, 64);
	sha1_update(&s, data, len);
	sha1_final(&s, inner);
	for (i = 0; i < 64; i++)
		pad[i] = k[i] ^ 0x5c;
	sha1_init(&s);
	sha1_update(&s, pad, 64);
	sha1_update(&s, inner, 20);
	sha1_final(&s, md);
}

void oracle_aes_ctr(const uint8_t *key, size_t key_bits, const uint8_t iv[16],
		    uint8_t *out, const uint8_t *in, size_t len)
{
	struct ocipher c;
	cipher_init(&c, MODE_CTR, key, key_bits);
	cipher_set_iv(&c, iv);
	cipher_update(&c, out, in, len, 1);
	cipher_free(&c);
}

int oracle_aes_gcm_encrypt(const uint8_t *key, size_t key_bits,
			   const uint8_t iv[12], const uint8_t *aad,
			   size_t aad_len, const uint8_t *in, uint8_t *out,
			   size_t len, uint8_t tag[16])
{
	struct ocipher c;
	cipher_init(&c, MODE_GCM, key, key_bits);
	cipher_set_iv(&c, iv);
	if (aad_len)
		cipher_update(&c, NULL, aad, aad_len, 1);
	if (len)
		cipher_update(&c, out, in, len, 1);
	gcm_tag(&c, tag);
	cipher_free(&c);
	return 0;
}

/* ----------------------------------------------------------- mbuf subset */

uint8_t *oracle_buf_alloc(size_t size) { return calloc(1, size ? size : 1); }
void oracle_buf_free(uint8_t *p) { free(p); }

static size_t left(const struct ombuf *mb)
{
	return mb->end > mb->pos ? mb->end - mb->pos : 0;
}

/* mbuf_write_mem growth: MAX(rsize, size ? 2*size : 512) (mbuf.c:235-260) */
static int mb_write(struct ombuf *mb, const uint8_t *p, size_t n)
{
	size_t rsize = mb->pos + n;
	if (rsize > mb->size) {
		size_t dsize = mb->size ? mb->size * 2 : 512;
		size_t ns = rsize > dsize ? rsize : dsize;
		uint8_t *nb = realloc(mb->buf, ns);
		if (!nb)
			return ENOMEM;
		memset(nb + mb->size, 0, ns - mb->size);
		mb->buf = nb;
		mb->size = ns;
	}
	memcpy(mb->buf + mb->pos, p, n);
	mb->pos += n;
	if (mb->pos > mb->end)
		mb->end = mb->pos;
	return 0;
}

static int mb_write_be32(struct ombuf *mb, uint32_t v)
{
	uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16),
			(uint8_t)(v >> 8), (uint8_t)v};
	return mb_write(mb, b, 4);
}

static uint32_t rd_be32(const uint8_t *p)
{
	return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 |
	       (uint32_t)p[2] << 8 | p[3];
}

/* -------------------------------------------------------- SRTP contexts */

struct oreplay {
	uint64_t bitmap;
	uint64_t lix;
};

struct ostream {                 /* src/srtp/srtp.h:29-38 */
	struct oreplay replay_rtp, replay_rtcp;
	uint32_t ssrc;
	uint32_t roc;
	uint16_t s_l;
	int s_l_set;
	uint32_t rtcp_index;
};

struct ocomp {                   /* src/srtp/srtp.h:42-49 */
	int has_aes;
	struct ocipher aes;
	int mode;
	int has_hmac;
	uint8_t k_a[20];
	uint8_t k_s[16];
	size_t tag_len;
	int encrypted;
};

struct osrtp {
	struct ocomp rtp, rtcp;
	struct ostream streams[8];
	int nstreams;
};

#define SRTP_MAX_STREAMS 8       /* src/srtp/stream.c:16-17 */

/* misc.c:44-73 */
int oracle_srtp_derive(uint8_t *out, size_t out_len, uint8_t label,
		       const uint8_t *master_key, size_t key_bytes,
		       const uint8_t *master_salt, size_t salt_bytes)
{
	static const uint8_t null[32];
	uint8_t x[16] = {0};

	if (!out || !master_key || !master_salt)
		return EINVAL;
	if (out_len > sizeof(null) || salt_bytes > sizeof(x))
		return EINVAL;
	memcpy(x, master_salt, salt_bytes);
	x[7] ^= label;
	oracle_aes_ctr(master_key, key_bytes * 8, x, out, null, out_len);
	return 0;
}

/* srtp.c:33-72 */
static int comp_init(struct ocomp *c, unsigned offs, const uint8_t *key,
		     size_t key_b, const uint8_t *s, size_t s_b, size_t tag_len,
		     int encrypted, int hash, int mode)
{
	uint8_t k_e[32];

	c->tag_len = tag_len;
	c->mode = mode;
	c->encrypted = encrypted;
	oracle_srtp_derive(k_e, key_b, (uint8_t)(0x00 + offs), key, key_b, s,
			   s_b);
	oracle_srtp_derive(c->k_a, 20, (uint8_t)(0x01 + offs), key, key_b, s,
			   s_b);
	oracle_srtp_derive(c->k_s, 14, (uint8_t)(0x02 + offs), key, key_b, s,
			   s_b);
	if (encrypted || mode == MODE_GCM) {
		cipher_init(&c->aes, mode, k_e, key_b * 8);
		c->has_aes = 1;
	}
	c->has_hmac = hash;
	return 0;
}

/* srtp.c:88-180 */
int oracle_srtp_alloc(struct osrtp **pp, int suite, const uint8_t *key,
		      size_t key_bytes, int flags)
{
	size_t cipher_bytes, salt_bytes, auth_bytes;
	int mode, hash;
	struct osrtp *s;

	if (!pp || !key)
		return EINVAL;
	switch (suite) {
	case 1: mode = MODE_CTR; cipher_bytes = 16; salt_bytes = 14;
		auth_bytes = 10; hash = 1; break;
	case 0: mode = MODE_CTR; cipher_bytes = 16; salt_bytes = 14;
		auth_bytes = 4; hash = 1; break;
	case 3: mode = MODE_CTR; cipher_bytes = 32; salt_bytes = 14;
		auth_bytes = 10; hash = 1; break;
	case 2: mode = MODE_CTR; cipher_bytes = 32; salt_bytes = 14;
		auth_bytes = 4; hash = 1; break;
	case 4: mode = MODE_GCM; cipher_bytes = 16; salt_bytes = 12;
		auth_bytes = 0; hash = 0; break;
	case 5: mode = MODE_GCM; cipher_bytes = 32; salt_bytes = 12;
		auth_bytes = 0; hash = 0; break;
	default:
		return ENOTSUP;
	}
	if (cipher_bytes + salt_bytes != key_bytes)
		return EINVAL;
	s = calloc(1, sizeof(*s));
	if (!s)
		return ENOMEM;
	comp_init(&s->rtp, 0, key, cipher_bytes, key + cipher_bytes,
		  salt_bytes, auth_bytes, 1, hash, mode);
	comp_init(&s->rtcp, 3, key, cipher_bytes, key + cipher_bytes,
		  salt_bytes, auth_bytes, !(flags & (1 << 1)), hash, mode);
	*pp = s;
	return 0;
}

void oracle_srtp_free(struct osrtp *s)
{
	if (!s)
		return;
	cipher_free(&s->rtp.aes);
	cipher_free(&s->rtcp.aes);
	free(s);
}

/* misc.c:108-120 */
const char *oracle_srtp_suite_name(int suite)
{
	switch (suite) {
	case 0: return "AES_CM_128_HMAC_SHA1_32";
	case 1: return "AES_CM_128_HMAC_SHA1_80";
	case 2: return "AES_256_CM_HMAC_SHA1_32";
	case 3: return "AES_256_CM_HMAC_SHA1_80";
	case 4: return "AEAD_AES_128_GCM";
	case 5: return "AEAD_AES_256_GCM";
	default: return "?";
	}
}

/* stream.c:29-84 (find or create; 9th SSRC -> ENOSR) */
static int stream_get(struct ostream **sp, struct osrtp *s, uint32_t ssrc)
{
	int i;
	for (i = 0; i < s->nstreams; i++)
		if (s->streams[i].ssrc == ssrc) {
			*sp = &s->streams[i];
			return 0;
		}
	if (s->nstreams >= SRTP_MAX_STREAMS)
		return ENOSR;
	memset(&s->streams[s->nstreams], 0, sizeof(s->streams[0]));
	s->streams[s->nstreams].ssrc = ssrc;
	*sp = &s->streams[s->nstreams++];
	return 0;
}

/* stream.c:87-109 */
static int stream_get_seq(struct ostream **sp, struct osrtp *s, uint32_t ssrc,
			  uint16_t seq)
{
	struct ostream *st;
	int err = stream_get(&st, s, ssrc);
	if (err)
		return err;
	if (!st->s_l_set) {
		st->s_l = seq;
		st->s_l_set = 1;
	}
	*sp = st;
	return 0;
}

/* replay.c:32-62, window 64 */
static int replay_check(struct oreplay *r, uint64_t ix)
{
	uint64_t diff;
	if (ix > r->lix) {
		diff = ix - r->lix;
		if (diff < 64) {
			r->bitmap <<= diff;
			r->bitmap |= 1;
		}
		else
			r->bitmap = 1;
		r->lix = ix;
		return 1;
	}
	diff = r->lix - ix;
	if (diff >= 64)
		return 0;
	if (r->bitmap & (1ULL << diff))
		return 0;
	r->bitmap |= (1ULL << diff);
	return 1;
}

/* misc.c:22-41 -- note `int v` holds roc-1/roc/roc+1 and is widened with
 * sign extension when multiplied by (uint64_t)65536 */
static uint64_t get_index(uint32_t roc, uint16_t s_l, uint16_t seq)
{
	int v;
	if (s_l < 32768) {
		if ((int)seq - (int)s_l > 32768)
			v = (int)((roc - 1) & 0xffffffffu);
		else
			v = (int)roc;
	}
	else {
		if ((int)s_l - 32768 > seq)
			v = (int)((roc + 1) & 0xffffffffu);
		else
			v = (int)roc;
	}
	return seq + (uint64_t)(int64_t)v * (uint64_t)65536;
}

/* misc.c:76-87 */
static void iv_calc(uint8_t iv[16], const uint8_t k_s[16], uint32_t ssrc,
		    uint64_t ix)
{
	uint32_t hi = (uint32_t)(ix >> 16);
	uint16_t lo = (uint16_t)ix;
	memcpy(iv, k_s, 4);
	iv[4] = k_s[4] ^ (uint8_t)(ssrc >> 24);
	iv[5] = k_s[5] ^ (uint8_t)(ssrc >> 16);
	iv[6] = k_s[6] ^ (uint8_t)(ssrc >> 8);
	iv[7] = k_s[7] ^ (uint8_t)ssrc;
	iv[8] = k_s[8] ^ (uint8_t)(hi >> 24);
	iv[9] = k_s[9] ^ (uint8_t)(hi >> 16);
	iv[10] = k_s[10] ^ (uint8_t)(hi >> 8);
	iv[11] = k_s[11] ^ (uint8_t)hi;
	iv[12] = k_s[12] ^ (uint8_t)(lo >> 8);
	iv[13] = k_s[13] ^ (uint8_t)lo;
	iv[14] = 0;
	iv[15] = 0;
}

/* misc.c:93-105 */
static void iv_calc_gcm(uint8_t iv[16], const uint8_t k_s[16], uint32_t ssrc,
			uint64_t ix)
{
	uint16_t w[6];
	int i;
	w[0] = 0;
	w[1] = (uint16_t)(ssrc >> 16);
	w[2] = (uint16_t)(ssrc & 0xffff);
	w[3] = (uint16_t)((ix >> 32) & 0xffff);
	w[4] = (uint16_t)((ix >> 16) & 0xffff);
	w[5] = (uint16_t)(ix & 0xffff);
	for (i = 0; i < 6; i++) {
		iv[2 * i] = k_s[2 * i] ^ (uint8_t)(w[i] >> 8);
		iv[2 * i + 1] = k_s[2 * i + 1] ^ (uint8_t)w[i];
	}
	iv[12] = iv[13] = iv[14] = iv[15] = 0;
}

struct ohdr {
	uint16_t seq;
	uint32_t ssrc;
};

/* rtp.c:88-137 -- including where mb->pos is left on each error */
static int rtp_hdr_decode(struct ohdr *h, struct ombuf *mb)
{
	uint8_t b0;
	unsigned cc, i;
	if (left(mb) < 12)
		return EBADMSG;
	b0 = mb->buf[mb->pos];
	h->seq = (uint16_t)(mb->buf[mb->pos + 2] << 8 | mb->buf[mb->pos + 3]);
	h->ssrc = rd_be32(mb->buf + mb->pos + 8);
	mb->pos += 12;
	cc = b0 & 0x0f;
	if (left(mb) < cc * 4)
		return EBADMSG;
	mb->pos += cc * 4;
	if (b0 & 0x10) {
		unsigned xlen;
		if (left(mb) < 4)
			return EBADMSG;
		xlen = (unsigned)(mb->buf[mb->pos + 2] << 8 | mb->buf[mb->pos + 3]);
		mb->pos += 4;
		if (left(mb) < xlen * 4)
			return EBADMSG;
		mb->pos += xlen * 4;
	}
	(void)i;
	return 0;
}

static void hmac_tag(const struct ocomp *c, const uint8_t *data, size_t len,
		     uint8_t md[20])
{
	oracle_hmac_sha1(c->k_a, 20, data, len, md);
}

/* srtp.c:183-285 */
int oracle_srtp_encrypt(struct osrtp *s, struct ombuf *mb)
{
	struct ostream *strm;
	struct ohdr hdr;
	struct ocomp *comp;
	size_t start;
	uint64_t ix;
	int err;

	if (!s || !mb)
		return EINVAL;
	comp = &s->rtp;
	start = mb->pos;
	err = rtp_hdr_decode(&hdr, mb);
	if (err)
		return err;
	err = stream_get_seq(&strm, s, hdr.ssrc, hdr.seq);
	if (err)
		return err;
	if ((int)hdr.seq - (int)strm->s_l <= -32768) {
		strm->roc++;
		strm->s_l = 0;
	}
	ix = 65536ULL * strm->roc + hdr.seq;

	if (comp->has_aes && comp->mode == MODE_CTR) {
		uint8_t iv[16];
		uint8_t *p = mb->buf + mb->pos;
		iv_calc(iv, comp->k_s, strm->ssrc, ix);
		cipher_set_iv(&comp->aes, iv);
		cipher_update(&comp->aes, p, p, left(mb), 1);
	}
	else if (comp->has_aes && comp->mode == MODE_GCM) {
		uint8_t iv[16], tag[16];
		uint8_t *p = mb->buf + mb->pos;
		iv_calc_gcm(iv, comp->k_s, strm->ssrc, ix);
		cipher_set_iv(&comp->aes, iv);
		cipher_update(&comp->aes, NULL, mb->buf + start,
			      mb->pos - start, 1);
		cipher_update(&comp->aes, p, p, left(mb), 1);
		gcm_tag(&comp->aes, tag);
		mb->pos = mb->end;
		err = mb_write(mb, tag, 16);
		if (err)
			return err;
	}

	if (comp->has_hmac) {
		const size_t tag_start = mb->end;
		uint8_t tag[20];
		mb->pos = tag_start;
		err = mb_write_be32(mb, strm->roc);
		if (err)
			return err;
		mb->pos = start;
		hmac_tag(comp, mb->buf + mb->pos, left(mb), tag);
		mb->pos = mb->end = tag_start;
		err = mb_write(mb, tag, comp->tag_len);
		if (err)
			return err;
	}

	if (hdr.seq > strm->s_l)
		strm->s_l = hdr.seq;
	mb->pos = start;
	return 0;
}

/* srtp.c:288-432 */
int oracle_srtp_decrypt(struct osrtp *s, struct ombuf *mb)
{
	struct ostream *strm;
	struct ohdr hdr;
	struct ocomp *comp;
	uint64_t ix;
	size_t start;
	int diff, err;

	if (!s || !mb)
		return EINVAL;
	comp = &s->rtp;
	start = mb->pos;
	err = rtp_hdr_decode(&hdr, mb);
	if (err)
		return err;
	err = stream_get_seq(&strm, s, hdr.ssrc, hdr.seq);
	if (err)
		return err;
	diff = (int)hdr.seq - (int)strm->s_l;
	if (diff > 32768)
		return ETIMEDOUT;
	if (diff <= -32768) {
		strm->roc++;
		strm->s_l = 0;
	}
	ix = get_index(strm->roc, strm->s_l, hdr.seq);

	if (comp->has_hmac) {
		uint8_t tag_calc[20], tag_pkt[20];
		size_t pld_start, tag_start;

		if (left(mb) < comp->tag_len)
			return EBADMSG;
		pld_start = mb->pos;
		tag_start = mb->end - comp->tag_len;
		memcpy(tag_pkt, mb->buf + tag_start, comp->tag_len);
		mb->pos = mb->end = tag_start;
		err = mb_write_be32(mb, strm->roc);
		if (err)
			return err;
		mb->pos = start;
		hmac_tag(comp, mb->buf + mb->pos, left(mb), tag_calc);
		mb->pos = pld_start;
		mb->end = tag_start;
		if (memcmp(tag_calc, tag_pkt, comp->tag_len))
			return EAUTH;
		if (!replay_check(&strm->replay_rtp, ix))
			return EALREADY;
	}

	if (comp->has_aes && comp->mode == MODE_CTR) {
		uint8_t iv[16];
		uint8_t *p = mb->buf + mb->pos;
		iv_calc(iv, comp->k_s, strm->ssrc, ix);
		cipher_set_iv(&comp->aes, iv);
		cipher_update(&comp->aes, p, p, left(mb), 0);
	}
	else if (comp->has_aes && comp->mode == MODE_GCM) {
		uint8_t iv[16], tag[16];
		uint8_t *p = mb->buf + mb->pos;
		size_t tag_start;

		iv_calc_gcm(iv, comp->k_s, strm->ssrc, ix);
		cipher_set_iv(&comp->aes, iv);
		cipher_update(&comp->aes, NULL, mb->buf + start,
			      mb->pos - start, 0);
		if (left(mb) < 16)
			return EBADMSG;
		tag_start = mb->end - 16;
		cipher_update(&comp->aes, p, p, tag_start - mb->pos, 0);
		gcm_tag(&comp->aes, tag);
		if (memcmp(tag, mb->buf + tag_start, 16))
			return EAUTH;
		mb->end = tag_start;
		if (!replay_check(&strm->replay_rtp, ix))
			return EALREADY;
	}

	if (hdr.seq > strm->s_l)
		strm->s_l = hdr.seq;
	mb->pos = start;
	return 0;
}

/* srtcp.c:19-28 */
static int get_rtcp_ssrc(uint32_t *ssrc, struct ombuf *mb)
{
	if (left(mb) < 8)
		return EBADMSG;
	mb->pos += 4;
	*ssrc = rd_be32(mb->buf + mb->pos);
	mb->pos += 4;
	return 0;
}

/* srtcp.c:31-140 */
int oracle_srtcp_encrypt(struct osrtp *s, struct ombuf *mb)
{
	struct ostream *strm;
	struct ocomp *rtcp;
	uint32_t ssrc, ep = 0;
	size_t start;
	int err;

	if (!s || !mb)
		return EINVAL;
	rtcp = &s->rtcp;
	start = mb->pos;
	err = get_rtcp_ssrc(&ssrc, mb);
	if (err)
		return err;
	err = stream_get(&strm, s, ssrc);
	if (err)
		return err;
	strm->rtcp_index = (strm->rtcp_index + 1) & 0x7fffffff;

	if (rtcp->has_aes && rtcp->mode == MODE_CTR) {
		uint8_t iv[16];
		uint8_t *p = mb->buf + mb->pos;
		iv_calc(iv, rtcp->k_s, ssrc, strm->rtcp_index);
		cipher_set_iv(&rtcp->aes, iv);
		cipher_update(&rtcp->aes, p, p, left(mb), 1);
		ep = 1;
	}
	else if (rtcp->has_aes && rtcp->mode == MODE_GCM) {
		uint8_t iv[16], tag[16], ixb[4];
		uint8_t *p = mb->buf + mb->pos;
		uint32_t v;
		ep = rtcp->encrypted ? 1 : 0;
		v = ep << 31 | strm->rtcp_index;
		ixb[0] = (uint8_t)(v >> 24); ixb[1] = (uint8_t)(v >> 16);
		ixb[2] = (uint8_t)(v >> 8); ixb[3] = (uint8_t)v;
		iv_calc_gcm(iv, rtcp->k_s, ssrc, strm->rtcp_index);
		cipher_set_iv(&rtcp->aes, iv);
		cipher_update(&rtcp->aes, NULL, mb->buf + start,
			      mb->pos - start, 1);
		if (rtcp->encrypted) {
			cipher_update(&rtcp->aes, NULL, ixb, 4, 1);
			cipher_update(&rtcp->aes, p, p, left(mb), 1);
		}
		else {
			cipher_update(&rtcp->aes, NULL, p, left(mb), 1);
			cipher_update(&rtcp->aes, NULL, ixb, 4, 1);
		}
		gcm_tag(&rtcp->aes, tag);
		mb->pos = mb->end;
		err = mb_write(mb, tag, 16);
		if (err)
			return err;
	}

	mb->pos = mb->end;
	err = mb_write_be32(mb, ep << 31 | strm->rtcp_index);
	if (err)
		return err;

	if (rtcp->has_hmac) {
		uint8_t tag[20];
		mb->pos = start;
		hmac_tag(rtcp, mb->buf + mb->pos, left(mb), tag);
		mb->pos = mb->end;
		err = mb_write(mb, tag, rtcp->tag_len);
		if (err)
			return err;
	}
	mb->pos = start;
	return 0;
}

/* srtcp.c:143-287 */
int oracle_srtcp_decrypt(struct osrtp *s, struct ombuf *mb)
{
	size_t start, eix_start, pld_start;
	struct ostream *strm;
	struct ocomp *rtcp;
	uint32_t v, ix, ssrc;
	int ep, err;

	if (!s || !mb)
		return EINVAL;
	rtcp = &s->rtcp;
	start = mb->pos;
	err = get_rtcp_ssrc(&ssrc, mb);
	if (err)
		return err;
	err = stream_get(&strm, s, ssrc);
	if (err)
		return err;
	pld_start = mb->pos;
	if (left(mb) < 4 + rtcp->tag_len)
		return EBADMSG;
	eix_start = mb->end - (4 + rtcp->tag_len);
	mb->pos = eix_start;
	v = rd_be32(mb->buf + mb->pos);
	mb->pos += 4;
	ep = (v >> 31) & 1;
	ix = v & 0x7fffffff;

	if (rtcp->has_hmac) {
		uint8_t tag[20], tag_pkt[20];
		const size_t tag_start = mb->pos;
		memcpy(tag_pkt, mb->buf + mb->pos, rtcp->tag_len);
		mb->pos += rtcp->tag_len;
		mb->pos = start;
		mb->end = tag_start;
		hmac_tag(rtcp, mb->buf + mb->pos, left(mb), tag);
		if (memcmp(tag, tag_pkt, rtcp->tag_len))
			return EAUTH;
		if (!replay_check(&strm->replay_rtcp, ix))
			return EALREADY;
	}

	mb->end = eix_start;

	if (rtcp->has_aes && ep && rtcp->mode == MODE_CTR) {
		uint8_t iv[16];
		uint8_t *p;
		mb->pos = pld_start;
		p = mb->buf + mb->pos;
		iv_calc(iv, rtcp->k_s, ssrc, ix);
		cipher_set_iv(&rtcp->aes, iv);
		cipher_update(&rtcp->aes, p, p, left(mb), 0);
	}
	else if (rtcp->has_aes && rtcp->mode == MODE_GCM) {
		uint8_t iv[16], tag[16];
		size_t tag_start;
		uint8_t *p;

		iv_calc_gcm(iv, rtcp->k_s, ssrc, ix);
		cipher_set_iv(&rtcp->aes, iv);
		cipher_update(&rtcp->aes, NULL, mb->buf + start,
			      pld_start - start, 0);
		mb->pos = pld_start;
		p = mb->buf + mb->pos;
		if (left(mb) < 16)
			return EBADMSG;
		tag_start = mb->end - 16;
		if (ep) {
			cipher_update(&rtcp->aes, NULL, mb->buf + eix_start, 4,
				      0);
			cipher_update(&rtcp->aes, p, p, tag_start - pld_start,
				      0);
		}
		else {
			cipher_update(&rtcp->aes, NULL, p,
				      tag_start - pld_start, 0);
			cipher_update(&rtcp->aes, NULL, mb->buf + eix_start, 4,
				      0);
		}
		gcm_tag(&rtcp->aes, tag);
		if (memcmp(tag, mb->buf + tag_start, 16))
			return EAUTH;
		mb->end = tag_start;
	}
	mb->pos = start;
	return 0;
}

/* ------------------------------------------------------- bench helper */

long oracle_bench_pairs(int suite, size_t len, long n)
{
	static const size_t kl[6] = {30, 30, 46, 46, 28, 44};
	uint8_t key[46];
	struct osrtp *tx = NULL, *rx = NULL;
	struct ombuf mb;
	long i, ok = 0;
	size_t b;

	for (b = 0; b < sizeof(key); b++)
		key[b] = (uint8_t)(b * 37 + 11);
	if (oracle_srtp_alloc(&tx, suite, key, kl[suite], 0) ||
	    oracle_srtp_alloc(&rx, suite, key, kl[suite], 0))
		return -1;
	mb.size = len + 64;
	mb.buf = calloc(1, mb.size);
	for (i = 0; i < n; i++) {
		uint16_t seq = (uint16_t)(65000 + i);
		mb.buf[0] = 0x80;
		mb.buf[2] = (uint8_t)(seq >> 8);
		mb.buf[3] = (uint8_t)seq;
		mb.buf[8] = 1; mb.buf[9] = 2; mb.buf[10] = 3; mb.buf[11] = 4;
		for (b = 12; b < len; b++)
			mb.buf[b] = (uint8_t)(b + (size_t)i);
		mb.pos = 0;
		mb.end = len;
		if (oracle_srtp_encrypt(tx, &mb))
			continue;
		mb.pos = 0;
		if (!oracle_srtp_decrypt(rx, &mb))
			ok++;
	}
	free(mb.buf);
	oracle_srtp_free(tx);
	oracle_srtp_free(rx);
	return ok;
}

/* stream state of ssrc (test helper: the state the reference keeps in
 * struct srtp_stream, src/srtp/srtp.h:29-38); -1 if no such stream */
int oracle_stream_state(const struct osrtp *s, uint32_t ssrc, uint32_t *roc,
			uint32_t *s_l, uint64_t *lix, uint64_t *bitmap)
{
	int i;
	for (i = 0; i < s->nstreams; i++) {
		const struct ostream *st = &s->streams[i];
		if (st->ssrc != ssrc)
			continue;
		*roc = st->roc;
		*s_l = st->s_l;
		*lix = st->replay_rtp.lix;
		*bitmap = st->replay_rtp.bitmap;
		return 0;
	}
	return -1;
}

/* test hook: set (or create) ssrc's receiver state -- a rank that starts
 * its shard from an assumed boundary state (tests/test_rxfold_cpu.py) */
int oracle_stream_set(struct osrtp *s, uint32_t ssrc, uint32_t roc,
		      uint32_t s_l, uint32_t s_l_set, uint64_t lix,
		      uint64_t bitmap)
{
	struct ostream *st;
	int err = stream_get(&st, s, ssrc);
	if (err)
		return err;
	st->roc = roc;
	st->s_l = (uint16_t)s_l;
	st->s_l_set = (uint8_t)s_l_set;
	st->replay_rtp.lix = lix;
	st->replay_rtp.bitmap = bitmap;
	return 0;
}
