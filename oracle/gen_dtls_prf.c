/*
 * gen_dtls_prf.c -- DTLS-SRTP keying golden vectors (TEST INFRASTRUCTURE).
 *
 * libre's tls_srtp_keyinfo() (src/tls/openssl/tls.c:1083-1157) asks OpenSSL
 * for SSL_export_keying_material(ssl, keymat, 2 * (key + salt),
 * "EXTRACTOR-dtls_srtp", no context) and splits keymat as
 *   client key | server key | client salt | server salt.
 * For (D)TLS 1.2 OpenSSL's exporter is the TLS 1.2 PRF (RFC 5246 5) over
 * the master secret with seed = label || client_random || server_random
 * (RFC 5705 4; ssl/t1_enc.c tls1_export_keying_material), P_<hash> with
 * the negotiated suite's handshake digest: SHA-256, or SHA-384 for the
 * *_SHA384 suites (cases with "prf":1).
 * This program evaluates that PRF with OpenSSL's own implementation
 * (EVP_PKEY_TLS1_PRF, the image's libcrypto) on deterministic inputs and
 * prints the inputs, the keying material and the split keys as JSON
 * (tests/golden/dtls_srtp_keying.json, scripts/make_dtls_golden.sh).
 */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <openssl/evp.h>
#include <openssl/kdf.h>
#include <openssl/opensslv.h>

static uint64_t s = 0xD715D715ull;

static uint8_t rnd8(void)
{
	s ^= s >> 12;
	s ^= s << 25;
	s ^= s >> 27;
	return (uint8_t)((s * 0x2545F4914F6CDD1Dull) >> 56);
}

static void hex(const char *k, const uint8_t *p, size_t n, int comma)
{
	size_t i;
	printf("\"%s\":\"", k);
	for (i = 0; i < n; i++)
		printf("%02x", p[i]);
	printf("\"%s", comma ? "," : "");
}

static int prf(const EVP_MD *md, const uint8_t *secret, size_t slen,
	       const uint8_t *seed, size_t seedlen, uint8_t *out,
	       size_t outlen)
{
	EVP_PKEY_CTX *pc = EVP_PKEY_CTX_new_id(EVP_PKEY_TLS1_PRF, NULL);
	int ok = pc && EVP_PKEY_derive_init(pc) > 0 &&
		 EVP_PKEY_CTX_set_tls1_prf_md(pc, md) > 0 &&
		 EVP_PKEY_CTX_set1_tls1_prf_secret(pc, secret, (int)slen) > 0 &&
		 EVP_PKEY_CTX_add1_tls1_prf_seed(pc, seed, (int)seedlen) > 0 &&
		 EVP_PKEY_derive(pc, out, &outlen) > 0;
	EVP_PKEY_CTX_free(pc);
	return ok ? 0 : -1;
}

int main(void)
{
	/* the four profiles tls_srtp_keyinfo maps (tls.c:1101-1132) */
	static const struct { int suite; const char *profile;
			      size_t key, salt; } P[4] = {
		{1, "SRTP_AES128_CM_SHA1_80", 16, 14},
		{0, "SRTP_AES128_CM_SHA1_32", 16, 14},
		{4, "SRTP_AEAD_AES_128_GCM", 16, 12},
		{5, "SRTP_AEAD_AES_256_GCM", 32, 12},
	};
	static const char label[] = "EXTRACTOR-dtls_srtp";
	int p, c, h, first = 1;

	printf("{\"generator\":\"oracle/gen_dtls_prf.c (%s EVP_PKEY_TLS1_PRF, "
	       "SHA-256 and SHA-384)\",\"label\":\"%s\",\"cases\":[\n",
	       OPENSSL_VERSION_TEXT, label);
	for (h = 0; h < 2; h++)
	for (p = 0; p < 4; p++) {
		for (c = 0; c < 8; c++) {
			uint8_t ms[48], cr[32], sr[32], seed[128], km[256];
			uint8_t cli[64], srv[64];
			const size_t size = P[p].key + P[p].salt;
			size_t i, sl = 0;
			for (i = 0; i < 48; i++) ms[i] = rnd8();
			for (i = 0; i < 32; i++) cr[i] = rnd8();
			for (i = 0; i < 32; i++) sr[i] = rnd8();
			memcpy(seed, label, strlen(label));
			sl = strlen(label);
			memcpy(seed + sl, cr, 32); sl += 32;
			memcpy(seed + sl, sr, 32); sl += 32;
			if (prf(h ? EVP_sha384() : EVP_sha256(), ms, 48, seed,
				sl, km, 2 * size)) {
				fprintf(stderr, "PRF failed\n");
				return 1;
			}
			/* the split of tls.c:1149-1154 */
			memcpy(cli, km, P[p].key);
			memcpy(srv, km + P[p].key, P[p].key);
			memcpy(cli + P[p].key, km + 2 * P[p].key, P[p].salt);
			memcpy(srv + P[p].key, km + 2 * P[p].key + P[p].salt,
			       P[p].salt);
			printf("%s{\"suite\":%d,\"profile\":\"%s\",\"prf\":%d,",
			       first ? "" : ",\n", P[p].suite, P[p].profile, h);
			first = 0;
			hex("master", ms, 48, 1);
			hex("client_random", cr, 32, 1);
			hex("server_random", sr, 32, 1);
			hex("keymat", km, 2 * size, 1);
			hex("cli_key", cli, size, 1);
			hex("srv_key", srv, size, 0);
			printf("}");
		}
	}
	printf("\n]}\n");
	return 0;
}
