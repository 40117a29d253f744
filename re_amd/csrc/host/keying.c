/*
 * keying.c -- DTLS-SRTP keying (include/re_srtp_keying.h): the split of
 * tls_srtp_keyinfo (src/tls/openssl/tls.c:1083-1157) on the host, the
 * exporter PRF for a batch of connections on the GPU (dtls_prf.hip).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include "re_mem.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"
#include "re_srtp_keying.h"
#include "../srtpgpu.h"
#include "fault.h"

/* the profiles tls_srtp_keyinfo maps (tls.c:1101-1132) */
static int profile(enum srtp_suite suite, size_t *key, size_t *salt)
{
	switch (suite) {
	case SRTP_AES_CM_128_HMAC_SHA1_80:
	case SRTP_AES_CM_128_HMAC_SHA1_32:
		*key = 16; *salt = 14; return 0;
	case SRTP_AES_128_GCM:
		*key = 16; *salt = 12; return 0;
	case SRTP_AES_256_GCM:
		*key = 32; *salt = 12; return 0;
	default:
		return ENOSYS;
	}
}

size_t srtp_dtls_key_size(enum srtp_suite suite)
{
	size_t k, s;
	return profile(suite, &k, &s) ? 0 : k + s;
}

int srtp_keyinfo_split(enum srtp_suite suite, const uint8_t *keymat,
		       uint8_t *cli_key, size_t cli_key_size,
		       uint8_t *srv_key, size_t srv_key_size)
{
	size_t key, salt;
	const uint8_t *p = keymat;
	int err;

	if (!keymat || !cli_key || !srv_key)
		return EINVAL;
	err = profile(suite, &key, &salt);
	if (err)
		return err;
	if (cli_key_size < key + salt || srv_key_size < key + salt)
		return EOVERFLOW;
	memcpy(cli_key, p, key);           p += key;
	memcpy(srv_key, p, key);           p += key;
	memcpy(cli_key + key, p, salt);    p += salt;
	memcpy(srv_key + key, p, salt);
	return 0;
}

int sgpu_dtls_prf(const uint8_t *in, uint32_t n, uint32_t stride,
		  uint32_t outlen, uint8_t *out);

int srtp_dtls_keying_many(const struct srtp_dtls_secret *sec, size_t n,
			  enum srtp_suite suite, uint8_t *cli_keys,
			  uint8_t *srv_keys)
{
	const size_t size = srtp_dtls_key_size(suite);
	uint8_t *km;
	size_t i;
	int err;

	if (!sec || !cli_keys || !srv_keys || n > UINT32_MAX / 256)
		return EINVAL;
	if (!size)
		return ENOSYS;
	if (!n)
		return 0;
	for (i = 0; i < n; i++)
		if (sec[i].prf != SRTP_DTLS_PRF_SHA256 &&
		    sec[i].prf != SRTP_DTLS_PRF_SHA384)
			return EINVAL;
	km = fi_malloc(n * 2 * size);
	if (!km)
		return ENOMEM;
	err = sgpu_dtls_prf((const uint8_t *)sec, (uint32_t)n,
			    (uint32_t)sizeof(*sec), (uint32_t)(2 * size), km);
	for (i = 0; !err && i < n; i++)
		err = srtp_keyinfo_split(suite, km + i * 2 * size,
					 cli_keys + i * size, size,
					 srv_keys + i * size, size);
	memset(km, 0, n * 2 * size);       /* mem_secclean in tls.c:1156 */
	free(km);
	return err;
}

int srtp_alloc_dtls_many(struct srtp **txv, struct srtp **rxv, size_t n,
			 enum srtp_suite suite,
			 const struct srtp_dtls_secret *sec, int is_client,
			 int flags)
{
	const size_t size = srtp_dtls_key_size(suite);
	uint8_t *cli, *srv;
	int err;

	if (!txv || !rxv || !sec)
		return EINVAL;
	if (!size)
		return ENOSYS;
	cli = fi_malloc((n ? n : 1) * size);
	srv = fi_malloc((n ? n : 1) * size);
	if (!cli || !srv) {
		err = ENOMEM;
		goto out;
	}
	err = srtp_dtls_keying_many(sec, n, suite, cli, srv);
	if (!err)
		err = srtp_alloc_many(txv, n, suite, is_client ? cli : srv,
				      size, flags);
	if (!err) {
		err = srtp_alloc_many(rxv, n, suite, is_client ? srv : cli,
				      size, flags);
		if (err) {
			size_t i;
			for (i = 0; i < n; i++)
				txv[i] = mem_deref(txv[i]);
		}
	}
 out:
	if (cli)
		memset(cli, 0, (n ? n : 1) * size);
	if (srv)
		memset(srv, 0, (n ? n : 1) * size);
	free(cli);
	free(srv);
	return err;
}
