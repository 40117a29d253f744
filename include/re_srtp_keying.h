/**
 * @file re_srtp_keying.h  DTLS-SRTP keying for SRTP contexts (extension).
 *
 * libre's tls_srtp_keyinfo() (src/tls/openssl/tls.c:1083-1157) exports
 * 2 * (key + salt) bytes of keying material per DTLS connection with the
 * label "EXTRACTOR-dtls_srtp" and splits them as
 *   client key | server key | client salt | server salt
 * into the client and server master key||salt that srtp_alloc() takes.
 * These functions do the same for many connections at once: the exporter
 * (RFC 5705 with the (D)TLS 1.2 PRF, RFC 5246 5) runs on the GPU, and the
 * contexts are set up by the batched srtp_alloc_many().
 *
 * The (D)TLS 1.2 PRF hash is the negotiated cipher suite's: P_SHA256 for
 * most suites, P_SHA384 for the *_SHA384 ones (RFC 5246 5, RFC 5289 3;
 * OpenSSL's default cipher list, which libre uses unless tls_set_ciphers
 * is called, tls.c:1185-1209, ranks ECDHE-*-AES256-GCM-SHA384 first).
 * Each connection names its own in srtp_dtls_secret.prf (what
 * SSL_CIPHER_get_handshake_digest() of the session's cipher gives).
 */
#ifndef RE_SRTP_KEYING_H
#define RE_SRTP_KEYING_H

#include "re_srtp.h"

#ifdef __cplusplus
extern "C" {
#endif

/** PRF hash of a (D)TLS 1.2 connection */
enum srtp_dtls_prf {
	SRTP_DTLS_PRF_SHA256 = 0,   /**< default (zero-initialised) */
	SRTP_DTLS_PRF_SHA384 = 1,   /**< the *_SHA384 cipher suites */
};

/** the DTLS 1.2 secrets of one connection (SSL_SESSION master key and the
 *  handshake randoms) and its PRF hash (enum srtp_dtls_prf; another value
 *  makes the call fail with EINVAL) */
struct srtp_dtls_secret {
	uint8_t master[48];
	uint8_t client_random[32];
	uint8_t server_random[32];
	uint32_t prf;
};

/** key + salt bytes of a suite (the key_bytes srtp_alloc takes); 0 for a
 *  suite DTLS-SRTP has no profile for (tls.c:1101-1132 maps 4 of 6) */
size_t srtp_dtls_key_size(enum srtp_suite suite);

/**
 * The split step of tls_srtp_keyinfo (tls.c:1140-1154): keymat holds
 * 2 * srtp_dtls_key_size(suite) exported bytes.  EINVAL, ENOSYS (suite
 * without a DTLS-SRTP profile), EOVERFLOW (an output too small) or 0.
 */
int srtp_keyinfo_split(enum srtp_suite suite, const uint8_t *keymat,
		       uint8_t *cli_key, size_t cli_key_size,
		       uint8_t *srv_key, size_t srv_key_size);

/**
 * n connections' keying material on the GPU, split like tls_srtp_keyinfo:
 * cli_keys / srv_keys receive n * srtp_dtls_key_size(suite) bytes.
 */
int srtp_dtls_keying_many(const struct srtp_dtls_secret *sec, size_t n,
			  enum srtp_suite suite, uint8_t *cli_keys,
			  uint8_t *srv_keys);

/**
 * Keying and contexts for n DTLS-SRTP endpoints: txv[i] protects with
 * this side's key (the client key if is_client), rxv[i] unprotects with
 * the peer's.  Freed with mem_deref() each.
 */
int srtp_alloc_dtls_many(struct srtp **txv, struct srtp **rxv, size_t n,
			 enum srtp_suite suite,
			 const struct srtp_dtls_secret *sec, int is_client,
			 int flags);

#ifdef __cplusplus
}
#endif

#endif
