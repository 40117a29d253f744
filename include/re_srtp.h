/**
 * @file re_srtp.h  Secure Real-time Transport Protocol (SRTP) -- drop-in
 *
 * MI355X-native replacement for libre's src/srtp.  The six declarations
 * below are the reference interface, unchanged
 * (baresip/re v4.10.0 include/re_srtp.h:8-30): same enum values, same
 * signatures, same ownership (struct srtp is allocated with mem_zalloc and
 * released with mem_deref) and the same errno results, bit-exact outputs.
 *
 * Each call replaces:
 *   srtp_alloc       src/srtp/srtp.c:88-180   (KDF + key schedule run on GPU)
 *   srtp_encrypt     src/srtp/srtp.c:183-285
 *   srtp_decrypt     src/srtp/srtp.c:288-432
 *   srtcp_encrypt    src/srtp/srtcp.c:31-140
 *   srtcp_decrypt    src/srtp/srtcp.c:143-287
 *   srtp_suite_name  src/srtp/misc.c:108-120
 *
 * Without a usable HIP device srtp_alloc() returns ENOSYS, exactly like the
 * reference's crypto-less stub backend (src/aes/stub.c); there is no CPU
 * fallback.  The batched extension lives in re_srtp_batch.h.
 */
#ifndef RE_SRTP_H
#define RE_SRTP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct mbuf;

enum srtp_suite {
	SRTP_AES_CM_128_HMAC_SHA1_32,
	SRTP_AES_CM_128_HMAC_SHA1_80,
	SRTP_AES_256_CM_HMAC_SHA1_32,
	SRTP_AES_256_CM_HMAC_SHA1_80,
	SRTP_AES_128_GCM,
	SRTP_AES_256_GCM,
};

enum srtp_flags {
	SRTP_UNENCRYPTED_SRTCP = 1<<1,
};

struct srtp;

int srtp_alloc(struct srtp **srtpp, enum srtp_suite suite,
	       const uint8_t *key, size_t key_bytes, int flags);
int srtp_encrypt(struct srtp *srtp, struct mbuf *mb);
int srtp_decrypt(struct srtp *srtp, struct mbuf *mb);
int srtcp_encrypt(struct srtp *srtp, struct mbuf *mb);
int srtcp_decrypt(struct srtp *srtp, struct mbuf *mb);

const char *srtp_suite_name(enum srtp_suite suite);

#ifdef __cplusplus
}
#endif

#endif
