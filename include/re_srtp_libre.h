/**
 * @file re_srtp_libre.h  The batched GPU SRTP transform as a libre UDP
 * helper (extension; LIBRE=1 builds only -- libre_srtp_amd_libre.so,
 * linked into libre).
 *
 * Registers on a libre struct udp_sock with udp_register_helper()
 * (include/re_udp.h:55-66, src/udp/udp.c:830-860), where an SRTP media
 * transform sits.  Its hooks queue each datagram udp_read() delivers
 * (src/udp/udp.c:149-211) and each one udp_send() sends (:484-507, :539)
 * and unprotect / protect the queue in one GPU batch when `batch` are
 * queued or `flush_ms` after the first (a libre timer: inside re_main).
 * Then every packet continues down the chain with udp_recv_helper() /
 * udp_send_helper() (:874-928): the helpers below, then the socket's
 * receive handler or sendto().  Bytes, pos/end and stream states are those
 * of srtp_decrypt() / srtp_encrypt() in datagram order; a datagram that
 * fails to unprotect is dropped and counted.  rtcp-mux sockets work: a
 * datagram whose payload type is RTCP's (rtp_pt_is_rtcp(), include/
 * re_rtp.h:333, as src/rtp/rtp.c:184-196 demultiplexes) takes the SRTCP
 * transform, srtcp_decrypt() / srtcp_encrypt().  Deviation: udp_send()
 * returns 0 when the packet is queued; a later failure is counted, not
 * returned.
 */
#ifndef RE_SRTP_LIBRE_H
#define RE_SRTP_LIBRE_H

#include <stddef.h>
#include <stdint.h>
#include "re_srtp.h"

#ifdef __cplusplus
extern "C" {
#endif

struct udp_sock;
struct srtp_udp_helper;

/**
 * Register on us at `layer` (libre helper layer, lower runs first on
 * receive).  rx / tx: the unprotect / protect contexts (either may be
 * NULL: that direction passes through).  batch: datagrams per GPU call;
 * slot: bytes per queued datagram (larger ones take the per-packet call,
 * in order); flush_ms: longest a queued datagram waits.  Freed (and
 * unregistered) with mem_deref().  0 or EINVAL / ENOMEM / ENOSYS.
 */
int srtp_udp_helper_alloc(struct srtp_udp_helper **hp, struct udp_sock *us,
			  int layer, struct srtp *rx, struct srtp *tx,
			  size_t batch, size_t slot, unsigned flush_ms);

/** run the queued datagrams now (send queue first) */
void srtp_udp_helper_flush(struct srtp_udp_helper *h);

/** counters: received / unprotected ok / sent / dropped */
void srtp_udp_helper_stats(const struct srtp_udp_helper *h, uint64_t *rx,
			   uint64_t *rx_ok, uint64_t *tx, uint64_t *dropped);

#ifdef __cplusplus
}
#endif

#endif
