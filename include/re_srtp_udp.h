/**
 * @file re_srtp_udp.h  Batched SRTP UDP helper (extension, no reference
 * counterpart beyond the helper hooks it replaces).
 *
 * In libre the SRTP transform sits in the UDP helper chain
 * (udp_register_helper, include/re_udp.h:55-71): udp_read() receives ONE
 * datagram into a new mbuf (src/udp/udp.c:149-211) and the helper's recv
 * hook calls srtp_decrypt() on it; udp_send_internal() runs the send hooks
 * (src/udp/udp.c:484-507), which call srtp_encrypt(), then sendto().
 *
 * struct srtp_udp is that helper for the GPU: it receives up to `batch`
 * datagrams with one recvmmsg() straight into a pinned host arena,
 * unprotects them in one srtp_decrypt_batch_dev() call and hands every
 * packet to the receive handler; the send side protects a batch of mbufs
 * with srtp_encrypt_batch_dev() and sends it with one sendmmsg().  Per
 * packet the results are exactly those of srtp_decrypt()/srtp_encrypt()
 * called in datagram order (re_srtp_batch.h semantics).
 */
#ifndef RE_SRTP_UDP_H
#define RE_SRTP_UDP_H

#include <sys/socket.h>
#include "re_srtp.h"

#ifdef __cplusplus
extern "C" {
#endif

struct srtp_udp;

/**
 * Receive handler, once per datagram in arrival order (udp_recv_h,
 * include/re_udp.h:21 plus the srtp_decrypt() result).  mb views the
 * pinned receive arena: [mb->pos, mb->end) is the unprotected RTP packet
 * when err == 0, or what srtp_decrypt() left on error.  Valid only during
 * the call: copy to keep.  err is srtp_decrypt()'s errno, or EMSGSIZE for
 * a datagram truncated to the slot size.
 */
typedef void (srtp_udp_recv_h)(const struct sockaddr_storage *src,
			       socklen_t srclen, struct mbuf *mb, int err,
			       void *arg);

/**
 * fd: a bound UDP socket (not owned).  rx / tx: the receive / send SRTP
 * contexts (either may be NULL; they may be the same context, as one
 * struct srtp may serve both directions).  batch: datagrams per
 * recvmmsg/sendmmsg and GPU call.  slot: bytes reserved per datagram
 * (>= largest datagram + tag; rounded up to 16).
 * Freed with mem_deref().  0 or an errno (ENOSYS without a HIP device).
 */
int srtp_udp_alloc(struct srtp_udp **sup, int fd, struct srtp *rx,
		   struct srtp *tx, size_t batch, size_t slot,
		   srtp_udp_recv_h *rh, void *arg);

/**
 * One receive round: recvmmsg() of up to `batch` datagrams (waiting at
 * most timeout_ms for the first, then taking what is queued), one GPU
 * unprotect of all of them, the handler per datagram.  Returns the number
 * of datagrams handled (0 on timeout) or -errno.
 *
 * Pipelined (srtp_udp_pipeline): the round's batch is queued on the GPU
 * and the previous round's batch is completed and handed to the handler
 * -- batch k+1 is read from the socket while the GPU unprotects batch k.
 * A round that receives nothing (timeout) hands over the batch in flight;
 * handler calls keep datagram order.
 */
int srtp_udp_recv(struct srtp_udp *su, int timeout_ms);

/**
 * Pipelining on (on != 0) or off (default) for both directions: two
 * arenas per direction, asynchronous batch calls (re_srtp_batch.h).
 * EBUSY while a received batch is still in flight (srtp_udp_recv until it
 * returns 0 first).
 */
int srtp_udp_pipeline(struct srtp_udp *su, int on);

/**
 * Protect mbv[0..n) (one GPU call per `batch` of them) and send each to
 * dst with sendmmsg().  The mbufs are not modified (the protected bytes
 * live in the send arena).  errv (optional): per packet srtp_encrypt()'s
 * errno -- packets with an error are not sent.  Every mbuf is checked
 * first (NULL, or longer than a slot: -EINVAL, nothing protected).
 * Returns the number of datagrams sent; if a GPU or socket error stops
 * the call after some were sent, that number, with errv[] holding the
 * errno for every packet not sent; -errno if none was sent.  A full
 * socket buffer is waited on for at most 2 s per sendmmsg.  Pipelined:
 * chunk j+1 is protected on the GPU while chunk j is sent.
 */
int srtp_udp_send(struct srtp_udp *su, const struct sockaddr *dst,
		  socklen_t dstlen, struct mbuf **mbv, int *errv, size_t n);

/** counters: datagrams received / unprotected ok / sent */
void srtp_udp_stats(const struct srtp_udp *su, uint64_t *rx, uint64_t *rx_ok,
		    uint64_t *tx);

/** where the time goes (nanoseconds, summed over the helper's life) */
enum {
	SRTP_UDP_RX_SYSCALL = 0,  /**< recvmmsg                            */
	SRTP_UDP_RX_GPU,          /**< waiting for unprotect + copies back  */
	SRTP_UDP_RX_DELIVER,      /**< the receive handler calls            */
	SRTP_UDP_TX_STAGE,        /**< mbufs into the pinned send arena     */
	SRTP_UDP_TX_GPU,          /**< waiting for protect + copies back    */
	SRTP_UDP_TX_SYSCALL,      /**< sendmmsg                             */
	SRTP_UDP_NSTAGE
};
void srtp_udp_times(const struct srtp_udp *su,
		    uint64_t ns[SRTP_UDP_NSTAGE]);

#ifdef __cplusplus
}
#endif

#endif
