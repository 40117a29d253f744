/*
 * udp_libre.c -- the batched GPU SRTP transform as a libre UDP helper
 * (include/re_srtp_libre.h).  LIBRE=1 builds only: compiled against
 * libre's own headers and linked into libre.
 *
 * In libre an SRTP transform is a helper on the socket's chain
 * (udp_register_helper, reference src/udp/udp.c:830-860): udp_read()
 * (:149-211) receives one datagram per poll event into a fresh mbuf and
 * walks the receive hooks; udp_send() -> udp_send_internal() (:484-507)
 * walks the send hooks in reverse before sendto().  This helper's hooks
 * take the datagram off the chain (return true) and queue its bytes in a
 * pinned arena; when `batch` datagrams are queued, or `flush_ms` after the
 * first one (a libre timer, so within the re_main loop), the queue is
 * unprotected / protected in ONE GPU batch call and every packet continues
 * down the chain exactly where it left it: udp_recv_helper() (:897-928:
 * the helpers below this one, then the socket's receive handler) with the
 * plaintext, udp_send_helper() (:874-886: the helpers below, then
 * sendto()) with the SRTP packet.  Per packet the bytes, pos/end and stream
 * states are those of srtp_decrypt()/srtp_encrypt() in datagram order; a
 * packet that fails to unprotect is dropped (counted), as an SRTP media
 * transform does.
 *
 * rtcp-mux (RFC 5761; libre demultiplexes it in src/rtp/rtp.c:184-196 by
 * rtp_pt_is_rtcp(), include/re_rtp.h:333): a datagram whose second byte
 * carries a payload type in 64..95 is RTCP and takes the SRTCP transform
 * (srtcp_decrypt / srtcp_encrypt semantics).  One queue keeps datagram
 * order; at a flush its RTP packets run as one srtp_*_batch_dev call and
 * its RTCP packets as one srtcp_*_batch_dev call on the same arena (the
 * two have separate state: ROC / s_l / RTP window vs SRTCP index / RTCP
 * window), then every packet continues down the chain in arrival order.
 */
#include <errno.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <netinet/in.h>
#include <sys/un.h>
/* libre's headers (LIBRE_INC), not its umbrella re.h: that one would
 * declare re_srtp.h a second time */
#include <re_types.h>
#include <re_atomic.h>
#include <re_mem.h>
#include <re_mbuf.h>
#include <re_list.h>
#include <re_sa.h>
#include <re_tmr.h>
#include <re_udp.h>
#include "re_srtp_batch.h"
#include "re_srtp_libre.h"
#include "../srtpgpu.h"

struct q {                      /* one direction's queue */
	uint8_t *h, *d;         /* pinned host / device arena */
	uint32_t *hw, *dw;      /* pos | end | cap */
	int32_t *he, *de;       /* per-packet errno */
	struct sa *sa;          /* source / destination per packet */
	size_t *pre;            /* the mbuf's pos before the packet */
	uint32_t *len;          /* packet length */
	uint8_t *rtcp;          /* the packet is RTCP (rtcp-mux) */
	uint32_t *win;          /* its index in the window arrays: the RTP
				   packets first, then the RTCP ones */
	size_t n;
};

/* include/re_rtp.h:333 rtp_pt_is_rtcp() on the second byte, as
 * src/rtp/rtp.c:184-196 demultiplexes rtcp-mux */
static bool is_rtcp(const uint8_t *p, size_t len)
{
	const uint8_t pt = len >= 2 ? (p[1] & 0x7f) : 0;
	return pt >= 64 && pt <= 95;
}

struct srtp_udp_helper {
	struct udp_helper *uh;
	struct udp_sock *us;
	struct srtp *rx, *tx;
	size_t batch, slot;
	uint64_t flush_ms;
	struct tmr tmr;
	struct q rq, sq;
	void *stream;
	uint64_t n_rx, n_rx_ok, n_tx, n_drop;
};

static void q_free(struct q *q)
{
	sgpu_host_free(q->h);
	sgpu_host_free(q->hw);
	sgpu_host_free(q->he);
	sgpu_free(q->d);
	sgpu_free(q->dw);
	sgpu_free(q->de);
	free(q->sa);
	free(q->pre);
	free(q->len);
	free(q->rtcp);
	free(q->win);
}

static int q_alloc(struct q *q, size_t batch, size_t slot)
{
	q->h = sgpu_host_alloc(batch * slot);
	q->d = sgpu_malloc(batch * slot);
	q->hw = sgpu_host_alloc(batch * 12);
	q->dw = sgpu_malloc(batch * 12);
	q->he = sgpu_host_alloc(batch * 4);
	q->de = sgpu_malloc(batch * 4);
	q->sa = calloc(batch, sizeof(*q->sa));
	q->pre = calloc(batch, sizeof(*q->pre));
	q->len = calloc(batch, sizeof(*q->len));
	q->rtcp = calloc(batch, sizeof(*q->rtcp));
	q->win = calloc(batch, sizeof(*q->win));
	return q->h && q->d && q->hw && q->dw && q->he && q->de && q->sa &&
	       q->pre && q->len && q->rtcp && q->win ? 0 : ENOMEM;
}

/* the queue's GPU calls: windows + arena up, the RTP packets as one
 * SRTP batch and the RTCP packets as one SRTCP batch, all down */
static int q_run(struct srtp_udp_helper *h, struct q *q, int prot,
		 struct srtp *ctx)
{
	const size_t n = q->n, used = n * h->slot;
	struct srtp_batch_dev b;
	size_t i, nrtp = 0, k;
	int err, pass;

	for (i = 0; i < n; i++)
		nrtp += !q->rtcp[i];
	for (i = 0, k = 0; i < n; i++) {
		const uint32_t base = (uint32_t)(i * h->slot);
		const size_t w = q->rtcp[i] ? nrtp + (i - k) : k;
		if (!q->rtcp[i])
			k++;
		q->win[i] = (uint32_t)w;
		q->hw[w] = base;
		q->hw[n + w] = base + q->len[i];
		q->hw[2 * n + w] = base + (uint32_t)h->slot;
	}
	err = sgpu_memcpy_h2d(q->d, q->h, used, h->stream);
	if (!err)
		err = sgpu_memcpy_h2d(q->dw, q->hw, n * 12, h->stream);
	for (pass = 0; pass < 2 && !err; pass++) {
		const size_t off = pass ? nrtp : 0;
		const size_t m = pass ? n - nrtp : nrtp;
		if (!m)
			continue;
		memset(&b, 0, sizeof(b));
		b.arena = q->d;
		b.arena_size = used;
		b.pos = q->dw + off;
		b.end = q->dw + n + off;
		b.cap = q->dw + 2 * n + off;
		b.err = q->de + off;
		b.n = m;
		b.stream = h->stream;
		if (!pass)
			err = prot ? srtp_encrypt_batch_dev(&ctx, 1, &b)
				   : srtp_decrypt_batch_dev(&ctx, 1, &b);
		else
			err = prot ? srtcp_encrypt_batch_dev(&ctx, 1, &b)
				   : srtcp_decrypt_batch_dev(&ctx, 1, &b);
	}
	if (!err)
		err = sgpu_memcpy_d2h(q->h, q->d, used, h->stream);
	if (!err)
		err = sgpu_memcpy_d2h(q->hw, q->dw, n * 8, h->stream);
	if (!err)
		err = sgpu_memcpy_d2h(q->he, q->de, n * 4, h->stream);
	if (!err)
		err = sgpu_stream_sync(h->stream);
	return err;
}

/* packet i of q as a fresh mbuf: its slot's bytes at the offset the
 * original mbuf had them, pos / end as the per-packet call leaves them */
static struct mbuf *q_mbuf(const struct srtp_udp_helper *h,
			   const struct q *q, size_t i)
{
	const uint32_t base = (uint32_t)(i * h->slot);
	const uint32_t w = q->win[i];
	const size_t len = q->hw[q->n + w] - base;
	struct mbuf *mb = mbuf_alloc(q->pre[i] + len);
	if (!mb)
		return NULL;
	mb->pos = mb->end = q->pre[i];
	if (mbuf_write_mem(mb, q->h + base, len)) {
		mem_deref(mb);
		return NULL;
	}
	mb->pos = q->pre[i] + (q->hw[w] - base);
	return mb;
}

static void flush_rx(struct srtp_udp_helper *h)
{
	struct q *q = &h->rq;
	size_t i;
	int err;

	if (!q->n)
		return;
	err = q_run(h, q, 0, h->rx);
	h->n_rx += q->n;
	for (i = 0; i < q->n; i++) {
		struct mbuf *mb;
		if (err || q->he[q->win[i]]) {
			h->n_drop++;
			continue;
		}
		mb = q_mbuf(h, q, i);
		if (!mb) {
			h->n_drop++;
			continue;
		}
		h->n_rx_ok++;
		udp_recv_helper(h->us, &q->sa[i], mb, h->uh);
		mem_deref(mb);
	}
	q->n = 0;
}

static void flush_tx(struct srtp_udp_helper *h)
{
	struct q *q = &h->sq;
	size_t i;
	int err;

	if (!q->n)
		return;
	err = q_run(h, q, 1, h->tx);
	for (i = 0; i < q->n; i++) {
		struct mbuf *mb;
		if (err || q->he[q->win[i]]) {
			h->n_drop++;
			continue;
		}
		mb = q_mbuf(h, q, i);
		if (!mb) {
			h->n_drop++;
			continue;
		}
		if (!udp_send_helper(h->us, &q->sa[i], mb, h->uh))
			h->n_tx++;
		mem_deref(mb);
	}
	q->n = 0;
}

void srtp_udp_helper_flush(struct srtp_udp_helper *h)
{
	if (!h)
		return;
	tmr_cancel(&h->tmr);
	flush_tx(h);
	flush_rx(h);
}

static void tmr_handler(void *arg)
{
	srtp_udp_helper_flush(arg);
}

/* queue [pos, end) of mb; false if it does not fit a slot (with room
 * for the SRTP tag, or SRTCP's E||index + tag) */
static bool q_push(struct srtp_udp_helper *h, struct q *q,
		   const struct sa *sa, const struct mbuf *mb)
{
	const size_t len = mbuf_get_left(mb);
	if (len + 20 > h->slot)
		return false;
	memcpy(q->h + q->n * h->slot, mbuf_buf(mb), len);
	q->len[q->n] = (uint32_t)len;
	q->rtcp[q->n] = is_rtcp(mbuf_buf(mb), len);
	sa_cpy(&q->sa[q->n], sa);
	q->pre[q->n] = mb->pos;
	q->n++;
	return true;
}

static bool recv_h(struct sa *src, struct mbuf *mb, void *arg)
{
	struct srtp_udp_helper *h = arg;

	if (!h->rx)
		return false;
	if (!q_push(h, &h->rq, src, mb)) {
		/* larger than a slot: in order, through the per-packet call,
		 * and on down the chain in place */
		flush_rx(h);
		h->n_rx++;
		if (is_rtcp(mbuf_buf(mb), mbuf_get_left(mb)) ?
		    srtcp_decrypt(h->rx, mb) : srtp_decrypt(h->rx, mb)) {
			h->n_drop++;
			return true;
		}
		h->n_rx_ok++;
		return false;
	}
	if (h->rq.n == h->batch)
		flush_rx(h);
	else if (h->rq.n == 1 && !tmr_isrunning(&h->tmr)) {
		tmr_start(&h->tmr, h->flush_ms, tmr_handler, h);
	}
	return true;
}

static bool send_h(int *err, struct sa *dst, struct mbuf *mb, void *arg)
{
	struct srtp_udp_helper *h = arg;

	if (!h->tx)
		return false;
	if (!q_push(h, &h->sq, dst, mb)) {
		flush_tx(h);
		*err = is_rtcp(mbuf_buf(mb), mbuf_get_left(mb)) ?
		       srtcp_encrypt(h->tx, mb) : srtp_encrypt(h->tx, mb);
		return *err != 0;       /* on down the chain, protected */
	}
	if (h->sq.n == h->batch)
		flush_tx(h);
	else if (h->sq.n == 1 && !tmr_isrunning(&h->tmr)) {
		tmr_start(&h->tmr, h->flush_ms, tmr_handler, h);
	}
	return true;
}

static void destructor(void *arg)
{
	struct srtp_udp_helper *h = arg;
	tmr_cancel(&h->tmr);
	mem_deref(h->uh);
	if (h->stream)
		sgpu_stream_sync(h->stream);
	q_free(&h->rq);
	q_free(&h->sq);
	sgpu_stream_destroy(h->stream);
}

int srtp_udp_helper_alloc(struct srtp_udp_helper **hp, struct udp_sock *us,
			  int layer, struct srtp *rx, struct srtp *tx,
			  size_t batch, size_t slot, unsigned flush_ms)
{
	struct srtp_udp_helper *h;
	int err;

	if (!hp || !us || (!rx && !tx) || !batch || batch > (1u << 16) ||
	    slot < 64 || slot > 65536)
		return EINVAL;
	slot = (slot + 15) & ~(size_t)15;
	h = mem_zalloc(sizeof(*h), destructor);
	if (!h)
		return ENOMEM;
	tmr_init(&h->tmr);
	h->us = us;
	h->rx = rx;
	h->tx = tx;
	h->batch = batch;
	h->slot = slot;
	h->flush_ms = flush_ms;
	h->stream = sgpu_stream_create();
	if (!h->stream) {
		err = ENOSYS;
		goto out;
	}
	err = q_alloc(&h->rq, batch, slot);
	if (!err)
		err = q_alloc(&h->sq, batch, slot);
	if (!err)
		err = udp_register_helper(&h->uh, us, layer, send_h, recv_h, h);
 out:
	if (err)
		mem_deref(h);
	else
		*hp = h;
	return err;
}

void srtp_udp_helper_stats(const struct srtp_udp_helper *h, uint64_t *rx,
			   uint64_t *rx_ok, uint64_t *tx, uint64_t *dropped)
{
	if (rx)
		*rx = h ? h->n_rx : 0;
	if (rx_ok)
		*rx_ok = h ? h->n_rx_ok : 0;
	if (tx)
		*tx = h ? h->n_tx : 0;
	if (dropped)
		*dropped = h ? h->n_drop : 0;
}
