/*
 * udp.c -- batched SRTP UDP helper (include/re_srtp_udp.h).
 *
 * The reference moves one datagram per event through the UDP helper chain:
 * udp_read() (src/udp/udp.c:149-211) recvfrom()s into a fresh mbuf and the
 * SRTP helper's recv hook unprotects it; udp_send_internal()
 * (src/udp/udp.c:484-507) runs the send hooks (srtp_encrypt) before
 * sendto().  Here a batch of datagrams lands with one recvmmsg() directly
 * in pinned host slots, crosses PCIe in one copy, is unprotected by one
 * device batch call and comes back in one copy; the send side mirrors it
 * with the protect batch call and sendmmsg().
 *
 * Pipelined mode (srtp_udp_pipeline): two arenas per direction.  Receive:
 * batch k+1 is read from the socket while the GPU unprotects batch k
 * (asynchronous batch call, srtp_batch_wait); batch k is handed to the
 * handler one call later.  Send: chunk j+1 is staged and queued while chunk
 * j is still on the GPU, and chunk j's datagrams go out while j+1 runs.
 * Results stay those of srtp_decrypt()/srtp_encrypt() in datagram order
 * (the asynchronous calls keep issue order on the contexts).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <time.h>
#include "re_mem.h"
#include "re_mbuf.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"
#include "re_srtp_udp.h"
#include "../srtpgpu.h"
#include "fault.h"

#define SEND_RETRY_MS 2000      /* bound on a full socket buffer */

struct dir {                    /* one arena: slots, windows, results */
	uint8_t *h, *d;         /* pinned host / device arena */
	uint32_t *hw, *dw;      /* pos | end | cap, pinned / device */
	int32_t *he, *de;       /* per-packet errno, pinned / device */
	struct mmsghdr *msg;
	struct iovec *iov;
	struct sockaddr_storage *src;
	size_t n;               /* packets staged / in flight */
	struct srtp_batch_ticket *tk;   /* in flight (pipelined) */
	struct srtp_batch_dev b;
	struct srtp *ctx;       /* the call's session array (one entry): it
				   must outlive an asynchronous call */
};

struct srtp_udp {
	int fd;
	struct srtp *rx, *tx;
	size_t batch, slot;
	struct dir in[2], out[2];
	int pipeline;
	int rcur;               /* receive arena to fill next */
	int rpend;              /* receive arena in flight, or -1 */
	void *stream, *cstream; /* batch calls / result copies */
	srtp_udp_recv_h *rh;
	void *arg;
	uint64_t n_rx, n_rx_ok, n_tx;
	uint64_t ns[SRTP_UDP_NSTAGE];
};

static uint64_t now_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static void dir_free(struct dir *d)
{
	sgpu_host_free(d->h);
	sgpu_host_free(d->hw);
	sgpu_host_free(d->he);
	sgpu_free(d->d);
	sgpu_free(d->dw);
	sgpu_free(d->de);
	free(d->msg);
	free(d->iov);
	free(d->src);
}

static int dir_alloc(struct dir *d, size_t batch, size_t slot)
{
	d->h = fi_sgpu_host_alloc(batch * slot);
	d->d = fi_sgpu_malloc(batch * slot);
	d->hw = fi_sgpu_host_alloc(batch * 12);
	d->dw = fi_sgpu_malloc(batch * 12);
	d->he = fi_sgpu_host_alloc(batch * 4);
	d->de = fi_sgpu_malloc(batch * 4);
	d->msg = fi_calloc(batch, sizeof(*d->msg));
	d->iov = fi_calloc(batch, sizeof(*d->iov));
	d->src = fi_calloc(batch, sizeof(*d->src));
	return d->h && d->d && d->hw && d->dw && d->he && d->de && d->msg &&
	       d->iov && d->src ? 0 : ENOMEM;
}

static void destructor(void *arg)
{
	struct srtp_udp *su = arg;
	int k;
	for (k = 0; k < 2; k++) {
		if (su->in[k].tk)
			(void)srtp_batch_wait(su->in[k].tk);
		if (su->out[k].tk)
			(void)srtp_batch_wait(su->out[k].tk);
	}
	if (su->stream)
		sgpu_stream_sync(su->stream);
	if (su->cstream)
		sgpu_stream_sync(su->cstream);
	for (k = 0; k < 2; k++) {
		dir_free(&su->in[k]);
		dir_free(&su->out[k]);
	}
	sgpu_stream_destroy(su->stream);
	sgpu_stream_destroy(su->cstream);
}

int srtp_udp_alloc(struct srtp_udp **sup, int fd, struct srtp *rx,
		   struct srtp *tx, size_t batch, size_t slot,
		   srtp_udp_recv_h *rh, void *arg)
{
	struct srtp_udp *su;
	int err, k;

	if (!sup || fd < 0 || !batch || batch > (1u << 20) || slot < 64 ||
	    slot > 65536 || (!rx && !tx))
		return EINVAL;
	slot = (slot + 15) & ~(size_t)15;
	if ((uint64_t)batch * slot > UINT32_MAX)
		return EINVAL;
	su = fi_mem_zalloc(sizeof(*su), destructor);
	if (!su)
		return ENOMEM;
	su->fd = fd;
	su->rx = rx;
	su->tx = tx;
	su->batch = batch;
	su->slot = slot;
	su->rh = rh;
	su->arg = arg;
	su->rpend = -1;
	su->stream = sgpu_stream_create();
	su->cstream = su->stream ? sgpu_stream_create() : NULL;
	if (!su->stream || !su->cstream) {
		err = ENOSYS;           /* no usable HIP device */
		goto out;
	}
	err = 0;
	for (k = 0; k < 2 && !err; k++) {
		err = dir_alloc(&su->in[k], batch, slot);
		if (!err)
			err = dir_alloc(&su->out[k], batch, slot);
	}
 out:
	if (err)
		mem_deref(su);
	else
		*sup = su;
	return err;
}

int srtp_udp_pipeline(struct srtp_udp *su, int on)
{
	if (!su)
		return EINVAL;
	if (su->rpend >= 0 || su->in[0].tk || su->in[1].tk)
		return EBUSY;   /* a receive batch is in flight: flush first */
	su->pipeline = on != 0;
	return 0;
}

/* windows + arena up, then the batch call (asynchronous when pipelined) */
static int gpu_issue(struct srtp_udp *su, struct dir *d, int prot,
		     struct srtp *ctx)
{
	struct srtp_batch_dev *b = &d->b;
	const size_t n = d->n, used = n * su->slot;
	int err;

	err = sgpu_memcpy_h2d(d->d, d->h, used, su->stream);
	if (!err)
		err = sgpu_memcpy_h2d(d->dw, d->hw, n * 12, su->stream);
	if (err)
		return err;
	memset(b, 0, sizeof(*b));
	b->arena = d->d;
	b->arena_size = used;
	b->pos = d->dw;
	b->end = d->dw + n;
	b->cap = d->dw + 2 * n;
	b->err = d->de;
	b->n = n;
	b->stream = su->stream;
	d->ctx = ctx;
	if (su->pipeline)
		return prot ? srtp_encrypt_batch_dev_async(&d->ctx, 1, b, &d->tk)
			    : srtp_decrypt_batch_dev_async(&d->ctx, 1, b, &d->tk);
	return prot ? srtp_encrypt_batch_dev(&d->ctx, 1, b)
		    : srtp_decrypt_batch_dev(&d->ctx, 1, b);
}

/* ... its completion, then arena, windows and results down (on the copy
 * stream when pipelined: the next batch may already run on the other) */
static int gpu_finish(struct srtp_udp *su, struct dir *d, int stage)
{
	const size_t n = d->n, used = n * su->slot;
	void *st = su->pipeline ? su->cstream : su->stream;
	const uint64_t t0 = now_ns();
	int err = 0;

	if (d->tk) {
		err = srtp_batch_wait(d->tk);
		d->tk = NULL;
	}
	if (!err)
		err = sgpu_memcpy_d2h(d->h, d->d, used, st);
	if (!err)
		err = sgpu_memcpy_d2h(d->hw, d->dw, n * 8, st);
	if (!err)
		err = sgpu_memcpy_d2h(d->he, d->de, n * 4, st);
	if (!err)
		err = sgpu_stream_sync(st);
	su->ns[stage] += now_ns() - t0;
	return err;
}

/* recvmmsg into d (non-blocking); number of datagrams or -errno */
static int rx_read(struct srtp_udp *su, struct dir *d)
{
	const uint64_t t0 = now_ns();
	size_t i, n;
	int r;

	for (i = 0; i < su->batch; i++) {
		d->iov[i].iov_base = d->h + i * su->slot;
		d->iov[i].iov_len = su->slot;
		memset(&d->msg[i].msg_hdr, 0, sizeof(d->msg[i].msg_hdr));
		d->msg[i].msg_hdr.msg_iov = &d->iov[i];
		d->msg[i].msg_hdr.msg_iovlen = 1;
		d->msg[i].msg_hdr.msg_name = &d->src[i];
		d->msg[i].msg_hdr.msg_namelen = sizeof(d->src[i]);
	}
	r = recvmmsg(su->fd, d->msg, (unsigned)su->batch, MSG_DONTWAIT, NULL);
	su->ns[SRTP_UDP_RX_SYSCALL] += now_ns() - t0;
	if (r < 0)
		return (errno == EAGAIN || errno == EWOULDBLOCK) ? 0 : -errno;
	n = (size_t)r;
	for (i = 0; i < n; i++) {
		const uint32_t base = (uint32_t)(i * su->slot);
		uint32_t len = d->msg[i].msg_len;
		if (d->msg[i].msg_hdr.msg_flags & MSG_TRUNC)
			len = 0;        /* reported as EMSGSIZE */
		d->hw[i] = base;
		d->hw[n + i] = base + len;
		d->hw[2 * n + i] = base + (uint32_t)su->slot;
	}
	d->n = n;
	return (int)n;
}

static void rx_deliver(struct srtp_udp *su, struct dir *d)
{
	const uint64_t t0 = now_ns();
	const size_t n = d->n;
	size_t i;

	su->n_rx += n;
	for (i = 0; i < n; i++) {
		struct mbuf mb;
		int e = (d->msg[i].msg_hdr.msg_flags & MSG_TRUNC) ? EMSGSIZE
								  : d->he[i];
		mb.buf = d->h;
		mb.size = (i + 1) * su->slot;
		mb.pos = d->hw[i];
		mb.end = d->hw[n + i];
		if (!e)
			su->n_rx_ok++;
		if (su->rh)
			su->rh(&d->src[i], d->msg[i].msg_hdr.msg_namelen, &mb,
			       e, su->arg);
	}
	d->n = 0;
	su->ns[SRTP_UDP_RX_DELIVER] += now_ns() - t0;
}

/* hand a batch over undecrypted with one error for every datagram (a
 * failed issue or completion): each received datagram still reaches the
 * handler exactly once */
static void rx_fail(struct srtp_udp *su, struct dir *d, int err)
{
	size_t i;
	for (i = 0; i < d->n; i++)
		d->he[i] = err;
	rx_deliver(su, d);
}

int srtp_udp_recv(struct srtp_udp *su, int timeout_ms)
{
	struct dir *d;
	struct pollfd pfd;
	int r, n, err, prev, done = 0;

	if (!su || !su->rx)
		return -EINVAL;
	d = &su->in[su->rcur];
	pfd.fd = su->fd;
	pfd.events = POLLIN;
	/* a batch in flight: take what is queued now, do not wait */
	r = poll(&pfd, 1, su->rpend >= 0 ? 0 : timeout_ms);
	if (r < 0)
		return -errno;
	n = r > 0 ? rx_read(su, d) : 0;
	if (n < 0)
		return n;
	prev = su->rpend;
	su->rpend = -1;
	if (n > 0) {
		/* batch k+1 queued behind batch k on the GPU */
		err = gpu_issue(su, d, 0, su->rx);
		if (err) {
			/* batch k is in flight: complete and deliver it
			 * first, then k+1 with the error */
			if (prev >= 0) {
				struct dir *p = &su->in[prev];
				if (gpu_finish(su, p, SRTP_UDP_RX_GPU))
					rx_fail(su, p, err);
				else
					rx_deliver(su, p);
			}
			rx_fail(su, d, err);
			return -err;
		}
		if (su->pipeline) {
			su->rpend = su->rcur;
			su->rcur ^= 1;
		}
		else {
			err = gpu_finish(su, d, SRTP_UDP_RX_GPU);
			if (err) {
				rx_fail(su, d, err);
				return -err;
			}
			done = n;
			rx_deliver(su, d);
		}
	}
	if (prev >= 0) {
		/* batch k: complete and hand over (k+1 was read meanwhile and
		 * runs on the GPU now) */
		struct dir *p = &su->in[prev];
		err = gpu_finish(su, p, SRTP_UDP_RX_GPU);
		if (err) {
			rx_fail(su, p, err);
			return -err;
		}
		done = (int)p->n;
		rx_deliver(su, p);
	}
	return done;
}

/* sendmmsg of chunk d's protected datagrams: 0 or errno, *nsent = the
 * datagrams that went out.  errv[i] = the protect result, or, after a
 * failed sendmmsg, the errno for each datagram that was not sent */
static int tx_send(struct srtp_udp *su, struct dir *d,
		   const struct sockaddr *dst, socklen_t dstlen, int *errv,
		   size_t *nsent)
{
	const uint64_t t0 = now_ns();
	const size_t m = d->n;
	size_t i, k, waited = 0;
	int err = 0;

	for (i = 0, k = 0; i < m; i++) {
		if (errv)
			errv[i] = d->he[i];
		if (d->he[i])
			continue;
		d->iov[k].iov_base = d->h + d->hw[i];
		d->iov[k].iov_len = d->hw[m + i] - d->hw[i];
		memset(&d->msg[k].msg_hdr, 0, sizeof(d->msg[k].msg_hdr));
		d->msg[k].msg_hdr.msg_iov = &d->iov[k];
		d->msg[k].msg_hdr.msg_iovlen = 1;
		d->msg[k].msg_hdr.msg_name = (void *)dst;
		d->msg[k].msg_hdr.msg_namelen = dstlen;
		k++;
	}
	for (i = 0; i < k;) {
		int r = sendmmsg(su->fd, d->msg + i, (unsigned)(k - i), 0);
		if (r < 0) {
			if (errno == EINTR)
				continue;
			if ((errno == EAGAIN || errno == EWOULDBLOCK ||
			     errno == ENOBUFS) && waited < SEND_RETRY_MS) {
				struct pollfd pfd = {su->fd, POLLOUT, 0};
				(void)poll(&pfd, 1, 10);
				waited += 10;
				continue;
			}
			err = errno;
			break;
		}
		i += (size_t)r;
	}
	su->ns[SRTP_UDP_TX_SYSCALL] += now_ns() - t0;
	su->n_tx += i;
	*nsent = i;
	if (err && errv) {
		/* the (i+1)-th protected datagram and every later one */
		size_t j, c = 0;
		for (j = 0; j < m; j++) {
			if (d->he[j])
				continue;
			if (c++ >= i)
				errv[j] = err;
		}
	}
	return err;
}

static void tx_stage(struct srtp_udp *su, struct dir *d, struct mbuf **mbv,
		     size_t m)
{
	const uint64_t t0 = now_ns();
	size_t i;
	for (i = 0; i < m; i++) {
		const struct mbuf *mb = mbv[i];
		const uint32_t base = (uint32_t)(i * su->slot);
		const size_t len = mb->end > mb->pos ? mb->end - mb->pos : 0;
		memcpy(d->h + base, mb->buf + mb->pos, len);
		d->hw[i] = base;
		d->hw[m + i] = base + (uint32_t)len;
		d->hw[2 * m + i] = base + (uint32_t)su->slot;
	}
	d->n = m;
	su->ns[SRTP_UDP_TX_STAGE] += now_ns() - t0;
}

int srtp_udp_send(struct srtp_udp *su, const struct sockaddr *dst,
		  socklen_t dstlen, struct mbuf **mbv, int *errv, size_t n)
{
	size_t done = 0, sent = 0, i, j, nch;
	int err = 0;

	if (!su || !su->tx || !dst || (!mbv && n))
		return -EINVAL;
	/* every packet is checked before anything is protected or sent */
	for (i = 0; i < n; i++) {
		const struct mbuf *mb = mbv[i];
		if (!mb || (mb->end > mb->pos ? mb->end - mb->pos : 0) >
		    su->slot)
			return -EINVAL;
	}
	nch = (n + su->batch - 1) / su->batch;
	/* chunk j on arena j % 2: stage + issue j, then finish + send j-1
	 * (pipelined: j-1's datagrams go out while j runs on the GPU) */
	for (j = 0; j <= nch && !err; j++) {
		if (j < nch) {
			struct dir *d = &su->out[j & 1];
			const size_t a = j * su->batch;
			const size_t m = n - a < su->batch ? n - a : su->batch;
			tx_stage(su, d, mbv + a, m);
			err = gpu_issue(su, d, 1, su->tx);
			if (err)
				break;
			if (!su->pipeline) {
				size_t r = 0;
				err = gpu_finish(su, d, SRTP_UDP_TX_GPU);
				if (err)
					break;
				err = tx_send(su, d, dst, dstlen,
					      errv ? errv + a : NULL, &r);
				sent += r;
				done = a + m;   /* the chunk's errv are set */
				continue;
			}
		}
		if (su->pipeline && j > 0) {
			struct dir *p = &su->out[(j - 1) & 1];
			size_t r = 0;
			err = gpu_finish(su, p, SRTP_UDP_TX_GPU);
			if (err)
				break;
			err = tx_send(su, p, dst, dstlen,
				      errv ? errv + (j - 1) * su->batch : NULL,
				      &r);
			sent += r;
			done = (j - 1) * su->batch + p->n;
		}
	}
	if (!err)
		return (int)sent;
	/* drain what is still in flight; the packets not sent get the errno
	 * (the ones before them went out and advanced the sender state) */
	for (i = 0; i < 2; i++)
		if (su->out[i].tk) {
			(void)srtp_batch_wait(su->out[i].tk);
			su->out[i].tk = NULL;
		}
	if (errv)
		for (i = done; i < n; i++)
			errv[i] = err;
	return sent ? (int)sent : -err;
}

void srtp_udp_stats(const struct srtp_udp *su, uint64_t *rx, uint64_t *rx_ok,
		    uint64_t *tx)
{
	if (rx)
		*rx = su ? su->n_rx : 0;
	if (rx_ok)
		*rx_ok = su ? su->n_rx_ok : 0;
	if (tx)
		*tx = su ? su->n_tx : 0;
}

void srtp_udp_times(const struct srtp_udp *su, uint64_t ns[SRTP_UDP_NSTAGE])
{
	int k;
	if (!ns)
		return;
	for (k = 0; k < SRTP_UDP_NSTAGE; k++)
		ns[k] = su ? su->ns[k] : 0;
}
