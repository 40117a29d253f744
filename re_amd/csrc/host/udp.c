/*
 * udp.c -- batched SRTP UDP helper (include/re_srtp_udp.h).
 *
 * The reference moves one datagram per event through the UDP helper chain:
 * udp_read() (src/udp/udp.c:149-211) recvfrom()s into a fresh mbuf and the
 * SRTP helper's recv hook unprotects it; udp_send_internal()
 * (src/udp/udp.c:484-507) runs the send hooks (srtp_encrypt) before
 * sendto().  Here a batch of datagrams lands with one recvmmsg() directly
 * in pinned host slots, crosses PCIe in one copy, is unprotected by one
 * srtp_decrypt_batch_dev() call and comes back in one copy; the send side
 * mirrors it with srtp_encrypt_batch_dev() and sendmmsg().
 */
#define _GNU_SOURCE
#include <errno.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include "re_mem.h"
#include "re_mbuf.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"
#include "re_srtp_udp.h"
#include "../srtpgpu.h"

struct dir {                    /* one direction's arena and windows */
	uint8_t *h, *d;         /* pinned host / device arena */
	uint32_t *hw, *dw;      /* pos | end | cap, pinned / device */
	int32_t *he, *de;       /* per-packet errno, pinned / device */
};

struct srtp_udp {
	int fd;
	struct srtp *rx, *tx;
	size_t batch, slot;
	struct dir in, out;
	struct mmsghdr *msg;
	struct iovec *iov;
	struct sockaddr_storage *src;
	void *stream;
	srtp_udp_recv_h *rh;
	void *arg;
	uint64_t n_rx, n_rx_ok, n_tx;
};

static void dir_free(struct dir *d)
{
	sgpu_host_free(d->h);
	sgpu_host_free(d->hw);
	sgpu_host_free(d->he);
	sgpu_free(d->d);
	sgpu_free(d->dw);
	sgpu_free(d->de);
}

static int dir_alloc(struct dir *d, size_t batch, size_t slot)
{
	d->h = sgpu_host_alloc(batch * slot);
	d->d = sgpu_malloc(batch * slot);
	d->hw = sgpu_host_alloc(batch * 12);
	d->dw = sgpu_malloc(batch * 12);
	d->he = sgpu_host_alloc(batch * 4);
	d->de = sgpu_malloc(batch * 4);
	return d->h && d->d && d->hw && d->dw && d->he && d->de ? 0 : ENOMEM;
}

static void destructor(void *arg)
{
	struct srtp_udp *su = arg;
	if (su->stream)
		sgpu_stream_sync(su->stream);
	dir_free(&su->in);
	dir_free(&su->out);
	sgpu_stream_destroy(su->stream);
	free(su->msg);
	free(su->iov);
	free(su->src);
}

int srtp_udp_alloc(struct srtp_udp **sup, int fd, struct srtp *rx,
		   struct srtp *tx, size_t batch, size_t slot,
		   srtp_udp_recv_h *rh, void *arg)
{
	struct srtp_udp *su;
	int err;

	if (!sup || fd < 0 || !batch || batch > (1u << 20) || slot < 64 ||
	    slot > 65536 || (!rx && !tx))
		return EINVAL;
	slot = (slot + 15) & ~(size_t)15;
	if ((uint64_t)batch * slot > UINT32_MAX)
		return EINVAL;
	su = mem_zalloc(sizeof(*su), destructor);
	if (!su)
		return ENOMEM;
	su->fd = fd;
	su->rx = rx;
	su->tx = tx;
	su->batch = batch;
	su->slot = slot;
	su->rh = rh;
	su->arg = arg;
	su->stream = sgpu_stream_create();
	su->msg = calloc(batch, sizeof(*su->msg));
	su->iov = calloc(batch, sizeof(*su->iov));
	su->src = calloc(batch, sizeof(*su->src));
	if (!su->stream) {
		err = ENOSYS;           /* no usable HIP device */
		goto out;
	}
	err = dir_alloc(&su->in, batch, slot);
	if (!err)
		err = dir_alloc(&su->out, batch, slot);
	if (!err && (!su->msg || !su->iov || !su->src))
		err = ENOMEM;
 out:
	if (err)
		mem_deref(su);
	else
		*sup = su;
	return err;
}

/* one GPU call over n packets laid out in d's slots: windows up, batch,
 * arena and results down (the caller's stream, one sync) */
static int gpu_batch(struct srtp_udp *su, struct dir *d, size_t n,
		     int (*fn)(struct srtp **, size_t, struct srtp_batch_dev *),
		     struct srtp *ctx)
{
	struct srtp_batch_dev b;
	size_t used = n * su->slot;
	int err;

	err = sgpu_memcpy_h2d(d->d, d->h, used, su->stream);
	if (!err)
		err = sgpu_memcpy_h2d(d->dw, d->hw, n * 12, su->stream);
	if (err)
		return err;
	memset(&b, 0, sizeof(b));
	b.arena = d->d;
	b.arena_size = used;
	b.pos = d->dw;
	b.end = d->dw + n;
	b.cap = d->dw + 2 * n;
	b.err = d->de;
	b.n = n;
	b.stream = su->stream;
	err = fn(&ctx, 1, &b);
	if (!err)
		err = sgpu_memcpy_d2h(d->h, d->d, used, su->stream);
	if (!err)
		err = sgpu_memcpy_d2h(d->hw, d->dw, n * 8, su->stream);
	if (!err)
		err = sgpu_memcpy_d2h(d->he, d->de, n * 4, su->stream);
	if (!err)
		err = sgpu_stream_sync(su->stream);
	return err;
}

int srtp_udp_recv(struct srtp_udp *su, int timeout_ms)
{
	struct dir *d;
	struct pollfd pfd;
	size_t i, n;
	int r, err;

	if (!su || !su->rx)
		return -EINVAL;
	d = &su->in;
	pfd.fd = su->fd;
	pfd.events = POLLIN;
	r = poll(&pfd, 1, timeout_ms);
	if (r < 0)
		return -errno;
	if (r == 0)
		return 0;
	for (i = 0; i < su->batch; i++) {
		su->iov[i].iov_base = d->h + i * su->slot;
		su->iov[i].iov_len = su->slot;
		memset(&su->msg[i].msg_hdr, 0, sizeof(su->msg[i].msg_hdr));
		su->msg[i].msg_hdr.msg_iov = &su->iov[i];
		su->msg[i].msg_hdr.msg_iovlen = 1;
		su->msg[i].msg_hdr.msg_name = &su->src[i];
		su->msg[i].msg_hdr.msg_namelen = sizeof(su->src[i]);
	}
	r = recvmmsg(su->fd, su->msg, (unsigned)su->batch, MSG_DONTWAIT,
		     NULL);
	if (r < 0)
		return (errno == EAGAIN || errno == EWOULDBLOCK) ? 0 : -errno;
	n = (size_t)r;
	for (i = 0; i < n; i++) {
		const uint32_t base = (uint32_t)(i * su->slot);
		uint32_t len = su->msg[i].msg_len;
		if (su->msg[i].msg_hdr.msg_flags & MSG_TRUNC)
			len = 0;        /* reported as EMSGSIZE below */
		d->hw[i] = base;
		d->hw[n + i] = base + len;
		d->hw[2 * n + i] = base + (uint32_t)su->slot;
	}
	err = gpu_batch(su, d, n, srtp_decrypt_batch_dev, su->rx);
	if (err)
		return -err;
	su->n_rx += n;
	for (i = 0; i < n; i++) {
		struct mbuf mb;
		int e = (su->msg[i].msg_hdr.msg_flags & MSG_TRUNC) ? EMSGSIZE
								   : d->he[i];
		mb.buf = d->h;
		mb.size = (i + 1) * su->slot;
		mb.pos = d->hw[i];
		mb.end = d->hw[n + i];
		if (!e)
			su->n_rx_ok++;
		if (su->rh)
			su->rh(&su->src[i], su->msg[i].msg_hdr.msg_namelen, &mb,
			       e, su->arg);
	}
	return (int)n;
}

int srtp_udp_send(struct srtp_udp *su, const struct sockaddr *dst,
		  socklen_t dstlen, struct mbuf **mbv, int *errv, size_t n)
{
	struct dir *d;
	size_t done = 0, sent = 0;
	int err;

	if (!su || !su->tx || !dst || (!mbv && n))
		return -EINVAL;
	d = &su->out;
	while (done < n) {
		const size_t m = n - done < su->batch ? n - done : su->batch;
		size_t i, k;
		for (i = 0; i < m; i++) {
			const struct mbuf *mb = mbv[done + i];
			const uint32_t base = (uint32_t)(i * su->slot);
			size_t len = mb && mb->end > mb->pos ? mb->end - mb->pos
							     : 0;
			if (!mb || len > su->slot)
				return -EINVAL;
			memcpy(d->h + base, mb->buf + mb->pos, len);
			d->hw[i] = base;
			d->hw[m + i] = base + (uint32_t)len;
			d->hw[2 * m + i] = base + (uint32_t)su->slot;
		}
		err = gpu_batch(su, d, m, srtp_encrypt_batch_dev, su->tx);
		if (err)
			return -err;
		for (i = 0, k = 0; i < m; i++) {
			if (errv)
				errv[done + i] = d->he[i];
			if (d->he[i])
				continue;
			su->iov[k].iov_base = d->h + d->hw[i];
			su->iov[k].iov_len = d->hw[m + i] - d->hw[i];
			memset(&su->msg[k].msg_hdr, 0, sizeof(su->msg[k].msg_hdr));
			su->msg[k].msg_hdr.msg_iov = &su->iov[k];
			su->msg[k].msg_hdr.msg_iovlen = 1;
			su->msg[k].msg_hdr.msg_name = (void *)dst;
			su->msg[k].msg_hdr.msg_namelen = dstlen;
			k++;
		}
		for (i = 0; i < k;) {
			int r = sendmmsg(su->fd, su->msg + i, (unsigned)(k - i), 0);
			if (r < 0) {
				if (errno == EINTR)
					continue;
				if (errno == EAGAIN || errno == EWOULDBLOCK ||
				    errno == ENOBUFS) {
					struct pollfd pfd = {su->fd, POLLOUT, 0};
					(void)poll(&pfd, 1, 10);
					continue;
				}
				return -errno;
			}
			i += (size_t)r;
		}
		sent += k;
		su->n_tx += k;
		done += m;
	}
	return (int)sent;
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
