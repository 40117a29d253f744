/*
 * rtcp_encode.hip -- batched RTCP compound encode on the GPU.
 *
 * A sender builds each compound packet with successive rtcp_encode() calls
 * on one mbuf (reference src/rtp/pkt.c:316 -> rtcp_vencode :136-313; the
 * report-block and SDES handlers rtcp_rr_encode rr.c:35-51 and
 * rtcp_sdes_encode sdes.c:36-76).  Here a batch of packets is described
 * by message descriptors (include/re_rtcp_batch.h struct rtcp_enc_msg) and
 * written into an HBM arena that srtcp_encrypt_batch_dev can protect in
 * place next.  One lane per packet: a sizing pass over its messages (the
 * errno of the first invalid one, ENOMEM past cap) and, when the packet is
 * valid, the write pass -- header, fixed words, report blocks / chunks /
 * sources / pool bytes, zero padding to 32 bits, the length field in words
 * minus one (pkt.c:296-310).  RTCP compounds are tens to hundreds of bytes
 * with a data-dependent layout, so the lane walks its packet serially.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include "re_rtcp_batch.h"
#include "../srtpgpu.h"

namespace {

struct enc {
	uint8_t *w;             /* write cursor, NULL in the sizing pass */
	uint32_t n;             /* bytes so far */
};

__device__ __forceinline__ void put8(enc &e, uint32_t v)
{
	if (e.w)
		e.w[e.n] = (uint8_t)v;
	e.n++;
}

__device__ __forceinline__ void put16(enc &e, uint32_t v)
{
	put8(e, v >> 8);
	put8(e, v);
}

__device__ __forceinline__ void put32(enc &e, uint32_t v)
{
	put16(e, v >> 16);
	put16(e, v);
}

__device__ __forceinline__ void putmem(enc &e, const uint8_t *p, uint32_t len)
{
	if (e.w)
		for (uint32_t i = 0; i < len; i++)
			e.w[e.n + i] = p[i];
	e.n += len;
}

struct arrays {
	const struct rtcp_enc_rb *rbv;
	const struct rtcp_enc_chunk *chunkv;
	const struct rtcp_enc_sdes *sdesv;
	const uint32_t *srcv;
	const uint8_t *pool;
	uint32_t nrb, nchunk, nsdes, nsrc, pool_size;
};

__device__ __forceinline__ bool in(uint32_t first, uint32_t num, uint32_t n)
{
	return (uint64_t)first + num <= n;
}

/* one rtcp_vencode call (pkt.c:136-313) appended at e.n; 0 or errno */
__device__ int message(enc &e, const struct rtcp_enc_msg &m, const arrays &a)
{
	const uint32_t start = e.n;
	e.n += 4;               /* the header is encoded last (pkt.c:153-154) */
	switch (m.pt) {
	case 200:               /* SR: sender info, then the report blocks */
	case 201:               /* RR */
		for (uint32_t i = 0; i < (m.pt == 200 ? 6u : 1u); i++)
			put32(e, m.w[i]);
		if (!in(m.first, m.num, a.nrb))
			return EINVAL;
		for (uint32_t i = 0; i < m.num; i++) {
			const struct rtcp_enc_rb &r = a.rbv[m.first + i];
			put32(e, r.ssrc);
			put32(e, (r.fraction & 0xff) << 24 |
				 (r.lost & 0xffffffu));
			put32(e, r.last_seq);
			put32(e, r.jitter);
			put32(e, r.lsr);
			put32(e, r.dlsr);
		}
		break;
	case 202:               /* SDES: one rtcp_sdes_encode per chunk */
		if (!in(m.first, m.num, a.nchunk))
			return EINVAL;
		for (uint32_t i = 0; i < m.num; i++) {
			const struct rtcp_enc_chunk &ch = a.chunkv[m.first + i];
			const uint32_t c0 = e.n;
			if (!ch.num || !in(ch.first, ch.num, a.nsdes))
				return EINVAL;          /* sdes.c:42 */
			put32(e, ch.src);
			for (uint32_t j = 0; j < ch.num; j++) {
				const struct rtcp_enc_sdes &it =
					a.sdesv[ch.first + j];
				if (it.len > 255 ||
				    !in(it.off, it.len, a.pool_size))
					return EINVAL;  /* sdes.c:57-60 */
				put8(e, it.type);
				put8(e, it.len);
				putmem(e, a.pool + it.off, it.len);
			}
			put8(e, 0);                     /* END */
			while ((e.n - c0) & 3)
				put8(e, 0);
		}
		break;
	case 203:               /* BYE: count sources, optional reason */
		if (!in(m.first, m.count, a.nsrc))
			return EINVAL;
		for (uint32_t i = 0; i < m.count; i++)
			put32(e, a.srcv[m.first + i]);
		if (m.flags & RTCP_ENC_REASON) {
			if (!in(m.off, m.len, a.pool_size))
				return EINVAL;
			put8(e, m.len);                 /* (uint8_t)str_len */
			putmem(e, a.pool + m.off, m.len);
		}
		break;
	case 204:               /* APP */
		put32(e, m.w[0]);
		put32(e, m.w[1]);                       /* name, 4 bytes */
		if (m.len) {
			if (m.len % 4)
				return EBADMSG;         /* pkt.c:199-203 */
			if (!in(m.off, m.len, a.pool_size))
				return EINVAL;
			putmem(e, a.pool + m.off, m.len);
		}
		break;
	case 192:               /* FIR (RFC 2032) */
		put32(e, m.w[0]);
		break;
	case 193:               /* NACK (RFC 2032) */
		put32(e, m.w[0]);
		put16(e, m.w[1]);
		put16(e, m.w[2]);
		break;
	case 205:               /* RTPFB */
	case 206:               /* PSFB */
	case 207:               /* XR */
		put32(e, m.w[0]);
		if (m.pt != 207)
			put32(e, m.w[1]);
		if (!in(m.off, m.len, a.pool_size))
			return EINVAL;
		putmem(e, a.pool + m.off, m.len);
		break;
	default:
		return EINVAL;                          /* pkt.c:249-250 */
	}
	while ((e.n - start) & 3)                       /* pkt.c:296-300 */
		put8(e, 0);
	if (e.w) {
		const uint32_t len = (e.n - start - 4) / 4;
		e.w[start] = (uint8_t)(0x80 | m.count);     /* pkt.c:92 */
		e.w[start + 1] = m.pt;
		e.w[start + 2] = (uint8_t)(len >> 8);
		e.w[start + 3] = (uint8_t)len;
	}
	return 0;
}

} /* namespace */

__global__ void k_rtcp_encode(uint8_t *__restrict__ arena, uint64_t asz,
			      const uint32_t *__restrict__ pos,
			      uint32_t *__restrict__ end,
			      const uint32_t *__restrict__ cap,
			      const uint32_t *__restrict__ mfirst,
			      const struct rtcp_enc_msg *__restrict__ msgv,
			      uint32_t nmsg, arrays a,
			      int32_t *__restrict__ errv, uint32_t n)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t p0 = pos[i], room = cap[i];
	const uint32_t m0 = mfirst[i], m1 = mfirst[i + 1];
	int err = 0;
	if (p0 > room || room > asz || m0 > m1 || m1 > nmsg)
		err = EINVAL;
	enc e = {nullptr, 0};
	for (uint32_t m = m0; !err && m < m1; m++)
		err = message(e, msgv[m], a);
	if (!err && e.n > room - p0)
		err = ENOMEM;
	if (!err) {
		e.w = arena + p0;
		e.n = 0;
		for (uint32_t m = m0; m < m1; m++)
			(void)message(e, msgv[m], a);
	}
	end[i] = err ? p0 : p0 + e.n;
	errv[i] = err;
}

extern "C" int sgpu_rtcp_encode(const struct rtcp_enc_batch *b)
{
	if (!b->n)
		return 0;
	arrays a = {b->rbv, b->chunkv, b->sdesv, b->srcv, b->pool, b->nrb,
		    b->nchunk, b->nsdes, b->nsrc, b->pool_size};
	const uint32_t n = (uint32_t)b->n;
	hipLaunchKernelGGL(k_rtcp_encode, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)b->stream, b->arena, b->arena_size,
			   b->pos, b->end, b->cap, b->mfirst, b->msgv, b->nmsg,
			   a, b->err, n);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
