/*
 * rtcp_walk.hip -- batched RTCP compound decode on the GPU.
 *
 * What libre's receive path does with a (decrypted) RTCP compound packet,
 * rtcp_recv_handler: `while (0 == rtcp_decode(&msg, mb))`
 * (reference src/rtp/rtp.c:164), for a whole batch at once.  One lane
 * walks one packet from its start, message by message, with exactly the
 * reference's cursor rules -- the walk advances by what each body parse
 * reads, not by the header length (pkt.c:369-538), a read past the end
 * returns 0 without moving (mbuf.c:376-452), padding is slurped to the next
 * 32-bit boundary of the message (pkt.c:536-538) -- and writes one
 * descriptor per decoded message (include/re_rtcp_batch.h struct
 * rtcp_desc) plus the errno of the call that ended the loop and where it
 * began.  Packets are small and independent; the walk is a short
 * data-dependent chain per packet, so one lane per packet.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include "re_rtcp_batch.h"
#include "../srtpgpu.h"

namespace {

struct cur {
	const uint8_t *p;
	uint32_t pos, end;
};

__device__ __forceinline__ uint32_t left(const cur &c)
{
	return c.end > c.pos ? c.end - c.pos : 0u;
}

/* mbuf_read_u8/_u16/_u32 + ntoh: 0 and no move past the end */
__device__ __forceinline__ uint32_t rd(cur &c, uint32_t n)
{
	if (n > left(c))
		return 0;
	uint32_t v = 0;
	for (uint32_t i = 0; i < n; i++)
		v = v << 8 | c.p[c.pos + i];
	c.pos += n;
	return v;
}

/* rtcp_rtpfb_twcc_decode (src/rtp/fb.c) on the cursor */
__device__ int twcc(cur &c, uint32_t n)
{
	if (left(c) < 8)
		return EBADMSG;
	(void)rd(c, 2);
	const uint32_t count = rd(c, 2);
	if (count == 0 || count > 32768)
		return EBADMSG;
	(void)rd(c, 4);
	uint64_t chunks = 0, sz = 0;
	for (uint32_t i = count; i > 0;) {
		if (left(c) < 2)
			return EBADMSG;
		const uint32_t chunk = rd(c, 2);
		uint32_t j;
		chunks += 2;
		if (chunk & 0x8000) {
			if (chunk & 0x4000) {
				for (j = 0; j < i && j < 7; j++)
					sz += (chunk >> (2 * (6 - j))) & 3;
			}
			else {
				for (j = 0; j < i && j < 14; j++)
					sz += (chunk >> (13 - j)) & 1;
			}
		}
		else {
			const uint32_t run = chunk & 0x1fffu;
			j = i < run ? i : run;
			sz += (uint64_t)j * ((chunk >> 13) & 3);
		}
		i -= j;
	}
	if (left(c) < sz)
		return EBADMSG;
	/* n * 4 - 8 - chunk bytes, in size_t: a short FCI wraps and fails */
	const uint64_t rest = (uint64_t)n * 4 - 8 - chunks;
	if (left(c) < rest)
		return EBADMSG;
	c.pos += (uint32_t)rest;
	return 0;
}

/* one rtcp_decode call; 0 with the descriptor, or EBADMSG */
__device__ int decode(cur &c, struct rtcp_desc &d)
{
	const uint32_t start = c.pos;
	if (left(c) < 4)
		return EBADMSG;
	const uint32_t b = rd(c, 1), pt = rd(c, 1), length = rd(c, 2);
	if ((b >> 6) != 2)
		return EBADMSG;
	const uint32_t rem = length * 4, count = b & 0x1f;
	if (left(c) < rem)
		return EBADMSG;
	uint32_t ssrc = 0, aux = 0;
	int err = 0;

	switch (pt) {
	case 200:       /* SR: sender info + count report blocks */
	case 201:       /* RR */
		if (left(c) < (pt == 200 ? 24u : 4u))
			return EBADMSG;
		ssrc = rd(c, 4);
		if (pt == 200) {
			c.pos += 8;             /* NTP timestamp */
			aux = rd(c, 4);         /* RTP timestamp */
			c.pos += 8;             /* packet / octet counts */
		}
		for (uint32_t i = 0; i < count; i++) {
			if (left(c) < 24)
				return EBADMSG;
			c.pos += 24;
		}
		break;
	case 202:       /* SDES: count chunks of items */
		for (uint32_t i = 0; i < count; i++) {
			if (left(c) < 4)
				return EBADMSG;
			const uint32_t c0 = c.pos;
			const uint32_t src = rd(c, 4);
			if (i == 0)
				ssrc = src;
			while (left(c) >= 1) {
				const uint32_t type = rd(c, 1);
				if (type == 0)
					break;
				if (left(c) < 1)
					return EBADMSG;
				const uint32_t len = rd(c, 1);
				if (left(c) < len)
					return EBADMSG;
				c.pos += len;
			}
			while (((c.pos - c0) & 3) && left(c))
				++c.pos;
		}
		break;
	case 203: {     /* BYE: count sources, optional reason */
		const uint32_t sz = count * 4;
		if (left(c) < sz)
			return EBADMSG;
		ssrc = count ? rd(c, 4) : 0;
		c.pos += sz - (count ? 4 : 0);
		if (rem > sz) {
			const uint32_t len = rd(c, 1);
			if (left(c) < len)
				return EBADMSG;
			c.pos += len;
		}
		break;
	}
	case 204:       /* APP */
		if (left(c) < 8)
			return EBADMSG;
		ssrc = rd(c, 4);
		aux = rd(c, 4);                 /* name */
		if (rem > 8) {
			if (left(c) < rem - 8)
				return EBADMSG;
			c.pos += rem - 8;
		}
		break;
	case 192:       /* FIR (RFC 2032) */
		if (left(c) < 4)
			return EBADMSG;
		ssrc = rd(c, 4);
		break;
	case 193:       /* NACK (RFC 2032) */
		if (left(c) < 8)
			return EBADMSG;
		ssrc = rd(c, 4);
		aux = rd(c, 4);                 /* fsn << 16 | blp */
		break;
	case 205:       /* RTPFB */
	case 206: {     /* PSFB */
		if (left(c) < 8 || length < 2)
			return EBADMSG;
		ssrc = rd(c, 4);
		aux = rd(c, 4);                 /* media source */
		uint32_t n = length - 2;
		if (pt == 205) {
			if (count == 1) {       /* generic NACK */
				if (left(c) < n * 4)
					return EBADMSG;
				c.pos += n * 4;
			}
			else if (count == 15) { /* transport-wide CC */
				if (left(c) < 8)
					return EBADMSG;
				err = twcc(c, n);
			}
		}
		else if (count == 2 || count == 15) {   /* SLI, AFB */
			if (left(c) < n * 4)
				return EBADMSG;
			c.pos += n * 4;
		}
		else if (count == 4) {                  /* FIR (RFC 5104) */
			n /= 2u;
			if (left(c) < n * 8)
				return EBADMSG;
			c.pos += n * 8;
		}
		break;
	}
	case 207: {     /* XR: the first report block */
		if (left(c) < 4)
			return EBADMSG;
		ssrc = rd(c, 4);
		const uint32_t bt = rd(c, 1);
		(void)rd(c, 1);
		const uint32_t bl = rd(c, 2);
		aux = bt << 16 | bl;
		if (bt == 4) {                  /* RRTR */
			if (bl != 2)
				return EBADMSG;
			(void)rd(c, 4);
			(void)rd(c, 4);
		}
		else if (bt == 5) {             /* DLRR */
			if (bl != 3)
				return EBADMSG;
			(void)rd(c, 4);
			(void)rd(c, 4);
			(void)rd(c, 4);
		}
		break;
	}
	default:        /* unknown type: skip the length */
		c.pos += rem;
		break;
	}
	if (err)
		return err;
	while (((c.pos - start) & 3) && left(c))
		++c.pos;
	d.off = start;
	d.size = c.pos - start;
	d.pt = (uint8_t)pt;
	d.count = (uint8_t)count;
	d.length = (uint16_t)length;
	d.ssrc = ssrc;
	d.aux = aux;
	return 0;
}

} /* namespace */

__global__ void k_rtcp_walk(const uint8_t *__restrict__ arena, uint64_t asz,
			    const uint32_t *__restrict__ pos,
			    const uint32_t *__restrict__ end, uint32_t n,
			    struct rtcp_desc *__restrict__ descv,
			    uint32_t maxmsg, uint32_t *__restrict__ nmsg,
			    int32_t *__restrict__ errv,
			    uint32_t *__restrict__ stopv)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t p0 = pos[i], p1 = end[i];
	if (p0 > p1 || p1 > asz) {
		nmsg[i] = 0;
		errv[i] = EINVAL;
		stopv[i] = 0;
		return;
	}
	cur c = {arena + p0, 0, p1 - p0};
	struct rtcp_desc *out = descv + (uint64_t)i * maxmsg;
	uint32_t k = 0;
	int err;
	for (;;) {
		const uint32_t at = c.pos;
		struct rtcp_desc d;
		err = decode(c, d);
		if (err) {
			stopv[i] = at;
			break;
		}
		if (k < maxmsg) {
			uint32_t *o = (uint32_t *)(out + k);
			o[0] = d.off;
			o[1] = d.size;
			o[2] = (uint32_t)d.pt | (uint32_t)d.count << 8 |
			       (uint32_t)d.length << 16;
			o[3] = d.ssrc;
			o[4] = d.aux;
		}
		k++;
	}
	nmsg[i] = k;
	errv[i] = err;
}

extern "C" int sgpu_rtcp_walk(const uint8_t *arena, uint64_t arena_size,
			      const uint32_t *pos, const uint32_t *end,
			      uint32_t n, struct rtcp_desc *descv,
			      uint32_t maxmsg, uint32_t *nmsg, int32_t *err,
			      uint32_t *stop, void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_rtcp_walk, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, arena, arena_size, pos, end, n,
			   descv, maxmsg, nmsg, err, stop);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
