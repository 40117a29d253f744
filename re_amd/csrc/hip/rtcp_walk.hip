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

/* the packet's item list (re_rtcp_batch.h struct rtcp_item): items past
 * max are counted, not written; a failed message's items are dropped by
 * resetting k */
struct sink {
	uint32_t *out;          /* packet's first item, 8 words each; NULL */
	uint32_t max, k, msg;
};

__device__ __forceinline__ uint32_t put(sink &s, uint32_t kind, uint32_t sub,
					uint32_t v0 = 0, uint32_t v1 = 0,
					uint32_t v2 = 0, uint32_t v3 = 0,
					uint32_t v4 = 0, uint32_t v5 = 0,
					uint32_t v6 = 0)
{
	const uint32_t k = s.k++;
	if (s.out && k < s.max) {
		uint32_t *o = s.out + 8 * (uint64_t)k;
		o[0] = s.msg | kind << 16 | sub << 24;
		o[1] = v0; o[2] = v1; o[3] = v2; o[4] = v3;
		o[5] = v4; o[6] = v5; o[7] = v6;
	}
	return k;
}

/* rewrite word j of an item already put (the SDES chunk's item count) */
__device__ __forceinline__ void patch(sink &s, uint32_t k, uint32_t j,
				      uint32_t v)
{
	if (s.out && k < s.max)
		s.out[8 * (uint64_t)k + 1 + j] = v;
}

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

/* rtcp_rtpfb_twcc_decode (src/rtp/fb.c:97-160) on the cursor */
__device__ int twcc(cur &c, uint32_t n, sink &s)
{
	if (left(c) < 8)
		return EBADMSG;
	const uint32_t seq = rd(c, 2);
	const uint32_t count = rd(c, 2);
	if (count == 0 || count > 32768)
		return EBADMSG;
	const uint32_t rf = rd(c, 4);
	const uint32_t c0 = c.pos;
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
	put(s, RTCP_ITEM_TWCC, 0, seq, count, rf >> 8, rf & 0xff, c0,
	    (uint32_t)chunks, (uint32_t)sz);
	return 0;
}

/* one rtcp_decode call (pkt.c:337-551); 0 with the descriptor and the
 * message's items, or EBADMSG */
__device__ int decode(cur &c, struct rtcp_desc &d, sink &s)
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
			const uint32_t ns = rd(c, 4), nf = rd(c, 4);
			aux = rd(c, 4);         /* RTP timestamp */
			const uint32_t ps = rd(c, 4), os = rd(c, 4);
			put(s, RTCP_ITEM_SR, 0, ns, nf, aux, ps, os);
		}
		for (uint32_t i = 0; i < count; i++) {
			/* rtcp_rr_decode (rr.c:55-72) */
			if (left(c) < 24)
				return EBADMSG;
			const uint32_t rs = rd(c, 4), w = rd(c, 4);
			const uint32_t ls = rd(c, 4), ji = rd(c, 4);
			const uint32_t lsr = rd(c, 4), dlsr = rd(c, 4);
			put(s, RTCP_ITEM_RB, 0, rs, w >> 24, w & 0xffffffu, ls,
			    ji, lsr, dlsr);
		}
		break;
	case 202:       /* SDES: count chunks of items (sdes.c:99-148) */
		for (uint32_t i = 0; i < count; i++) {
			if (left(c) < 4)
				return EBADMSG;
			const uint32_t c0 = c.pos;
			const uint32_t src = rd(c, 4);
			const uint32_t ck = put(s, RTCP_ITEM_SDES_CHUNK, 0, src);
			uint32_t items = 0;
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
				put(s, RTCP_ITEM_SDES, type, len, c.pos);
				items++;
				c.pos += len;
			}
			patch(s, ck, 1, items);
			while (((c.pos - c0) & 3) && left(c))
				++c.pos;
		}
		break;
	case 203: {     /* BYE: count sources, optional reason */
		const uint32_t sz = count * 4;
		if (left(c) < sz)
			return EBADMSG;
		for (uint32_t i = 0; i < count; i++) {
			const uint32_t src = rd(c, 4);
			if (i == 0)
				ssrc = src;
			put(s, RTCP_ITEM_BYE_SRC, 0, src);
		}
		if (rem > sz) {
			const uint32_t len = rd(c, 1);
			if (left(c) < len)
				return EBADMSG;
			put(s, RTCP_ITEM_BYE_REASON, 0, len, c.pos);
			c.pos += len;
		}
		break;
	}
	case 204: {     /* APP */
		if (left(c) < 8)
			return EBADMSG;
		ssrc = rd(c, 4);
		aux = rd(c, 4);                 /* name */
		uint32_t doff = 0, dlen = 0;
		if (rem > 8) {
			if (left(c) < rem - 8)
				return EBADMSG;
			doff = c.pos;
			dlen = rem - 8;
			c.pos += rem - 8;
		}
		put(s, RTCP_ITEM_APP, count, ssrc, aux, doff, dlen);
		break;
	}
	case 192:       /* FIR (RFC 2032) */
		if (left(c) < 4)
			return EBADMSG;
		ssrc = rd(c, 4);
		put(s, RTCP_ITEM_FIR, 0, ssrc);
		break;
	case 193: {     /* NACK (RFC 2032) */
		if (left(c) < 8)
			return EBADMSG;
		ssrc = rd(c, 4);
		const uint32_t fsn = rd(c, 2), blp = rd(c, 2);
		aux = fsn << 16 | blp;
		put(s, RTCP_ITEM_NACK, 0, ssrc, fsn, blp);
		break;
	}
	case 205:       /* RTPFB (fb.c:170-215) */
	case 206: {     /* PSFB (fb.c:226-307) */
		if (left(c) < 8 || length < 2)
			return EBADMSG;
		ssrc = rd(c, 4);
		aux = rd(c, 4);                 /* media source */
		uint32_t n = length - 2;
		const uint32_t fb = put(s, RTCP_ITEM_FB, count, ssrc, aux, n);
		if (pt == 205) {
			if (count == 1) {       /* generic NACK */
				if (left(c) < n * 4)
					return EBADMSG;
				for (uint32_t i = 0; i < n; i++) {
					const uint32_t pid = rd(c, 2);
					put(s, RTCP_ITEM_GNACK, 0, pid, rd(c, 2));
				}
			}
			else if (count == 15) { /* transport-wide CC */
				if (left(c) < 8)
					return EBADMSG;
				err = twcc(c, n, s);
			}
		}
		else if (count == 2) {                  /* SLI */
			if (left(c) < n * 4)
				return EBADMSG;
			for (uint32_t i = 0; i < n; i++) {
				const uint32_t v = rd(c, 4);
				put(s, RTCP_ITEM_SLI, 0, v >> 19 & 0x1fff,
				    v >> 6 & 0x1fff, v & 0x3f);
			}
		}
		else if (count == 15) {                 /* AFB */
			if (left(c) < n * 4)
				return EBADMSG;
			put(s, RTCP_ITEM_AFB, 0, c.pos, n * 4);
			c.pos += n * 4;
		}
		else if (count == 4) {                  /* FIR (RFC 5104) */
			n /= 2u;
			patch(s, fb, 2, n);
			if (left(c) < n * 8)
				return EBADMSG;
			for (uint32_t i = 0; i < n; i++) {
				const uint32_t fs = rd(c, 4);
				const uint32_t sq = rd(c, 1);
				c.pos += 3;
				put(s, RTCP_ITEM_PSFB_FIR, 0, fs, sq);
			}
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
		put(s, RTCP_ITEM_XR, 0, ssrc, bt, bl);
		if (bt == 4) {                  /* RRTR */
			if (bl != 2)
				return EBADMSG;
			const uint32_t hi = rd(c, 4);
			put(s, RTCP_ITEM_RRTR, 0, hi, rd(c, 4));
		}
		else if (bt == 5) {             /* DLRR */
			if (bl != 3)
				return EBADMSG;
			const uint32_t ds = rd(c, 4), lrr = rd(c, 4);
			put(s, RTCP_ITEM_DLRR, 0, ds, lrr, rd(c, 4));
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
			    struct rtcp_item *__restrict__ itemv,
			    uint32_t maxitem, uint32_t *__restrict__ nitem,
			    int32_t *__restrict__ errv,
			    uint32_t *__restrict__ stopv)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t p0 = pos[i], p1 = end[i];
	if (p0 > p1 || p1 > asz) {
		nmsg[i] = 0;
		if (nitem)
			nitem[i] = 0;
		errv[i] = EINVAL;
		stopv[i] = 0;
		return;
	}
	cur c = {arena + p0, 0, p1 - p0};
	struct rtcp_desc *out = descv + (uint64_t)i * maxmsg;
	sink s = {itemv ? (uint32_t *)(itemv + (uint64_t)i * maxitem) : NULL,
		  maxitem, 0, 0};
	uint32_t k = 0;
	int err;
	for (;;) {
		const uint32_t at = c.pos, k0 = s.k;
		struct rtcp_desc d;
		s.msg = k & 0xffffu;
		err = decode(c, d, s);
		if (err) {
			s.k = k0;       /* the failed message's items */
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
	if (nitem)
		nitem[i] = s.k;
	errv[i] = err;
}

extern "C" int sgpu_rtcp_walk(const uint8_t *arena, uint64_t arena_size,
			      const uint32_t *pos, const uint32_t *end,
			      uint32_t n, struct rtcp_desc *descv,
			      uint32_t maxmsg, uint32_t *nmsg,
			      struct rtcp_item *itemv, uint32_t maxitem,
			      uint32_t *nitem, int32_t *err, uint32_t *stop,
			      void *stream)
{
	if (!n)
		return 0;
	hipLaunchKernelGGL(k_rtcp_walk, dim3((n + 255) / 256), dim3(256), 0,
			   (hipStream_t)stream, arena, arena_size, pos, end, n,
			   descv, maxmsg, nmsg, itemv, maxitem, nitem, err, stop);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
