/*
 * rtcp_oracle.c -- CPU restatement of libre's RTCP compound decode loop.
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle, never linked into re_amd/).
 * Restates what rtcp_recv_handler (/root/reference/src/rtp/rtp.c:164) gets
 * from `while (0 == rtcp_decode(&msg, mb))` over one compound packet:
 *
 *   src/rtp/pkt.c:115-133  rtcp_hdr_decode
 *   src/rtp/pkt.c:337-551  rtcp_decode (per-type body parse, padding slurp)
 *   src/rtp/rr.c:55-72     rtcp_rr_decode
 *   src/rtp/sdes.c:99-148  rtcp_sdes_decode
 *   src/rtp/fb.c           rtcp_rtpfb_decode, rtcp_rtpfb_twcc_decode,
 *                          rtcp_psfb_decode
 *   src/mbuf/mbuf.c:376-452 mbuf_read_mem / _u8 / _u16 / _u32: a read past
 *                          the end returns 0 and does not move the cursor
 *
 * Output per decoded message: off, size, pt, count, length, ssrc, aux
 * (oracle/gen_rtcp_golden.c documents the fields); the return value is the
 * errno of the call that ended the loop (EBADMSG) and *stop the offset it
 * began at.  Pinned by tests/golden/rtcp_decode_golden.json.gz (the
 * reference itself, oracle/gen_rtcp_golden.c).
 */
#include <errno.h>
#include <stdint.h>
#include <stddef.h>
#include "srtp_oracle.h"

struct cur {
	const uint8_t *p;
	size_t pos, end;
};

static size_t left(const struct cur *c)
{
	return c->end > c->pos ? c->end - c->pos : 0;
}

/* mbuf_read_u8/u16/u32 (network order here; the reference ntoh's) */
static uint32_t rd(struct cur *c, size_t n)
{
	uint32_t v = 0;
	size_t i;
	if (n > left(c))
		return 0;
	for (i = 0; i < n; i++)
		v = v << 8 | c->p[c->pos + i];
	c->pos += n;
	return v;
}

static int twcc(struct cur *c, uint32_t n)
{
	uint32_t count, i;
	size_t chunks = 0, sz = 0, j;

	if (left(c) < 8)
		return EBADMSG;
	(void)rd(c, 2);                         /* seq */
	count = rd(c, 2);
	if (count == 0 || count > 32768)
		return EBADMSG;
	(void)rd(c, 4);                         /* reftime | fbcount */
	for (i = count; i > 0;) {
		uint32_t chunk;
		if (left(c) < 2)
			return EBADMSG;
		chunk = rd(c, 2);
		chunks += 2;
		if (chunk & 0x8000) {
			if (chunk & 0x4000) {
				for (j = 0; j < i && j < 7; j++)
					sz += chunk >> (2 * (7 - 1 - j)) & 3;
			}
			else {
				for (j = 0; j < i && j < 14; j++)
					sz += (chunk >> (14 - 1 - j)) & 1;
			}
		}
		else {
			for (j = 0; j < i && j < (chunk & 0x1fffu); j++)
				sz += (chunk >> 13) & 3;
		}
		i -= (uint32_t)j;
	}
	if (left(c) < sz)
		return EBADMSG;
	sz = (size_t)n * 4 - 8 - chunks;        /* size_t: may wrap */
	if (left(c) < sz)
		return EBADMSG;
	c->pos += sz;
	return 0;
}

/* one rtcp_decode call; 0 and the message fields, or EBADMSG */
static int decode(struct cur *c, uint32_t *f)
{
	const size_t start = c->pos;
	uint32_t b, pt, count, length, i, n;
	size_t rem, sz;
	int err = 0;

	if (left(c) < 4)
		return EBADMSG;
	b = rd(c, 1);
	pt = rd(c, 1);
	length = rd(c, 2);
	if ((b >> 6) != 2)
		return EBADMSG;
	rem = (size_t)length * 4;
	if (left(c) < rem)
		return EBADMSG;
	count = b & 0x1f;
	f[5] = f[6] = 0;

	switch (pt) {
	case 200:       /* SR */
		if (left(c) < 24)
			return EBADMSG;
		f[5] = rd(c, 4);
		(void)rd(c, 4);
		(void)rd(c, 4);
		f[6] = rd(c, 4);                /* rtp_ts */
		(void)rd(c, 4);
		(void)rd(c, 4);
		for (i = 0; i < count && !err; i++) {
			if (left(c) < 24)
				err = EBADMSG;
			else
				c->pos += 24;
		}
		break;
	case 201:       /* RR */
		if (left(c) < 4)
			return EBADMSG;
		f[5] = rd(c, 4);
		for (i = 0; i < count && !err; i++) {
			if (left(c) < 24)
				err = EBADMSG;
			else
				c->pos += 24;
		}
		break;
	case 202:       /* SDES */
		for (i = 0; i < count && !err; i++) {
			size_t c0;
			uint32_t src;
			if (left(c) < 4) {
				err = EBADMSG;
				break;
			}
			c0 = c->pos;
			src = rd(c, 4);
			if (i == 0)
				f[5] = src;
			while (left(c) >= 1) {
				uint32_t type = rd(c, 1), len;
				if (type == 0)
					break;
				if (left(c) < 1) {
					err = EBADMSG;
					break;
				}
				len = rd(c, 1);
				if (left(c) < len) {
					err = EBADMSG;
					break;
				}
				c->pos += len;
			}
			if (err)
				break;
			while ((c->pos - c0) & 3 && left(c))
				++c->pos;
		}
		break;
	case 203:       /* BYE */
		sz = (size_t)count * 4;
		if (left(c) < sz)
			return EBADMSG;
		for (i = 0; i < count; i++) {
			uint32_t s = rd(c, 4);
			if (i == 0)
				f[5] = s;
		}
		if (rem > sz) {
			const size_t len = rd(c, 1);
			if (left(c) < len)
				return EBADMSG;
			c->pos += len;
		}
		break;
	case 204:       /* APP */
		if (left(c) < 8)
			return EBADMSG;
		f[5] = rd(c, 4);
		f[6] = rd(c, 4);                /* name */
		if (rem > 8) {
			if (left(c) < rem - 8)
				return EBADMSG;
			c->pos += rem - 8;
		}
		break;
	case 192:       /* FIR */
		if (left(c) < 4)
			return EBADMSG;
		f[5] = rd(c, 4);
		break;
	case 193:       /* NACK */
		if (left(c) < 8)
			return EBADMSG;
		f[5] = rd(c, 4);
		f[6] = rd(c, 2) << 16;
		f[6] |= rd(c, 2);
		break;
	case 205:       /* RTPFB */
	case 206:       /* PSFB */
		if (left(c) < 8)
			return EBADMSG;
		if (length < 2)
			return EBADMSG;
		f[5] = rd(c, 4);
		f[6] = rd(c, 4);
		n = length - 2;
		if (pt == 205) {
			if (count == 1) {               /* generic NACK */
				if (left(c) < (size_t)n * 4)
					return EBADMSG;
				c->pos += (size_t)n * 4;
			}
			else if (count == 15) {         /* TWCC */
				if (left(c) < 8)
					return EBADMSG;
				err = twcc(c, n);
			}
		}
		else if (count == 2 || count == 15) {   /* SLI, AFB */
			if (left(c) < (size_t)n * 4)
				return EBADMSG;
			c->pos += (size_t)n * 4;
		}
		else if (count == 4) {                  /* FIR */
			n /= 2u;
			if (left(c) < (size_t)n * 8)
				return EBADMSG;
			c->pos += (size_t)n * 8;
		}
		break;
	case 207:       /* XR */
		if (left(c) < 4)
			return EBADMSG;
		f[5] = rd(c, 4);
		{
			uint32_t bt = rd(c, 1), bl;
			(void)rd(c, 1);
			bl = rd(c, 2);
			f[6] = bt << 16 | bl;
			if (bt == 4) {
				if (bl != 2)
					return EBADMSG;
				(void)rd(c, 4);
				(void)rd(c, 4);
			}
			else if (bt == 5) {
				if (bl != 3)
					return EBADMSG;
				(void)rd(c, 4);
				(void)rd(c, 4);
				(void)rd(c, 4);
			}
		}
		break;
	default:
		c->pos += rem;
		break;
	}
	if (err)
		return err;
	while ((c->pos - start) & 3 && left(c))
		++c->pos;
	f[0] = (uint32_t)start;
	f[1] = (uint32_t)(c->pos - start);
	f[2] = pt;
	f[3] = count;
	f[4] = length;
	return 0;
}

int oracle_rtcp_walk(const uint8_t *p, size_t len, uint32_t *desc,
		     uint32_t maxmsg, uint32_t *nmsg, uint32_t *stop)
{
	struct cur c = {p, 0, len};
	uint32_t f[7], k;
	int err;

	*nmsg = 0;
	for (;;) {
		const size_t at = c.pos;
		err = decode(&c, f);
		if (err) {
			*stop = (uint32_t)at;
			return err;
		}
		if (*nmsg < maxmsg)
			for (k = 0; k < 7; k++)
				desc[7 * *nmsg + k] = f[k];
		(*nmsg)++;
	}
}
