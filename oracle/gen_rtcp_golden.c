/*
 * gen_rtcp_golden.c -- RTCP compound-decode golden vectors (TEST
 * INFRASTRUCTURE ONLY).
 *
 * Linked against the reference sources compiled by oracle/Makefile (target
 * `ref`: src/rtp/pkt.c, rr.c, sdes.c, fb.c and their mbuf/mem closure, the
 * image's gcc, no reference build system).  For every generated RTCP
 * compound packet it runs the reference receive loop exactly as
 * rtcp_recv_handler does (/root/reference/src/rtp/rtp.c:164:
 * `while (0 == rtcp_decode(&msg, mb))`) and records, per decoded message,
 *
 *   [off, size, pt, count, length, ssrc, aux]
 *
 *   off    message start (bytes from the packet start)
 *   size   bytes that rtcp_decode consumed for it (mb->pos delta, padding
 *          slurp included -- pkt.c:536-538)
 *   pt, count, length   the decoded header (pkt.c:115-133)
 *   ssrc   the first SSRC field of the message body: SR/RR sender, first
 *          SDES chunk's src, first BYE source, APP src, FIR/NACK ssrc,
 *          RTPFB/PSFB ssrc_packet, XR ssrc (0: none -- SDES/BYE with
 *          count 0, unknown types)
 *   aux    one second field: SR rtp_ts, APP name (big-endian word), NACK
 *          fsn << 16 | blp, RTPFB/PSFB ssrc_media, XR bt << 16 |
 *          block_len, else 0
 *
 * and the errno of the call that ended the loop with the offset where that
 * call began ("err", "stop").  The packets are well-formed compounds of every
 * message type pkt.c decodes (SR/RR with report blocks, SDES chunks and
 * items, BYE with and without reason, APP, FIR, NACK, generic NACK, TWCC,
 * PLI/SLI/AFB/FIR, XR RRTR/DLRR, unknown types), then the same with
 * truncations, bad versions, bad lengths and counts, and random bytes.
 *
 * Usage: oracle/_ref/gen_rtcp_golden > tests/golden/rtcp_decode_golden.json
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <re.h>

static uint64_t rng_s = 0x7C7C7C7Cull;

static uint64_t rnd(void)
{
	rng_s ^= rng_s >> 12;
	rng_s ^= rng_s << 25;
	rng_s ^= rng_s >> 27;
	return rng_s * 0x2545F4914F6CDD1Dull;
}

static uint32_t rndn(uint32_t n) { return (uint32_t)(rnd() % n); }

/* ---- packet builder ---------------------------------------------------- */
struct pb {
	uint8_t b[2048];
	size_t n;
};

static void u8(struct pb *p, uint32_t v)
{
	if (p->n < sizeof(p->b))
		p->b[p->n++] = (uint8_t)v;
}

static void u16(struct pb *p, uint32_t v) { u8(p, v >> 8); u8(p, v); }
static void u32(struct pb *p, uint32_t v) { u16(p, v >> 16); u16(p, v); }

/* header with the length field patched in by hdr_end */
static size_t hdr(struct pb *p, uint32_t count, uint32_t pt)
{
	size_t at = p->n;
	u8(p, 0x80 | (count & 0x1f));
	u8(p, pt);
	u16(p, 0);
	return at;
}

static void hdr_end(struct pb *p, size_t at)
{
	size_t len;
	while ((p->n - at) & 3)
		u8(p, 0);
	len = (p->n - at - 4) / 4;
	p->b[at + 2] = (uint8_t)(len >> 8);
	p->b[at + 3] = (uint8_t)len;
}

static void rr_block(struct pb *p)
{
	int i;
	for (i = 0; i < 6; i++)
		u32(p, (uint32_t)rnd());
}

static void msg_sr(struct pb *p)
{
	uint32_t k = rndn(4), i;
	size_t at = hdr(p, k, 200);
	for (i = 0; i < 6; i++)
		u32(p, (uint32_t)rnd());
	for (i = 0; i < k; i++)
		rr_block(p);
	hdr_end(p, at);
}

static void msg_rr(struct pb *p)
{
	uint32_t k = rndn(4), i;
	size_t at = hdr(p, k, 201);
	u32(p, (uint32_t)rnd());
	for (i = 0; i < k; i++)
		rr_block(p);
	hdr_end(p, at);
}

static void msg_sdes(struct pb *p)
{
	uint32_t k = rndn(4), i, j;
	size_t at = hdr(p, k, 202);
	for (i = 0; i < k; i++) {
		size_t c0 = p->n;
		uint32_t items = rndn(4);
		u32(p, (uint32_t)rnd());
		for (j = 0; j < items; j++) {
			uint32_t len = rndn(20), t;
			u8(p, 1 + rndn(8));
			u8(p, len);
			for (t = 0; t < len; t++)
				u8(p, 'a' + rndn(26));
		}
		u8(p, 0);               /* END, then pad the chunk */
		while ((p->n - c0) & 3)
			u8(p, 0);
	}
	hdr_end(p, at);
}

static void msg_bye(struct pb *p)
{
	uint32_t k = rndn(4), i;
	size_t at = hdr(p, k, 203);
	for (i = 0; i < k; i++)
		u32(p, (uint32_t)rnd());
	if (rndn(2)) {
		uint32_t len = rndn(16);
		u8(p, len);
		for (i = 0; i < len; i++)
			u8(p, 'A' + rndn(26));
	}
	hdr_end(p, at);
}

static void msg_app(struct pb *p)
{
	uint32_t i, words = rndn(4);
	size_t at = hdr(p, rndn(32), 204);
	u32(p, (uint32_t)rnd());
	u32(p, 0x54455354);     /* "TEST" */
	for (i = 0; i < words; i++)
		u32(p, (uint32_t)rnd());
	hdr_end(p, at);
}

static void msg_fir(struct pb *p)
{
	size_t at = hdr(p, 0, 192);
	u32(p, (uint32_t)rnd());
	hdr_end(p, at);
}

static void msg_nack(struct pb *p)
{
	size_t at = hdr(p, 0, 193);
	u32(p, (uint32_t)rnd());
	u16(p, (uint32_t)rnd());
	u16(p, (uint32_t)rnd());
	hdr_end(p, at);
}

static void msg_rtpfb(struct pb *p)
{
	uint32_t i, n, fmt = rndn(3) == 0 ? 15 : (rndn(4) ? 1 : 3);
	size_t at = hdr(p, fmt, 205);
	u32(p, (uint32_t)rnd());
	u32(p, (uint32_t)rnd());
	if (fmt == 1) {
		n = 1 + rndn(4);
		for (i = 0; i < n; i++)
			u32(p, (uint32_t)rnd());
	}
	else if (fmt == 15) {
		/* transport-wide CC: base seq, count, reftime|fbcount, chunks
		 * (run length / status vectors), then one delta byte per
		 * received packet (small deltas) */
		uint32_t count = 1 + rndn(20), left = count, deltas = 0;
		u16(p, (uint32_t)rnd());
		u16(p, count);
		u32(p, (uint32_t)rnd());
		while (left) {
			uint32_t kind = rndn(3), run, j;
			if (kind == 0) {        /* run length, symbol 1 */
				run = 1 + rndn(left);
				u16(p, (1u << 13) | run);
				deltas += run;
				left -= run;
			}
			else if (kind == 1) {   /* 1-bit status vector */
				uint32_t v = 0x8000 | (rndn(0x4000));
				u16(p, v);
				for (j = 0; j < 14 && j < left; j++)
					deltas += (v >> (13 - j)) & 1;
				left -= j;
			}
			else {                  /* 2-bit status vector */
				uint32_t v = 0xC000, s;
				for (j = 0; j < 7; j++) {
					s = rndn(2);    /* 0 or 1 */
					v |= s << (2 * (6 - j));
				}
				u16(p, v);
				for (j = 0; j < 7 && j < left; j++)
					deltas += (v >> (2 * (6 - j))) & 3;
				left -= j;
			}
		}
		for (i = 0; i < deltas; i++)
			u8(p, rndn(256));
	}
	hdr_end(p, at);
}

static void msg_psfb(struct pb *p)
{
	static const uint32_t fmts[] = {1, 2, 4, 15, 7};
	uint32_t i, n, fmt = fmts[rndn(5)];
	size_t at = hdr(p, fmt, 206);
	u32(p, (uint32_t)rnd());
	u32(p, (uint32_t)rnd());
	n = fmt == 1 ? 0 : 1 + rndn(3);
	if (fmt == 4)
		n *= 2;
	for (i = 0; i < n; i++)
		u32(p, (uint32_t)rnd());
	hdr_end(p, at);
}

static void msg_xr(struct pb *p)
{
	uint32_t bt = rndn(3) ? 4 + rndn(2) : 6, bl, i;
	size_t at = hdr(p, 0, 207);
	u32(p, (uint32_t)rnd());
	bl = bt == 4 ? 2 : bt == 5 ? 3 : 1 + rndn(3);
	u8(p, bt);
	u8(p, 0);
	u16(p, bl);
	for (i = 0; i < bl; i++)
		u32(p, (uint32_t)rnd());
	hdr_end(p, at);
}

static void msg_unknown(struct pb *p)
{
	uint32_t i, words = rndn(4);
	size_t at = hdr(p, rndn(32), rndn(2) ? 208 : 199);
	for (i = 0; i < words; i++)
		u32(p, (uint32_t)rnd());
	hdr_end(p, at);
}

static void (*const builders[])(struct pb *) = {
	msg_sr, msg_rr, msg_sdes, msg_bye, msg_app, msg_fir, msg_nack,
	msg_rtpfb, msg_psfb, msg_xr, msg_unknown,
};
#define NB (sizeof(builders) / sizeof(builders[0]))

/* ---- the reference receive loop ---------------------------------------- */
static int first = 1;

static uint32_t be32(const void *p)
{
	const uint8_t *b = p;
	return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 |
	       (uint32_t)b[2] << 8 | b[3];
}

static void fields(const struct rtcp_msg *m, uint32_t *ssrc, uint32_t *aux)
{
	*ssrc = *aux = 0;
	switch (m->hdr.pt) {
	case RTCP_SR:
		*ssrc = m->r.sr.ssrc;
		*aux = m->r.sr.rtp_ts;
		break;
	case RTCP_RR:
		*ssrc = m->r.rr.ssrc;
		break;
	case RTCP_SDES:
		if (m->hdr.count && m->r.sdesv)
			*ssrc = m->r.sdesv[0].src;
		break;
	case RTCP_BYE:
		if (m->hdr.count)
			*ssrc = m->r.bye.srcv[0];
		break;
	case RTCP_APP:
		*ssrc = m->r.app.src;
		*aux = be32(m->r.app.name);
		break;
	case RTCP_FIR:
		*ssrc = m->r.fir.ssrc;
		break;
	case RTCP_NACK:
		*ssrc = m->r.nack.ssrc;
		*aux = (uint32_t)m->r.nack.fsn << 16 | m->r.nack.blp;
		break;
	case RTCP_RTPFB:
	case RTCP_PSFB:
		*ssrc = m->r.fb.ssrc_packet;
		*aux = m->r.fb.ssrc_media;
		break;
	case RTCP_XR:
		*ssrc = m->r.xr.ssrc;
		*aux = (uint32_t)m->r.xr.bt << 16 | m->r.xr.block_len;
		break;
	default:
		break;
	}
}

static void emit(const uint8_t *pkt, size_t len)
{
	struct mbuf *mb = mbuf_alloc(len + 1);
	struct rtcp_msg *msg;
	size_t i, start;
	int err, nm = 0;

	if (!mb) {
		fprintf(stderr, "ENOMEM\n");
		exit(1);
	}
	(void)mbuf_write_mem(mb, pkt, len);
	mb->pos = 0;
	printf("%s\n{\"pkt\":\"", first ? "" : ",");
	first = 0;
	for (i = 0; i < len; i++)
		printf("%02x", pkt[i]);
	printf("\",\"msgs\":[");
	for (;;) {
		uint32_t ssrc, aux;
		start = mb->pos;
		err = rtcp_decode(&msg, mb);
		if (err)
			break;
		fields(msg, &ssrc, &aux);
		printf("%s[%zu,%zu,%u,%u,%u,%u,%u]", nm++ ? "," : "", start,
		       mb->pos - start, msg->hdr.pt, msg->hdr.count,
		       msg->hdr.length, ssrc, aux);
		mem_deref(msg);
	}
	printf("],\"err\":%d,\"stop\":%zu}", err, start);
	mem_deref(mb);
}

int main(void)
{
	struct pb p;
	int c, k;
	uint32_t i;

	printf("{\"generator\":\"oracle/gen_rtcp_golden.c (reference "
	       "src/rtp/pkt.c rtcp_decode loop, rtp.c:164)\",\"cases\":[");

	/* every message type alone, several times */
	for (c = 0; c < (int)NB; c++)
		for (k = 0; k < 12; k++) {
			p.n = 0;
			builders[c](&p);
			emit(p.b, p.n);
		}
	/* compounds of 1..8 messages */
	for (k = 0; k < 400; k++) {
		uint32_t m = 1 + rndn(8);
		p.n = 0;
		for (i = 0; i < m; i++)
			builders[rndn(NB)](&p);
		emit(p.b, p.n);
	}
	/* malformed: truncation at every kind of position, a bad version, a
	 * bad length (short / long), a bad count, trailing junk */
	for (k = 0; k < 1200; k++) {
		uint32_t m = 1 + rndn(4), kind = rndn(6), at;
		p.n = 0;
		for (i = 0; i < m; i++)
			builders[rndn(NB)](&p);
		at = rndn((uint32_t)p.n);
		switch (kind) {
		case 0:
			p.n = at;
			break;
		case 1:
			p.b[at & ~3u] ^= 0x40 << rndn(2);
			break;
		case 2:
			at &= ~3u;
			p.b[at + 3] = (uint8_t)(p.b[at + 3] + 1 + rndn(3));
			break;
		case 3:
			at &= ~3u;
			p.b[at + 3] = (uint8_t)(p.b[at + 3] - 1 - rndn(2));
			break;
		case 4:
			p.b[at & ~3u] = (uint8_t)((p.b[at & ~3u] & 0xe0) |
						  rndn(32));
			break;
		default: {
			uint32_t j, extra = 1 + rndn(12);
			for (j = 0; j < extra; j++)
				u8(&p, rnd());
		}
		}
		emit(p.b, p.n);
	}
	/* random bytes with an RTCP-looking first byte */
	for (k = 0; k < 300; k++) {
		uint32_t len = rndn(96);
		for (i = 0; i < len; i++)
			p.b[i] = (uint8_t)rnd();
		if (len)
			p.b[0] = 0x80 | (p.b[0] & 0x3f);
		if (len > 1)
			p.b[1] = (uint8_t)(192 + rndn(17));
		emit(p.b, len);
	}
	printf("\n]}\n");
	return 0;
}
