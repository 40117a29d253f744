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
 * Usage: scripts/make_rtcp_golden.sh (decode cases; `encode`: rtcp_encode
 * cases, tests/golden/rtcp_encode_golden.json.gz)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <re.h>
#include "rtcp.h"          /* rtcp_rr_encode, rtcp_encode_h (src/rtp) */

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

/* ---- the decoded contents as items (include/re_rtcp_batch.h struct
 * rtcp_item): [msg, kind, sub, v0..v6, "hex"], where the reference copied
 * variable data out of the packet (SDES item data, BYE reason, APP data)
 * the offset word is 0 and "hex" holds the copied bytes; TWCC chunks /
 * deltas and AFB stay in the packet (mbuf_alloc_ref) and their offsets
 * are the reference's own ---- */
static int nitem;

static void item(int msg, int kind, int sub, uint32_t v0, uint32_t v1,
		 uint32_t v2, uint32_t v3, uint32_t v4, uint32_t v5,
		 uint32_t v6, const uint8_t *data, size_t dlen)
{
	size_t i;
	printf("%s[%d,%d,%d,%u,%u,%u,%u,%u,%u,%u,\"", nitem++ ? "," : "", msg,
	       kind, sub, v0, v1, v2, v3, v4, v5, v6);
	for (i = 0; i < dlen; i++)
		printf("%02x", data[i]);
	printf("\"]");
}

static void items(const struct rtcp_msg *m, int k)
{
	uint32_t i, j;
	switch (m->hdr.pt) {
	case RTCP_SR:
		item(k, 1, 0, m->r.sr.ntp_sec, m->r.sr.ntp_frac, m->r.sr.rtp_ts,
		     m->r.sr.psent, m->r.sr.osent, 0, 0, NULL, 0);
		/*@fallthrough@*/
	case RTCP_RR: {
		const struct rtcp_rr *rrv = m->hdr.pt == RTCP_SR ?
			m->r.sr.rrv : m->r.rr.rrv;
		for (i = 0; i < m->hdr.count; i++)
			item(k, 2, 0, rrv[i].ssrc, rrv[i].fraction,
			     (uint32_t)rrv[i].lost & 0xffffffu, rrv[i].last_seq,
			     rrv[i].jitter, rrv[i].lsr, rrv[i].dlsr, NULL, 0);
		break;
	}
	case RTCP_SDES:
		for (i = 0; i < m->hdr.count && m->r.sdesv; i++) {
			const struct rtcp_sdes *sd = &m->r.sdesv[i];
			item(k, 3, 0, sd->src, sd->n, 0, 0, 0, 0, 0, NULL, 0);
			for (j = 0; j < sd->n; j++)
				item(k, 4, sd->itemv[j].type,
				     sd->itemv[j].length, 0, 0, 0, 0, 0, 0,
				     (const uint8_t *)sd->itemv[j].data,
				     sd->itemv[j].length);
		}
		break;
	case RTCP_BYE:
		for (i = 0; i < m->hdr.count; i++)
			item(k, 5, 0, m->r.bye.srcv[i], 0, 0, 0, 0, 0, 0, NULL,
			     0);
		if (m->r.bye.reason)
			item(k, 6, 0, (uint32_t)strlen(m->r.bye.reason), 0, 0,
			     0, 0, 0, 0, (const uint8_t *)m->r.bye.reason,
			     strlen(m->r.bye.reason));
		break;
	case RTCP_APP:
		item(k, 7, m->hdr.count, m->r.app.src,
		     be32(m->r.app.name), 0, (uint32_t)m->r.app.data_len, 0,
		     0, 0, m->r.app.data, m->r.app.data_len);
		break;
	case RTCP_FIR:
		item(k, 8, 0, m->r.fir.ssrc, 0, 0, 0, 0, 0, 0, NULL, 0);
		break;
	case RTCP_NACK:
		item(k, 9, 0, m->r.nack.ssrc, m->r.nack.fsn, m->r.nack.blp, 0,
		     0, 0, 0, NULL, 0);
		break;
	case RTCP_RTPFB:
	case RTCP_PSFB:
		item(k, 10, m->hdr.count, m->r.fb.ssrc_packet,
		     m->r.fb.ssrc_media, m->r.fb.n, 0, 0, 0, 0, NULL, 0);
		if (m->hdr.pt == RTCP_RTPFB && m->hdr.count == RTCP_RTPFB_GNACK)
			for (i = 0; i < m->r.fb.n; i++)
				item(k, 11, 0, m->r.fb.fci.gnackv[i].pid,
				     m->r.fb.fci.gnackv[i].blp, 0, 0, 0, 0, 0,
				     NULL, 0);
		else if (m->hdr.pt == RTCP_RTPFB &&
			 m->hdr.count == RTCP_RTPFB_TWCC) {
			const struct twcc *t = m->r.fb.fci.twccv;
			if (t->deltas->pos != t->chunks->end) {
				fprintf(stderr, "TWCC deltas not after chunks\n");
				exit(1);
			}
			item(k, 12, 0, t->seq, t->count, t->reftime, t->fbcount,
			     (uint32_t)t->chunks->pos,
			     (uint32_t)(t->chunks->end - t->chunks->pos),
			     (uint32_t)(t->deltas->end - t->deltas->pos), NULL,
			     0);
		}
		else if (m->hdr.pt == RTCP_PSFB &&
			 m->hdr.count == RTCP_PSFB_SLI)
			for (i = 0; i < m->r.fb.n; i++)
				item(k, 13, 0, m->r.fb.fci.sliv[i].first,
				     m->r.fb.fci.sliv[i].number,
				     m->r.fb.fci.sliv[i].picid, 0, 0, 0, 0, NULL,
				     0);
		else if (m->hdr.pt == RTCP_PSFB &&
			 m->hdr.count == RTCP_PSFB_AFB)
			item(k, 14, 0, (uint32_t)m->r.fb.fci.afb->pos,
			     (uint32_t)(m->r.fb.fci.afb->end -
					m->r.fb.fci.afb->pos), 0, 0, 0, 0, 0,
			     NULL, 0);
		else if (m->hdr.pt == RTCP_PSFB &&
			 m->hdr.count == RTCP_PSFB_FIR)
			for (i = 0; i < m->r.fb.n; i++)
				item(k, 15, 0, m->r.fb.fci.firv[i].ssrc,
				     m->r.fb.fci.firv[i].seq_n, 0, 0, 0, 0, 0,
				     NULL, 0);
		break;
	case RTCP_XR:
		item(k, 16, 0, m->r.xr.ssrc, m->r.xr.bt, m->r.xr.block_len, 0,
		     0, 0, 0, NULL, 0);
		if (m->r.xr.bt == RTCP_XR_RRTR)
			item(k, 17, 0, m->r.xr.rb.rrtrb.ntp_msw,
			     m->r.xr.rb.rrtrb.ntp_lsw, 0, 0, 0, 0, 0, NULL, 0);
		else if (m->r.xr.bt == RTCP_XR_DLRR)
			item(k, 18, 0, m->r.xr.rb.dlrrb.ssrc,
			     m->r.xr.rb.dlrrb.lrr, m->r.xr.rb.dlrrb.dlrr, 0, 0,
			     0, 0, NULL, 0);
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
	struct rtcp_msg *msgv[256];
	int nkeep = 0;
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
		if (nkeep < 256)
			msgv[nkeep++] = msg;
		else
			mem_deref(msg);
	}
	printf("],\"items\":[");
	nitem = 0;
	for (i = 0; i < (size_t)nkeep; i++) {
		items(msgv[i], (int)i);
		mem_deref(msgv[i]);
	}
	printf("],\"err\":%d,\"stop\":%zu}", err, start);
	mem_deref(mb);
}

/* ---- encode cases (`gen_rtcp_golden encode`) --------------------------
 * Random compound specs in the form of include/re_rtcp_batch.h
 * (struct rtcp_enc_msg and its arrays), each packet built by the
 * reference's own rtcp_encode() calls on one mbuf (src/rtp/pkt.c:316,
 * rtcp_vencode :136-313) with rtcp_rr_encode (rr.c:35) / rtcp_sdes_encode
 * (sdes.c:36) / raw-byte handlers; the output bytes, or the errno of the
 * first call that failed. */
#define EMAX 64
struct espec {
	uint32_t msg[EMAX][14];         /* pt count flags w0..w5 first num off
					   len */
	uint32_t nmsg;
	uint32_t rb[EMAX * 4][7];
	uint32_t nrb;
	uint32_t chunk[EMAX * 4][3];
	uint32_t nchunk;
	uint32_t sdes[EMAX * 16][3];
	uint32_t nsdes;
	uint32_t src[EMAX * 4];
	uint32_t nsrc;
	uint8_t pool[16384];
	uint32_t npool;
};

struct ectx {
	const struct espec *e;
	const uint32_t *m;
};

static int ench_rb(struct mbuf *mb, void *arg)
{
	const struct ectx *x = arg;
	uint32_t i;
	int err = 0;
	for (i = 0; i < x->m[10] && !err; i++) {
		const uint32_t *r = x->e->rb[x->m[9] + i];
		struct rtcp_rr rr;
		memset(&rr, 0, sizeof(rr));
		rr.ssrc = r[0];
		rr.fraction = r[1] & 0xff;
		rr.lost = (int)(r[2] << 8) >> 8;
		rr.last_seq = r[3];
		rr.jitter = r[4];
		rr.lsr = r[5];
		rr.dlsr = r[6];
		err = rtcp_rr_encode(mb, &rr);
	}
	return err;
}

static int ench_sdes(struct mbuf *mb, void *arg)
{
	const struct ectx *x = arg;
	uint32_t i, j;
	int err = 0;
	for (i = 0; i < x->m[10] && !err; i++) {
		const uint32_t *ch = x->e->chunk[x->m[9] + i];
		char str[4][300];
		int ty[4];
		for (j = 0; j < ch[2] && j < 4; j++) {
			const uint32_t *it = x->e->sdes[ch[1] + j];
			ty[j] = (int)it[0];
			memcpy(str[j], x->e->pool + it[2], it[1]);
			str[j][it[1]] = 0;
		}
		switch (ch[2]) {
		case 0: err = rtcp_sdes_encode(mb, ch[0], 0); break;
		case 1: err = rtcp_sdes_encode(mb, ch[0], 1, ty[0], str[0]);
			break;
		case 2: err = rtcp_sdes_encode(mb, ch[0], 2, ty[0], str[0],
					       ty[1], str[1]);
			break;
		case 3: err = rtcp_sdes_encode(mb, ch[0], 3, ty[0], str[0],
					       ty[1], str[1], ty[2], str[2]);
			break;
		default: err = rtcp_sdes_encode(mb, ch[0], 4, ty[0], str[0],
						ty[1], str[1], ty[2], str[2],
						ty[3], str[3]);
			break;
		}
	}
	return err;
}

static int ench_raw(struct mbuf *mb, void *arg)
{
	const struct ectx *x = arg;
	return x->m[13] ? mbuf_write_mem(mb, x->e->pool + x->m[12], x->m[13])
			: 0;
}

/* pool bytes of the given alphabet (no NUL: the reference takes C strings) */
static uint32_t pool_str(struct espec *e, uint32_t len)
{
	uint32_t off = e->npool, i;
	for (i = 0; i < len; i++)
		e->pool[e->npool++] = (uint8_t)('!' + rndn(94));
	return off;
}

static uint32_t pool_raw(struct espec *e, uint32_t len)
{
	uint32_t off = e->npool, i;
	for (i = 0; i < len; i++)
		e->pool[e->npool++] = (uint8_t)rnd();
	return off;
}

static void espec_msg(struct espec *e, int bad)
{
	static const uint32_t pts[] = {200, 201, 202, 203, 204, 192, 193, 205,
				       206, 207};
	uint32_t *m = e->msg[e->nmsg++], i, j;
	memset(m, 0, 14 * 4);
	m[0] = pts[rndn(10)];
	if (bad == 1 || bad == 2)
		m[0] = 202;
	else if (bad == 3)
		m[0] = 204;
	m[1] = rndn(8) ? rndn(32) : rndn(256);  /* count > 31: pkt.c:92 */
	for (i = 0; i < 6; i++)
		m[3 + i] = (uint32_t)rnd();
	switch (m[0]) {
	case 200:
	case 201:
		m[9] = e->nrb;
		m[10] = rndn(4);
		for (i = 0; i < m[10]; i++)
			for (j = 0; j < 7; j++)
				e->rb[e->nrb + i][j] = (uint32_t)rnd();
		e->nrb += m[10];
		if (rndn(8))
			m[1] = m[10];   /* as callers set it, mostly */
		break;
	case 202:
		m[9] = e->nchunk;
		m[10] = bad ? 1 + rndn(3) : rndn(4);
		for (i = 0; i < m[10]; i++) {
			uint32_t *ch = e->chunk[e->nchunk + i];
			ch[0] = (uint32_t)rnd();
			ch[1] = e->nsdes;
			ch[2] = (bad == 1 && i == 0) ? 0 : 1 + rndn(4);
			for (j = 0; j < ch[2]; j++) {
				uint32_t *it = e->sdes[e->nsdes++];
				it[0] = 1 + rndn(8);
				it[1] = (bad == 2 && j == 0) ? 256 + rndn(20)
							      : rndn(40);
				it[2] = pool_str(e, it[1]);
			}
		}
		e->nchunk += m[10];
		if (rndn(8))
			m[1] = m[10];
		break;
	case 203:
		m[1] = rndn(5);
		m[9] = e->nsrc;
		for (i = 0; i < m[1]; i++)
			e->src[e->nsrc++] = (uint32_t)rnd();
		if (rndn(2)) {
			m[2] = 1;
			m[13] = rndn(8) ? rndn(30) : 250 + rndn(60);
			m[12] = pool_str(e, m[13]);
		}
		break;
	case 204:
		m[13] = bad == 3 ? 1 + 4 * rndn(4) + rndn(3) : 4 * rndn(5);
		m[12] = pool_raw(e, m[13]);
		break;
	case 205:
	case 206:
	case 207:
		m[13] = 4 * rndn(6) + (rndn(6) ? 0 : 1 + rndn(3));
		m[12] = pool_raw(e, m[13]);
		break;
	default:
		break;
	}
	if (bad == 4)
		m[0] = 194 + rndn(6);           /* no such type: EINVAL */
}

static int espec_encode(const struct espec *e, uint32_t k, struct mbuf *mb)
{
	const uint32_t *m = e->msg[k];
	struct ectx x = {e, m};
	const uint32_t *w = m + 3;
	uint8_t name[4];
	switch (m[0]) {
	case 200:
		return rtcp_encode(mb, RTCP_SR, m[1], w[0], w[1], w[2], w[3],
				   w[4], w[5], ench_rb, &x);
	case 201:
		return rtcp_encode(mb, RTCP_RR, m[1], w[0], ench_rb, &x);
	case 202:
		return rtcp_encode(mb, RTCP_SDES, m[1], ench_sdes, &x);
	case 203: {
		char reason[400];
		memcpy(reason, e->pool + m[12], m[13]);
		reason[m[13]] = 0;
		return rtcp_encode(mb, RTCP_BYE, m[1], e->src + m[9],
				   m[2] ? reason : NULL);
	}
	case 204:
		name[0] = (uint8_t)(w[1] >> 24);
		name[1] = (uint8_t)(w[1] >> 16);
		name[2] = (uint8_t)(w[1] >> 8);
		name[3] = (uint8_t)w[1];
		return rtcp_encode(mb, RTCP_APP, m[1], w[0], name,
				   m[13] ? e->pool + m[12] : NULL,
				   (size_t)m[13]);
	case 192:
		return rtcp_encode(mb, RTCP_FIR, m[1], w[0]);
	case 193:
		return rtcp_encode(mb, RTCP_NACK, m[1], w[0], w[1], w[2]);
	case 205:
	case 206:
		return rtcp_encode(mb, (enum rtcp_type)m[0], m[1], w[0], w[1],
				   ench_raw, &x);
	case 207:
		return rtcp_encode(mb, RTCP_XR, m[1], w[0], ench_raw, &x);
	default:
		return rtcp_encode(mb, (enum rtcp_type)m[0], m[1], w[0]);
	}
}

static void put_arr(const char *name, const uint32_t *a, uint32_t n,
		    uint32_t width)
{
	uint32_t i, j;
	printf(",\"%s\":[", name);
	for (i = 0; i < n; i++) {
		printf("%s", i ? "," : "");
		if (width > 1)
			printf("[");
		for (j = 0; j < width; j++)
			printf("%s%u", j ? "," : "", a[i * width + j]);
		if (width > 1)
			printf("]");
	}
	printf("]");
}

static int encode_main(void)
{
	static struct espec e;
	int k, first_case = 1;
	uint32_t i;

	rng_s = 0xE5C0DEull;
	printf("{\"generator\":\"oracle/gen_rtcp_golden.c encode (reference "
	       "src/rtp/pkt.c rtcp_encode, rr.c rtcp_rr_encode, sdes.c "
	       "rtcp_sdes_encode)\",\"cases\":[");
	for (k = 0; k < 1500; k++) {
		struct mbuf *mb = mbuf_alloc(256);
		uint32_t nm = 1 + rndn(6);
		/* one case in 8 carries one invalid message */
		int bad = rndn(8) ? 0 : 1 + (int)rndn(4), err = 0;
		uint32_t badat = rndn(nm);
		memset(&e, 0, sizeof(e));
		for (i = 0; i < nm; i++)
			espec_msg(&e, i == badat ? bad : 0);
		for (i = 0; i < nm && !err; i++)
			err = espec_encode(&e, i, mb);
		printf("%s\n{", first_case ? "" : ",");
		first_case = 0;
		printf("\"err\":%d", err);
		put_arr("msgs", &e.msg[0][0], e.nmsg, 14);
		put_arr("rb", &e.rb[0][0], e.nrb, 7);
		put_arr("chunks", &e.chunk[0][0], e.nchunk, 3);
		put_arr("sdes", &e.sdes[0][0], e.nsdes, 3);
		put_arr("srcs", e.src, e.nsrc, 1);
		printf(",\"pool\":\"");
		for (i = 0; i < e.npool; i++)
			printf("%02x", e.pool[i]);
		printf("\",\"out\":\"");
		if (!err)
			for (i = 0; i < mb->end; i++)
				printf("%02x", mb->buf[i]);
		printf("\"}");
		mem_deref(mb);
	}
	printf("\n]}\n");
	return 0;
}

int main(int argc, char **argv)
{
	struct pb p;
	int c, k;
	uint32_t i;

	if (argc > 1 && !strcmp(argv[1], "encode"))
		return encode_main();

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
