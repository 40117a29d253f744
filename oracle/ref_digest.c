/*
 * ref_digest.c -- whole-arena reference digests (TEST INFRASTRUCTURE ONLY).
 *
 * Linked against the reference src/srtp compiled by oracle/Makefile
 * (target `ref`, the image's libcrypto).  For a BASELINE.json config it
 * rebuilds the exact packet arena re_amd/workload.py builds (same
 * xorshift64* generators, same slot layout), runs the reference
 * srtp_encrypt (src/srtp/srtp.c:183-285) over every packet in array order,
 * then srtp_decrypt (srtp.c:288-432) of the protected arena with fresh
 * receiver contexts, and prints SHA-256 digests of the arena, the end
 * array, the per-packet errnos and the final stream states after each
 * direction.  tests/golden/fullsize_digests.json is this program's output
 * for configs 1-4 and for the shapes beyond them (scripts/
 * make_fullsize_digests.sh); the -m gpu tests compare the HIP path's
 * full-size outputs with it:
 *
 *   5  the config-5 stream: 2M x 1200 B, one SSRC (two 1M shards of it)
 *   6  config 2 over 2 SSRCs of one session (packet i -> SSRC i mod 2,
 *      per-SSRC seq from 65000)
 *   7  SRTCP, config-2 arena shape (1M x 1200-B RTCP packets, CM128/HMAC80,
 *      srtcp_encrypt/srtcp_decrypt, src/srtp/srtcp.c:31-287)
 *   8  SRTCP, config-3 shape (AEAD_AES_256_GCM)
 *   9  config 2 with forged packets: after protect, every packet i with
 *      i % 1000 == 999 gets payload byte 20 (arena offset pos + 32)
 *      flipped (^ 0x40) -- 1048 EAUTH verdicts, the receiver states and the
 *      post-error bytes (ciphertext kept, ROC over the tag) pinned
 *  10  config 4 (64K sessions, mixed lengths) with the same forgeries
 *  11  config 3 (AEAD_AES_256_GCM) with the same forgeries -- the GCM
 *      EAUTH side effects (payload left decrypted in place, end not
 *      trimmed: srtp.c:394-411) pinned at full size
 *  12  shape 7 (SRTCP, CM128/HMAC80) with the same forgeries, and every
 *      packet i with i % 1000 == 499 replaced after protect by a copy of
 *      packet i - 1's protected bytes (same SRTCP index: EALREADY after a
 *      good tag, the tag trimmed, srtcp.c:199-209)
 *
 *   ref_digest <config> [npkts]
 *
 * `ref_digest shards 8 1048576` (shards() below) pins config 5 whole: the
 * 8M-packet stream cut into the 8 ranks' shards, per-shard digests and the
 * reference's stream states at every boundary
 * (tests/golden/config5_shards.json).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <openssl/sha.h>
#include <re.h>
#include "srtp.h"               /* reference src/srtp/srtp.h (stream state) */

#define GOLDEN 0x9E3779B97F4A7C15ull
#define SEED_PAYLOAD 0x5EED5EEDull
#define SEED_KEYS 0xC0FFEEull
#define SSRC_BASE 0x01020304u
#define BLOCK_PKTS 65536u

static const size_t keylen[6]  = {16, 16, 32, 32, 16, 32};
static const size_t saltlen[6] = {14, 14, 14, 14, 12, 12};

static uint64_t xs(uint64_t *s)
{
	*s ^= *s >> 12;
	*s ^= *s << 25;
	*s ^= *s >> 27;
	return *s * 0x2545F4914F6CDD1Dull;
}

static uint64_t xs_init(uint64_t seed, uint64_t i)
{
	uint64_t s = seed ^ (GOLDEN * (i + 1));
	return s ? s : GOLDEN;
}

/* LE bytes of generator i's outputs (workload.py xs_bytes) */
static void xs_fill(uint8_t *out, size_t n, uint64_t seed, uint64_t i)
{
	uint64_t s = xs_init(seed, i);
	size_t o;
	for (o = 0; o < n; o += 8) {
		uint64_t v = xs(&s);
		uint8_t b[8];
		int k;
		for (k = 0; k < 8; k++)
			b[k] = (uint8_t)(v >> (8 * k));
		memcpy(out + o, b, n - o < 8 ? n - o : 8);
	}
}

struct cfg {
	int suite;
	size_t n;
	size_t length;          /* 0: mixed 200/1400 */
	size_t nsess;
	unsigned s0;
	int test_key;
	unsigned nssrc;         /* SSRCs of session 0: packet i -> i mod nssrc */
	int rtcp;               /* SRTCP (workload.make_rtcp_arena) */
	unsigned forge;         /* forge packet i when i % forge == forge-1 */
	unsigned replay;        /* packet i when i % replay == replay/2 - 1:
				   a copy of protected packet i - 1 */
};

#define NCFG 13
static const struct cfg CFG[NCFG] = {
	{0, 0, 0, 0, 0, 0, 1, 0},
	{1, 1024, 160, 1, 1, 1, 1, 0},
	{1, 1u << 20, 1200, 1, 65000, 0, 1, 0},
	{5, 1u << 20, 1200, 1, 65000, 0, 1, 0},
	{1, 1u << 20, 0, 1u << 16, 65000, 0, 1, 0},
	{1, 2u << 20, 1200, 1, 65000, 0, 1, 0},
	{1, 1u << 20, 1200, 1, 65000, 0, 2, 0},
	{1, 1u << 20, 1200, 1, 65000, 0, 1, 1},
	{5, 1u << 20, 1200, 1, 65000, 0, 1, 1},
	{1, 1u << 20, 1200, 1, 65000, 0, 1, 0, 1000},
	{1, 1u << 20, 0, 1u << 16, 65000, 0, 1, 0, 1000},
	{5, 1u << 20, 1200, 1, 65000, 0, 1, 0, 1000},
	{1, 1u << 20, 1200, 1, 65000, 0, 1, 1, 1000, 1000},
};

static void hex(const uint8_t *p, size_t n)
{
	size_t i;
	putchar('"');
	for (i = 0; i < n; i++)
		printf("%02x", p[i]);
	putchar('"');
}

static void sha(const void *p, size_t n)
{
	uint8_t md[32];
	SHA256(p, n, md);
	hex(md, 32);
}

/* per stream row k (session k, or stream k of session 0 when nssrc > 1):
 * roc u32, s_l u32, replay_rtp lix u64, bitmap u64 (LE).  SRTCP rows:
 * rtcp_index u32, 0, replay_rtcp lix, bitmap */
static void states(struct srtp **ctx, size_t nrows, int by_stream, int rtcp,
		   uint32_t ssrc0, uint8_t *buf)
{
	size_t k;
	for (k = 0; k < nrows; k++) {
		struct srtp_stream *st = NULL;
		struct srtp *c = ctx[by_stream ? 0 : k];
		uint8_t *o = buf + 24 * k;
		struct le *le;
		memset(o, 0, 24);
		for (le = c->streaml.head; le; le = le->next) {
			struct srtp_stream *x = le->data;
			if (x->ssrc == ssrc0 + (uint32_t)k)
				st = x;
		}
		if (!st)
			continue;
		if (rtcp) {
			memcpy(o, &st->rtcp_index, 4);
			memcpy(o + 8, &st->replay_rtcp.lix, 8);
			memcpy(o + 16, &st->replay_rtcp.bitmap, 8);
			continue;
		}
		memcpy(o, &st->roc, 4);
		{
			uint32_t sl = st->s_l;
			memcpy(o + 4, &sl, 4);
		}
		memcpy(o + 8, &st->replay_rtp.lix, 8);
		memcpy(o + 16, &st->replay_rtp.bitmap, 8);
	}
}

static void emit(const char *name, const uint8_t *arena, size_t n,
		 size_t slot, const uint32_t *end, const int32_t *err,
		 struct srtp **ctx, size_t nrows, int by_stream, int rtcp,
		 uint8_t *stbuf)
{
	size_t b, nerr = 0, i;
	for (i = 0; i < n; i++)
		nerr += err[i] != 0;
	printf(",\"%s\":{\"arena\":", name);
	sha(arena, n * slot);
	printf(",\"blocks\":[");
	for (b = 0; b * BLOCK_PKTS < n; b++) {
		size_t m = n - b * BLOCK_PKTS < BLOCK_PKTS ? n - b * BLOCK_PKTS
							   : BLOCK_PKTS;
		if (b)
			putchar(',');
		sha(arena + b * BLOCK_PKTS * slot, m * slot);
	}
	printf("],\"end\":");
	sha(end, n * 4);
	printf(",\"err\":");
	sha(err, n * 4);
	printf(",\"nerr\":%zu,\"states\":", nerr);
	states(ctx, nrows, by_stream, rtcp, SSRC_BASE, stbuf);
	sha(stbuf, 24 * nrows);
	if (nrows == 1) {
		printf(",\"state0\":");
		hex(stbuf, 24);
	}
	printf(",\"pkt0\":");
	hex(arena, end[0]);
	printf(",\"pktN\":");
	hex(arena + (n - 1) * slot, end[n - 1] - (n - 1) * slot);
	printf("}");
}

/* one stream state of the reference, as srtp_stream_import takes it */
static void emit_state(const char *name, struct srtp *ctx)
{
	struct le *le;
	const struct srtp_stream *st = NULL;
	for (le = ctx->streaml.head; le; le = le->next)
		if (((struct srtp_stream *)le->data)->ssrc == SSRC_BASE)
			st = le->data;
	printf("\"%s\":", name);
	if (!st) {
		printf("null");
		return;
	}
	printf("{\"roc\":%u,\"s_l\":%u,\"s_l_set\":%d,\"lix\":%llu,"
	       "\"bitmap\":%llu}", st->roc, (unsigned)st->s_l, st->s_l_set ? 1 : 0,
	       (unsigned long long)st->replay_rtp.lix,
	       (unsigned long long)st->replay_rtp.bitmap);
}

/*
 * BASELINE config 5 whole: one stream of world x per packets (seq from
 * 65000, 1200 B, AES_CM_128_HMAC_SHA1_80), cut into `world` contiguous
 * shards of `per` packets as bench.py --gpus N cuts it.  One reference
 * sender and one receiver run over the whole stream in order (shard by
 * shard: the sender's and the receiver's sequences are each the sequential
 * reference's; only one shard's arena is held at a time).  Per shard: the
 * sender's and receiver's stream states at its start (what rank r must
 * import), and the arena / end / errno digests and final states after its
 * protect and its unprotect, with the arena laid out as rank r holds it
 * (workload.make_arena(per, 1200, s0=shard_seq0(r), first=r*per)).
 *
 *   ref_digest shards <world> <per>
 */
static int shards(size_t world, size_t per)
{
	const size_t length = 1200, slot = (length + 16 + 15) & ~(size_t)15;
	const unsigned s0 = 65000;
	const size_t klen = keylen[1] + saltlen[1];
	uint8_t key[64], *arena = calloc(per, slot);
	uint32_t *pos = calloc(per, 4), *end = calloc(per, 4);
	int32_t *err = calloc(per, 4);
	struct srtp *tx, *rx;
	size_t r, i;

	if (!arena || !pos || !end || !err) {
		fprintf(stderr, "out of memory\n");
		return 1;
	}
	xs_fill(key, klen, SEED_KEYS, 0);
	if (srtp_alloc(&tx, 1, key, klen, 0) || srtp_alloc(&rx, 1, key, klen, 0)) {
		fprintf(stderr, "srtp_alloc failed\n");
		return 1;
	}
	printf("{\"generator\":\"oracle/ref_digest.c shards (reference src/srtp"
	       " + OpenSSL)\",\"config\":5,\"suite\":1,\"world\":%zu,\"per\":%zu,"
	       "\"s0\":%u,\"length\":%zu,\"slot\":%zu,\"shards\":[",
	       world, per, s0, length, slot);
	for (r = 0; r < world; r++) {
		const uint64_t first = (uint64_t)r * per;
		for (i = 0; i < per; i++) {
			const uint64_t g = first + i;
			uint8_t *p = arena + i * slot;
			const uint32_t ts = (uint32_t)(160u * g);
			const uint16_t seq = (uint16_t)(s0 + g);
			memset(p, 0, slot);
			p[0] = 0x80;
			p[2] = (uint8_t)(seq >> 8);
			p[3] = (uint8_t)seq;
			p[4] = (uint8_t)(ts >> 24); p[5] = (uint8_t)(ts >> 16);
			p[6] = (uint8_t)(ts >> 8);  p[7] = (uint8_t)ts;
			p[8] = (uint8_t)(SSRC_BASE >> 24);
			p[9] = (uint8_t)(SSRC_BASE >> 16);
			p[10] = (uint8_t)(SSRC_BASE >> 8);
			p[11] = (uint8_t)SSRC_BASE;
			xs_fill(p + 12, length - 12, SEED_PAYLOAD, g);
			pos[i] = (uint32_t)(i * slot);
			end[i] = pos[i] + (uint32_t)length;
		}
		printf("%s{\"rank\":%zu,\"first\":%llu,\"seq0\":%u,", r ? "," : "",
		       r, (unsigned long long)first, (unsigned)(uint16_t)(s0 + first));
		emit_state("tx_in", tx);
		putchar(',');
		emit_state("rx_in", rx);
		printf(",\"plain\":");
		sha(arena, per * slot);
		for (int dir = 0; dir < 2; dir++) {
			size_t nerr = 0;
			for (i = 0; i < per; i++) {
				struct mbuf mb;
				mb.buf = arena;
				mb.size = pos[i] + slot;
				mb.pos = pos[i];
				mb.end = end[i];
				err[i] = dir ? srtp_decrypt(rx, &mb)
					     : srtp_encrypt(tx, &mb);
				end[i] = (uint32_t)mb.end;
				nerr += err[i] != 0;
			}
			printf(",\"%s\":{\"arena\":", dir ? "unprotect" : "protect");
			sha(arena, per * slot);
			printf(",\"end\":");
			sha(end, per * 4);
			printf(",\"err\":");
			sha(err, per * 4);
			printf(",\"nerr\":%zu,\"pkt0\":", nerr);
			hex(arena, end[0]);
			printf(",");
			emit_state("state", dir ? rx : tx);
			printf("}");
		}
		printf("}");
		fflush(stdout);
	}
	printf("]}\n");
	mem_deref(tx);
	mem_deref(rx);
	free(arena);
	free(pos);
	free(end);
	free(err);
	return 0;
}

int main(int argc, char **argv)
{
	int c;
	if (argc > 1 && !strcmp(argv[1], "shards"))
		return shards(argc > 2 ? (size_t)atol(argv[2]) : 8,
			      argc > 3 ? (size_t)atol(argv[3]) : (size_t)1 << 20);
	c = argc > 1 ? atoi(argv[1]) : 0;
	struct cfg cf;
	size_t n, slot, maxlen, i, klen, nrows;
	uint8_t *arena, *keys, *stbuf;
	uint32_t *pos, *end, *len, *sess, *cnt;
	int32_t *err;
	struct srtp **tx, **rx;

	if (c < 1 || c >= NCFG) {
		fprintf(stderr, "usage: %s <config 1-%d> [npkts]\n", argv[0],
			NCFG - 1);
		return 2;
	}
	cf = CFG[c];
	n = argc > 2 ? (size_t)atol(argv[2]) : cf.n;
	klen = keylen[cf.suite] + saltlen[cf.suite];
	maxlen = cf.length ? cf.length : 1400;
	/* workload.make_arena / slot_size: SRTCP and mixed-length slots
	 * 64-B aligned, the rest 16-B aligned */
	slot = cf.rtcp ? (maxlen + 20 + 63) & ~(size_t)63
	       : !cf.length ? (maxlen + 16 + 63) & ~(size_t)63
			    : (maxlen + 16 + 15) & ~(size_t)15;
	nrows = cf.nssrc > 1 ? cf.nssrc : cf.nsess;

	arena = calloc(n, slot);
	pos = calloc(n, 4);
	end = calloc(n, 4);
	len = calloc(n, 4);
	sess = calloc(n, 4);
	err = calloc(n, 4);
	cnt = calloc(cf.nsess > cf.nssrc ? cf.nsess : cf.nssrc, 4);
	keys = calloc(cf.nsess, klen);
	stbuf = calloc(nrows, 24);
	tx = calloc(cf.nsess, sizeof(*tx));
	rx = calloc(cf.nsess, sizeof(*rx));
	if (!arena || !pos || !end || !len || !sess || !err || !cnt || !keys ||
	    !stbuf || !tx || !rx) {
		fprintf(stderr, "out of memory\n");
		return 1;
	}

	/* keys (workload.make_keys, or the test/srtp.c:524-528 key) */
	for (i = 0; i < cf.nsess; i++) {
		if (cf.test_key) {
			memset(keys, 0x22, 16);
			memset(keys + 16, 0x44, 14);
		}
		else {
			xs_fill(keys + i * klen, klen, SEED_KEYS, i);
		}
		if (srtp_alloc(&tx[i], cf.suite, keys + i * klen, klen, 0) ||
		    srtp_alloc(&rx[i], cf.suite, keys + i * klen, klen, 0)) {
			fprintf(stderr, "srtp_alloc failed\n");
			return 1;
		}
	}

	/* arena (workload.make_arena) */
	for (i = 0; i < n; i++) {
		uint8_t *p = arena + i * slot;
		uint32_t ssrc, ts = (uint32_t)(160u * (uint64_t)i);
		uint16_t seq;
		if (cf.length) {
			len[i] = (uint32_t)cf.length;
		}
		else {
			uint64_t s = xs_init(SEED_PAYLOAD + 1, i);
			len[i] = (xs(&s) >> 63) ? 1400 : 200;
		}
		if (cf.nsess > 1) {
			uint64_t s = xs_init(SEED_PAYLOAD + 2, i);
			sess[i] = (uint32_t)((xs(&s) >> 32) % cf.nsess);
		}
		{
			/* stream of the packet: its session, or i mod nssrc */
			uint32_t k = cf.nssrc > 1 ? (uint32_t)(i % cf.nssrc)
						  : sess[i];
			seq = (uint16_t)(cf.s0 + cnt[k]++);
			ssrc = SSRC_BASE + k;
		}
		p[0] = 0x80;
		p[1] = 0;
		p[2] = (uint8_t)(seq >> 8);
		p[3] = (uint8_t)seq;
		p[4] = (uint8_t)(ts >> 24); p[5] = (uint8_t)(ts >> 16);
		p[6] = (uint8_t)(ts >> 8);  p[7] = (uint8_t)ts;
		p[8] = (uint8_t)(ssrc >> 24); p[9] = (uint8_t)(ssrc >> 16);
		p[10] = (uint8_t)(ssrc >> 8); p[11] = (uint8_t)ssrc;
		xs_fill(p + 12, len[i] - 12, SEED_PAYLOAD, i);
		if (cf.rtcp) {
			/* workload.make_rtcp_arena: an SR-typed header, length
			 * field len/4 - 1, SSRC_BASE (bytes 8-11 keep the RTP
			 * SSRC) */
			uint16_t w = (uint16_t)(len[i] / 4 - 1);
			p[0] = 0x80;
			p[1] = 200;
			p[2] = (uint8_t)(w >> 8);
			p[3] = (uint8_t)w;
			p[4] = (uint8_t)(SSRC_BASE >> 24);
			p[5] = (uint8_t)(SSRC_BASE >> 16);
			p[6] = (uint8_t)(SSRC_BASE >> 8);
			p[7] = (uint8_t)SSRC_BASE;
		}
		pos[i] = (uint32_t)(i * slot);
		end[i] = pos[i] + len[i];
	}

	printf("{\"config\":%d,\"suite\":%d,\"n\":%zu,\"slot\":%zu,"
	       "\"nsess\":%zu,\"nssrc\":%u,\"rtcp\":%d,\"forge\":%u,"
	       "\"replay\":%u,\"plain\":", c, cf.suite, n, slot, cf.nsess,
	       cf.nssrc, cf.rtcp, cf.forge, cf.replay);
	sha(arena, n * slot);

	/* protect every packet in array order, in place (the slot has room
	 * for the tag: mbuf_write_mem never reallocates) */
	for (i = 0; i < n; i++) {
		struct mbuf mb;
		mb.buf = arena;
		mb.size = pos[i] + slot;
		mb.pos = pos[i];
		mb.end = end[i];
		err[i] = cf.rtcp ? srtcp_encrypt(tx[sess[i]], &mb)
				 : srtp_encrypt(tx[sess[i]], &mb);
		end[i] = (uint32_t)mb.end;
	}
	emit("protect", arena, n, slot, end, err, tx, nrows, cf.nssrc > 1,
	     cf.rtcp, stbuf);
	if (cf.forge)
		for (i = 0; i < n; i++)
			if (i % cf.forge == cf.forge - 1)
				arena[pos[i] + 32] ^= 0x40;
	if (cf.replay)
		for (i = 1; i < n; i++)
			if (i % cf.replay == cf.replay / 2 - 1) {
				memcpy(arena + pos[i], arena + pos[i - 1], slot);
				end[i] = pos[i] + (end[i - 1] - pos[i - 1]);
			}

	for (i = 0; i < n; i++) {
		struct mbuf mb;
		mb.buf = arena;
		mb.size = pos[i] + slot;
		mb.pos = pos[i];
		mb.end = end[i];
		err[i] = cf.rtcp ? srtcp_decrypt(rx[sess[i]], &mb)
				 : srtp_decrypt(rx[sess[i]], &mb);
		end[i] = (uint32_t)mb.end;
	}
	emit("unprotect", arena, n, slot, end, err, rx, nrows, cf.nssrc > 1,
	     cf.rtcp, stbuf);
	printf("}\n");

	for (i = 0; i < cf.nsess; i++) {
		mem_deref(tx[i]);
		mem_deref(rx[i]);
	}
	return 0;
}
