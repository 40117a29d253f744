/*
 * gen_golden.c -- golden-vector generator (TEST INFRASTRUCTURE ONLY).
 *
 * Linked against the reference libre sources compiled by oracle/Makefile
 * (target `ref`).  It drives the reference API exactly as the reference's
 * own tests do (test/srtp.c) and records every call's inputs and outputs
 * (errno, mbuf pos/end/size, buffer bytes) as JSON on stdout.  The output is
 * committed as tests/golden/srtp_golden.json; the product and the C
 * restatement (oracle/srtp_oracle.c) are both checked against it.
 *
 * Usage: oracle/_ref/gen_golden > tests/golden/srtp_golden.json
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <openssl/opensslv.h>
#include <re.h>

/* ---- deterministic PRNG (xorshift64*) ---------------------------------- */
static uint64_t rng_s = 0x5EED5EEDull;

static uint64_t rnd(void)
{
	rng_s ^= rng_s >> 12;
	rng_s ^= rng_s << 25;
	rng_s ^= rng_s >> 27;
	return rng_s * 0x2545F4914F6CDD1Dull;
}

static uint32_t rndn(uint32_t n) { return (uint32_t)(rnd() % n); }

/* ---- JSON helpers ------------------------------------------------------ */
static int first_scn = 1, first_op = 1;

static void hexout(const uint8_t *p, size_t n)
{
	size_t i;
	putchar('"');
	for (i = 0; i < n; i++)
		printf("%02x", p[i]);
	putchar('"');
}

static const uint8_t *cur_keys[8];
static size_t cur_keylen[8];
static int cur_suite[8], cur_flags[8];
static struct srtp *cur_ctx[8];
static int n_ctx;

static void scn_begin(const char *name)
{
	printf("%s\n{\"name\":\"%s\",\"ctxs\":[", first_scn ? "" : ",", name);
	first_scn = 0;
	n_ctx = 0;
}

static int ctx_add(int suite, const uint8_t *key, size_t key_len, int flags)
{
	int err = srtp_alloc(&cur_ctx[n_ctx], suite, key, key_len, flags);
	if (err) {
		fprintf(stderr, "srtp_alloc failed %d\n", err);
		exit(1);
	}
	cur_keys[n_ctx] = key;
	cur_keylen[n_ctx] = key_len;
	cur_suite[n_ctx] = suite;
	cur_flags[n_ctx] = flags;
	return n_ctx++;
}

static void ctxs_emit_and_open_ops(void)
{
	int i;
	for (i = 0; i < n_ctx; i++) {
		printf("%s{\"suite\":%d,\"flags\":%d,\"key\":", i ? "," : "",
		       cur_suite[i], cur_flags[i]);
		hexout(cur_keys[i], cur_keylen[i]);
		printf("}");
	}
	printf("],\"ops\":[");
	first_op = 1;
}

static void scn_end(void)
{
	int i;
	printf("]}");
	for (i = 0; i < n_ctx; i++)
		cur_ctx[i] = mem_deref(cur_ctx[i]);
}

enum opk { OP_SRTP_ENC, OP_SRTP_DEC, OP_SRTCP_ENC, OP_SRTCP_DEC };
static const char *opname[] = {"srtp_encrypt", "srtp_decrypt",
			       "srtcp_encrypt", "srtcp_decrypt"};

/*
 * Run one reference call on a fresh mbuf built from (buf[0:end], size, pos)
 * with zero bytes in [end, size).  Records everything; returns the output
 * buffer (malloc'd, len *outlen) so callers can chain tx -> rx.
 */
static uint8_t *run_op(int ctx, enum opk op, const uint8_t *in, size_t size,
		       size_t pos, size_t end, int *errp, size_t *pos_o,
		       size_t *end_o)
{
	struct mbuf *mb = mbuf_alloc(size);
	size_t rec;
	uint8_t *copy;
	int err = 0;

	memset(mb->buf, 0, size);
	memcpy(mb->buf, in, end);
	mb->pos = pos;
	mb->end = end;

	switch (op) {
	case OP_SRTP_ENC:  err = srtp_encrypt(cur_ctx[ctx], mb);  break;
	case OP_SRTP_DEC:  err = srtp_decrypt(cur_ctx[ctx], mb);  break;
	case OP_SRTCP_ENC: err = srtcp_encrypt(cur_ctx[ctx], mb); break;
	case OP_SRTCP_DEC: err = srtcp_decrypt(cur_ctx[ctx], mb); break;
	}

	rec = mb->end > end ? mb->end : end;

	printf("%s\n {\"ctx\":%d,\"op\":\"%s\",\"size\":%zu,\"pos\":%zu,"
	       "\"end\":%zu,\"in\":", first_op ? "" : ",", ctx, opname[op],
	       size, pos, end);
	first_op = 0;
	hexout(in, end);
	printf(",\"err\":%d,\"pos_o\":%zu,\"end_o\":%zu,\"size_o\":%zu,"
	       "\"out\":", err, mb->pos, mb->end, mb->size);
	hexout(mb->buf, rec);
	printf("}");

	copy = malloc(rec + 64);
	memcpy(copy, mb->buf, rec);
	if (errp)  *errp = err;
	if (pos_o) *pos_o = mb->pos;
	if (end_o) *end_o = mb->end;
	mem_deref(mb);
	return copy;
}

/* ---- packet builders --------------------------------------------------- */

/* RTP header per RFC 3550 (rtp_hdr_encode layout), optional CSRC / ext. */
static size_t build_rtp(uint8_t *p, uint16_t seq, uint32_t ts, uint32_t ssrc,
			unsigned cc, int ext, unsigned xlen, size_t plen,
			int payload_kind)
{
	size_t n = 0, i;
	p[n++] = (uint8_t)(0x80 | (ext ? 0x10 : 0) | (cc & 0xf));
	p[n++] = (uint8_t)(rndn(2) << 7 | rndn(128));
	p[n++] = seq >> 8; p[n++] = seq & 0xff;
	p[n++] = ts >> 24; p[n++] = ts >> 16; p[n++] = ts >> 8; p[n++] = ts;
	p[n++] = ssrc >> 24; p[n++] = ssrc >> 16; p[n++] = ssrc >> 8;
	p[n++] = ssrc;
	for (i = 0; i < cc; i++) {
		uint32_t c = (uint32_t)rnd();
		memcpy(p + n, &c, 4); n += 4;
	}
	if (ext) {
		p[n++] = 0xbe; p[n++] = 0xde;
		p[n++] = xlen >> 8; p[n++] = xlen & 0xff;
		for (i = 0; i < 4 * xlen; i++)
			p[n++] = (uint8_t)rnd();
	}
	for (i = 0; i < plen; i++)
		p[n++] = payload_kind ? (uint8_t)rnd() : (uint8_t)i;
	return n;
}

/* RTCP compound-ish packet: header(4) + SSRC(4) + body. */
static size_t build_rtcp(uint8_t *p, uint32_t ssrc, size_t body)
{
	size_t n = 0, i, words = (8 + body) / 4 - 1;
	p[n++] = 0x81; p[n++] = (uint8_t)(200 + rndn(5));
	p[n++] = (uint8_t)(words >> 8); p[n++] = (uint8_t)words;
	p[n++] = ssrc >> 24; p[n++] = ssrc >> 16; p[n++] = ssrc >> 8;
	p[n++] = ssrc;
	for (i = 0; i < body; i++)
		p[n++] = (uint8_t)rnd();
	return n;
}

static const uint8_t key46[46] = {
	0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22,
	0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22,
	0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22,
	0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22,
	0x44, 0x44, 0x44, 0x44, 0x44, 0x44, 0x44,
	0x44, 0x44, 0x44, 0x44, 0x44, 0x44, 0x44,
};

static const size_t keylen[6]  = {16, 16, 32, 32, 16, 32};
static const size_t saltlen[6] = {14, 14, 14, 14, 12, 12};
static const size_t taglen[6]  = {4, 10, 4, 10, 16, 16};

static uint8_t rkeys[64][46];
static int n_rkeys;

static const uint8_t *random_key(void)
{
	uint8_t *k = rkeys[n_rkeys++ % 64];
	size_t i;
	for (i = 0; i < 46; i++)
		k[i] = (uint8_t)rnd();
	return k;
}

/* ---- scenarios ---------------------------------------------------------- */

/* test/srtp.c:514-570 -- libsrtp known-answer packet */
static void scn_libsrtp(void)
{
	static const uint8_t mk[30] = {
		0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22,
		0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22, 0x22,
		0x44, 0x44, 0x44, 0x44, 0x44, 0x44, 0x44,
		0x44, 0x44, 0x44, 0x44, 0x44, 0x44, 0x44};
	uint8_t p[64];
	size_t n = 0;

	scn_begin("libsrtp_kat");
	ctx_add(SRTP_AES_CM_128_HMAC_SHA1_80, mk, 30, 0);
	ctx_add(SRTP_AES_CM_128_HMAC_SHA1_32, mk, 30, 0);
	ctxs_emit_and_open_ops();

	memcpy(p, "\x80\x00\x00\x01\x00\x00\x00\x00\x01\x02\x03\x04", 12);
	memset(p + 12, 0xa5, 20);
	n = 32;
	free(run_op(0, OP_SRTP_ENC, p, 512, 0, n, NULL, NULL, NULL));

	/* test/srtp.c:583-632 -- SRTCP BYE, reason "b" */
	memcpy(p, "\x81\xcb\x00\x02\x01\x02\x03\x04\x01\x62\x00\x00", 12);
	free(run_op(1, OP_SRTCP_ENC, p, 512, 0, 12, NULL, NULL, NULL));
	scn_end();
}

/* test/srtp.c:321-409 (test_srtp_loop), recorded */
static void scn_loop(int suite, size_t offset, uint16_t seq)
{
	char name[64];
	uint8_t p[256];
	int i, tx, rx;

	snprintf(name, sizeof(name), "srtp_loop_s%d_o%zu_q%u", suite, offset,
		 seq);
	scn_begin(name);
	tx = ctx_add(suite, key46, keylen[suite] + saltlen[suite], 0);
	rx = ctx_add(suite, key46, keylen[suite] + saltlen[suite], 0);
	ctxs_emit_and_open_ops();

	for (i = 0; i < 10; i++) {
		static const uint8_t fixed[20] = {
			0x55, 0x55, 0x55, 0x55, 0x11, 0x11, 0x11, 0x11,
			0xee, 0xee, 0xee, 0xee, 0x11, 0x11, 0x11, 0x11,
			0x55, 0x55, 0x55, 0x55};
		size_t end, e2;
		uint8_t *c;
		int err;

		memset(p, 0, sizeof(p));
		p[offset + 0] = 0x80;
		p[offset + 2] = seq >> 8; p[offset + 3] = seq & 0xff;
		p[offset + 8] = 0x31; p[offset + 9] = 0x32;
		p[offset + 10] = 0x33; p[offset + 11] = 0x34;
		memcpy(p + offset + 12, fixed, 20);
		end = offset + 32;
		seq++;

		c = run_op(tx, OP_SRTP_ENC, p, offset + 32, offset, end, &err,
			   NULL, &e2);
		free(run_op(rx, OP_SRTP_DEC, c, e2, offset, e2, NULL, NULL,
			    NULL));
		free(c);
	}
	scn_end();
}

/*
 * Randomised SRTP send/receive session covering reordering, ROC wrap, loss,
 * tampering, replay, truncation, CSRC/extension headers, multiple SSRCs
 * (up to > 8 for ENOSR) and offsets.
 */
static void scn_random_srtp(int suite, int idx, int nssrc, int npkt,
			    int big)
{
	char name[64];
	uint8_t *held[8];
	size_t held_len[8], held_off[8];
	int nheld = 0;
	uint32_t ssrcs[12];
	uint16_t seqs[12];
	int i, tx, rx;
	const uint8_t *k = random_key();

	snprintf(name, sizeof(name), "srtp_random_s%d_%d", suite, idx);
	scn_begin(name);
	tx = ctx_add(suite, k, keylen[suite] + saltlen[suite], 0);
	rx = ctx_add(suite, k, keylen[suite] + saltlen[suite], 0);
	ctxs_emit_and_open_ops();

	for (i = 0; i < nssrc; i++) {
		ssrcs[i] = (uint32_t)rnd();
		seqs[i] = (uint16_t)(rndn(4) == 0 ? 65536 - 1 - rndn(20)
				     : rnd());
	}

	for (i = 0; i < npkt; i++) {
		static uint8_t p[4096];
		int s = (int)rndn((uint32_t)nssrc);
		size_t off = rndn(3) == 0 ? 4 * rndn(5) : 0;
		unsigned cc = rndn(6) == 0 ? rndn(3) : 0;
		int ext = rndn(6) == 0;
		unsigned xlen = ext ? rndn(3) : 0;
		size_t plen, n, cap, e2, p2;
		uint8_t *c;
		int err, r;

		if (big && rndn(8) == 0)
			plen = rndn(2) ? 1188 : 1388;
		else
			plen = rndn(70);

		/* sequence evolution: mostly +1, sometimes jumps/reorder */
		r = (int)rndn(40);
		if (r == 0)
			seqs[s] = (uint16_t)(seqs[s] + 30000 + rndn(5000));
		else if (r == 1)
			seqs[s] = (uint16_t)(seqs[s] - 1 - rndn(70));
		else if (r == 2)
			seqs[s] = (uint16_t)(seqs[s] + 40 + rndn(60));
		else
			seqs[s] = (uint16_t)(seqs[s] + 1);

		memset(p, 0, off);
		n = off + build_rtp(p + off, seqs[s], (uint32_t)rnd(),
				    ssrcs[s], cc, ext, xlen, plen, 1);
		/* capacity: sometimes exact (forces mbuf growth) */
		cap = rndn(3) == 0 ? n : n + 32;

		c = run_op(tx, OP_SRTP_ENC, p, cap, off, n, &err, &p2, &e2);
		if (err) {
			free(c);
			continue;
		}

		r = (int)rndn(20);
		if (r == 0) {          /* tamper: flip one byte */
			c[off + rndn((uint32_t)(e2 - off))] ^=
				(uint8_t)(1u << rndn(8));
		}
		else if (r == 1 && e2 - off > 2) {   /* truncate */
			e2 = off + rndn((uint32_t)(e2 - off));
		}
		else if (r == 2) {     /* drop */
			free(c);
			continue;
		}
		else if (r == 3 && nheld < 8) {   /* hold for reordering */
			held[nheld] = c;
			held_len[nheld] = e2;
			held_off[nheld] = off;
			nheld++;
			continue;
		}

		free(run_op(rx, OP_SRTP_DEC, c, e2, off, e2, NULL, NULL,
			    NULL));
		if (rndn(15) == 0) {   /* replay the same packet */
			free(run_op(rx, OP_SRTP_DEC, c, e2, off, e2, NULL,
				    NULL, NULL));
		}
		free(c);

		if (nheld && rndn(4) == 0) {
			nheld--;
			free(run_op(rx, OP_SRTP_DEC, held[nheld],
				    held_len[nheld], held_off[nheld],
				    held_len[nheld], NULL, NULL, NULL));
			free(held[nheld]);
		}
	}
	while (nheld--) {
		free(run_op(rx, OP_SRTP_DEC, held[nheld], held_len[nheld],
			    held_off[nheld], held_len[nheld], NULL, NULL,
			    NULL));
		free(held[nheld]);
	}
	scn_end();
}

/* test/srtp.c:811-869 (test_srtp_random): every truncation, both ways */
static void scn_truncations(int suite)
{
	char name[64];
	uint8_t p[128];
	size_t n, i;
	int c;

	snprintf(name, sizeof(name), "srtp_truncations_s%d", suite);
	scn_begin(name);
	c = ctx_add(suite, key46, keylen[suite] + saltlen[suite], 0);
	ctxs_emit_and_open_ops();

	n = build_rtp(p, 1234, 0, 0x31323334, 0, 0, 0, 0, 0);
	memset(p + n, 0xd5, 32);
	n += 32;
	for (i = 0; i < n; i++) {
		free(run_op(c, OP_SRTP_ENC, p, 1024, 0, i, NULL, NULL, NULL));
		free(run_op(c, OP_SRTP_DEC, p, 1024, 0, i, NULL, NULL, NULL));
	}
	/* also: truncated CSRC / extension headers */
	n = build_rtp(p, 77, 0, 0x31323334, 3, 1, 2, 8, 0);
	for (i = 10; i <= n; i++) {
		free(run_op(c, OP_SRTP_ENC, p, 1024, 0, i, NULL, NULL, NULL));
	}
	scn_end();
}

/* test/srtp.c:687-734 (test_srtp_replay): shared tx/rx context */
static void scn_shared_ctx(int suite)
{
	char name[64];
	uint8_t p[128];
	size_t n, e2;
	uint8_t *c;
	int ctx, k;

	snprintf(name, sizeof(name), "srtp_shared_ctx_s%d", suite);
	scn_begin(name);
	ctx = ctx_add(suite, key46, keylen[suite] + saltlen[suite], 0);
	ctxs_emit_and_open_ops();

	for (k = 0; k < 2; k++) {
		n = build_rtp(p, 42, 0, 0x31323334, 0, 0, 0, 20, 0);
		c = run_op(ctx, OP_SRTP_ENC, p, 1024, 0, n, NULL, NULL, &e2);
		free(run_op(ctx, OP_SRTP_DEC, c, 1024, 0, e2, NULL, NULL,
			    NULL));
		free(c);
	}
	scn_end();
}

/* test/srtp.c:412-500 (test_srtcp_loop) + randomised SRTCP */
static void scn_random_srtcp(int suite, int flags, int idx, int npkt)
{
	char name[64];
	int i, tx, rx;
	uint32_t ssrcs[10];
	int nssrc = 1 + (int)rndn(3);
	const uint8_t *k = random_key();

	snprintf(name, sizeof(name), "srtcp_random_s%d_f%d_%d", suite, flags,
		 idx);
	scn_begin(name);
	tx = ctx_add(suite, k, keylen[suite] + saltlen[suite], flags);
	rx = ctx_add(suite, k, keylen[suite] + saltlen[suite], 0);
	ctxs_emit_and_open_ops();

	if (idx == 3)
		nssrc = 10;
	for (i = 0; i < nssrc; i++)
		ssrcs[i] = (uint32_t)rnd();

	for (i = 0; i < npkt; i++) {
		static uint8_t p[2048];
		size_t off = rndn(3) == 0 ? 4 : 0;
		size_t body = 4 * rndn(20), n, e2, cap;
		uint8_t *c;
		int err, r;

		if (rndn(8) == 0)
			body = 4 * (250 + rndn(100));
		memset(p, 0, off);
		n = off + build_rtcp(p + off, ssrcs[rndn((uint32_t)nssrc)],
				     body);
		cap = rndn(3) == 0 ? n : n + 64;

		c = run_op(tx, OP_SRTCP_ENC, p, cap, off, n, &err, NULL, &e2);
		if (err) {
			free(c);
			continue;
		}
		r = (int)rndn(16);
		if (r == 0)
			c[off + rndn((uint32_t)(e2 - off))] ^=
				(uint8_t)(1u << rndn(8));
		else if (r == 1)
			e2 = off + rndn((uint32_t)(e2 - off));
		else if (r == 2) {
			free(c);
			continue;
		}
		free(run_op(rx, OP_SRTCP_DEC, c, e2, off, e2, NULL, NULL,
			    NULL));
		if (rndn(10) == 0)
			free(run_op(rx, OP_SRTCP_DEC, c, e2, off, e2, NULL,
				    NULL, NULL));
		free(c);
	}
	scn_end();
}

/* test/srtp.c:872-925 (test_srtcp_random) */
static void scn_srtcp_truncations(int suite)
{
	char name[64];
	uint8_t p[128];
	size_t n, i;
	int c;

	snprintf(name, sizeof(name), "srtcp_truncations_s%d", suite);
	scn_begin(name);
	c = ctx_add(suite, key46, keylen[suite] + saltlen[suite], 0);
	ctxs_emit_and_open_ops();

	memcpy(p, "\x82\xcb\x00\x04\x12\x34\x56\x78\x00\xab\xcd\xef"
	       "\x04\x63\x69\x61\x6f\x00\x00\x00", 20);
	memset(p + 20, 0xd5, 32);
	n = 52;
	for (i = 0; i < n; i++) {
		free(run_op(c, OP_SRTCP_ENC, p, 1024, 0, i, NULL, NULL, NULL));
		free(run_op(c, OP_SRTCP_DEC, p, 1024, 0, i, NULL, NULL, NULL));
	}
	scn_end();
}

/* srtp_alloc argument validation (srtp.c:98-158) */
static void alloc_errors(void)
{
	static const uint8_t zk[64];
	int s, first = 1;
	size_t len;

	printf("],\"alloc\":[");
	for (s = -1; s <= 7; s++) {
		for (len = 0; len <= 48; len += 2) {
			struct srtp *ctx = NULL;
			int err = srtp_alloc(&ctx, (enum srtp_suite)s, zk, len,
					     0);
			printf("%s[%d,%zu,%d]", first ? "" : ",", s, len, err);
			first = 0;
			mem_deref(ctx);
		}
	}
	printf("],\"names\":[");
	for (s = -1; s <= 7; s++)
		printf("%s\"%s\"", s == -1 ? "" : ",",
		       srtp_suite_name((enum srtp_suite)s));
	printf("]");
}

/* ---- primitive known answers, computed by the reference primitives ------ */
int srtp_derive(uint8_t *out, size_t out_len, uint8_t label,
		const uint8_t *master_key, size_t key_bytes,
		const uint8_t *master_salt, size_t salt_bytes);

static void hexparse(uint8_t *o, const char *h, size_t n)
{
	size_t i;
	for (i = 0; i < n; i++) {
		unsigned v;
		sscanf(h + 2 * i, "%2x", &v);
		o[i] = (uint8_t)v;
	}
}

/* RFC 3711 B.3, RFC 6188 7.2 and SRTCP labels (test/srtp.c:197-318) */
static void prim_kdf(void)
{
	static const struct { const char *key, *salt; int label, outlen; }
	v[] = {
		{"E1F97A0D3E018BE0D64FA32C06DE4139", "0EC675AD498AFEEBB6960B3AABE6", 0, 16},
		{"E1F97A0D3E018BE0D64FA32C06DE4139", "0EC675AD498AFEEBB6960B3AABE6", 1, 20},
		{"E1F97A0D3E018BE0D64FA32C06DE4139", "0EC675AD498AFEEBB6960B3AABE6", 2, 14},
		{"E1F97A0D3E018BE0D64FA32C06DE4139", "0EC675AD498AFEEBB6960B3AABE6", 3, 16},
		{"E1F97A0D3E018BE0D64FA32C06DE4139", "0EC675AD498AFEEBB6960B3AABE6", 4, 20},
		{"E1F97A0D3E018BE0D64FA32C06DE4139", "0EC675AD498AFEEBB6960B3AABE6", 5, 14},
		{"f0f04914b513f2763a1b1fa130f10e2998f6f6e43e4309d1e622a0e332b9f1b6", "3b04803de51ee7c96423ab5b78d2", 0, 32},
		{"f0f04914b513f2763a1b1fa130f10e2998f6f6e43e4309d1e622a0e332b9f1b6", "3b04803de51ee7c96423ab5b78d2", 1, 20},
		{"f0f04914b513f2763a1b1fa130f10e2998f6f6e43e4309d1e622a0e332b9f1b6", "3b04803de51ee7c96423ab5b78d2", 2, 14},
	};
	size_t i;
	printf(",\"kdf\":[");
	for (i = 0; i < sizeof(v) / sizeof(v[0]); i++) {
		uint8_t key[32], salt[14], out[32];
		size_t kl = strlen(v[i].key) / 2;
		hexparse(key, v[i].key, kl);
		hexparse(salt, v[i].salt, 14);
		srtp_derive(out, (size_t)v[i].outlen, (uint8_t)v[i].label,
			    key, kl, salt, 14);
		printf("%s{\"key\":\"%s\",\"salt\":\"%s\",\"label\":%d,\"out\":",
		       i ? "," : "", v[i].key, v[i].salt, v[i].label);
		hexout(out, (size_t)v[i].outlen);
		printf("}");
	}
	printf("]");
}

/* AES-GCM vectors of test/aes.c:172-396, run through src/aes/openssl */
static void prim_gcm(void)
{
	static const struct { const char *k, *iv, *p, *a; } v[] = {
		{"b52c505a37d78eda5dd34f20c22540ea1b58963cf8e5bf8ffa85f9f2492505b4", "516c33929df5a3284ff463d7", "", ""},
		{"31bdadd96698c204aa9ce1448ea94ae1fb4a9a0b3c9d773b51bb1822666b8f22", "0d18e06c7c725ac9e362e1ce", "2db5168e932556f8089a0622981d017d", ""},
		{"92e11dcdaa866f5ce790fd24501f92509aacf4cb8b1339d50c9c1240935dd08b", "ac93a1a6145299bde902f21a", "2d71bcfa914e4ac045b2aa60955fad24", "1e0889016f67601c8ebea4943bc23ad6"},
		{"eebc1f57487f51921c0465665f8ae6d1658bb26de6f8a069a3520293a572078f", "99aa3e68ed8173a0eed06684", "f56e87055bc32d0eeb31b2eacc2bf2a5", "4d23c3cec334b49bdb370c437fec78de"},
	};
	size_t i;
	printf(",\"gcm\":[");
	for (i = 0; i < sizeof(v) / sizeof(v[0]); i++) {
		uint8_t key[32], iv[16] = {0}, pt[64], aad[64], ct[64], tag[16];
		size_t pl = strlen(v[i].p) / 2, al = strlen(v[i].a) / 2;
		struct aes *aes = NULL;
		hexparse(key, v[i].k, 32);
		hexparse(iv, v[i].iv, 12);
		hexparse(pt, v[i].p, pl);
		hexparse(aad, v[i].a, al);
		aes_alloc(&aes, AES_MODE_GCM, key, 256, iv);
		if (al)
			aes_encr(aes, NULL, aad, al);
		if (pl)
			aes_encr(aes, ct, pt, pl);
		aes_get_authtag(aes, tag, 16);
		mem_deref(aes);
		printf("%s{\"key\":\"%s\",\"iv\":\"%s\",\"pt\":\"%s\",\"aad\":\"%s\",\"ct\":",
		       i ? "," : "", v[i].k, v[i].iv, v[i].p, v[i].a);
		hexout(ct, pl);
		printf(",\"tag\":");
		hexout(tag, 16);
		printf("}");
	}
	printf("]");
}

/* HMAC-SHA1 over random lengths through src/hmac/openssl (hmac.c:78-95) */
static void prim_hmac(void)
{
	size_t i;
	printf(",\"hmac\":[");
	for (i = 0; i < 24; i++) {
		uint8_t key[20], data[1500], md[20];
		size_t dl = i < 12 ? i * 7 : 50 + rndn(1400), k;
		struct hmac *h = NULL;
		for (k = 0; k < 20; k++) key[k] = (uint8_t)rnd();
		for (k = 0; k < dl; k++) data[k] = (uint8_t)rnd();
		hmac_create(&h, HMAC_HASH_SHA1, key, 20);
		if (dl)
			hmac_digest(h, md, 20, data, dl);
		else
			memset(md, 0, 20);  /* hmac_digest rejects len 0 */
		mem_deref(h);
		printf("%s{\"key\":", i ? "," : "");
		hexout(key, 20);
		printf(",\"data\":");
		hexout(data, dl);
		printf(",\"mac\":");
		hexout(md, 20);
		printf("}");
	}
	printf("]");
}

int main(void)
{
	int s, i;

	printf("{\"generator\":\"oracle/gen_golden.c\","
	       "\"reference\":\"baresip/re v4.10.0 src/srtp (OpenSSL %s)\","
	       "\"scenarios\":[", OPENSSL_VERSION_TEXT);

	scn_libsrtp();
	for (s = 0; s < 6; s++) {
		scn_loop(s, 0, 3);
		scn_loop(s, 4, 65530);
	}
	for (s = 0; s < 6; s++) {
		scn_random_srtp(s, 0, 1, 80, 1);
		scn_random_srtp(s, 1, 3, 120, 0);
		scn_truncations(s);
		scn_shared_ctx(s);
	}
	scn_random_srtp(1, 2, 11, 60, 0);   /* > 8 SSRCs: ENOSR */
	scn_random_srtp(4, 2, 11, 60, 0);
	for (s = 0; s < 6; s++) {
		for (i = 0; i < 2; i++)
			scn_random_srtcp(s, 0, i, 40);
		scn_random_srtcp(s, 2, 2, 40);   /* SRTP_UNENCRYPTED_SRTCP */
		scn_srtcp_truncations(s);
	}
	scn_random_srtcp(1, 0, 3, 40);      /* > 8 SSRCs */

	alloc_errors();
	prim_kdf();
	prim_gcm();
	prim_hmac();
	printf("}\n");
	return 0;
}
