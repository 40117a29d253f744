/*
 * srtp.c -- host side of the MI355X SRTP/SRTCP path (plain C).
 *
 * Keeps all SRTP *state* exactly as the reference does (struct srtp_stream,
 * src/srtp/srtp.h:29-38): stream table with the 8-SSRC cap
 * (src/srtp/stream.c:16-109), sender ROC/s_l (srtp.c:203-213, 279-280),
 * receiver index estimation (misc.c:22-41), replay windows
 * (replay.c:32-62), SRTCP index (srtcp.c:54).  Every cipher/MAC operation
 * is delegated to the GPU through the C-ABI shim (../srtpgpu.h); there is
 * no CPU crypto anywhere in the product.
 *
 * Batches.  Each packet is *planned* on the host in array order -- the
 * exact sequence of checks, state updates and mbuf pos/end moves of the
 * reference call -- producing one GPU job.  Unprotect outcomes depend on
 * the MAC/tag verdict, which is only known after the GPU ran, so planning
 * speculates "authentic" and the verdicts are folded afterwards: if a
 * packet turns out forged, planning is replayed from a state snapshot with
 * the known verdicts, and only packets whose job changed run again (a
 * device-resident packet that was already decrypted in place is first
 * restored by re-applying its keystream).  The results are identical to
 * sequential per-packet calls.
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "re_mem.h"
#include "re_mbuf.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"
#include "../srtpgpu.h"

#ifndef EAUTH
#define EAUTH 217               /* include/re_types.h:215-217 */
#endif

#define SRTP_MAX_STREAMS 8      /* src/srtp/stream.c:16-17 */

enum { OP_RTP_ENC = 0, OP_RTP_DEC = 1, OP_RTCP_ENC = 2, OP_RTCP_DEC = 3 };

struct replay {
	uint64_t bitmap;
	uint64_t lix;
};

struct srtp_stream {
	struct replay replay_rtp;
	struct replay replay_rtcp;
	uint32_t ssrc;
	uint32_t roc;
	uint16_t s_l;
	uint8_t s_l_set;
	uint32_t rtcp_index;
};

struct comp {
	int has_aes;
	int mode;               /* SGPU_MODE_* */
	int has_hmac;
	int encrypted;
	uint32_t tag_len;
	uint32_t nr;
	uint32_t dev;           /* sgpu_comp index in the device table */
};

struct srtp {
	struct comp rtp, rtcp;
	struct srtp_stream streams[SRTP_MAX_STREAMS];
	unsigned nstreams;
	uint32_t slot;
	int dev;
};

/* ------------------------------------------------------------------ */
/* device table slots                                                  */

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static uint32_t *g_free;
static uint32_t g_nfree, g_free_cap, g_next_slot;
static int g_gpu_state;         /* 0 unknown, 1 ok, -1 unavailable */

static int gpu_ready(void)
{
	int r;
	pthread_mutex_lock(&g_lock);
	if (g_gpu_state == 0) {
		int e = sgpu_init();
		g_gpu_state = e ? -1 : 1;
		if (e)
			fprintf(stderr, "re_srtp_amd: no HIP device usable "
				"(%s); srtp_alloc returns ENOSYS\n",
				sgpu_last_error());
	}
	r = g_gpu_state;
	pthread_mutex_unlock(&g_lock);
	return r == 1;
}

const char *srtp_gpu_error(void)
{
	return sgpu_last_error();
}

static int slots_get(uint32_t *slots, size_t n)
{
	size_t i;
	int err;
	pthread_mutex_lock(&g_lock);
	for (i = 0; i < n; i++)
		slots[i] = g_nfree ? g_free[--g_nfree] : g_next_slot++;
	err = sgpu_table_reserve(g_next_slot);
	pthread_mutex_unlock(&g_lock);
	return err;
}

static void slot_put(uint32_t s)
{
	pthread_mutex_lock(&g_lock);
	if (g_nfree == g_free_cap) {
		uint32_t nc = g_free_cap ? 2 * g_free_cap : 256;
		uint32_t *nf = realloc(g_free, nc * sizeof(*nf));
		if (nf) {
			g_free = nf;
			g_free_cap = nc;
		}
	}
	if (g_nfree < g_free_cap)
		g_free[g_nfree++] = s;
	pthread_mutex_unlock(&g_lock);
}

/* ------------------------------------------------------------------ */
/* srtp_alloc (srtp.c:88-180)                                          */

static void destructor(void *arg)
{
	struct srtp *srtp = arg;
	slot_put(srtp->slot);
}

struct suite_par {
	int mode;
	uint32_t cipher_bytes, salt_bytes, auth_bytes;
	int hash;
};

static int suite_params(enum srtp_suite suite, struct suite_par *p)
{
	switch (suite) {
	case SRTP_AES_CM_128_HMAC_SHA1_80:
		*p = (struct suite_par){SGPU_MODE_CTR, 16, 14, 10, 1}; return 0;
	case SRTP_AES_CM_128_HMAC_SHA1_32:
		*p = (struct suite_par){SGPU_MODE_CTR, 16, 14, 4, 1}; return 0;
	case SRTP_AES_256_CM_HMAC_SHA1_80:
		*p = (struct suite_par){SGPU_MODE_CTR, 32, 14, 10, 1}; return 0;
	case SRTP_AES_256_CM_HMAC_SHA1_32:
		*p = (struct suite_par){SGPU_MODE_CTR, 32, 14, 4, 1}; return 0;
	case SRTP_AES_128_GCM:
		*p = (struct suite_par){SGPU_MODE_GCM, 16, 12, 0, 0}; return 0;
	case SRTP_AES_256_GCM:
		*p = (struct suite_par){SGPU_MODE_GCM, 32, 12, 0, 0}; return 0;
	default:
		return ENOTSUP;
	}
}

static void comp_set(struct comp *c, const struct suite_par *p, int encrypted,
		     uint32_t dev)
{
	c->mode = p->mode;
	c->encrypted = encrypted;
	c->has_aes = encrypted || p->mode == SGPU_MODE_GCM;  /* srtp.c:59 */
	c->has_hmac = p->hash;
	c->tag_len = p->auth_bytes;
	c->nr = p->cipher_bytes / 4 + 6;
	c->dev = dev;
}

int srtp_alloc_many(struct srtp **srtpv, size_t n, enum srtp_suite suite,
		    const uint8_t *keys, size_t key_bytes, int flags)
{
	struct suite_par p;
	struct sgpu_keyreq *req = NULL;
	uint32_t *slots = NULL;
	size_t i;
	int err;

	if (!srtpv || !keys)
		return EINVAL;
	err = suite_params(suite, &p);
	if (err)
		return err;
	if (p.cipher_bytes + p.salt_bytes != key_bytes)
		return EINVAL;
	if (!gpu_ready())
		return ENOSYS;

	req = calloc(n ? n : 1, sizeof(*req));
	slots = calloc(n ? n : 1, sizeof(*slots));
	if (!req || !slots) {
		err = ENOMEM;
		goto out;
	}
	err = slots_get(slots, n);
	if (err)
		goto out;
	for (i = 0; i < n; i++) {
		memcpy(req[i].master, keys + i * key_bytes, key_bytes);
		req[i].cipher_bytes = p.cipher_bytes;
		req[i].salt_bytes = p.salt_bytes;
		req[i].tag_len = p.auth_bytes;
		req[i].mode = (uint32_t)p.mode;
		req[i].hash = (uint32_t)p.hash;
		req[i].rtcp_encrypted = !(flags & SRTP_UNENCRYPTED_SRTCP);
	}
	pthread_mutex_lock(&g_lock);
	err = sgpu_setup_sessions(req, slots, (uint32_t)n);
	pthread_mutex_unlock(&g_lock);
	if (err) {
		for (i = 0; i < n; i++)
			slot_put(slots[i]);
		goto out;
	}
	for (i = 0; i < n; i++) {
		struct srtp *s = mem_zalloc(sizeof(*s), destructor);
		if (!s) {
			size_t k;
			for (k = i; k < n; k++)
				slot_put(slots[k]);
			while (i--)
				srtpv[i] = mem_deref(srtpv[i]);
			err = ENOMEM;
			goto out;
		}
		s->slot = slots[i];
		s->dev = sgpu_get_device();
		comp_set(&s->rtp, &p, 1, 2 * slots[i]);
		comp_set(&s->rtcp, &p, !(flags & SRTP_UNENCRYPTED_SRTCP),
			 2 * slots[i] + 1);
		srtpv[i] = s;
	}
 out:
	free(req);
	free(slots);
	return err;
}

int srtp_alloc(struct srtp **srtpp, enum srtp_suite suite,
	       const uint8_t *key, size_t key_bytes, int flags)
{
	if (!srtpp || !key)
		return EINVAL;
	return srtp_alloc_many(srtpp, 1, suite, key, key_bytes, flags);
}

/* misc.c:108-120 */
const char *srtp_suite_name(enum srtp_suite suite)
{
	switch (suite) {
	case SRTP_AES_CM_128_HMAC_SHA1_32:  return "AES_CM_128_HMAC_SHA1_32";
	case SRTP_AES_CM_128_HMAC_SHA1_80:  return "AES_CM_128_HMAC_SHA1_80";
	case SRTP_AES_256_CM_HMAC_SHA1_32:  return "AES_256_CM_HMAC_SHA1_32";
	case SRTP_AES_256_CM_HMAC_SHA1_80:  return "AES_256_CM_HMAC_SHA1_80";
	case SRTP_AES_128_GCM:              return "AEAD_AES_128_GCM";
	case SRTP_AES_256_GCM:              return "AEAD_AES_256_GCM";
	default:                            return "?";
	}
}

/* ------------------------------------------------------------------ */
/* stream table, index, replay                                          */

/* stream.c:29-84: find by SSRC in creation order; the 9th -> ENOSR */
static int stream_get(struct srtp_stream **sp, struct srtp *s, uint32_t ssrc)
{
	unsigned i;
	for (i = 0; i < s->nstreams; i++)
		if (s->streams[i].ssrc == ssrc) {
			*sp = &s->streams[i];
			return 0;
		}
	if (s->nstreams >= SRTP_MAX_STREAMS)
		return ENOSR;
	memset(&s->streams[s->nstreams], 0, sizeof(s->streams[0]));
	s->streams[s->nstreams].ssrc = ssrc;
	*sp = &s->streams[s->nstreams++];
	return 0;
}

/* stream.c:87-109 */
static int stream_get_seq(struct srtp_stream **sp, struct srtp *s,
			  uint32_t ssrc, uint16_t seq)
{
	struct srtp_stream *st;
	int err = stream_get(&st, s, ssrc);
	if (err)
		return err;
	if (!st->s_l_set) {
		st->s_l = seq;
		st->s_l_set = 1;
	}
	*sp = st;
	return 0;
}

/* replay.c:32-62 (64-packet window) */
static int replay_check(struct replay *r, uint64_t ix)
{
	uint64_t diff;
	if (ix > r->lix) {
		diff = ix - r->lix;
		if (diff < 64) {
			r->bitmap <<= diff;
			r->bitmap |= 1;
		}
		else
			r->bitmap = 1;
		r->lix = ix;
		return 1;
	}
	diff = r->lix - ix;
	if (diff >= 64)
		return 0;
	if (r->bitmap & (1ULL << diff))
		return 0;
	r->bitmap |= (1ULL << diff);
	return 1;
}

/* misc.c:22-41, including the `int v` sign extension of roc+-1 */
static uint64_t get_index(uint32_t roc, uint16_t s_l, uint16_t seq)
{
	int32_t v;
	if (s_l < 32768) {
		if ((int)seq - (int)s_l > 32768)
			v = (int32_t)(roc - 1);
		else
			v = (int32_t)roc;
	}
	else {
		if ((int)s_l - 32768 > seq)
			v = (int32_t)(roc + 1);
		else
			v = (int32_t)roc;
	}
	return seq + (uint64_t)(int64_t)v * 65536ull;
}

/* ------------------------------------------------------------------ */
/* per-packet planning                                                  */

struct pinfo {
	uint32_t start, end, size;
	uint32_t hdr_len;       /* UINT32_MAX on EBADMSG */
	uint32_t err_pos;       /* bytes consumed before EBADMSG */
	uint32_t ssrc;
	uint16_t seq;
	uint32_t eix[3];        /* RTCP: BE word at end-4-tl, tl = 0, 4, 10 */
	uint8_t fixed;          /* device arena: size is a hard cap */
};

struct rec {
	int32_t err;
	uint32_t pos_o, end_o, size_o;
	uint8_t has_job;
	uint8_t need_run;
	uint8_t ran;
	uint8_t vd;             /* verdict bits of the last run */
	uint8_t need_undo;
	uint32_t in_end;        /* stage bytes [start, in_end) */
	uint32_t ext_end;       /* GPU may write up to here */
	struct sgpu_job job;
	struct sgpu_job ran_job;
	uint32_t save;          /* original tag word (device path undo) */
};

static uint32_t grow(uint32_t size, uint32_t need)
{
	/* mbuf_write_mem growth (src/mbuf/mbuf.c:244-252) */
	if (need > size) {
		uint32_t d = size ? size * 2 : 512;
		size = need > d ? need : d;
	}
	return size;
}

/* RTP header parse over host bytes (rtp.c:88-137) */
static void parse_rtp(struct pinfo *pi, const uint8_t *buf)
{
	const uint32_t left = pi->end > pi->start ? pi->end - pi->start : 0;
	const uint8_t *b = buf + pi->start;
	uint32_t cc, hl = 12;

	pi->hdr_len = UINT32_MAX;
	pi->err_pos = 0;
	if (left < 12)
		return;
	cc = b[0] & 0x0f;
	pi->seq = (uint16_t)(b[2] << 8 | b[3]);
	pi->ssrc = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 |
		   (uint32_t)b[10] << 8 | b[11];
	if (left - hl < 4 * cc) {
		pi->err_pos = hl;
		return;
	}
	hl += 4 * cc;
	if (b[0] & 0x10) {
		uint32_t xl;
		if (left - hl < 4) {
			pi->err_pos = hl;
			return;
		}
		xl = (uint32_t)b[hl + 2] << 8 | b[hl + 3];
		hl += 4;
		if (left - hl < 4 * xl) {
			pi->err_pos = hl;
			return;
		}
		hl += 4 * xl;
	}
	pi->hdr_len = hl;
}

static uint32_t rd_be32(const uint8_t *p)
{
	return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 |
	       (uint32_t)p[2] << 8 | p[3];
}

static void parse_rtcp(struct pinfo *pi, const uint8_t *buf)
{
	const uint32_t left = pi->end > pi->start ? pi->end - pi->start : 0;
	static const uint32_t tl[3] = {0, 4, 10};
	int k;
	pi->hdr_len = UINT32_MAX;
	pi->err_pos = 0;
	if (left < 8)
		return;
	pi->ssrc = rd_be32(buf + pi->start + 4);
	pi->hdr_len = 8;
	for (k = 0; k < 3; k++)
		pi->eix[k] = left >= 8 + 4 + tl[k] ?
			rd_be32(buf + pi->end - 4 - tl[k]) : 0;
}

static int same_job(const struct sgpu_job *a, const struct sgpu_job *b)
{
	return memcmp(a, b, sizeof(*a)) == 0;
}

/* decide the verdict for this plan: known from an identical previous run,
 * or speculated authentic (then the job must run) */
static int verdict_for(struct rec *r)
{
	if (r->ran && same_job(&r->job, &r->ran_job)) {
		r->need_run = 0;
		return (r->vd & SV_TAG_OK) != 0;
	}
	r->need_run = 1;
	return 1;
}

static void no_job(struct rec *r, int err, uint32_t pos, uint32_t end,
		   uint32_t size)
{
	r->err = err;
	r->pos_o = pos;
	r->end_o = end;
	r->size_o = size;
	r->has_job = 0;
	r->need_run = 0;
}

static void job_base(struct rec *r, const struct comp *c,
		     const struct pinfo *pi, uint32_t ssrc, uint64_t ix)
{
	memset(&r->job, 0, sizeof(r->job));
	r->job.off = pi->start;
	r->job.comp = c->dev;
	r->job.ssrc = ssrc;
	r->job.ixhi = (uint32_t)(ix >> 16);
	r->job.ixlo = (uint16_t)ix;
	r->has_job = 1;
}

/*
 * Device arenas cannot grow the way mbuf_write_mem does; a protect whose
 * appended tag/trailer would not fit in cap[i] fails with ENOMEM right
 * after the stream lookup, before the ROC/index/s_l updates (documented
 * deviation of the batch extension; the mbuf API grows like the
 * reference).
 */
static int cap_short(const struct pinfo *pi, const struct comp *c, int rtcp)
{
	uint32_t need;
	if (!pi->fixed)
		return 0;
	if (rtcp)
		need = (c->mode == SGPU_MODE_GCM ? 16u : 0u) + 4u + c->tag_len;
	else
		need = c->mode == SGPU_MODE_GCM ? 16u
		       : (c->tag_len > 4 ? c->tag_len : 4u);
	return (uint64_t)pi->end + need > pi->size;
}

/* srtp_encrypt, srtp.c:183-285 */
static void plan_rtp_enc(struct srtp *s, const struct pinfo *pi,
			 struct rec *r)
{
	const struct comp *c = &s->rtp;
	struct srtp_stream *st;
	uint32_t start = pi->start, end = pi->end, size = pi->size, pld;
	uint64_t ix;
	int err;

	if (pi->hdr_len == UINT32_MAX) {
		no_job(r, EBADMSG, start + pi->err_pos, end, size);
		return;
	}
	pld = start + pi->hdr_len;
	err = stream_get_seq(&st, s, pi->ssrc, pi->seq);
	if (err) {
		no_job(r, err, pld, end, size);
		return;
	}
	if (cap_short(pi, c, 0)) {
		no_job(r, ENOMEM, pld, end, size);
		return;
	}
	if ((int)pi->seq - (int)st->s_l <= -32768) {
		st->roc++;
		st->s_l = 0;
	}
	ix = 65536ULL * st->roc + pi->seq;

	job_base(r, c, pi, st->ssrc, ix);
	r->job.c_off = pi->hdr_len;
	r->job.c_len = end - pld;
	r->in_end = end;
	r->ext_end = end;
	if (c->has_aes && c->mode == SGPU_MODE_CTR) {
		r->job.flags |= SJ_CIPHER;
	}
	else if (c->has_aes && c->mode == SGPU_MODE_GCM) {
		r->job.flags |= SJ_CIPHER | SJ_GCM;
		r->job.a_len = pi->hdr_len;
		r->job.tag_off = end - start;
		size = grow(size, end + 16);
		end += 16;
		r->ext_end = end;
	}
	if (c->has_hmac) {
		r->job.flags |= SJ_HMAC | SJ_TRAILER;
		r->job.a_len = end - start;
		r->job.trailer = st->roc;
		r->job.tag_off = end - start;
		size = grow(size, end + 4);
		size = grow(size, end + c->tag_len);
		end += c->tag_len;
		r->ext_end = end;
	}
	r->job.flags |= SJ_PROTECT;
	(void)verdict_for(r);
	if (pi->seq > st->s_l)
		st->s_l = pi->seq;
	r->err = 0;
	r->pos_o = start;
	r->end_o = end;
	r->size_o = size;
}

/* srtp_decrypt, srtp.c:288-432 */
static void plan_rtp_dec(struct srtp *s, const struct pinfo *pi,
			 struct rec *r)
{
	const struct comp *c = &s->rtp;
	struct srtp_stream *st;
	uint32_t start = pi->start, end = pi->end, size = pi->size, pld;
	uint64_t ix;
	int diff, err, ok;

	if (pi->hdr_len == UINT32_MAX) {
		no_job(r, EBADMSG, start + pi->err_pos, end, size);
		return;
	}
	pld = start + pi->hdr_len;
	err = stream_get_seq(&st, s, pi->ssrc, pi->seq);
	if (err) {
		no_job(r, err, pld, end, size);
		return;
	}
	diff = (int)pi->seq - (int)st->s_l;
	if (diff > 32768) {
		no_job(r, ETIMEDOUT, pld, end, size);
		return;
	}
	if (diff <= -32768) {
		st->roc++;
		st->s_l = 0;
	}
	ix = get_index(st->roc, st->s_l, pi->seq);

	if (c->has_hmac) {
		uint32_t tag_start;
		struct replay rp;
		int rp_ok;

		if (end - pld < c->tag_len) {
			no_job(r, EBADMSG, pld, end, size);
			return;
		}
		tag_start = end - c->tag_len;
		/* MAC over hdr‖ct‖ROC; the ROC is written at tag_start
		 * (srtp.c:342-344) by the kernel (SJ_ROC_AT_TAG) */
		job_base(r, c, pi, st->ssrc, ix);
		r->job.flags = SJ_HMAC | SJ_TRAILER | SJ_ROC_AT_TAG;
		r->job.a_len = tag_start - start;
		r->job.trailer = st->roc;
		r->job.tag_off = tag_start - start;
		r->job.c_off = pi->hdr_len;
		r->job.c_len = tag_start - pld;
		r->in_end = end;
		r->ext_end = end;
		/* the replay verdict if the tag is authentic decides whether
		 * the kernel decrypts (srtp.c:367-382) */
		rp = st->replay_rtp;
		rp_ok = replay_check(&rp, ix);
		if (rp_ok && c->has_aes && c->mode == SGPU_MODE_CTR)
			r->job.flags |= SJ_CIPHER | SJ_CIPHER_IF_OK;
		ok = verdict_for(r);
		if (!ok) {
			r->err = EAUTH;
			r->pos_o = pld;
			r->end_o = tag_start;
			r->size_o = size;
			return;
		}
		st->replay_rtp = rp;
		if (!rp_ok) {
			r->err = EALREADY;
			r->pos_o = pld;
			r->end_o = tag_start;
			r->size_o = size;
			return;
		}
		end = tag_start;
	}
	else if (c->has_aes && c->mode == SGPU_MODE_GCM) {
		uint32_t tag_start;
		if (end - pld < 16) {
			no_job(r, EBADMSG, pld, end, size);
			return;
		}
		tag_start = end - 16;
		job_base(r, c, pi, st->ssrc, ix);
		r->job.flags = SJ_GCM | SJ_CIPHER;
		r->job.a_len = pi->hdr_len;
		r->job.c_off = pi->hdr_len;
		r->job.c_len = tag_start - pld;
		r->job.tag_off = tag_start - start;
		r->in_end = end;
		r->ext_end = end;
		ok = verdict_for(r);
		if (!ok) {
			/* plaintext stays in place, end untouched (srtp.c:404) */
			r->err = EAUTH;
			r->pos_o = pld;
			r->end_o = end;
			r->size_o = size;
			return;
		}
		end = tag_start;
		if (!replay_check(&st->replay_rtp, ix)) {
			r->err = EALREADY;
			r->pos_o = pld;
			r->end_o = end;
			r->size_o = size;
			return;
		}
	}
	if (pi->seq > st->s_l)
		st->s_l = pi->seq;
	r->err = 0;
	r->pos_o = start;
	r->end_o = end;
	r->size_o = size;
}

/* srtcp_encrypt, srtcp.c:31-140 */
static void plan_rtcp_enc(struct srtp *s, const struct pinfo *pi,
			  struct rec *r)
{
	const struct comp *c = &s->rtcp;
	struct srtp_stream *st;
	uint32_t start = pi->start, end = pi->end, size = pi->size, ep = 0;
	uint32_t eword;
	int err;

	if (pi->hdr_len == UINT32_MAX) {
		no_job(r, EBADMSG, start, end, size);
		return;
	}
	err = stream_get(&st, s, pi->ssrc);
	if (err) {
		no_job(r, err, start + 8, end, size);
		return;
	}
	if (cap_short(pi, c, 1)) {
		no_job(r, ENOMEM, start + 8, end, size);
		return;
	}
	st->rtcp_index = (st->rtcp_index + 1) & 0x7fffffff;

	job_base(r, c, pi, pi->ssrc, st->rtcp_index);
	r->in_end = end;
	r->job.c_off = 8;
	r->job.c_len = end - (start + 8);
	if (c->has_aes && c->mode == SGPU_MODE_CTR) {
		r->job.flags |= SJ_CIPHER;
		ep = 1;
	}
	else if (c->has_aes && c->mode == SGPU_MODE_GCM) {
		ep = c->encrypted ? 1 : 0;
		r->job.flags |= SJ_GCM | SJ_TRAILER;
		r->job.trailer = ep << 31 | st->rtcp_index;
		if (c->encrypted) {
			r->job.flags |= SJ_CIPHER;
			r->job.a_len = 8;
		}
		else {
			r->job.a_len = end - start;
			r->job.c_len = 0;
		}
		r->job.tag_off = end - start;
		size = grow(size, end + 16);
		end += 16;
	}
	eword = ep << 31 | st->rtcp_index;
	r->job.flags |= SJ_STORE_TRAIL;
	r->job.t_off = end - start;
	r->job.trailer = eword;
	size = grow(size, end + 4);
	end += 4;
	if (c->has_hmac) {
		r->job.flags |= SJ_HMAC | SJ_TRAILER;
		r->job.a_len = end - 4 - start;
		r->job.tag_off = end - start;
		size = grow(size, end + c->tag_len);
		end += c->tag_len;
	}
	r->job.flags |= SJ_PROTECT;
	r->ext_end = end;
	(void)verdict_for(r);
	r->err = 0;
	r->pos_o = start;
	r->end_o = end;
	r->size_o = size;
}

/* srtcp_decrypt, srtcp.c:143-287 */
static void plan_rtcp_dec(struct srtp *s, const struct pinfo *pi,
			  struct rec *r)
{
	const struct comp *c = &s->rtcp;
	struct srtp_stream *st;
	uint32_t start = pi->start, end = pi->end, size = pi->size;
	uint32_t pld, eix_start, v, ix;
	int ep, err;

	if (pi->hdr_len == UINT32_MAX) {
		no_job(r, EBADMSG, start, end, size);
		return;
	}
	pld = start + 8;
	err = stream_get(&st, s, pi->ssrc);
	if (err) {
		no_job(r, err, pld, end, size);
		return;
	}
	if (end - pld < 4 + c->tag_len) {
		no_job(r, EBADMSG, pld, end, size);
		return;
	}
	eix_start = end - (4 + c->tag_len);
	v = pi->eix[c->tag_len == 0 ? 0 : (c->tag_len == 4 ? 1 : 2)];
	ep = (v >> 31) & 1;
	ix = v & 0x7fffffff;

	job_base(r, c, pi, pi->ssrc, ix);
	r->in_end = end;
	r->ext_end = end;
	if (c->has_hmac) {
		const uint32_t tag_start = eix_start + 4;
		struct replay rp;
		int rp_ok, ok;

		r->job.flags = SJ_HMAC;
		r->job.a_len = tag_start - start;
		r->job.tag_off = tag_start - start;
		r->job.c_off = 8;
		r->job.c_len = eix_start - pld;
		rp = st->replay_rtcp;
		rp_ok = replay_check(&rp, ix);
		if (rp_ok && c->has_aes && ep && c->mode == SGPU_MODE_CTR)
			r->job.flags |= SJ_CIPHER | SJ_CIPHER_IF_OK;
		ok = verdict_for(r);
		if (!ok) {
			r->err = EAUTH;
			r->pos_o = start;
			r->end_o = tag_start;
			r->size_o = size;
			return;
		}
		st->replay_rtcp = rp;
		if (!rp_ok) {
			r->err = EALREADY;
			r->pos_o = start;
			r->end_o = tag_start;
			r->size_o = size;
			return;
		}
		end = eix_start;
	}
	else {
		end = eix_start;
	}
	if (c->has_aes && ep && c->mode == SGPU_MODE_CTR) {
		/* decrypted by the kernel (CIPHER_IF_OK) */
	}
	else if (c->has_aes && c->mode == SGPU_MODE_GCM) {
		uint32_t tag_start;
		int ok;
		if (eix_start - pld < 16) {
			no_job(r, EBADMSG, pld, end, size);
			return;
		}
		tag_start = eix_start - 16;
		r->job.flags = SJ_GCM | SJ_TRAILER;
		r->job.trailer = v;
		r->job.tag_off = tag_start - start;
		if (ep) {
			r->job.flags |= SJ_CIPHER;
			r->job.a_len = 8;
			r->job.c_off = 8;
			r->job.c_len = tag_start - pld;
		}
		else {
			r->job.a_len = tag_start - start;
			r->job.c_off = 8;
			r->job.c_len = 0;
		}
		ok = verdict_for(r);
		if (!ok) {
			r->err = EAUTH;
			r->pos_o = pld;
			r->end_o = end;
			r->size_o = size;
			return;
		}
		end = tag_start;
	}
	else if (!c->has_hmac) {
		r->has_job = 0;
	}
	r->err = 0;
	r->pos_o = start;
	r->end_o = end;
	r->size_o = size;
}

/* ------------------------------------------------------------------ */
/* the batch engine                                                     */

struct engine {
	int op;
	size_t n;
	struct srtp **sess;        /* per packet session */
	struct pinfo *pi;
	struct rec *rec;
	/* snapshot of every distinct session's stream state */
	struct srtp **uniq;
	size_t nuniq;
	struct srtp *snap;
};

static void snap_take(struct engine *E)
{
	size_t i;
	for (i = 0; i < E->nuniq; i++)
		E->snap[i] = *E->uniq[i];
}

static void snap_restore(struct engine *E)
{
	size_t i;
	for (i = 0; i < E->nuniq; i++)
		*E->uniq[i] = E->snap[i];
}

static size_t plan_all(struct engine *E)
{
	size_t i, need = 0;
	for (i = 0; i < E->n; i++) {
		struct rec *r = &E->rec[i];
		r->has_job = 0;
		switch (E->op) {
		case OP_RTP_ENC:  plan_rtp_enc(E->sess[i], &E->pi[i], r);  break;
		case OP_RTP_DEC:  plan_rtp_dec(E->sess[i], &E->pi[i], r);  break;
		case OP_RTCP_ENC: plan_rtcp_enc(E->sess[i], &E->pi[i], r); break;
		case OP_RTCP_DEC: plan_rtcp_dec(E->sess[i], &E->pi[i], r); break;
		}
		if (!r->has_job)
			r->need_run = 0;
		if (r->need_run)
			need++;
	}
	return need;
}

static int engine_init(struct engine *E, int op, size_t n,
		       struct srtp **sessv, size_t nsess, const uint32_t *sidx)
{
	size_t i;
	memset(E, 0, sizeof(*E));
	E->op = op;
	E->n = n;
	E->sess = malloc((n ? n : 1) * sizeof(*E->sess));
	E->pi = calloc(n ? n : 1, sizeof(*E->pi));
	E->rec = calloc(n ? n : 1, sizeof(*E->rec));
	E->uniq = malloc((nsess ? nsess : 1) * sizeof(*E->uniq));
	E->snap = malloc((nsess ? nsess : 1) * sizeof(*E->snap));
	if (!E->sess || !E->pi || !E->rec || !E->uniq || !E->snap)
		return ENOMEM;
	for (i = 0; i < n; i++) {
		uint32_t k = sidx ? sidx[i] : 0;
		if (k >= nsess || !sessv[k])
			return EINVAL;
		E->sess[i] = sessv[k];
	}
	/* distinct sessions referenced (array order of sessv) */
	{
		uint8_t *used = calloc(nsess ? nsess : 1, 1);
		if (!used)
			return ENOMEM;
		for (i = 0; i < n; i++)
			used[sidx ? sidx[i] : 0] = 1;
		for (i = 0; i < nsess; i++)
			if (used[i])
				E->uniq[E->nuniq++] = sessv[i];
		free(used);
	}
	return 0;
}

static void engine_free(struct engine *E)
{
	free(E->sess);
	free(E->pi);
	free(E->rec);
	free(E->uniq);
	free(E->snap);
}

/* ---- GPU rounds ----------------------------------------------------- */

struct pool {
	uint8_t *h;             /* pinned host */
	uint8_t *d;             /* device */
	size_t cap;
};

struct ws {
	void *stream;
	struct pool ctl;        /* jobs | verdict | save */
	struct pool stage;      /* host path: packet bytes */
	struct pool hdr;        /* device path: pos/end, parsed headers */
	uint32_t *cls_idx;
	size_t cls_cap;
};

static __thread struct ws *t_ws;

static struct ws *ws_get(void)
{
	if (!t_ws) {
		t_ws = calloc(1, sizeof(*t_ws));
		if (!t_ws)
			return NULL;
		t_ws->stream = sgpu_stream_create();
		if (!t_ws->stream) {
			free(t_ws);
			t_ws = NULL;
		}
	}
	return t_ws;
}

static int pool_reserve(struct ws *w, struct pool *p, size_t bytes)
{
	size_t c;
	if (bytes <= p->cap)
		return 0;
	c = bytes + bytes / 2 + 4096;
	sgpu_stream_sync(w->stream);
	sgpu_host_free(p->h);
	sgpu_free(p->d);
	p->h = sgpu_host_alloc(c);
	p->d = sgpu_malloc(c);
	if (!p->h || !p->d) {
		sgpu_host_free(p->h);
		sgpu_free(p->d);
		p->h = p->d = NULL;
		p->cap = 0;
		return ENOMEM;
	}
	p->cap = c;
	return 0;
}

static int idx_reserve(struct ws *w, size_t n)
{
	if (n > w->cls_cap) {
		size_t c = n + n / 2 + 64;
		uint32_t *ix = realloc(w->cls_idx, c * sizeof(*ix));
		if (!ix)
			return ENOMEM;
		w->cls_idx = ix;
		w->cls_cap = c;
	}
	return 0;
}

static const struct comp *op_comp(int op, const struct srtp *s)
{
	return (op == OP_RTP_ENC || op == OP_RTP_DEC) ? &s->rtp : &s->rtcp;
}

/* kernel class of a job: (mode, nr, shift) -> 0..15 */
static unsigned job_class(const struct sgpu_job *j, const struct comp *c)
{
	unsigned mode = (j->flags & SJ_GCM) ? 1u : 0u;
	unsigned nr14 = c->nr == 14 ? 1u : 0u;
	unsigned shift = mode ? 0u : ((j->c_off >> 2) & 3u);
	return mode << 3 | nr14 << 2 | shift;
}

enum { SEL_RUN = 0, SEL_UNDO = 1 };

static int undo_job(const struct rec *r, struct sgpu_job *u)
{
	if (!(r->ran && (r->vd & SV_CIPHERED)))
		return 0;
	*u = r->ran_job;
	if (u->flags & SJ_GCM)
		u->flags = SJ_GCM | SJ_CIPHER | SJ_UNDO;
	else
		u->flags = SJ_CIPHER;
	return 1;
}

/*
 * Build the class-sorted job list (pinned), upload it and launch.  SEL_RUN
 * takes every planned job with need_run; SEL_UNDO takes the re-apply-
 * keystream jobs of packets about to be re-run.  joff (optional) maps a
 * packet to its byte offset in the device arena.  Returns #jobs in *pm.
 */
static int round_launch(struct ws *w, struct engine *E, int sel,
			uint8_t *arena_d, uint64_t asz, const uint32_t *joff,
			int prot, uint32_t *pm)
{
	uint32_t cnt[16] = {0}, start[17], k, m = 0;
	size_t i, need = 0;
	struct sgpu_job *jh, *jd;
	uint8_t *vd;
	int err;

	for (i = 0; i < E->n; i++) {
		const struct rec *r = &E->rec[i];
		struct sgpu_job u;
		if (sel == SEL_RUN ? r->need_run : (r->need_run && undo_job(r, &u)))
			need++;
	}
	*pm = 0;
	if (!need)
		return 0;
	err = pool_reserve(w, &w->ctl, need * (sizeof(struct sgpu_job) + 5));
	if (!err)
		err = idx_reserve(w, need);
	if (err)
		return err;
	jh = (struct sgpu_job *)w->ctl.h;
	jd = (struct sgpu_job *)w->ctl.d;
	vd = w->ctl.d + need * sizeof(struct sgpu_job);

	for (i = 0; i < E->n; i++) {
		const struct rec *r = &E->rec[i];
		struct sgpu_job u;
		const struct sgpu_job *j = &r->job;
		if (sel == SEL_RUN) {
			if (!r->need_run)
				continue;
		}
		else {
			if (!(r->need_run && undo_job(r, &u)))
				continue;
			j = &u;
		}
		cnt[job_class(j, op_comp(E->op, E->sess[i]))]++;
	}
	start[0] = 0;
	for (k = 0; k < 16; k++)
		start[k + 1] = start[k] + cnt[k];
	memset(cnt, 0, sizeof(cnt));
	for (i = 0; i < E->n; i++) {
		const struct rec *r = &E->rec[i];
		struct sgpu_job u, jb;
		unsigned c;
		uint32_t slot;
		if (sel == SEL_RUN) {
			if (!r->need_run)
				continue;
			jb = r->job;
		}
		else {
			if (!(r->need_run && undo_job(r, &u)))
				continue;
			jb = u;
		}
		c = job_class(&jb, op_comp(E->op, E->sess[i]));
		slot = start[c] + cnt[c]++;
		if (joff)
			jb.off = joff[i];
		jh[slot] = jb;
		w->cls_idx[slot] = (uint32_t)i;
		m++;
	}
	err = sgpu_memcpy_h2d(jd, jh, m * sizeof(struct sgpu_job), w->stream);
	if (err)
		return err;
	for (k = 0; k < 16; k++) {
		uint32_t a = start[k], b = start[k + 1];
		if (a == b)
			continue;
		err = sgpu_run_class(arena_d, asz, jd + a, b - a, vd + a,
				     (uint32_t *)(vd + m) + a, (k >> 3) & 1,
				     (k >> 2) & 1 ? 14 : 10, (int)(k & 3),
				     sel == SEL_RUN ? prot : 0, w->stream);
		if (err)
			return err;
	}
	*pm = m;
	return 0;
}

/* D2H of verdicts + saved tag words for the m jobs just launched */
static int round_fetch(struct ws *w, uint32_t m)
{
	size_t off = (size_t)m * sizeof(struct sgpu_job);
	if (!m)
		return 0;
	return sgpu_memcpy_d2h(w->ctl.h + off, w->ctl.d + off, (size_t)m * 5,
			       w->stream);
}

static void round_collect(struct ws *w, struct engine *E, uint32_t m)
{
	const uint8_t *v = w->ctl.h + (size_t)m * sizeof(struct sgpu_job);
	const uint32_t *sv = (const uint32_t *)(v + m);
	uint32_t k;
	for (k = 0; k < m; k++) {
		struct rec *r = &E->rec[w->cls_idx[k]];
		r->ran = 1;
		r->ran_job = r->job;
		r->vd = v[k];
		if (r->job.flags & SJ_ROC_AT_TAG)
			r->save = sv[k];
	}
}

/* ---- host-resident front-end (mbufs) -------------------------------- */

static int run_mbufs(int op, struct srtp *srtp, struct mbuf **mbv, int *errv,
		     size_t n)
{
	const int prot = op == OP_RTP_ENC || op == OP_RTCP_ENC;
	struct engine E;
	struct ws *w;
	uint8_t **outp = NULL;      /* where packet i's GPU output lives */
	uint8_t *keep = NULL;       /* per-packet copies across rounds */
	uint32_t *soff = NULL;      /* staging offsets */
	size_t *koff = NULL, i, round;
	int err;

	if (!srtp || !mbv)
		return EINVAL;
	for (i = 0; i < n; i++)
		if (!mbv[i])
			return EINVAL;
	err = engine_init(&E, op, n, &srtp, 1, NULL);
	if (err)
		goto out;
	outp = calloc(n ? n : 1, sizeof(*outp));
	soff = calloc(n ? n : 1, sizeof(*soff));
	koff = calloc(n ? n : 1, sizeof(*koff));
	if (!outp || !soff || !koff) {
		err = ENOMEM;
		goto out;
	}
	for (i = 0; i < n; i++) {
		struct mbuf *mb = mbv[i];
		struct pinfo *pi = &E.pi[i];
		pi->start = (uint32_t)mb->pos;
		pi->end = (uint32_t)mb->end;
		pi->size = (uint32_t)mb->size;
		if (op == OP_RTP_ENC || op == OP_RTP_DEC)
			parse_rtp(pi, mb->buf);
		else
			parse_rtcp(pi, mb->buf);
	}
	w = ws_get();
	if (!w) {
		err = ENOMEM;
		goto out;
	}

	snap_take(&E);
	for (round = 0;; round++) {
		size_t need, bytes = 0;
		uint32_t m;

		snap_restore(&E);
		need = plan_all(&E);
		if (!need)
			break;
		if (round > n + 2) {
			err = EIO;
			goto out;
		}
		if (round == 1) {
			/* staging is about to be reused: move outputs aside */
			size_t tot = 0;
			for (i = 0; i < n; i++)
				if (outp[i]) {
					koff[i] = tot;
					tot += E.rec[i].ext_end - E.pi[i].start;
				}
			keep = malloc(tot ? tot : 1);
			if (!keep) {
				err = ENOMEM;
				goto out;
			}
		}
		if (round >= 1) {
			for (i = 0; i < n; i++)
				if (outp[i] && outp[i] != keep + koff[i]) {
					memcpy(keep + koff[i], outp[i],
					       E.rec[i].ext_end - E.pi[i].start);
					outp[i] = keep + koff[i];
				}
		}
		/* stage the packets that need a run at 16-B aligned offsets */
		for (i = 0; i < n; i++) {
			const struct rec *r = &E.rec[i];
			if (!r->need_run)
				continue;
			soff[i] = (uint32_t)bytes;
			bytes += ((r->ext_end - E.pi[i].start) + 31u) & ~15u;
		}
		err = pool_reserve(w, &w->stage, bytes);
		if (err)
			goto out;
		for (i = 0; i < n; i++) {
			const struct rec *r = &E.rec[i];
			if (!r->need_run)
				continue;
			memcpy(w->stage.h + soff[i], mbv[i]->buf + E.pi[i].start,
			       r->in_end - E.pi[i].start);
		}
		err = sgpu_memcpy_h2d(w->stage.d, w->stage.h, bytes, w->stream);
		if (!err) {
			/* job offsets are relative to the packet start */
			for (i = 0; i < n; i++)
				if (E.rec[i].need_run)
					E.rec[i].job.off = E.pi[i].start;
			err = round_launch(w, &E, SEL_RUN, w->stage.d, bytes,
					   soff, prot, &m);
		}
		if (!err)
			err = round_fetch(w, m);
		if (!err)
			err = sgpu_memcpy_d2h(w->stage.h, w->stage.d, bytes,
					      w->stream);
		if (!err)
			err = sgpu_stream_sync(w->stream);
		if (err)
			goto out;
		round_collect(w, &E, m);
		for (i = 0; i < n; i++)
			if (E.rec[i].need_run)
				outp[i] = w->stage.h + soff[i];
	}

	/* unpack: bytes, mbuf size growth (same policy), pos/end, errno */
	for (i = 0; i < n; i++) {
		const struct rec *r = &E.rec[i];
		struct mbuf *mb = mbv[i];
		const struct pinfo *pi = &E.pi[i];
		if (r->size_o > mb->size) {
			err = mbuf_resize(mb, r->size_o);
			if (err)
				goto out;
		}
		if (r->has_job && outp[i])
			memcpy(mb->buf + pi->start, outp[i],
			       r->ext_end - pi->start);
		mb->pos = r->pos_o;
		mb->end = r->end_o;
		if (errv)
			errv[i] = r->err;
	}
 out:
	free(outp);
	free(keep);
	free(soff);
	free(koff);
	engine_free(&E);
	return err;
}

int srtp_encrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
		       size_t n)
{
	return run_mbufs(OP_RTP_ENC, srtp, mbv, errv, n);
}

int srtp_decrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
		       size_t n)
{
	return run_mbufs(OP_RTP_DEC, srtp, mbv, errv, n);
}

int srtcp_encrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
			size_t n)
{
	return run_mbufs(OP_RTCP_ENC, srtp, mbv, errv, n);
}

int srtcp_decrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
			size_t n)
{
	return run_mbufs(OP_RTCP_DEC, srtp, mbv, errv, n);
}

static int one(int op, struct srtp *srtp, struct mbuf *mb)
{
	int e = 0, err;
	if (!srtp || !mb)
		return EINVAL;
	err = run_mbufs(op, srtp, &mb, &e, 1);
	return err ? err : e;
}

int srtp_encrypt(struct srtp *srtp, struct mbuf *mb)
{
	return one(OP_RTP_ENC, srtp, mb);
}

int srtp_decrypt(struct srtp *srtp, struct mbuf *mb)
{
	return one(OP_RTP_DEC, srtp, mb);
}

int srtcp_encrypt(struct srtp *srtp, struct mbuf *mb)
{
	return one(OP_RTCP_ENC, srtp, mb);
}

int srtcp_decrypt(struct srtp *srtp, struct mbuf *mb)
{
	return one(OP_RTCP_DEC, srtp, mb);
}

/* ---- device-resident front-end ---------------------------------------- */

static int run_batch(int op, struct srtp **sessv, size_t nsess,
		     struct srtp_batch *b)
{
	const int prot = op == OP_RTP_ENC || op == OP_RTCP_ENC;
	const int rtcp = op == OP_RTCP_ENC || op == OP_RTCP_DEC;
	struct engine E;
	struct ws *w;
	void *stream;
	size_t i, round, n;
	uint32_t *pe_h;
	struct sgpu_hdr *hd_h;
	uint32_t *eix_h;
	int err;

	if (!sessv || !nsess || !b || !b->arena || !b->pos || !b->end ||
	    !b->cap || !b->err)
		return EINVAL;
	n = b->n;
	if (n > UINT32_MAX / 2 || b->arena_size > UINT32_MAX)
		return EINVAL;
	for (i = 0; i < n; i++)
		if ((b->pos[i] & 3) || b->end[i] > b->cap[i] ||
		    b->cap[i] > b->arena_size || b->pos[i] > b->end[i])
			return EINVAL;
	err = engine_init(&E, op, n, sessv, nsess, b->sess);
	if (err)
		goto out;
	w = ws_get();
	if (!w) {
		err = ENOMEM;
		goto out;
	}
	stream = b->stream ? b->stream : w->stream;

	/* 1. header parse on the device: pos/end up, parsed headers down */
	err = pool_reserve(w, &w->hdr, n * (8 + sizeof(struct sgpu_hdr) + 12));
	if (err)
		goto out;
	pe_h = (uint32_t *)w->hdr.h;
	memcpy(pe_h, b->pos, n * 4);
	memcpy(pe_h + n, b->end, n * 4);
	hd_h = (struct sgpu_hdr *)(w->hdr.h + 8 * n);
	eix_h = (uint32_t *)(w->hdr.h + 8 * n + n * sizeof(struct sgpu_hdr));
	err = sgpu_memcpy_h2d(w->hdr.d, w->hdr.h, 8 * n, stream);
	if (!err)
		err = sgpu_parse_headers(b->arena, (const uint32_t *)w->hdr.d,
					 (const uint32_t *)w->hdr.d + n,
					 (struct sgpu_hdr *)(w->hdr.d + 8 * n),
					 rtcp && op == OP_RTCP_DEC ?
					 (uint32_t *)(w->hdr.d + 8 * n +
						      n * sizeof(struct sgpu_hdr))
					 : NULL,
					 (uint32_t)n, rtcp, stream);
	if (!err)
		err = sgpu_memcpy_d2h(w->hdr.h + 8 * n, w->hdr.d + 8 * n,
				      n * (sizeof(struct sgpu_hdr) +
					   (op == OP_RTCP_DEC ? 12 : 0)),
				      stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		goto out;
	for (i = 0; i < n; i++) {
		struct pinfo *pi = &E.pi[i];
		const struct sgpu_hdr *h = &hd_h[i];
		pi->start = b->pos[i];
		pi->end = b->end[i];
		pi->size = b->cap[i];
		pi->fixed = 1;
		pi->hdr_len = h->hdr_len;
		pi->err_pos = h->err_pos;
		pi->ssrc = h->ssrc;
		pi->seq = h->seq;
		if (op == OP_RTCP_DEC)
			memcpy(pi->eix, eix_h + 3 * i, 12);
	}

	/* 2. plan / run rounds; in-place results */
	snap_take(&E);
	for (round = 0;; round++) {
		size_t need;
		uint32_t m = 0, mu = 0;

		snap_restore(&E);
		need = plan_all(&E);
		if (!need)
			break;
		if (round > n + 2) {
			err = EIO;
			goto out;
		}
		if (round > 0) {
			/* restore tag words overwritten by SJ_ROC_AT_TAG and
			 * re-apply keystreams of packets that must re-run */
			size_t nr = 0;
			uint32_t *wo, *wv;
			for (i = 0; i < n; i++) {
				const struct rec *r = &E.rec[i];
				if (r->need_run && r->ran &&
				    (r->ran_job.flags & SJ_ROC_AT_TAG))
					nr++;
			}
			if (nr) {
				err = pool_reserve(w, &w->stage, nr * 8);
				if (err)
					goto out;
				wo = (uint32_t *)w->stage.h;
				wv = wo + nr;
				nr = 0;
				for (i = 0; i < n; i++) {
					const struct rec *r = &E.rec[i];
					if (r->need_run && r->ran &&
					    (r->ran_job.flags & SJ_ROC_AT_TAG)) {
						wo[nr] = r->ran_job.off +
							 r->ran_job.tag_off;
						wv[nr] = r->save;
						nr++;
					}
				}
				err = sgpu_memcpy_h2d(w->stage.d, w->stage.h,
						      nr * 8, stream);
				if (!err)
					err = sgpu_store_words(b->arena,
						(const uint32_t *)w->stage.d,
						(const uint32_t *)w->stage.d + nr,
						(uint32_t)nr, stream);
				if (err)
					goto out;
			}
			err = round_launch(w, &E, SEL_UNDO, b->arena,
					   b->arena_size, NULL, 0, &mu);
			if (!err)
				err = sgpu_stream_sync(stream);
			if (err)
				goto out;
		}
		err = round_launch(w, &E, SEL_RUN, b->arena, b->arena_size,
				   NULL, prot, &m);
		if (!err)
			err = round_fetch(w, m);
		if (!err)
			err = sgpu_stream_sync(stream);
		if (err)
			goto out;
		round_collect(w, &E, m);
	}
	for (i = 0; i < n; i++) {
		const struct rec *r = &E.rec[i];
		b->pos[i] = r->pos_o;
		b->end[i] = r->end_o;
		b->err[i] = r->err;
	}
 out:
	engine_free(&E);
	return err;
}

int srtp_encrypt_batch(struct srtp **sessv, size_t nsess,
		       struct srtp_batch *b)
{
	return run_batch(OP_RTP_ENC, sessv, nsess, b);
}

int srtp_decrypt_batch(struct srtp **sessv, size_t nsess,
		       struct srtp_batch *b)
{
	return run_batch(OP_RTP_DEC, sessv, nsess, b);
}

int srtcp_encrypt_batch(struct srtp **sessv, size_t nsess,
			struct srtp_batch *b)
{
	return run_batch(OP_RTCP_ENC, sessv, nsess, b);
}

int srtcp_decrypt_batch(struct srtp **sessv, size_t nsess,
			struct srtp_batch *b)
{
	return run_batch(OP_RTCP_DEC, sessv, nsess, b);
}

/* ---- stream state export / import ------------------------------------ */

int srtp_stream_export(const struct srtp *srtp, uint32_t ssrc,
		       struct srtp_stream_state *st)
{
	unsigned i;
	if (!srtp || !st)
		return EINVAL;
	for (i = 0; i < srtp->nstreams; i++) {
		const struct srtp_stream *s = &srtp->streams[i];
		if (s->ssrc != ssrc)
			continue;
		memset(st, 0, sizeof(*st));
		st->replay_rtp_bitmap = s->replay_rtp.bitmap;
		st->replay_rtp_lix = s->replay_rtp.lix;
		st->replay_rtcp_bitmap = s->replay_rtcp.bitmap;
		st->replay_rtcp_lix = s->replay_rtcp.lix;
		st->ssrc = s->ssrc;
		st->roc = s->roc;
		st->s_l = s->s_l;
		st->s_l_set = s->s_l_set;
		st->rtcp_index = s->rtcp_index;
		return 0;
	}
	return ENOENT;
}

int srtp_stream_import(struct srtp *srtp, const struct srtp_stream_state *st)
{
	struct srtp_stream *s;
	int err;
	if (!srtp || !st)
		return EINVAL;
	err = stream_get(&s, srtp, st->ssrc);
	if (err)
		return err;
	s->replay_rtp.bitmap = st->replay_rtp_bitmap;
	s->replay_rtp.lix = st->replay_rtp_lix;
	s->replay_rtcp.bitmap = st->replay_rtcp_bitmap;
	s->replay_rtcp.lix = st->replay_rtcp_lix;
	s->roc = st->roc;
	s->s_l = st->s_l;
	s->s_l_set = st->s_l_set;
	s->rtcp_index = st->rtcp_index;
	return 0;
}

/* ---- diagnostics: per-kernel-class device time (HIP events) ----------- */

void srtp_gpu_prof(int enable)
{
	sgpu_prof_enable(enable);
}

void srtp_gpu_prof_read(double ms[32], uint64_t launches[32],
			uint64_t jobs[32])
{
	sgpu_prof_read(ms, launches, jobs);
}
