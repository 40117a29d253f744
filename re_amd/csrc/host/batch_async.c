/*
 * batch_async.c -- the public batch entry points (re_srtp_batch.h), the
 * asynchronous tickets (srtp_*_batch_dev_async / srtp_batch_wait: up to
 * TK_MAX pending calls per thread, chained by gate words), stream state
 * export / import, the RTCP compound encode / decode entry points
 * (re_rtcp_batch.h) and the profiler switches.  Split out of srtp.c.
 */
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "re_mem.h"
#include "re_mbuf.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"
#include "re_rtcp_batch.h"
#include "../srtpgpu.h"
#include "fault.h"
#include "pool.h"
#include "srtp_int.h"

/* ---- asynchronous device batches (re_srtp_batch.h) -------------------- */

#define TK_MAX   4              /* pending calls per thread */
#define TK_GATES 64             /* per-thread gate words (a ring > TK_MAX) */

enum { TK_PLANNED = 1, TK_MPLANNED = 2, TK_SPLANNED = 3, TK_DONE = 4 };

struct srtp_batch_ticket {
	struct srtp_batch_ticket *next;
	pthread_t owner;
	uint64_t seq;
	int kind;               /* TK_* */
	int result;             /* TK_DONE: the call's result */
	struct dcall k;
	void *ev;               /* recorded after the launches */
};

static __thread struct srtp_batch_ticket *t_tk_head, *t_tk_tail;
static __thread uint64_t t_tk_seq, t_tk_done;
static __thread int t_tk_n;
static __thread void *t_tk_stream;
static __thread uint32_t *t_gates;
static __thread struct ws *t_aws[TK_MAX + 1];
static __thread int t_naws;

static int run_dev(int op, struct srtp **sessv, size_t nsess,
		   struct srtp_batch_dev *d);
static int dev_staged(int op, struct srtp **sessv, size_t nsess,
		      struct srtp_batch_dev *d);

/* complete the thread's oldest pending call (its result stays in the
 * ticket until srtp_batch_wait) */
static void tk_finish_one(void)
{
	struct srtp_batch_ticket *t = t_tk_head;
	struct dcall *k = &t->k;
	int r;

	r = sgpu_event_sync(t->ev);
	if (!r)
		r = t->kind == TK_PLANNED ? dev_planned_finish(k) :
		    t->kind == TK_SPLANNED ? dev_splanned_finish(k)
					   : dev_mplanned_finish(k);
	t_tk_head = t->next;
	if (!t_tk_head)
		t_tk_tail = NULL;
	t_tk_n--;
	t_tk_done = t->seq;
	__atomic_store_n(&t_own->done, t->seq, __ATOMIC_RELEASE);
	t_aws[t_naws++] = k->w;
	sgpu_event_destroy(t->ev);
	t->ev = NULL;
	if (r == -2) {
		/* gated behind an earlier call that the host completed:
		 * nothing was modified, run it now */
		count(&g_cnt_gated, 1);
		r = run_dev(k->op, k->sessv, k->nsess, &k->d);
	}
	else if (r == -1) {
		r = sess_host(k->sessv, k->nsess);
		/* a second SSRC in a single-stream plan: the per-stream one */
		if (!r && t->kind == TK_PLANNED && (k->pfail & SPF_SSRC))
			r = dev_splanned(k->op, k->sessv[0], &k->d);
		/* a session over the counting grouping's bound: the radix
		 * sort */
		else if (!r && t->kind == TK_MPLANNED && (k->pfail & SPF_SEG) &&
			 !k->radix) {
			uint32_t pf = 0;
			r = dev_mplanned_(k->op, k->sessv, k->nsess, &k->d, 1,
					  &pf);
		}
		else if (!r)
			r = -1;
		if (r == -1)
			r = dev_staged(k->op, k->sessv, k->nsess, &k->d);
	}
	t->result = r;
	t->kind = TK_DONE;
	table_unlock();         /* held since the call was issued */
}

/* this thread has asynchronous calls pending (their sessions must not
 * be handed to another thread's shared launch) */
int tk_pending(void)
{
	return t_tk_head != NULL;
}

/* complete every pending call of this thread (before any other entry
 * point: those see the sessions as the calls in order leave them) */
void tk_drain(void)
{
	while (t_tk_head)
		tk_finish_one();
}

static void tk_drain_upto(uint64_t seq)
{
	while (t_tk_head && t_tk_done < seq)
		tk_finish_one();
}

static int batch_async(int op, struct srtp **sessv, size_t nsess,
		       struct srtp_batch_dev *d,
		       struct srtp_batch_ticket **tp)
{
	struct srtp_batch_ticket *t;
	struct dcall *k;
	size_t i;
	int kind = 0, err;

	if (!tp || !sessv || !nsess || !d || !d->arena || !d->pos ||
	    !d->end || !d->cap || !d->err)
		return EINVAL;
	for (i = 0; i < nsess; i++)
		if (!sessv[i])
			return EINVAL;
	if (d->n > UINT32_MAX / 4 || d->arena_size > UINT32_MAX)
		return EINVAL;
	t = fi_calloc(1, sizeof(*t));
	if (!t)
		return ENOMEM;
	t->owner = pthread_self();
	*tp = t;
	env_init();
	if (!tk_me()) {
		t->kind = TK_DONE;
		t->result = ENOMEM;
		return 0;
	}
	/* the chain's gate words are ordered by the stream */
	if (t_tk_n && t_tk_stream != d->stream)
		tk_drain();
	while (t_tk_n >= TK_MAX)
		tk_finish_one();
	if (!t_gates) {
		t_gates = fi_sgpu_malloc(TK_GATES * 4);
		if (!t_gates || sgpu_memset(t_gates, 0, TK_GATES * 4, NULL) ||
		    sgpu_stream_sync(NULL)) {
			t->kind = TK_DONE;
			t->result = ENOMEM;
			return 0;
		}
	}
	if (d->n && (op == OP_RTP_ENC || op == OP_RTP_DEC) &&
	    !g_env.noplan && !g_env.general) {
		if (nsess == 1 && !d->sess)
			kind = TK_PLANNED;
		else if (nsess > 1 && d->sess)
			kind = TK_MPLANNED;
	}
	if (kind == TK_PLANNED) {
		struct srtp *s = sessv[0];
		uint64_t p = s->pend_p > s->pend_m ? s->pend_p : s->pend_m;
		/* plans from the host copy of its state: the pending calls
		 * on it complete first (this thread's; another thread's
		 * make sess_host return EBUSY) */
		if (s->pend_own == t_own && p > t_tk_done)
			tk_drain_upto(p);
		table_rdlock();
		err = sess_host(&s, 1);
		table_unlock();
		if (err)
			kind = 0;
		else if (s->nstreams > 1 || g_env.splan ||
			 (!s->nstreams &&
			  __atomic_load_n(&g_fresh_multi, __ATOMIC_RELAXED)))
			kind = TK_SPLANNED;
	}
	if (!kind) {
		tk_drain();
		table_rdlock();
		t->result = run_dev(op, sessv, nsess, d);
		table_unlock();
		t->kind = TK_DONE;
		return 0;
	}
	k = &t->k;
	k->op = op;
	k->sessv = sessv;
	k->nsess = nsess;
	k->d = *d;
	k->w = t_naws ? t_aws[--t_naws] : ws_new();
	if (!k->w) {
		t->kind = TK_DONE;
		t->result = ENOMEM;
		return 0;
	}
	t->seq = t_tk_seq + 1;
	k->pred = t_tk_n ? &t_gates[t_tk_tail->seq % TK_GATES] : NULL;
	k->gate = &t_gates[t->seq % TK_GATES];
	k->pend = t->seq;
	k->done = t_tk_done;
	t->ev = sgpu_event_create();
	table_rdlock();         /* until the call completes (tk_finish_one) */
	err = t->ev ? 0 : ENOMEM;
	if (!err)
		err = kind == TK_PLANNED ? dev_planned_issue(k) :
		      kind == TK_SPLANNED ? dev_splanned_issue(k)
					  : dev_mplanned_issue(k);
	if (!err)
		err = sgpu_event_record(t->ev, d->stream);
	if (err) {
		/* nothing queued that completes the call: run it here */
		t_aws[t_naws++] = k->w;
		if (t->ev)
			sgpu_event_destroy(t->ev);
		t->ev = NULL;
		table_unlock();
		if (err == -1) {
			tk_drain();
			table_rdlock();
			err = sess_host(sessv, nsess);
			if (!err)
				err = run_dev(op, sessv, nsess, d);
			table_unlock();
		}
		t->kind = TK_DONE;
		t->result = err;
		return 0;
	}
	t_tk_seq = t->seq;
	t->kind = kind;
	if (kind == TK_PLANNED || kind == TK_SPLANNED) {
		sessv[0]->pend_p = t->seq;
		sessv[0]->pend_own = t_own;
	}
	if (t_tk_tail)
		t_tk_tail->next = t;
	else
		t_tk_head = t;
	t_tk_tail = t;
	t_tk_n++;
	t_tk_stream = d->stream;
	return 0;
}

int srtp_encrypt_batch_dev_async(struct srtp **sessv, size_t nsess,
				 struct srtp_batch_dev *b,
				 struct srtp_batch_ticket **tp)
{
	return batch_async(OP_RTP_ENC, sessv, nsess, b, tp);
}

int srtp_decrypt_batch_dev_async(struct srtp **sessv, size_t nsess,
				 struct srtp_batch_dev *b,
				 struct srtp_batch_ticket **tp)
{
	return batch_async(OP_RTP_DEC, sessv, nsess, b, tp);
}

int srtp_batch_wait(struct srtp_batch_ticket *t)
{
	int r;
	if (!t || !pthread_equal(t->owner, pthread_self()))
		return EINVAL;
	while (t->kind != TK_DONE)
		tk_finish_one();
	r = t->result;
	free(t);
	return r;
}

/* any other batch: stage the device arrays through the host engine */
static int dev_staged(int op, struct srtp **sessv, size_t nsess,
		      struct srtp_batch_dev *d)
{
	const size_t n = d->n;
	struct srtp_batch hb;
	uint32_t *hpos = fi_malloc(n * 4), *hend = fi_malloc(n * 4);
	uint32_t *hcap = fi_malloc(n * 4), *hsess = d->sess ? fi_malloc(n * 4) : NULL;
	int32_t *herrv = fi_malloc(n * 4);
	void *stream = d->stream;
	int err = 0, r;

	if (!hpos || !hend || !hcap || !herrv || (d->sess && !hsess)) {
		err = ENOMEM;
		goto out;
	}
	err = sgpu_memcpy_d2h(hpos, d->pos, n * 4, stream);
	if (!err)
		err = sgpu_memcpy_d2h(hend, d->end, n * 4, stream);
	if (!err)
		err = sgpu_memcpy_d2h(hcap, d->cap, n * 4, stream);
	if (!err && d->sess)
		err = sgpu_memcpy_d2h(hsess, d->sess, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		goto out;
	memset(&hb, 0, sizeof(hb));
	hb.arena = d->arena;
	hb.arena_size = d->arena_size;
	hb.pos = hpos;
	hb.end = hend;
	hb.cap = hcap;
	hb.err = herrv;
	hb.sess = hsess;
	hb.n = n;
	hb.stream = stream;
	t_noplan = 1;
	r = run_batch(op, sessv, nsess, &hb);
	t_noplan = 0;
	if (r) {
		err = r;
		goto out;
	}
	err = sgpu_memcpy_h2d(d->pos, hpos, n * 4, stream);
	if (!err)
		err = sgpu_memcpy_h2d(d->end, hend, n * 4, stream);
	if (!err)
		err = sgpu_memcpy_h2d(d->err, herrv, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
 out:
	free(hpos);
	free(hend);
	free(hcap);
	free(hsess);
	free(herrv);
	return err;
}

static int run_dev(int op, struct srtp **sessv, size_t nsess,
		   struct srtp_batch_dev *d)
{
	size_t k;
	if (!sessv || !nsess || !d || !d->arena || !d->pos || !d->end ||
	    !d->cap || !d->err)
		return EINVAL;
	for (k = 0; k < nsess; k++)
		if (!sessv[k])
			return EINVAL;
	if (d->n == 0)
		return 0;
	if (d->n > UINT32_MAX / 4 || d->arena_size > UINT32_MAX)
		return EINVAL;
	/* many sessions: planned on the device against the resident states */
	if ((op == OP_RTP_ENC || op == OP_RTP_DEC) && nsess > 1 && d->sess &&
	    !g_env.noplan && !g_env.general) {
		int r = dev_mplanned(op, sessv, nsess, d);
		if (r >= 0)
			return r;
	}
	{
		int err = sess_host(sessv, nsess);
		if (err)
			return err;
	}
	if ((op == OP_RTP_ENC || op == OP_RTP_DEC) && nsess == 1 &&
	    !d->sess && !g_env.noplan && !g_env.general) {
		/* one stream: the single-stream planner (with the device verdict
		 * fold); several SSRCs (or a plan rejected for a second one):
		 * the per-stream planner */
		uint32_t pf = SPF_SSRC;
		int r = -1;
		if (sessv[0]->nstreams <= 1 && !g_env.splan &&
		    (sessv[0]->nstreams ||
		     !__atomic_load_n(&g_fresh_multi, __ATOMIC_RELAXED)))
			r = dev_planned(op, sessv[0], d, &pf);
		if (r == -1 && (pf & SPF_SSRC))
			r = dev_splanned(op, sessv[0], d);
		if (r >= 0)
			return r;
	}
	if ((op == OP_RTCP_ENC || op == OP_RTCP_DEC) && nsess == 1 &&
	    !d->sess && sessv[0]->nstreams <= 1 &&
	    !g_env.noplan && !g_env.general) {
		int r = dev_planned_rtcp(op, sessv[0], d);
		if (r >= 0)
			return r;
	}
	return dev_staged(op, sessv, nsess, d);
}

enum { HOSTW = 0, DEV = 1 };

/* public batch entry: the device table stays in place for the call */
static int locked(int kind, int op, struct srtp **sessv, size_t nsess,
		  void *b)
{
	int err;
	tk_drain();
	table_rdlock();
	if (kind == DEV) {
		err = run_dev(op, sessv, nsess, b);
	}
	else {
		err = sessv ? sess_host(sessv, nsess) : 0;
		if (!err)
			err = run_batch(op, sessv, nsess, b);
	}
	table_unlock();
	return err;
}

int srtp_encrypt_batch_dev(struct srtp **sessv, size_t nsess,
			   struct srtp_batch_dev *b)
{
	return locked(DEV, OP_RTP_ENC, sessv, nsess, b);
}

int srtp_decrypt_batch_dev(struct srtp **sessv, size_t nsess,
			   struct srtp_batch_dev *b)
{
	return locked(DEV, OP_RTP_DEC, sessv, nsess, b);
}

int srtcp_encrypt_batch_dev(struct srtp **sessv, size_t nsess,
			    struct srtp_batch_dev *b)
{
	return locked(DEV, OP_RTCP_ENC, sessv, nsess, b);
}

int srtcp_decrypt_batch_dev(struct srtp **sessv, size_t nsess,
			    struct srtp_batch_dev *b)
{
	return locked(DEV, OP_RTCP_DEC, sessv, nsess, b);
}

int srtp_encrypt_batch(struct srtp **sessv, size_t nsess,
		       struct srtp_batch *b)
{
	return locked(HOSTW, OP_RTP_ENC, sessv, nsess, b);
}

int srtp_decrypt_batch(struct srtp **sessv, size_t nsess,
		       struct srtp_batch *b)
{
	return locked(HOSTW, OP_RTP_DEC, sessv, nsess, b);
}

int srtcp_encrypt_batch(struct srtp **sessv, size_t nsess,
			struct srtp_batch *b)
{
	return locked(HOSTW, OP_RTCP_ENC, sessv, nsess, b);
}

int srtcp_decrypt_batch(struct srtp **sessv, size_t nsess,
			struct srtp_batch *b)
{
	return locked(HOSTW, OP_RTCP_DEC, sessv, nsess, b);
}

/* ---- stream state export / import ------------------------------------ */

int srtp_stream_export(const struct srtp *srtp, uint32_t ssrc,
		       struct srtp_stream_state *st)
{
	unsigned i;
	struct srtp *sp = (struct srtp *)srtp;  /* state cache refresh */
	int err;
	if (!srtp || !st)
		return EINVAL;
	tk_drain();
	table_rdlock();
	err = sess_host(&sp, 1);
	table_unlock();
	if (err)
		return err;
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
	tk_drain();
	table_rdlock();
	err = sess_host(&srtp, 1);
	table_unlock();
	if (err)
		return err;
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

/* ---- RTCP compound decode (include/re_rtcp_batch.h) ------------------- */

int rtcp_decode_full_batch_dev(const uint8_t *arena, size_t arena_size,
			       const uint32_t *pos, const uint32_t *end,
			       size_t n, struct rtcp_desc *descv,
			       uint32_t maxmsg, uint32_t *nmsg,
			       struct rtcp_item *itemv, uint32_t maxitem,
			       uint32_t *nitem, int32_t *err, uint32_t *stop,
			       void *stream)
{
	if (!n)
		return 0;
	if (!arena || !pos || !end || !nmsg || !err || !stop ||
	    (maxmsg && !descv) || (maxitem && (!itemv || !nitem)) ||
	    (itemv && !nitem) || n > UINT32_MAX ||
	    (uint64_t)n * maxmsg > ((uint64_t)1 << 40) ||
	    (uint64_t)n * maxitem > ((uint64_t)1 << 40))
		return EINVAL;
	if (!gpu_ready())
		return ENOSYS;
	return sgpu_rtcp_walk(arena, arena_size, pos, end, (uint32_t)n, descv,
			      maxmsg, nmsg, maxitem ? itemv : NULL, maxitem,
			      nitem, err, stop, stream);
}

int rtcp_decode_batch_dev(const uint8_t *arena, size_t arena_size,
			  const uint32_t *pos, const uint32_t *end, size_t n,
			  struct rtcp_desc *descv, uint32_t maxmsg,
			  uint32_t *nmsg, int32_t *err, uint32_t *stop,
			  void *stream)
{
	return rtcp_decode_full_batch_dev(arena, arena_size, pos, end, n,
					  descv, maxmsg, nmsg, NULL, 0, NULL,
					  err, stop, stream);
}

/* ---- RTCP compound encode (include/re_rtcp_batch.h) ------------------- */

int rtcp_encode_batch_dev(const struct rtcp_enc_batch *b)
{
	if (!b)
		return EINVAL;
	if (!b->n)
		return 0;
	if (!b->arena || !b->pos || !b->end || !b->cap || !b->mfirst ||
	    !b->err || b->n >= UINT32_MAX || b->arena_size > UINT32_MAX ||
	    (b->nmsg && !b->msgv) || (b->nrb && !b->rbv) ||
	    (b->nchunk && !b->chunkv) || (b->nsdes && !b->sdesv) ||
	    (b->nsrc && !b->srcv) || (b->pool_size && !b->pool))
		return EINVAL;
	if (!gpu_ready())
		return ENOSYS;
	return sgpu_rtcp_encode(b);
}

/* ---- diagnostics: per-kernel-class device time (HIP events) ----------- */

void srtp_gpu_prof(int enable)
{
	sgpu_prof_enable(enable);
}

void srtp_gpu_prof_read(double ms[32], uint64_t launches[32],
			uint64_t jobs[32])
{
	sgpu_prof_read(ms, launches, jobs, NULL);
}

void srtp_gpu_prof_read_named(double ms[32], uint64_t launches[32],
			      uint64_t jobs[32], char names[32][48])
{
	sgpu_prof_read(ms, launches, jobs, names);
}
