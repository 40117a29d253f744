/*
 * batch_dev.c -- fully device-resident batches (srtp_*_batch_dev):
 * packets, positions and stream state stay in HBM and the plan runs on the
 * device -- one stream planned inside the crypto launch (k_ctr_fused.h,
 * fz_issue / fz_finish), one stream by the planner kernels
 * (dev_planned), several streams of one session (plan_streams.hip), SRTCP
 * (dev_planned_rtcp) and many sessions with resident state
 * (dev_mplanned).  Each call is a struct dcall between its launches
 * (*_issue) and its completion (*_finish), so the synchronous calls and the
 * asynchronous tickets (batch_async.c) share it.  Split out of srtp.c.
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

/* ---- fully device-resident batches ------------------------------------ */



/* single-stream RTP batch planned and processed on the device: the
 * launches (no host synchronisation) */
static int fz_issue(struct dcall *k, int sync);
static int fz_finish(struct dcall *k, int sync);

static int lp_issue(struct dcall *k, int sync);
static int lp_finish(struct dcall *k, int sync);

int dev_planned_issue(struct dcall *k)
{
	if (!g_env.noplanfuse) {
		if (k->sessv[0]->rtp.mode == SGPU_MODE_CTR && !g_env.lplan) {
			k->fused = 1;
			return fz_issue(k, 0);
		}
		k->fused = 2;
		return lp_issue(k, 0);
	}
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &s->rtp;
	const size_t n = d->n;
	const uint32_t T = c0->mode == SGPU_MODE_GCM ? 16u : c0->tag_len;
	const uint32_t need = prot ? (c0->mode == SGPU_MODE_GCM ? 16u :
			      (T > 4 ? T : 4u)) : 0u;
	struct sgpu_plan_out *po, *po_d;
	struct sgpu_fold_out *fo_d;
	struct sgpu_hdr *hd_d;
	uint64_t *desc_d;
	uint32_t *scr, *es_d, *save_d, *nfail_d, *flist_d;
	uint32_t cm = c0->dev;
	uint8_t *vd_d;
	void *stream = d->stream;       /* NULL: the default (null) stream */
	size_t foff;
	int err;

	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 12);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 9 + 72);
	if (!err)
		err = pool_reserve(w, &w->cm, 4);
	/* pl: plan out | plan scratch | fold out | fold scratch */
	foff = (sizeof(struct sgpu_plan_out) + (n / 256 + 8) * 4 + 63) & ~63ul;
	k->foff = foff;
	if (!err)
		err = pool_reserve(w, &w->pl, foff + 64 + (n / 256 + 4) * 20);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (err)
		return err;
	hd_d = (struct sgpu_hdr *)w->hd.d;
	desc_d = (uint64_t *)w->dsc.d;
	nfail_d = (uint32_t *)w->vs.d;
	save_d = (uint32_t *)(w->vs.d + 64);
	vd_d = w->vs.d + 64 + n * 4;
	flist_d = (uint32_t *)(w->vs.d + ((64 + n * 5 + 3) & ~(size_t)3));
	po = (struct sgpu_plan_out *)w->pl.h;
	po_d = (struct sgpu_plan_out *)w->pl.d;
	scr = (uint32_t *)(w->pl.d + sizeof(*po));
	es_d = (uint32_t *)w->es.d;

	plan_in(&k->in, s, (uint32_t)n, prot, T, need);
	{
		/* one launch: parse + end copy + zeroed counters + comp map */
		struct sgpu_prologue pro = {
			es_d, nfail_d, (uint32_t *)po_d, 1,
			(uint32_t)(sizeof(*po) / 4), (uint32_t *)w->cm.d, cm, NULL, NULL,
			0, 0, 0, 0, NULL, 0};
		k->in.zeroed = 1;
		err = sgpu_parse_prologue(d->arena, d->arena_size, d->pos,
					  d->end, hd_d, NULL, (uint32_t)n, 0,
					  &pro, stream);
	}
	k->in.pred = k->pred;   /* the gate check rides in k_plan_count */
	if (!err)
		err = sgpu_plan_rtp(&k->in, hd_d, d->pos, es_d, d->cap,
				    d->arena_size, desc_d, scr, po_d, stream);
	if (!err) {
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, NULL,
			(const uint32_t *)w->cm.d, NULL, 0, (uint32_t)n, vd_d,
			save_d, nfail_d, 0, 1, NULL, 0, flist_d, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0,
				  po_d, prot, stream);
	}
	/* unprotect: the verdict fold queued behind the kernels (nothing to
	 * do without a miss), so a forged packet neither gates the next
	 * chained call nor waits for the host (sgpu_fold_rtp) */
	k->devfold = !prot && !g_env.nodevfold;
	fo_d = (struct sgpu_fold_out *)(w->pl.d + foff);
	if (!err && k->devfold)
		err = sgpu_fold_rtp(1, nfail_d, &k->in, hd_d, desc_d, vd_d, es_d,
				    d->pos, d->end, d->err,
				    c0->mode == SGPU_MODE_GCM,
				    (uint32_t *)(w->pl.d + foff + 64), fo_d,
				    stream);
	/* results, gate word and the miss count next to the plan: one
	 * launch, one copy into pinned memory */
	if (!err)
		err = sgpu_plan_finish(&po_d->fail, es_d, d->end, d->err,
				       (uint32_t)n,
				       prot ? (int32_t)T : -(int32_t)T, nfail_d,
				       k->gate, &po_d->nfail,
				       k->devfold ? &fo_d->fail : NULL, stream);
	if (!err && k->devfold)
		err = sgpu_fold_rtp(2, nfail_d, &k->in, hd_d, desc_d, vd_d, es_d,
				    d->pos, d->end, d->err,
				    c0->mode == SGPU_MODE_GCM,
				    (uint32_t *)(w->pl.d + foff + 64), fo_d,
				    stream);
	/* plan out and fold out in one copy */
	if (!err)
		err = sgpu_memcpy_d2h(po, po_d, k->devfold ? foff + sizeof(*fo_d)
							  : sizeof(*po), stream);
	return err;
}

/* ... after its launches completed: 0 / errno, -1 not plannable or a
 * forged packet the host must fold (nothing modified), -2 gated by the
 * chained call before (nothing modified) */
int dev_planned_finish(struct dcall *k)
{
	if (k->fused == 1)
		return fz_finish(k, 0);
	if (k->fused == 2)
		return lp_finish(k, 0);
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &s->rtp;
	const size_t n = d->n;
	const unsigned ns0 = s->nstreams;
	const size_t foff = k->foff;
	struct sgpu_plan_out *po = (struct sgpu_plan_out *)w->pl.h;
	struct sgpu_plan_out *po_d = (struct sgpu_plan_out *)w->pl.d;
	struct sgpu_hdr *hd_d = (struct sgpu_hdr *)w->hd.d;
	uint64_t *desc_d = (uint64_t *)w->dsc.d;
	uint32_t *nfail_d = (uint32_t *)w->vs.d;
	uint32_t *save_d = (uint32_t *)(w->vs.d + 64);
	uint8_t *vd_d = w->vs.d + 64 + n * 4;
	uint32_t *es_d = (uint32_t *)w->es.d;
	void *stream = d->stream;
	struct srtp_stream old;
	uint32_t nfail;
	int err = 0;

	nfail = po->nfail;
	k->pfail = po->fail;
	if (po->fail) {
		if (po->fail & SPF_PRED)
			return -2;
		if ((po->fail & SPF_SSRC) && !ns0)
			__atomic_store_n(&g_fresh_multi, 1, __ATOMIC_RELAXED);
		count(&g_cnt_rejects, 1);
		return -1;
	}
	count(&g_cnt_dplans, 1);
	if (nfail)
		count(&g_cnt_misses, nfail);
	plan_apply(s, po, prot, n, &old);
	if (!nfail)
		return 0;
	/* a forged packet: fold the verdicts on the device.  The kernels
	 * already left each forged packet as srtp_decrypt does (HMAC: the
	 * ciphertext restored, the ROC over the tag; GCM: decrypted in
	 * place); the fold checks that the speculated rollovers and indices
	 * hold under the true s_l and writes the EAUTH results, s_l and the
	 * replay window (sgpu_fold_rtp). */
	if (!prot && k->devfold) {
		/* folded on the device behind the kernels (dev_planned_issue);
		 * its verdict came back with the plan */
		const struct sgpu_fold_out *fo =
			(const struct sgpu_fold_out *)(w->pl.h + foff);
		if (!fo->fail) {
			struct srtp_stream *st = &s->streams[0];
			st->s_l = (uint16_t)fo->s_l;
			st->replay_rtp.lix = fo->lix;
			st->replay_rtp.bitmap = fo->bitmap;
			count(&g_cnt_devfolds, 1);
			return 0;
		}
	}
	count(&g_cnt_folds, 1);
	/* undo on the device, fold on the host engine */
	{
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, NULL,
			(const uint32_t *)w->cm.d, NULL, 0, (uint32_t)n, vd_d,
			save_d, nfail_d, 1, 1, NULL, 0, NULL, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0,
				  po_d, prot, stream);
	}
	if (!err)
		err = sgpu_memcpy_d2d(d->end, es_d, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	plan_unapply(s, ns0, &old);
	return -1;
}


/* ---- one stream, planned inside the crypto launch (k_ctr_fused.h) ----- */

#define FZ_HEAD 64u             /* ticket word, padded */

/*
 * Single-stream AES-CM batch planned inside its crypto launch
 * (srtpgpu.h struct sgpu_fused): one launch parses, plans and encrypts /
 * decrypts.  Synchronous calls (dev_fused): with no forged packet nothing
 * else runs on the device; forged packets get their ciphertext back
 * (k_ctr_refix_list) and the device verdict fold (sgpu_fold_rtp) after the
 * synchronisation showed a miss.  Asynchronous calls (dev_planned_issue):
 * the refix and fold are queued behind the launch (each exits at once
 * without a miss) with the chained gate word, so no host round trip is
 * needed.  A rejected plan or a fold the device cannot settle: every
 * processed packet undone (sgpu_fused_undo), the ends restored, and -1
 * (k->pfail: the plan's SPF_* bits, 0 for a fold) -- the caller plans on
 * the host, as for the separate device planner.
 *
 * w->fz: ticket | (plan out, fold out) x 2 | look-back words
 */
#define FZ_FO_OFF ((sizeof(struct sgpu_plan_out) + 63u) & ~(size_t)63)
#define FZ_SLOT (FZ_FO_OFF + 64u)

/* the workspace's pinned completion word for synchronous single-stream
 * calls (srtp_gpu_tune syncspin), once */
static int sync_word(struct ws *w)
{
	if (!w->sy_word) {
		w->sy_word = fi_sgpu_host_alloc(4);
		if (w->sy_word)
			*w->sy_word = 0;
	}
	return w->sy_word != NULL;
}

/* wait for a synchronous call: its post's completion word when it has one
 * (spinning, the stream asked now and then whether it stopped without
 * it: a fault), else the stream */
static int sync_wait(struct dcall *k, void *stream)
{
	unsigned long i;
	if (!k->spin)
		return sgpu_stream_sync(stream);
	for (i = 1;; i++) {
		int q;
		if (__atomic_load_n(k->w->sy_word, __ATOMIC_ACQUIRE) == k->spin)
			return 0;
		if (i & 1023) {
			__builtin_ia32_pause();
			continue;
		}
		q = sgpu_stream_query(stream);
		if (q == EAGAIN)
			continue;
		if (__atomic_load_n(k->w->sy_word, __ATOMIC_ACQUIRE) == k->spin)
			return 0;
		return q ? q : EIO;
	}
}

/* a single-stream call's plan out back to its pinned mirror, behind the
 * crypto launch; an asynchronous call also sets its chained gate word
 * (out->fail || out->nfail: the plan failed or a tag did not verify --
 * forged packets' restore and verdict fold run when the call is waited
 * for, as for a synchronous call, and a chained call queued behind one
 * with misses is gated and re-run; the zero-miss fold launches cost every
 * call ~25 us, a miss costs the call behind it a host round trip) */
static int plan_out_back(struct dcall *k, int sync, struct sgpu_plan_out *out,
			 void *host, void *stream)
{
	int err = 0;
	k->devfold = 0;
	if (!g_env.nopost) {
		/* a synchronous call with srtp_gpu_tune syncspin: waited for
		 * by the post's completion word, not a stream synchronisation */
		uint32_t *done = NULL;
		if (sync && g_env.syncspin && sync_word(k->w))
			done = k->w->sy_word;
		k->spin = done ? ++k->w->sy_seq : 0;
		if (k->spin == 0 && done)
			k->spin = ++k->w->sy_seq;       /* never 0 */
		return sgpu_plan_post(out, host, sizeof(*out),
				      sync ? NULL : k->gate, done, k->spin,
				      stream);
	}
	if (!sync && k->gate)
		err = sgpu_plan_finish(&out->fail, NULL, NULL, NULL, 0, 0,
				       &out->nfail, k->gate, NULL, NULL, stream);
	if (!err)
		err = sgpu_memcpy_d2h(host, out, sizeof(*out), stream);
	return err;
}

static int fz_issue(struct dcall *k, int sync)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	const struct comp *c0 = &s->rtp;
	const size_t n = d->n;
	const uint32_t T = c0->tag_len;
	const uint32_t need = prot ? (T > 4 ? T : 4u) : 0u;
	const uint32_t B = sgpu_fused_block();
	const uint32_t nblk = (uint32_t)((n + B - 1) / B);
	struct ws *w = k->w;
	struct sgpu_fused *F = &k->fz;
	void *stream = d->stream;
	uint8_t *fz;
	size_t poff;
	int err;

	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 8);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 9 + 72);
	if (!err)
		err = pool_reserve(w, &w->cm, 4);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)
		err = pool_reserve(w, &w->pl, 64 + (n / 256 + 4) * 20);
	if (!err)
		err = pool_reserve(w, &w->fz, FZ_HEAD + 2 * FZ_SLOT +
				   (size_t)nblk * 8);
	if (err)
		return err;
	fz = w->fz.d;
	{
		/* srtp_gpu_tune fzepoch (a test hook, one-shot for whichever
		 * thread's fused launch comes next): the look-back words are
		 * zeroed with it, so words of an epoch used since the last
		 * zeroing can never match */
		const long e = __atomic_exchange_n(&g_env.fzepoch, 0,
						   __ATOMIC_RELAXED);
		if (e > 0 && e <= 0xffff)
			w->fz_d = NULL;
		if (w->fz_d != fz || w->fz_epoch == 0 ||
		    w->fz_epoch > 0xffffu) {
			/* a new pool (or the look-back epoch wrapped):
			 * counters, plan outs and look-back words from zero */
			err = sgpu_memset(fz, 0, w->fz.cap, stream);
			if (err)
				return err;
			w->fz_d = fz;
			w->fz_epoch = 1;
			w->fz_tbase = 0;
			w->fz_par = 0;
		}
		if (e > 0 && e <= 0xffff)
			w->fz_epoch = (uint32_t)e;
	}
	poff = FZ_HEAD + (size_t)w->fz_par * FZ_SLOT;
	k->foff = poff;

	memset(F, 0, sizeof(*F));
	plan_in(&F->in, s, (uint32_t)n, prot, T, need);
	F->in.zeroed = 1;
	F->in.pred = k->pred;   /* the chained call before: its gate word */
	F->pos = d->pos;
	F->end = d->end;
	F->cap = d->cap;
	F->err = d->err;
	F->es = (uint32_t *)w->es.d;
	F->hdr = (struct sgpu_hdr *)w->hd.d;
	F->desc = (uint64_t *)w->dsc.d;
	if (!prot) {
		F->save = (uint32_t *)(w->vs.d + 64);
		F->verdict = w->vs.d + 64 + n * 4;
		F->flist = (uint32_t *)(w->vs.d +
					((64 + n * 5 + 3) & ~(size_t)3));
	}
	F->out = (struct sgpu_plan_out *)(fz + poff);
	F->out_next = (struct sgpu_plan_out *)(fz + FZ_HEAD +
					       (size_t)(w->fz_par ^ 1) * FZ_SLOT);
	F->cm_out = (uint32_t *)w->cm.d;
	F->agg = (unsigned long long *)(fz + FZ_HEAD + 2 * FZ_SLOT);
	F->ticket = (uint32_t *)fz;
	F->tbase = w->fz_tbase;
	F->epoch = w->fz_epoch;
	F->comp = c0->dev;
	F->delta = prot ? (int32_t)T : -(int32_t)T;
	err = sgpu_run_fused(d->arena, d->arena_size, F, (int)c0->nr, stream);
	if (err) {
		w->fz_d = NULL;         /* counters unknown: from zero next time */
		return err;
	}
	w->fz_tbase += F->ntickets;
	w->fz_epoch++;
	w->fz_par ^= 1;
	return plan_out_back(k, sync, F->out, w->fz.h + poff, stream);
}

/* ... after its launches completed: 0 / errno, -1 not plannable or a
 * forged packet the host must fold (nothing modified), -2 gated by the
 * chained call before (nothing modified) */
static int fz_finish(struct dcall *k, int sync)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	const struct comp *c0 = &s->rtp;
	const size_t n = d->n;
	const unsigned ns0 = s->nstreams;
	struct ws *w = k->w;
	struct sgpu_fused *F = &k->fz;
	const size_t poff = k->foff;
	const struct sgpu_plan_out *po =
		(const struct sgpu_plan_out *)(w->fz.h + poff);
	const struct sgpu_fold_out *fo =
		(const struct sgpu_fold_out *)(w->fz.h + poff + FZ_FO_OFF);
	void *stream = d->stream;
	struct srtp_stream old;
	int err;

	k->pfail = po->fail;
	if (po->fail) {
		/* no work that counts: nothing (gated) or undone */
		sgpu_prof_void(F->prof_id);
		if (po->fail & SPF_PRED)
			return -2;      /* every workgroup did nothing */
		if (po->fail & (SPF_BAD | SPF_SLOW))
			w->fz_d = NULL; /* ticket / look-back state from zero */
		if (po->fail & SPF_SLOW)
			count(&g_cnt_lbtimeout, 1);
		if ((po->fail & SPF_SSRC) && !ns0)
			__atomic_store_n(&g_fresh_multi, 1, __ATOMIC_RELAXED);
		count(&g_cnt_rejects, 1);
		goto undo;
	}
	plan_apply(s, po, prot, n, &old);
	count(&g_cnt_fused, 1);
	if (!po->nfail)
		return 0;
	count(&g_cnt_misses, po->nfail);
	(void)sync;
	if (!g_env.nodevfold) {
		/* forged packets: ciphertext back, verdicts folded on the
		 * device; its outcome comes back in one copy */
		struct sgpu_fold_out *fo_d =
			(struct sgpu_fold_out *)(w->fz.d + poff + FZ_FO_OFF);
		err = sgpu_fused_refix(d->arena, d->arena_size, F,
				       (int)c0->nr, stream);
		if (!err)
			err = sgpu_fold_rtp(0, &F->out->nfail, &F->in, F->hdr,
					    F->desc, F->verdict, F->es, d->pos,
					    d->end, d->err, 0,
					    (uint32_t *)(w->pl.d + 64), fo_d,
					    stream);
		if (!err)
			err = sgpu_memcpy_d2h(w->fz.h + poff + FZ_FO_OFF, fo_d,
					      sizeof(*fo), stream);
		if (!err)
			err = sgpu_stream_sync(stream);
		if (err)
			return err;
		k->devfold = 1;
	}
	if (k->devfold && !fo->fail) {
		struct srtp_stream *st = &s->streams[0];
		st->s_l = (uint16_t)fo->s_l;
		st->replay_rtp.lix = fo->lix;
		st->replay_rtp.bitmap = fo->bitmap;
		count(&g_cnt_devfolds, 1);
		return 0;
	}
	/* the fold cannot be settled on the device (or nodevfold): undo --
	 * forged packets still decrypted are re-encrypted with the rest --
	 * and fold on the host */
	count(&g_cnt_folds, 1);
	plan_unapply(s, ns0, &old);
 undo:
	if (po->hl0 != 0xffffffffu) {
		F->shift = (po->hl0 >> 2) & 3u;
		err = sgpu_fused_undo(d->arena, d->arena_size, F, (int)c0->nr,
				      prot, stream);
		if (err)
			return err;
	}
	err = sgpu_memcpy_d2d(d->end, F->es, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	return err ? err : -1;
}

/* synchronous (dev_planned): -1 not plannable (nothing modified;
 * *pfail: why, 0 for a forged packet the host must fold), else 0 /
 * errno */
static int dev_fused(int op, struct srtp *s, struct srtp_batch_dev *d,
		     uint32_t *pfail)
{
	struct dcall k;
	int err;
	memset(&k, 0, sizeof(k));
	k.op = op;
	k.sessv = &s;
	k.nsess = 1;
	k.d = *d;
	k.w = ws_get();
	*pfail = 0;
	if (!k.w)
		return ENOMEM;
	{
		/* where a synchronous call's host time goes (counters
		 * sync_ns_issue / _wait / _finish) */
		const uint64_t t0 = mono_ns();
		uint64_t t1, t2;
		err = fz_issue(&k, 1);
		t1 = mono_ns();
		if (!err)
			err = sync_wait(&k, d->stream);
		t2 = mono_ns();
		if (err)
			return err;
		err = fz_finish(&k, 1);
		count(&g_cnt_sync_calls, 1);
		count(&g_ns_sync_issue, t1 - t0);
		count(&g_ns_sync_wait, t2 - t1);
		count(&g_ns_sync_finish, mono_ns() - t2);
	}
	*pfail = k.pfail;
	return err;
}

/* ---- one stream, the one-launch planner in front of the lean kernels -- */

/*
 * k_lp_plan (k_ctr_fused.h) plans the batch in one launch -- the in-launch
 * plan of k_ctr_fused as a kernel of its own: hdr, es, desc, the plan out
 * with the class guards skip[], the results of every packet planned -- and
 * the lean crypto kernel runs behind it, guarded by skip[] and out->fail
 * (AES-CM: k_ctr_fast_any) or by out->fail (GCM: k_gcmu), counting its
 * tag misses into out->nfail.  A rejected plan wrote no byte of the arena
 * (the crypto launch did nothing): only the ends are put back.  Forged
 * packets: as dev_fused (the restore of their ciphertext and the verdict
 * fold after the synchronisation; queued behind for asynchronous calls).
 * Same workspace state as fz_issue (w->fz: tickets, epochs, plan outs).
 */
/* the fused / one-launch planners' workspace state (w->fz: ticket |
 * (plan out, fold out) x 2 | look-back words for nblk workgroups), zeroed
 * on a new pool, an epoch wrap or the fzepoch hook */
static int fz_prepare(struct ws *w, uint32_t nblk, void *stream)
{
	int err = pool_reserve(w, &w->fz, FZ_HEAD + 2 * FZ_SLOT +
			       (size_t)nblk * 8);
	const long e = __atomic_exchange_n(&g_env.fzepoch, 0,
					   __ATOMIC_RELAXED);
	if (err)
		return err;
	if (e > 0 && e <= 0xffff)
		w->fz_d = NULL;
	if (w->fz_d != w->fz.d || w->fz_epoch == 0 ||
	    w->fz_epoch > 0xffffu) {
		err = sgpu_memset(w->fz.d, 0, w->fz.cap, stream);
		if (err)
			return err;
		w->fz_d = w->fz.d;
		w->fz_epoch = 1;
		w->fz_tbase = 0;
		w->fz_par = 0;
	}
	if (e > 0 && e <= 0xffff)
		w->fz_epoch = (uint32_t)e;
	return 0;
}

static int lp_issue(struct dcall *k, int sync)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	const struct comp *c0 = &s->rtp;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const size_t n = d->n;
	const uint32_t T = gcm ? 16u : c0->tag_len;
	const uint32_t need = prot ? (gcm ? 16u : (T > 4 ? T : 4u)) : 0u;
	const uint32_t B = sgpu_fused_block();
	const uint32_t nblk = (uint32_t)((n + B - 1) / B);
	struct ws *w = k->w;
	struct sgpu_fused *F = &k->fz;
	void *stream = d->stream;
	uint8_t *fz;
	size_t poff;
	int err;

	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 8);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 9 + 72);
	if (!err)
		err = pool_reserve(w, &w->cm, 4);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)
		err = pool_reserve(w, &w->pl, 64 + (n / 256 + 4) * 20);
	if (!err)
		err = fz_prepare(w, nblk, stream);
	if (err)
		return err;
	fz = w->fz.d;
	poff = FZ_HEAD + (size_t)w->fz_par * FZ_SLOT;
	k->foff = poff;

	memset(F, 0, sizeof(*F));
	plan_in(&F->in, s, (uint32_t)n, prot, T, need);
	F->in.zeroed = 1;
	F->in.pred = k->pred;
	F->pos = d->pos;
	F->end = d->end;
	F->cap = d->cap;
	F->err = d->err;
	F->es = (uint32_t *)w->es.d;
	F->hdr = (struct sgpu_hdr *)w->hd.d;
	F->desc = (uint64_t *)w->dsc.d;
	if (!prot) {
		F->save = (uint32_t *)(w->vs.d + 64);
		F->verdict = w->vs.d + 64 + n * 4;
		F->flist = gcm ? NULL : (uint32_t *)(w->vs.d +
				     ((64 + n * 5 + 3) & ~(size_t)3));
	}
	F->out = (struct sgpu_plan_out *)(fz + poff);
	F->out_next = (struct sgpu_plan_out *)(fz + FZ_HEAD +
					       (size_t)(w->fz_par ^ 1) * FZ_SLOT);
	F->cm_out = (uint32_t *)w->cm.d;
	F->agg = (unsigned long long *)(fz + FZ_HEAD + 2 * FZ_SLOT);
	F->ticket = (uint32_t *)fz;
	F->tbase = w->fz_tbase;
	F->epoch = w->fz_epoch;
	F->comp = c0->dev;
	F->delta = prot ? (int32_t)T : -(int32_t)T;
	err = sgpu_run_fzplan(d->arena, d->arena_size, F, stream);
	if (err) {
		w->fz_d = NULL;
		return err;
	}
	w->fz_tbase += F->ntickets;
	w->fz_epoch++;
	w->fz_par ^= 1;
	{
		/* the crypto launch behind the plan's guards */
		struct sgpu_compact C = {
			d->pos, F->es, F->hdr, F->desc, NULL, F->cm_out, NULL, 0,
			(uint32_t)n, F->verdict, F->save, &F->out->nfail, 0,
			gcm ? 1 : 2, gcm ? &F->out->fail : F->out->skip, 0,
			F->flist, gcm ? NULL : &F->out->fail};
		err = sgpu_run_compact(d->arena, d->arena_size, &C, c0->mode,
				       (int)c0->nr, gcm ? 0 : -1, prot, stream);
		if (err)
			return err;
	}
	return plan_out_back(k, sync, F->out, w->fz.h + poff, stream);
}

static int lp_finish(struct dcall *k, int sync)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	const struct comp *c0 = &s->rtp;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const size_t n = d->n;
	const unsigned ns0 = s->nstreams;
	struct ws *w = k->w;
	struct sgpu_fused *F = &k->fz;
	const size_t poff = k->foff;
	const struct sgpu_plan_out *po =
		(const struct sgpu_plan_out *)(w->fz.h + poff);
	const struct sgpu_fold_out *fo =
		(const struct sgpu_fold_out *)(w->fz.h + poff + FZ_FO_OFF);
	void *stream = d->stream;
	struct srtp_stream old;
	int err;

	k->pfail = po->fail;
	if (po->fail) {
		if (po->fail & SPF_PRED)
			return -2;      /* every workgroup did nothing */
		if (po->fail & (SPF_BAD | SPF_SLOW))
			w->fz_d = NULL;
		if (po->fail & SPF_SLOW)
			count(&g_cnt_lbtimeout, 1);
		if ((po->fail & SPF_SSRC) && !ns0)
			__atomic_store_n(&g_fresh_multi, 1, __ATOMIC_RELAXED);
		count(&g_cnt_rejects, 1);
		if (g_env.times)
			fprintf(stderr, "re_srtp plan n=%zu %s: rejected "
				"(SPF %#x)\n", n, prot ? "protect" : "unprotect",
				po->fail);
		/* the crypto launch did nothing: only the ends the plan wrote
		 * go back */
		err = sgpu_memcpy_d2d(d->end, F->es, n * 4, stream);
		if (!err)
			err = sgpu_stream_sync(stream);
		return err ? err : -1;
	}
	plan_apply(s, po, prot, n, &old);
	count(&g_cnt_lplans, 1);
	if (!po->nfail)
		return 0;
	count(&g_cnt_misses, po->nfail);
	(void)sync;
	if (!g_env.nodevfold) {
		struct sgpu_fold_out *fo_d =
			(struct sgpu_fold_out *)(w->fz.d + poff + FZ_FO_OFF);
		err = 0;
		if (!gcm)
			err = sgpu_fused_refix(d->arena, d->arena_size, F,
					       (int)c0->nr, stream);
		if (!err)
			err = sgpu_fold_rtp(0, &F->out->nfail, &F->in, F->hdr,
					    F->desc, F->verdict, F->es, d->pos,
					    d->end, d->err, gcm,
					    (uint32_t *)(w->pl.d + 64), fo_d,
					    stream);
		if (!err)
			err = sgpu_memcpy_d2h(w->fz.h + poff + FZ_FO_OFF, fo_d,
					      sizeof(*fo), stream);
		if (!err)
			err = sgpu_stream_sync(stream);
		if (err)
			return err;
		k->devfold = 1;
	}
	if (k->devfold && !fo->fail) {
		struct srtp_stream *st = &s->streams[0];
		st->s_l = (uint16_t)fo->s_l;
		st->replay_rtp.lix = fo->lix;
		st->replay_rtp.bitmap = fo->bitmap;
		count(&g_cnt_devfolds, 1);
		return 0;
	}
	/* the fold cannot be settled on the device (or nodevfold): every
	 * processed packet back to its bytes, the host folds */
	count(&g_cnt_folds, 1);
	plan_unapply(s, ns0, &old);
	if (gcm) {
		struct sgpu_compact C = {
			d->pos, F->es, F->hdr, F->desc, NULL, F->cm_out, NULL, 0,
			(uint32_t)n, F->verdict, F->save, &F->out->nfail, 1, 1,
			NULL, 0, NULL, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0, F->out, prot,
				  stream);
	}
	else {
		F->shift = (po->hl0 >> 2) & 3u;
		err = sgpu_fused_undo(d->arena, d->arena_size, F, (int)c0->nr,
				      prot, stream);
	}
	if (!err)
		err = sgpu_memcpy_d2d(d->end, F->es, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	return err ? err : -1;
}

/* synchronous (dev_planned): -1 not plannable (nothing modified;
 * *pfail: why, 0 for a forged packet the host must fold), else 0 /
 * errno */
static int dev_lplanned(int op, struct srtp *s, struct srtp_batch_dev *d,
			uint32_t *pfail)
{
	struct dcall k;
	int err;
	memset(&k, 0, sizeof(k));
	k.op = op;
	k.sessv = &s;
	k.nsess = 1;
	k.d = *d;
	k.w = ws_get();
	*pfail = 0;
	if (!k.w)
		return ENOMEM;
	err = lp_issue(&k, 1);
	if (!err)
		err = sgpu_stream_sync(d->stream);
	if (err)
		return err;
	err = lp_finish(&k, 1);
	*pfail = k.pfail;
	return err;
}

/* synchronous: -1 not plannable (nothing modified; *pfail: why, 0 for a
 * forged packet the host must fold), else 0 / errno */
int dev_planned(int op, struct srtp *s, struct srtp_batch_dev *d,
		       uint32_t *pfail)
{
	struct dcall k;
	int err;
	if (!g_env.noplanfuse) {
		if (s->rtp.mode == SGPU_MODE_CTR && !g_env.lplan)
			return dev_fused(op, s, d, pfail);
		return dev_lplanned(op, s, d, pfail);
	}
	memset(&k, 0, sizeof(k));
	k.op = op;
	k.sessv = &s;
	k.nsess = 1;
	k.d = *d;
	k.w = ws_get();
	if (!k.w)
		return ENOMEM;
	err = dev_planned_issue(&k);
	if (!err)
		err = sgpu_stream_sync(d->stream);
	if (err)
		return err;
	err = dev_planned_finish(&k);
	*pfail = k.pfail;
	return err;
}

/* ---- one session, several streams (plan_streams.hip) ------------------ */

static void splan_in(struct sgpu_splan_in *in, const struct srtp *s,
		     uint32_t n, int prot, uint32_t T, uint32_t need)
{
	unsigned k;
	memset(in, 0, sizeof(*in));
	in->n = n;
	in->prot = (uint32_t)prot;
	in->tag = T;
	in->need = need;
	in->maxlen = SGPU_CACHED_MAX(s->rtp.mode);
	in->nst = s->nstreams;
	for (k = 0; k < s->nstreams; k++) {
		const struct srtp_stream *x = &s->streams[k];
		in->st[k].ssrc = x->ssrc;
		in->st[k].roc = x->roc;
		in->st[k].s_l = x->s_l;
		in->st[k].flags = SST_EXISTS | (x->s_l_set ? SST_SL_SET : 0);
		in->st[k].lix = x->replay_rtp.lix;
		in->st[k].bitmap = x->replay_rtp.bitmap;
	}
}

/* stream states after an accepted plan: streams with packets in the batch
 * advance, new SSRCs are appended in first-appearance order (stream_new,
 * stream.c:45-67) */
static void splan_apply(struct srtp *s, const struct sgpu_splan_out *po,
			int prot)
{
	unsigned k;
	for (k = 0; k < po->nst && k < SRTP_MAX_STREAMS; k++) {
		struct srtp_stream *x = &s->streams[k];
		if (!po->cnt[k])
			continue;
		if (k >= s->nstreams) {
			memset(x, 0, sizeof(*x));
			x->ssrc = po->ssrc[k];
		}
		x->s_l_set = 1;
		x->roc += po->wraps[k];
		x->s_l = (uint16_t)po->s_l_last[k];
		if (!prot)
			x->replay_rtp = plan_replay(&x->replay_rtp, po->tail_ix[k],
						    po->cnt[k]);
	}
	if (po->nst > s->nstreams)
		s->nstreams = po->nst;
}

/* the launches (no host synchronisation) */
int dev_splanned_issue(struct dcall *k)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &s->rtp;
	const size_t n = d->n;
	const uint32_t T = c0->mode == SGPU_MODE_GCM ? 16u : c0->tag_len;
	const uint32_t need = prot ? (c0->mode == SGPU_MODE_GCM ? 16u :
			      (T > 4 ? T : 4u)) : 0u;
	const size_t scr = sgpu_splan_scratch((uint32_t)n);
	struct sgpu_splan_out *po, *po_d;
	struct sgpu_hdr *hd_d;
	uint64_t *desc_d;
	uint32_t *es_d, *save_d, *nfail_d;
	uint8_t *vd_d;
	void *stream = d->stream;
	int err;

	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 12);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 5 + 64);
	if (!err)
		err = pool_reserve(w, &w->cm, 4);
	if (!err)
		err = pool_reserve(w, &w->pl, sizeof(struct sgpu_splan_out) + 64);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)
		err = pool_reserve(w, &w->mscr, scr);
	if (err)
		return err;
	hd_d = (struct sgpu_hdr *)w->hd.d;
	desc_d = (uint64_t *)w->dsc.d;
	nfail_d = (uint32_t *)w->vs.d;
	save_d = (uint32_t *)(w->vs.d + 64);
	vd_d = w->vs.d + 64 + n * 4;
	po = (struct sgpu_splan_out *)w->pl.h;
	po_d = (struct sgpu_splan_out *)w->pl.d;
	es_d = (uint32_t *)w->es.d;

	splan_in(&k->sin, s, (uint32_t)n, prot, T, need);
	{
		struct sgpu_prologue pro = {
			es_d, nfail_d, (uint32_t *)po_d, 1,
			(uint32_t)(sizeof(*po) / 4), (uint32_t *)w->cm.d,
			c0->dev, NULL, NULL, 0, 0, 0, 0, NULL, 0};
		k->sin.zeroed = 1;
		err = sgpu_parse_prologue(d->arena, d->arena_size, d->pos,
					  d->end, hd_d, NULL, (uint32_t)n, 0,
					  &pro, stream);
	}
	if (!err && k->pred)
		err = sgpu_gate_pred(k->pred, &po_d->base.fail, stream);
	if (!err)
		err = sgpu_splan_rtp(&k->sin, hd_d, d->pos, es_d, d->cap,
				     d->arena_size, desc_d, w->mscr.d, scr, po_d,
				     stream);
	if (!err) {
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, NULL,
			(const uint32_t *)w->cm.d, NULL, 0, (uint32_t)n, vd_d,
			save_d, nfail_d, 0, 1, NULL, 0, NULL, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0,
				  &po_d->base, prot, stream);
	}
	if (!err)
		err = sgpu_plan_finish(&po_d->base.fail, es_d, d->end, d->err,
				       (uint32_t)n,
				       prot ? (int32_t)T : -(int32_t)T, nfail_d,
				       k->gate, &po_d->base.nfail, NULL, stream);
	if (!err)
		err = sgpu_memcpy_d2h(po, po_d, sizeof(*po), stream);
	return err;
}

/* ... after its launches completed: 0 / errno, -1 not plannable or a
 * forged packet (undone on the device; the host folds), -2 gated by the
 * chained call before (nothing modified) */
int dev_splanned_finish(struct dcall *k)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp *s = k->sessv[0];
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &s->rtp;
	const size_t n = d->n;
	const struct sgpu_splan_out *po = (const struct sgpu_splan_out *)w->pl.h;
	struct sgpu_splan_out *po_d = (struct sgpu_splan_out *)w->pl.d;
	const uint32_t nfail = po->base.nfail;
	int err;

	k->pfail = po->base.fail;
	if (po->base.fail) {
		if (po->base.fail & SPF_PRED)
			return -2;
		count(&g_cnt_rejects, 1);
		return -1;
	}
	count(&g_cnt_splans, 1);
	if (!s->nstreams && po->nst <= 1)
		__atomic_store_n(&g_fresh_multi, 0, __ATOMIC_RELAXED);
	if (!nfail) {
		splan_apply(s, po, prot);
		return 0;
	}
	count(&g_cnt_misses, nfail);
	count(&g_cnt_folds, 1);
	/* a forged packet: undo on the device, fold on the host engine */
	{
		struct sgpu_compact C = {
			d->pos, (uint32_t *)w->es.d, (struct sgpu_hdr *)w->hd.d,
			(uint64_t *)w->dsc.d, NULL, (const uint32_t *)w->cm.d,
			NULL, 0, (uint32_t)n, w->vs.d + 64 + n * 4,
			(uint32_t *)(w->vs.d + 64), (uint32_t *)w->vs.d, 1, 1,
			NULL, 0, NULL, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0, &po_d->base,
				  prot, d->stream);
	}
	if (!err)
		err = sgpu_memcpy_d2d(d->end, w->es.d, n * 4, d->stream);
	if (!err)
		err = sgpu_stream_sync(d->stream);
	return err ? err : -1;
}

/* synchronous: -1 not plannable or folded on the host (nothing
 * modified), else 0 / errno */
int dev_splanned(int op, struct srtp *s, struct srtp_batch_dev *d)
{
	struct dcall k;
	int err;
	memset(&k, 0, sizeof(k));
	k.op = op;
	k.sessv = &s;
	k.nsess = 1;
	k.d = *d;
	k.w = ws_get();
	if (!k.w)
		return ENOMEM;
	err = dev_splanned_issue(&k);
	if (!err)
		err = sgpu_stream_sync(d->stream);
	if (err)
		return err;
	return dev_splanned_finish(&k);
}

/* the SRTCP plan input of a batch of n packets on session s */
static void rplan_in(struct sgpu_rplan_in *in, const struct srtp *s,
		     uint32_t n, int prot)
{
	const struct comp *c0 = &s->rtcp;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const uint32_t T = c0->tag_len;             /* 0 for GCM */
	memset(in, 0, sizeof(*in));
	in->n = n;
	in->prot = (uint32_t)prot;
	in->ssrc_any = !s->nstreams;
	in->ssrc = s->nstreams ? s->streams[0].ssrc : 0;
	in->rtcp_index = s->nstreams ? s->streams[0].rtcp_index : 0;
	in->lix = s->nstreams ? s->streams[0].replay_rtcp.lix : 0;
	in->bitmap = s->nstreams ? s->streams[0].replay_rtcp.bitmap : 0;
	in->tag = T;
	in->gcm = (uint32_t)gcm;
	in->hmac = (uint32_t)c0->has_hmac;
	in->encrypted = (uint32_t)(gcm ? c0->encrypted : c0->has_aes);
	in->need = 4u + T + (gcm ? 16u : 0u);
	in->maxlen = SGPU_CACHED_MAX(c0->mode);
}

/* the stream (stream.c:45-67) and its SRTCP state after an accepted
 * plan; *old: the state before */
static void rplan_apply(struct srtp *s, const struct sgpu_plan_out *po,
			int prot, size_t n, struct srtp_stream *old)
{
	if (!s->nstreams) {
		memset(&s->streams[0], 0, sizeof(s->streams[0]));
		s->streams[0].ssrc = po->ssrc0;
		s->nstreams = 1;
	}
	*old = s->streams[0];
	if (prot)
		s->streams[0].rtcp_index =
			(s->streams[0].rtcp_index + (uint32_t)n) & 0x7fffffffu;
	else if (s->rtcp.has_hmac)
		s->streams[0].replay_rtcp =
			plan_replay(&s->streams[0].replay_rtcp, po->tail_ix, n);
}

/*
 * Single-stream SRTCP batch planned in one launch (k_rp_plan: the parse,
 * every check of k_plan_rtcp, desc) in front of the single-key crypto
 * kernel, which it guards with out->fail and whose misses it counts in
 * out->nfail, then the guarded results; one copy and one
 * synchronisation.  -1: not plannable (nothing modified) or a forged
 * packet (undone), else 0 / errno.
 */
static int dev_lplanned_rtcp(int op, struct srtp *s, struct srtp_batch_dev *d)
{
	const int prot = op == OP_RTCP_ENC;
	const struct comp *c0 = &s->rtcp;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const size_t n = d->n;
	const uint32_t grow = 4u + c0->tag_len + (gcm ? 16u : 0u);
	const unsigned ns0 = s->nstreams;
	struct srtp_stream old;
	struct sgpu_rfused R;
	struct sgpu_plan_out *po, *po_d;
	uint8_t *vd_d;
	uint32_t *save_d;
	void *stream = d->stream;
	struct ws *w = ws_get();
	size_t poff;
	int err;

	if (!w)
		return ENOMEM;
	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 8);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 5 + 64);
	if (!err)
		err = pool_reserve(w, &w->cm, 4);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)
		err = fz_prepare(w, 1, stream);
	if (err)
		return err;
	poff = FZ_HEAD + (size_t)w->fz_par * FZ_SLOT;
	po = (struct sgpu_plan_out *)(w->fz.h + poff);
	po_d = (struct sgpu_plan_out *)(w->fz.d + poff);
	save_d = (uint32_t *)(w->vs.d + 64);
	vd_d = w->vs.d + 64 + n * 4;
	memset(&R, 0, sizeof(R));
	rplan_in(&R.in, s, (uint32_t)n, prot);
	R.pos = d->pos;
	R.end = d->end;
	R.cap = d->cap;
	R.err = d->err;
	R.es = (uint32_t *)w->es.d;
	R.hdr = (struct sgpu_hdr *)w->hd.d;
	R.desc = (uint64_t *)w->dsc.d;
	R.out = po_d;
	R.out_next = (struct sgpu_plan_out *)(w->fz.d + FZ_HEAD +
					      (size_t)(w->fz_par ^ 1) * FZ_SLOT);
	R.cm_out = (uint32_t *)w->cm.d;
	R.comp = c0->dev;
	R.delta = prot ? (int32_t)grow : -(int32_t)grow;
	err = sgpu_run_rpplan(d->arena, d->arena_size, &R, stream);
	if (err) {
		w->fz_d = NULL;
		return err;
	}
	w->fz_par ^= 1;
	{
		/* CTR: the lean kernel's SRTCP form (srtp_gpu_tune nolean: the
		 * general compact kernel) */
		struct sgpu_compact C = {
			d->pos, R.es, R.hdr, R.desc, NULL, R.cm_out, NULL, 0,
			(uint32_t)n, vd_d, save_d, &po_d->nfail, 0,
			gcm || g_env.nolean ? 1 : 4, &po_d->fail, 1, NULL, NULL};
		err = sgpu_run_compact(d->arena, d->arena_size, &C, c0->mode,
				       (int)c0->nr, gcm ? 0 : 2, prot, stream);
	}
	if (!err)   /* the results, guarded by the plan */
		err = sgpu_plan_results(&po_d->fail, R.es, d->end, d->err,
					(uint32_t)n, R.delta, stream);
	if (!err)
		err = g_env.nopost ? sgpu_memcpy_d2h(po, po_d, sizeof(*po), stream)
				   : sgpu_plan_post(po_d, po, sizeof(*po), NULL,
						    NULL, 0, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	if (po->fail) {
		/* the crypto launch and the results did nothing */
		count(&g_cnt_rejects, 1);
		if (g_env.times)
			fprintf(stderr, "re_srtp rtcp plan n=%zu %s: rejected "
				"(SPF %#x)\n", n, prot ? "protect" : "unprotect",
				po->fail);
		return -1;
	}
	count(&g_cnt_rplans, 1);
	rplan_apply(s, po, prot, n, &old);
	if (!po->nfail)
		return 0;
	count(&g_cnt_misses, po->nfail);
	count(&g_cnt_folds, 1);
	/* a forged packet: undo on the device, fold on the host engine */
	{
		struct sgpu_compact C = {
			d->pos, R.es, R.hdr, R.desc, NULL, R.cm_out, NULL, 0,
			(uint32_t)n, vd_d, save_d, &po_d->nfail, 1, gcm ? 0 : 1,
			&po_d->fail, 1, NULL, NULL};
		err = sgpu_run_compact(d->arena, d->arena_size, &C, c0->mode,
				       (int)c0->nr, gcm ? 0 : 2, 0, stream);
	}
	if (!err)
		err = sgpu_memcpy_d2d(d->end, R.es, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	s->streams[0] = old;
	s->nstreams = ns0;
	return -1;
}

/*
 * Single-stream SRTCP batch planned and processed on the device (the
 * SRTCP counterpart of dev_planned): by default the one-launch plan above;
 * srtp_gpu_tune noplanfuse: k_parse (with the E || index words),
 * k_plan_rtcp, the compact crypto launch, the per-packet results; one host
 * synchronisation.  -1: not plannable or a forged packet (undone), else 0
 * / errno.
 */
int dev_planned_rtcp(int op, struct srtp *s, struct srtp_batch_dev *d)
{
	if (!g_env.noplanfuse)
		return dev_lplanned_rtcp(op, s, d);
	const int prot = op == OP_RTCP_ENC;
	const struct comp *c0 = &s->rtcp;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const size_t n = d->n;
	const uint32_t T = c0->tag_len;             /* 0 for GCM */
	const uint32_t grow = 4u + T + (gcm ? 16u : 0u);
	const unsigned ns0 = s->nstreams;
	struct srtp_stream old;
	struct sgpu_rplan_in in;
	struct sgpu_plan_out *po, *po_d;
	struct sgpu_hdr *hd_d;
	uint64_t *desc_d;
	uint32_t *es_d, *save_d, *nfail_d, *eix_d, nfail, cm = c0->dev;
	uint8_t *vd_d;
	void *stream = d->stream;
	struct ws *w = ws_get();
	int err;

	if (!w)
		return ENOMEM;
	err = pool_reserve(w, &w->hd, n * (sizeof(struct sgpu_hdr) + 12));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 12);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 5 + 64);
	if (!err)
		err = pool_reserve(w, &w->cm, 4);
	if (!err)
		err = pool_reserve(w, &w->pl, sizeof(struct sgpu_plan_out) + 64);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (err)
		return err;
	hd_d = (struct sgpu_hdr *)w->hd.d;
	eix_d = (uint32_t *)(w->hd.d + n * sizeof(struct sgpu_hdr));
	desc_d = (uint64_t *)w->dsc.d;
	nfail_d = (uint32_t *)w->vs.d;
	save_d = (uint32_t *)(w->vs.d + 64);
	vd_d = w->vs.d + 64 + n * 4;
	po = (struct sgpu_plan_out *)w->pl.h;
	po_d = (struct sgpu_plan_out *)w->pl.d;
	es_d = (uint32_t *)w->es.d;

	memset(&in, 0, sizeof(in));
	in.n = (uint32_t)n;
	in.prot = (uint32_t)prot;
	in.ssrc_any = !s->nstreams;
	in.ssrc = s->nstreams ? s->streams[0].ssrc : 0;
	in.rtcp_index = s->nstreams ? s->streams[0].rtcp_index : 0;
	in.lix = s->nstreams ? s->streams[0].replay_rtcp.lix : 0;
	in.bitmap = s->nstreams ? s->streams[0].replay_rtcp.bitmap : 0;
	in.tag = T;
	in.gcm = (uint32_t)gcm;
	in.hmac = (uint32_t)c0->has_hmac;
	in.encrypted = (uint32_t)(gcm ? c0->encrypted : c0->has_aes);
	in.need = grow;
	in.maxlen = SGPU_CACHED_MAX(c0->mode);
	{
		/* parse (+ E || index words) + end copy + zeroed counters and
		 * plan + comp map, one launch */
		struct sgpu_prologue pro = {
			es_d, nfail_d, (uint32_t *)po_d, 1,
			(uint32_t)(sizeof(*po) / 4), (uint32_t *)w->cm.d, cm, NULL, NULL,
			0, 0, 0, 0, NULL, 0};
		err = sgpu_parse_prologue(d->arena, d->arena_size, d->pos,
					  d->end, hd_d, prot ? NULL : eix_d,
					  (uint32_t)n, 1, &pro, stream);
	}
	if (!err)
		err = sgpu_plan_rtcp(&in, hd_d, eix_d, d->pos, es_d, d->cap,
				     d->arena_size, desc_d, po_d, stream);
	if (!err) {
		/* CTR: the lean kernel's SRTCP form (srtp_gpu_tune nolean:
		 * the general compact kernel) */
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, NULL,
			(const uint32_t *)w->cm.d, NULL, 0, (uint32_t)n, vd_d,
			save_d, nfail_d, 0, gcm || g_env.nolean ? 1 : 4,
			gcm ? &po_d->fail : &po_d->skip[2], 1, NULL, NULL};
		err = sgpu_run_compact(d->arena, d->arena_size, &C, c0->mode,
				       (int)c0->nr, gcm ? 0 : 2, prot, stream);
	}
	if (!err)
		err = sgpu_plan_finish(&po_d->fail, es_d, d->end, d->err,
				       (uint32_t)n,
				       prot ? (int32_t)grow : -(int32_t)grow,
				       nfail_d, NULL, &po_d->nfail, NULL, stream);
	if (!err)
		err = sgpu_memcpy_d2h(po, po_d, sizeof(*po), stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	nfail = po->nfail;
	if (po->fail) {
		count(&g_cnt_rejects, 1);
		return -1;
	}
	count(&g_cnt_rplans, 1);
	/* the stream (stream.c:45-67) and its SRTCP state after the batch */
	if (!s->nstreams) {
		memset(&s->streams[0], 0, sizeof(s->streams[0]));
		s->streams[0].ssrc = po->ssrc0;
		s->nstreams = 1;
	}
	old = s->streams[0];
	if (prot)
		s->streams[0].rtcp_index =
			(s->streams[0].rtcp_index + (uint32_t)n) & 0x7fffffffu;
	else if (c0->has_hmac)
		s->streams[0].replay_rtcp =
			plan_replay(&s->streams[0].replay_rtcp, po->tail_ix, n);
	if (!nfail)
		return 0;
	count(&g_cnt_misses, nfail);
	count(&g_cnt_folds, 1);
	/* a forged packet: undo on the device, fold on the host engine */
	{
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, NULL,
			(const uint32_t *)w->cm.d, NULL, 0, (uint32_t)n, vd_d,
			save_d, nfail_d, 1, gcm ? 0 : 1,
			gcm ? &po_d->fail : &po_d->skip[2], 1, NULL, NULL};
		err = sgpu_run_compact(d->arena, d->arena_size, &C, c0->mode,
				       (int)c0->nr, gcm ? 0 : 2, 0, stream);
	}
	if (!err)
		err = sgpu_memcpy_d2d(d->end, es_d, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	s->streams[0] = old;
	s->nstreams = ns0;
	return -1;
}

/*
 * Many sessions with at most one RTP stream each, every array in HBM: the
 * multi-session device planner (plan_multi.hip) plus the compact kernels
 * in length order, against the session states resident in HBM
 * (sgpu_sst_*); host work is one O(sessions) pass (slot map, residency).
 * The launches; -1: not plannable (after a synchronisation; nothing
 * modified).
 */
/* the multi-session verdict fold over the call's planner scratch (phase:
 * sgpu_mfold_rtp; nfail: the kernels' miss count, device, or NULL) */
static int mfold(struct dcall *k, int phase, const uint32_t *nfail,
		 const struct sgpu_sstate *sin_d, struct sgpu_sstate *sout_d,
		 size_t scr)
{
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const size_t n = d->n;
	struct sgpu_mplan_in in;
	memset(&in, 0, sizeof(in));
	in.n = (uint32_t)n;
	in.nsess = (uint32_t)k->nsess;
	return sgpu_mfold_rtp(phase, nfail, &in, (const struct sgpu_hdr *)w->hd.d,
			      d->sess, (const uint64_t *)w->dsc.d,
			      w->vs.d + 64 + n * 4, (const uint32_t *)w->es.d,
			      d->pos, d->end, d->err,
			      k->sessv[0]->rtp.mode == SGPU_MODE_GCM, sin_d,
			      sout_d, w->mscr.d, scr,
			      (uint32_t *)(w->pl.d + k->foff + 64),
			      (struct sgpu_fold_out *)(w->pl.d + k->foff),
			      d->stream);
}

/*
 * The bucket planner (plan_buckets.hip, srtpgpu.h struct sgpu_bplan): the
 * same plan, verdict fold and resident states as below, in three launches
 * around the crypto instead of ~17 plus the fold's five.
 *
 * w->bp: ticket words | bin counters | bucket counters (BP_HEAD, zero
 * between calls) | bucket entries | sorted | fail words | sseg | sout |
 * launch order
 */
#define BP_HEAD (512u + 4u * SGPU_BP_NBMAX)

static int dev_bplanned_issue(struct dcall *k, uint32_t bshift, uint32_t nb,
			      uint32_t cap)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp **sessv = k->sessv;
	const size_t nsess = k->nsess;
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &sessv[0]->rtp;
	const size_t n = d->n;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const uint32_t T = gcm ? 16u : c0->tag_len;
	const size_t na = (n + SGPU_BP_BLOCK * SGPU_BP_PPT - 1) /
			  (SGPU_BP_BLOCK * SGPU_BP_PPT);
	struct sgpu_bplan *B = &k->bp;
	struct sgpu_sstate *up_h, *up_d;
	uint8_t *need_h, *need_d, *p;
	uint32_t *cm_h;
	void *stream = d->stream;
	const int times = g_env.times;
	int err;

	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 8);
	if (!err)   /* nfail | save | verdict | forged list */
		err = pool_reserve(w, &w->vs, n * 9 + 72);
	if (!err)
		err = pool_reserve(w, &w->cm, nsess * 4);
	k->foff = (sizeof(struct sgpu_plan_out) + 63) & ~(size_t)63;
	if (!err)   /* plan out | fold out */
		err = pool_reserve(w, &w->pl, k->foff + 64);
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)   /* uploads | need */
		err = pool_reserve(w, &w->ms,
				   nsess * (sizeof(struct sgpu_sstate) + 1));
	if (!err)
		err = pool_reserve(w, &w->bp, BP_HEAD +
				   sgpu_bplan_scratch((uint32_t)n,
						      (uint32_t)nsess, nb, cap) +
				   n * 4 + 256);
	if (err)
		return err;
	if (w->bp_d != w->bp.d) {
		/* a new pool (or a call that did not finish): counters and
		 * tickets from zero */
		err = sgpu_memset(w->bp.d, 0, BP_HEAD, stream);
		if (err)
			return err;
		w->bp_d = w->bp.d;
	}
	memset(B, 0, sizeof(*B));
	B->n = (uint32_t)n;
	B->nsess = (uint32_t)nsess;
	B->prot = (uint32_t)prot;
	B->tag = T;
	B->need = prot ? (gcm ? 16u : (T > 4 ? T : 4u)) : 0u;
	B->maxlen = SGPU_CACHED_MAX(c0->mode);
	B->bshift = bshift;
	B->nb = nb;
	B->cap = cap;
	B->delta = prot ? (int32_t)T : -(int32_t)T;
	B->gcm = (uint32_t)gcm;
	k->devfold = !prot && !g_env.nodevfold;
	B->nofold = (uint32_t)!k->devfold;
	B->pos = d->pos;
	B->end = d->end;
	B->capv = d->cap;
	B->sess = d->sess;
	B->posw = d->pos;
	B->endw = d->end;
	B->err = d->err;
	B->es = (uint32_t *)w->es.d;
	B->hdr = (struct sgpu_hdr *)w->hd.d;
	B->desc = (uint64_t *)w->dsc.d;
	p = w->bp.d;
	B->ticket = (uint32_t *)p;
	B->obins = (uint32_t *)(p + 64);
	B->bcount = (uint32_t *)(p + 512);
	p += BP_HEAD;
#define BP_TAKE(ptr, bytes)                                                  \
	do {                                                                 \
		(ptr) = (void *)p;                                           \
		p += ((size_t)(bytes) + 255) & ~(size_t)255;                 \
	} while (0)
	BP_TAKE(B->tmp, (size_t)nb * cap * 16);
	BP_TAKE(B->sorted, (size_t)nb * cap * 4);
	BP_TAKE(B->afail, na * 4);
	BP_TAKE(B->sseg, nsess * 4);
	BP_TAKE(B->sout, nsess * sizeof(struct sgpu_sstate));
	BP_TAKE(B->order, n * 4);
#undef BP_TAKE
	B->sst = sgpu_sst_table();
	B->out = (struct sgpu_plan_out *)w->pl.d;
	B->fo = (struct sgpu_fold_out *)(w->pl.d + k->foff);
	B->pred = k->pred;
	B->gate = k->gate;
	B->nfail = (uint32_t *)w->vs.d;
	B->verdict = w->vs.d + 64 + n * 4;
	B->flist = !prot && !gcm && k->devfold ?
		   (uint32_t *)(w->vs.d + ((64 + n * 5 + 3) & ~(size_t)3)) : NULL;
	/* parse, checks, bucket slots: no session state needed, so it runs
	 * while the host walks the sessions */
	err = sgpu_bplan_scatter(d->arena, d->arena_size, B, stream);
	if (err) {
		w->bp_d = NULL;
		return err;
	}
	cm_h = (uint32_t *)w->cm.h;
	up_h = (struct sgpu_sstate *)w->ms.h;
	need_h = (uint8_t *)(up_h + nsess);
	up_d = (struct sgpu_sstate *)w->ms.d;
	need_d = (uint8_t *)(up_d + nsess);
	k->t[0] = times ? now_ms() : 0;
	if (mplan_gather_res(sessv, nsess, up_h, cm_h, need_h, &k->nup,
			     k->pend, k->done)) {
		/* the scatter only wrote scratch -- and the bucket counters,
		 * zeroed again before the workspace's next call */
		w->bp_d = NULL;
		err = sgpu_stream_sync(stream);
		return err ? err : -1;
	}
	k->t[1] = times ? now_ms() : 0;
	/* the slot map and the states the device lacks go up on the
	 * workspace's own stream (overlapping the kernels queued before on the
	 * call's stream); the call's stream waits for them before the plan */
	if (!w->upev)
		w->upev = sgpu_event_create();
	if (!w->upev) {
		w->bp_d = NULL;
		sgpu_stream_sync(stream);
		return ENOMEM;
	}
	srv_stop(w);
	err = sgpu_memcpy_h2d(w->cm.d, cm_h, nsess * 4, w->stream);
	if (!err && k->nup)
		err = sgpu_memcpy_h2d(up_d, up_h,
				      nsess * (sizeof(struct sgpu_sstate) + 1),
				      w->stream);
	if (!err)
		err = sgpu_event_record(w->upev, w->stream);
	if (!err)
		err = sgpu_stream_wait(stream, w->upev);
	if (err) {
		/* no copy may still read the host buffers */
		sgpu_stream_sync(w->stream);
		w->bp_d = NULL;
		return err;
	}
	B->cm = (const uint32_t *)w->cm.d;
	B->upneed = k->nup ? need_d : NULL;
	B->up = up_d;
	err = sgpu_bplan_plan(B, stream);
	if (!err) {
		/* the crypto launches behind the plan's guards (the class
		 * guards skip[] and the fail word), in its order */
		struct sgpu_compact C = {
			d->pos, B->es, B->hdr, B->desc, d->sess,
			(const uint32_t *)w->cm.d, B->order, 0, (uint32_t)n,
			(uint8_t *)B->verdict, (uint32_t *)(w->vs.d + 64),
			B->nfail, 0, 0, NULL, 0, (uint32_t *)B->flist,
			&B->out->fail};
		err = run_classes(d->arena, d->arena_size, C, c0,
				  B->out, prot, stream);
	}
	/* plan out and fold out back in one piece: written by the finish
	 * launch itself (srtp_gpu_tune nopost: one copy behind it) */
	B->outbytes = (uint32_t)(k->foff + sizeof(struct sgpu_fold_out));
	B->outh = g_env.nopost ? NULL : (uint32_t *)w->pl.h;
	if (!err)
		err = sgpu_bplan_finish(B, stream);
	if (err) {
		w->bp_d = NULL;
		return err;
	}
	if (g_env.nopost)
		err = sgpu_memcpy_d2h(w->pl.h, w->pl.d, B->outbytes, stream);
	k->t[2] = times ? now_ms() : 0;
	return err;
}

int dev_mplanned_issue(struct dcall *k)
{
	{
		uint32_t bsh, nb, cap;
		if (!k->radix && !g_env.mpradix && !g_env.nobucket &&
		    !sgpu_bplan_geometry((uint32_t)k->d.n, (uint32_t)k->nsess,
					 &bsh, &nb, &cap)) {
			k->bucket = 1;
			return dev_bplanned_issue(k, bsh, nb, cap);
		}
		k->bucket = 0;
	}

	const int prot = k->op == OP_RTP_ENC;
	struct srtp **sessv = k->sessv;
	const size_t nsess = k->nsess;
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &sessv[0]->rtp;
	const size_t n = d->n;
	const uint32_t T = c0->mode == SGPU_MODE_GCM ? 16u : c0->tag_len;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	struct sgpu_plan_out *po, *po_d;
	struct sgpu_fold_out *fo_d;
	struct sgpu_sstate *up_h, *up_d, *sin_d, *sout_d;
	struct sgpu_mplan_in in;
	struct sgpu_hdr *hd_d;
	uint64_t *desc_d;
	uint32_t *es_d, *save_d, *nfail_d, *cm_h, *order_d, bits = 1;
	uint8_t *vd_d, *need_h, *need_d;
	size_t scr;
	void *stream = d->stream;
	const int times = g_env.times;
	int err;

	while (bits < 32 && ((size_t)1 << bits) < nsess)
		bits++;
	scr = sgpu_mplan_scratch((uint32_t)n, (uint32_t)nsess);
	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 12);
	if (!err)   /* verdict | save | nfail | forged list */
		err = pool_reserve(w, &w->vs, n * 9 + 72);
	if (!err)
		err = pool_reserve(w, &w->cm, nsess * 4);
	/* pl: plan out | fold out | fold scratch (multi-session fold) */
	k->foff = (sizeof(struct sgpu_plan_out) + 63) & ~(size_t)63;
	if (!err)
		err = pool_reserve(w, &w->pl, k->foff + 64 +
				   sgpu_mfold_scratch((uint32_t)n));
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)
		err = pool_reserve(w, &w->ms,
				   nsess * (3 * sizeof(struct sgpu_sstate) + 1));
	if (!err)   /* scratch, the launch order (n words), then the parse
		     * prologue's window-check words (one per 256 packets) */
		err = pool_reserve(w, &w->mscr, scr + n * 4 + (n / 256 + 1) * 4);
	if (err)
		return err;
	hd_d = (struct sgpu_hdr *)w->hd.d;
	desc_d = (uint64_t *)w->dsc.d;
	nfail_d = (uint32_t *)w->vs.d;
	save_d = (uint32_t *)(w->vs.d + 64);
	vd_d = w->vs.d + 64 + n * 4;
	po = (struct sgpu_plan_out *)w->pl.h;
	po_d = (struct sgpu_plan_out *)w->pl.d;
	es_d = (uint32_t *)w->es.d;
	cm_h = (uint32_t *)w->cm.h;
	/* ms: st_in | st_out | uploads | need (device; host: the uploads) */
	sin_d = (struct sgpu_sstate *)w->ms.d;
	sout_d = sin_d + nsess;
	up_d = sout_d + nsess;
	need_d = (uint8_t *)(up_d + nsess);
	up_h = (struct sgpu_sstate *)w->ms.h + 2 * nsess;
	need_h = (uint8_t *)(up_h + nsess);
	order_d = (uint32_t *)(w->mscr.d + scr);
	/* parse + end copy (the kernels keep reading the input windows) +
	 * zeroed miss counter + the planner's window checks, one launch */
	memset(&in, 0, sizeof(in));
	in.wchk = (const uint32_t *)(w->mscr.d + scr + n * 4);
	{
		/* zeroes the plan out too (k_mp_iota ORs into it) and the
		 * counting grouping's per-session counters */
		const int radix = k->radix || g_env.mpradix || nsess > 65536;
		struct sgpu_prologue pro = {es_d, nfail_d, (uint32_t *)po_d, 1,
					    (uint32_t)(sizeof(*po) / 4), NULL, 0,
					    (uint32_t *)in.wchk, d->cap,
					    (uint32_t)prot, T,
					    prot ? (gcm ? 16u : (T > 4 ? T : 4u))
						 : 0u,
					    SGPU_CACHED_MAX(c0->mode),
					    radix ? NULL :
					    sgpu_mplan_counters(w->mscr.d,
								(uint32_t)n,
								(uint32_t)nsess),
					    radix ? 0u :
					    sgpu_mplan_counter_words(
						    (uint32_t)nsess)};
		in.radix = (uint32_t)radix;
		in.cnt_zeroed = !radix;
		err = sgpu_parse_prologue(d->arena, d->arena_size, d->pos,
					  d->end, hd_d, NULL, (uint32_t)n, 0,
					  &pro, stream);
		if (err)
			return err;
	}
	in.n = (uint32_t)n;
	in.nsess = (uint32_t)nsess;
	in.prot = (uint32_t)prot;
	in.tag = T;
	in.need = prot ? (gcm ? 16u : (T > 4 ? T : 4u)) : 0u;
	in.maxlen = SGPU_CACHED_MAX(c0->mode);
	in.key_bits = bits;
	in.out_zeroed = 1;
	/* the sort by session needs no session state: it runs while the
	 * host walks the sessions */
	err = sgpu_mplan_rtp_phase(1, &in, hd_d, d->pos, es_d, d->cap,
				   d->arena_size, d->sess, sin_d, sout_d,
				   desc_d, w->mscr.d, scr, po_d, order_d,
				   stream);
	if (!err && k->pred)
		err = sgpu_gate_pred(k->pred, &po_d->fail, stream);
	if (err)
		return err;
	/* one pass over the sessions: suite check, slot map, and the states
	 * the device does not hold yet (none once sessions are resident) */
	k->t[0] = times ? now_ms() : 0;
	if (mplan_gather_res(sessv, nsess, up_h, cm_h, need_h, &k->nup,
			     k->pend, k->done)) {
		/* the queued sort only wrote scratch */
		err = sgpu_stream_sync(stream);
		return err ? err : -1;
	}
	k->t[1] = times ? now_ms() : 0;
	/* the slot map and the states the device lacks (64K fresh sessions:
	 * 2 MB) go up on the workspace's own stream, so the copy overlaps
	 * the kernels queued before it on the call's stream (the sort above,
	 * or the previous call's crypto launch) instead of following them;
	 * the call's stream waits for it before k_sst_load.  Nothing queued
	 * before reads cm or the uploads, and the workspace is not reused
	 * before the call completes. */
	if (!w->upev)
		w->upev = sgpu_event_create();
	if (!w->upev)
		return ENOMEM;
	srv_stop(w);
	err = sgpu_memcpy_h2d(w->cm.d, cm_h, nsess * 4, w->stream);
	if (!err && k->nup)
		err = sgpu_memcpy_h2d(up_d, up_h,
				      nsess * (sizeof(struct sgpu_sstate) + 1),
				      w->stream);
	if (!err)
		err = sgpu_event_record(w->upev, w->stream);
	if (!err)
		err = sgpu_stream_wait(stream, w->upev);
	if (err) {
		/* no copy may still read the host buffers */
		sgpu_stream_sync(w->stream);
		return err;
	}
	if (!err)
		err = sgpu_sst_load((const uint32_t *)w->cm.d,
				    k->nup ? need_d : NULL, up_d,
				    (uint32_t)nsess, sin_d, stream);
	if (!err)
		err = sgpu_mplan_rtp_phase(2, &in, hd_d, d->pos, es_d, d->cap,
					   d->arena_size, d->sess, sin_d,
					   sout_d, desc_d, w->mscr.d, scr, po_d,
					   order_d, stream);
	if (!err) {
		/* unprotect (CTR): forged packets are listed and restored
		 * behind the kernel, for the device fold (dev_mplanned_finish) */
		uint32_t *flist_d = (uint32_t *)(w->vs.d +
						 ((64 + n * 5 + 3) & ~(size_t)3));
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, d->sess,
			(const uint32_t *)w->cm.d, order_d, 0, (uint32_t)n,
			vd_d, save_d, nfail_d, 0, 0, NULL, 0,
			!prot && !gcm && !g_env.nodevfold ? flist_d : NULL, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0,
				  po_d, prot, stream);
	}
	/* unprotect: the verdict fold queued behind the kernels (it does
	 * nothing without a miss), so a forged packet neither gates the next
	 * chained call nor waits for the host: srtp.c:310-321, 342-359,
	 * 426-427 per session segment (sgpu_mfold_rtp) */
	k->devfold = !prot && !g_env.nodevfold;
	fo_d = (struct sgpu_fold_out *)(w->pl.d + k->foff);
	if (!err && k->devfold)
		err = mfold(k, 1, nfail_d, sin_d, sout_d, scr);
	if (!err)
		err = sgpu_plan_finish(&po_d->fail, es_d, d->end, d->err,
				       (uint32_t)n,
				       prot ? (int32_t)T : -(int32_t)T, nfail_d,
				       k->gate, &po_d->nfail,
				       k->devfold ? &fo_d->fail : NULL, stream);
	if (!err && k->devfold)
		err = mfold(k, 2, nfail_d, sin_d, sout_d, scr);
	/* the new states replace the resident ones if the plan held and
	 * every tag verified or the fold held (else the host folds from the
	 * old ones) */
	if (!err)
		err = sgpu_sst_commit((const uint32_t *)w->cm.d, sout_d,
				      (uint32_t)nsess, &po_d->fail,
				      k->devfold ? &fo_d->fail : nfail_d, stream);
	/* plan out and fold out in one copy */
	if (!err)
		err = sgpu_memcpy_d2h(po, po_d, k->foff + sizeof(*fo_d), stream);
	k->t[2] = times ? now_ms() : 0;
	return err;
}

/* ... after its launches completed: 0 / errno, -1 not plannable or a
 * forged packet (undone; the host folds), -2 gated by the chained call
 * before (nothing modified) */
int dev_mplanned_finish(struct dcall *k)
{
	const int prot = k->op == OP_RTP_ENC;
	struct srtp **sessv = k->sessv;
	struct srtp_batch_dev *d = &k->d;
	struct ws *w = k->w;
	const struct comp *c0 = &sessv[0]->rtp;
	const size_t n = d->n;
	struct sgpu_plan_out *po = (struct sgpu_plan_out *)w->pl.h;
	struct sgpu_plan_out *po_d = (struct sgpu_plan_out *)w->pl.d;
	struct sgpu_hdr *hd_d = (struct sgpu_hdr *)w->hd.d;
	uint64_t *desc_d = (uint64_t *)w->dsc.d;
	uint32_t *nfail_d = (uint32_t *)w->vs.d;
	uint32_t *save_d = (uint32_t *)(w->vs.d + 64);
	uint8_t *vd_d = w->vs.d + 64 + n * 4;
	uint32_t *es_d = (uint32_t *)w->es.d;
	void *stream = d->stream;
	uint32_t nfail = po->nfail;
	int err;

	k->pfail = po->fail;
	if (g_env.times)
		fprintf(stderr, "re_srtp mplan n=%zu nsess=%zu up=%u: gather "
			"%.3f submit %.3f wait %.3f ms\n", n, k->nsess, k->nup,
			k->t[1] - k->t[0], k->t[2] - k->t[1],
			now_ms() - k->t[2]);
	if (po->fail) {
		if (po->fail & SPF_PRED)
			return -2;
		count(&g_cnt_rejects, 1);
		return -1;
	}
	count(&g_cnt_mplans, 1);
	if (!nfail)
		return 0;
	count(&g_cnt_misses, nfail);
	/* a forged packet: fold the verdicts on the device, per session
	 * (sgpu_mfold_rtp).  The kernels left each forged packet as
	 * srtp_decrypt does (HMAC: ciphertext restored, the ROC over the tag;
	 * GCM: decrypted in place); the fold checks the speculation under the
	 * true s_l and writes the EAUTH results and the touched sessions'
	 * states, which then replace the resident ones. */
	if (!prot && k->devfold) {
		/* folded on the device behind the kernels (dev_mplanned_issue);
		 * its verdict came back with the plan */
		const struct sgpu_fold_out *fo =
			(const struct sgpu_fold_out *)(w->pl.h + k->foff);
		if (!fo->fail) {
			count(&g_cnt_devfolds, 1);
			return 0;
		}
	}
	count(&g_cnt_folds, 1);
	/* undo on the device, fold on the host engine */
	{
		struct sgpu_compact C = {
			d->pos, es_d, hd_d, desc_d, d->sess,
			(const uint32_t *)w->cm.d, NULL, 0, (uint32_t)n, vd_d,
			save_d, nfail_d, 1, 0, NULL, 0, NULL, NULL};
		err = run_classes(d->arena, d->arena_size, C, c0,
				  po_d, prot, stream);
	}
	if (!err)
		err = sgpu_memcpy_d2d(d->end, es_d, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	return -1;      /* resident states untouched: the host folds */
}

/* synchronous: -1 not plannable (nothing modified), else 0 / errno */
int dev_mplanned_(int op, struct srtp **sessv, size_t nsess,
			 struct srtp_batch_dev *d, int radix, uint32_t *pfail)
{
	struct dcall k;
	int err;
	memset(&k, 0, sizeof(k));
	k.op = op;
	k.sessv = sessv;
	k.nsess = nsess;
	k.d = *d;
	k.radix = radix;
	k.w = ws_get();
	if (!k.w)
		return ENOMEM;
	err = dev_mplanned_issue(&k);
	if (!err)
		err = sgpu_stream_sync(d->stream);
	if (err)
		return err;
	err = dev_mplanned_finish(&k);
	*pfail = k.pfail;
	return err;
}

/* a session with more than SGPU_MP_SEGMAX packets (SPF_SEG): re-planned
 * with the radix-sort grouping */
int dev_mplanned(int op, struct srtp **sessv, size_t nsess,
			struct srtp_batch_dev *d)
{
	uint32_t pf = 0;
	int r = dev_mplanned_(op, sessv, nsess, d, g_env.mpradix, &pf);
	if (r == -1 && (pf & SPF_SEG) && !g_env.mpradix)
		r = dev_mplanned_(op, sessv, nsess, d, 1, &pf);
	return r;
}
