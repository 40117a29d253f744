/*
 * rxfold.c -- the cross-rank replay fold of one SRTP stream unprotected
 * by several ranks (include/re_srtp_batch.h srtp_rx_index, _dev,
 * srtp_rx_fold): the ranks' per-packet records and the
 * reference receiver replayed over the whole stream.
 */
#include "srtp_int.h"

/* ---- cross-rank replay fold (include/re_srtp_batch.h) ----------------- */

/* the rank's own receiver over one packet (srtp.c:310-321 + the s_l
 * update of :426-427); ok: rtp_hdr_decode succeeded.  0 or EINVAL (another
 * SSRC) */
struct rx_walk {
	uint32_t ssrc, roc;
	uint16_t s_l;
	uint8_t set;
};

static int rx_step(struct rx_walk *x, int ok, uint32_t ssrc, uint16_t seq,
		   int32_t res, struct srtp_rx_rec *r)
{
	int diff;
	r->ix = 0;
	r->res = res;
	r->seq = 0;
	r->pad = 0;
	if (!ok) {
		r->stage = SRTP_RX_NOHDR;
		return 0;
	}
	if (ssrc != x->ssrc)
		return EINVAL;
	r->seq = seq;
	if (!x->set) {
		x->s_l = seq;
		x->set = 1;
	}
	diff = (int)seq - (int)x->s_l;
	if (diff > 32768) {
		r->stage = SRTP_RX_NOIX;
		return 0;
	}
	if (diff <= -32768) {
		x->roc++;
		x->s_l = 0;
	}
	r->stage = SRTP_RX_IX;
	r->ix = get_index(x->roc, x->s_l, seq);
	if (res == 0 && seq > x->s_l)
		x->s_l = seq;
	return 0;
}

static int rx_walk_packed(const struct srtp_stream_state *st0,
			  const uint32_t *pk, const int32_t *rh, size_t n,
			  struct srtp_rx_rec *rec);

/* srtp_rx_index: packets [lo, hi) parsed into the packed words of
 * k_rx_pack (seq | ok << 16 | other SSRC << 17) */
struct rxp {
	const struct srtp_stream_state *st0;
	const uint8_t *arena;
	const uint32_t *pos, *end;
	uint32_t *pk;
};

static void rxp_part(void *arg, size_t lo, size_t hi)
{
	const struct rxp *q = arg;
	size_t i;
	for (i = lo; i < hi; i++) {
		struct pinfo pi;
		memset(&pi, 0, sizeof(pi));
		pi.start = q->pos[i];
		pi.end = q->end[i];
		parse_rtp(&pi, q->arena);
		q->pk[i] = pi.hdr_len == UINT32_MAX ? 0u :
			   (uint32_t)pi.seq | 1u << 16 |
			   (pi.ssrc != q->st0->ssrc ? 1u << 17 : 0u);
	}
}

int srtp_rx_index(const struct srtp_stream_state *st0, const uint8_t *arena,
		  const uint32_t *pos, const uint32_t *end,
		  const int32_t *res, size_t n, struct srtp_rx_rec *rec)
{
	uint32_t *pk;
	int err;

	if (!st0 || (n && (!arena || !pos || !end || !res || !rec)))
		return EINVAL;
	if (!n)
		return 0;
	/* the headers parsed here (in parts: one cold line per packet of
	 * the arena), then the walk of srtp_rx_index_dev */
	pk = fi_malloc(n * sizeof(*pk));
	if (!pk)
		return ENOMEM;
	{
		struct rxp q = {st0, arena, pos, end, pk};
		par_for(n, 16384, rxp_part, &q);
	}
	err = rx_walk_packed(st0, pk, res, n, rec);
	free(pk);
	return err;
}

/*
 * The walk over packed words (k_rx_pack: seq | ok << 16 | other SSRC << 17
 * | res << 24, or res from rh) in parallel parts: part k > 0 guesses its
 * start state by a cold walk over the W packets before it (the receiver's
 * s_l is the newest accepted in-window seq, which a few hundred packets
 * re-establish) and walks with a relative ROC; then, in order, each
 * guess is checked against the previous part's true end state -- a part
 * whose guess was wrong is walked again from the true state, a right one
 * gets its ROC base added to its indices (get_index is linear in the ROC
 * while it stays below 2^31, which the caller checks).  Same records as
 * the sequential walk.
 */
enum { RXW_PARTS = 16, RXW_WARM = 512 };

struct rxw {
	const uint32_t *pk;
	const int32_t *rh;
	struct srtp_rx_rec *rec;
	size_t n;
	struct rx_walk st0;
	struct rx_walk guess[RXW_PARTS], end[RXW_PARTS];
	int bad[RXW_PARTS];
	uint32_t base[RXW_PARTS];
};

static size_t rxw_lo(const struct rxw *q, size_t k)
{
	return q->n * k / RXW_PARTS;
}

/* packets [lo, hi) from *x; 1 if one has another SSRC */
static int rxw_walk(const struct rxw *q, struct rx_walk *x, size_t lo,
		    size_t hi, int store)
{
	size_t i;
	for (i = lo; i < hi; i++) {
		const uint32_t v = q->pk[i];
		const int32_t r = q->rh ? q->rh[i] : (int32_t)(v >> 24);
		struct srtp_rx_rec tmp;
		if ((v >> 17) & 1)
			return 1;
		(void)rx_step(x, (v >> 16) & 1, x->ssrc, (uint16_t)v, r,
			      store ? &q->rec[i] : &tmp);
	}
	return 0;
}

static void rxw_part(void *arg, size_t k0, size_t k1)
{
	struct rxw *q = arg;
	size_t k;
	for (k = k0; k < k1; k++) {
		const size_t lo = rxw_lo(q, k), hi = rxw_lo(q, k + 1);
		struct rx_walk x = q->st0;
		if (k) {
			x.roc = 0;
			x.set = 0;
			x.s_l = 0;
			q->bad[k] = rxw_walk(q, &x, lo > RXW_WARM ? lo - RXW_WARM : 0,
					     lo, 0);
			x.roc = 0;      /* relative from here */
			q->guess[k] = x;
		}
		q->bad[k] |= rxw_walk(q, &x, lo, hi, 1);
		q->end[k] = x;
	}
}

static void rxw_fix(void *arg, size_t k0, size_t k1)
{
	struct rxw *q = arg;
	size_t k, i;
	for (k = k0; k < k1; k++) {
		const uint64_t add = (uint64_t)q->base[k] << 16;
		if (!add)
			continue;
		for (i = rxw_lo(q, k); i < rxw_lo(q, k + 1); i++)
			if (q->rec[i].stage == SRTP_RX_IX)
				q->rec[i].ix += add;
	}
}

static int rx_walk_packed(const struct srtp_stream_state *st0,
			  const uint32_t *pk, const int32_t *rh, size_t n,
			  struct srtp_rx_rec *rec)
{
	struct rxw *q;
	struct rx_walk x;
	size_t k;
	int fix = 0;

	x.ssrc = st0->ssrc;
	x.roc = st0->roc;
	x.s_l = st0->s_l;
	x.set = st0->s_l_set;
	if (n < 65536 || g_env.rxseq ||
	    (uint64_t)st0->roc + n + 2 >= 0x7fffffffull) {
		struct rxw one = {.pk = pk, .rh = rh, .rec = rec, .n = n};
		return rxw_walk(&one, &x, 0, n, 1) ? EINVAL : 0;
	}
	q = fi_calloc(1, sizeof(*q));
	if (!q)
		return ENOMEM;
	q->pk = pk;
	q->rh = rh;
	q->rec = rec;
	q->n = n;
	q->st0 = x;
	par_for(RXW_PARTS, 1, rxw_part, q);
	for (k = 0; k < RXW_PARTS; k++)
		if (q->bad[k]) {
			free(q);
			return EINVAL;
		}
	for (k = 1; k < RXW_PARTS; k++) {
		struct rx_walk t = q->end[k - 1];       /* the true start */
		if (t.set != q->guess[k].set ||
		    (t.set && t.s_l != q->guess[k].s_l)) {
			/* a wrong guess: this part again, exactly */
			count(&g_cnt_rxw_redo, 1);
			(void)rxw_walk(q, &t, rxw_lo(q, k), rxw_lo(q, k + 1), 1);
			q->end[k] = t;
			continue;
		}
		q->base[k] = t.roc;
		fix |= t.roc != 0;
		q->end[k].roc += t.roc;
	}
	if (fix)
		par_for(RXW_PARTS, 1, rxw_fix, q);
	free(q);
	return 0;
}

int srtp_rx_index_dev(const struct srtp_stream_state *st0,
		      const uint8_t *arena, size_t arena_size,
		      const uint32_t *pos, const uint32_t *end,
		      const int32_t *res, size_t n, struct srtp_rx_rec *rec,
		      void *stream)
{
	const uint32_t *pk;
	const int32_t *rh = NULL;
	struct ws *w;
	size_t i;
	int err, wide = 0;

	if (!st0 || (n && (!arena || !pos || !end || !res || !rec)) ||
	    n > UINT32_MAX)
		return EINVAL;
	if (!n)
		return 0;
	if (!gpu_ready())
		return ENOSYS;
	w = ws_get();
	if (!w)
		return ENOMEM;
	/* the headers parsed where the packets lie (k_parse: rtp_hdr_decode,
	 * rtp.c:88-137) and packed with the results, 4 B per packet down:
	 * the arena stays on the device */
	err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->es, n * 4);
	if (!err)
		err = sgpu_parse_headers(arena, arena_size, pos, end,
					 (struct sgpu_hdr *)w->hd.d, NULL,
					 (uint32_t)n, 0, stream);
	if (!err)
		err = sgpu_rx_pack((const struct sgpu_hdr *)w->hd.d, res,
				   st0->ssrc, (uint32_t *)w->es.d, (uint32_t)n,
				   stream);
	if (!err)
		err = sgpu_memcpy_d2h(w->es.h, w->es.d, n * 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
	if (err)
		return err;
	pk = (const uint32_t *)w->es.h;
	for (i = 0; i < n; i++)
		wide |= (pk[i] >> 23) & 1;
	if (wide) {
		/* a result outside 0..255 (not an errno): all of them */
		err = pool_reserve(w, &w->hd, n * 4);
		if (!err)
			err = sgpu_memcpy_d2h(w->hd.h, res, n * 4, stream);
		if (!err)
			err = sgpu_stream_sync(stream);
		if (err)
			return err;
		rh = (const int32_t *)w->hd.h;
	}
	return rx_walk_packed(st0, pk, rh, n, rec);
}

/*
 * The fold's walk (the reference receiver from the true state, srtp.c
 * :310-321 index step, :355-368 / :413-429 replay verdicts; the rank's
 * verdict void where the index or the replay verdict differs) over
 * records [lo, hi) from *x.  Returns the first void position (hi: none);
 * the state is then the one before it.  RXF_REL: the ROC is relative to
 * an unknown base -- instead of comparing indices, rec.ix - ix must be
 * one constant *D over the part (a different one is a void); *vmin is
 * the least ROC value get_index used.  RXF_WARM: state only (a guess of
 * a part's start), no verdicts, nothing stops it.
 */
enum { RXF_EXACT, RXF_REL, RXF_WARM, RXF_PARTS = 16, RXF_WARMN = 512,
       RXF_R0 = 2 };

struct rxf_state {
	struct replay rp;
	uint32_t roc;
	uint16_t s_l;
	uint8_t set;
};

static size_t rxf_walk(struct rxf_state *x, const struct srtp_rx_rec *rec,
		       int32_t *err, size_t lo, size_t hi, int mode,
		       uint64_t *D, int *hasD, int64_t *vmin)
{
	size_t i;
	for (i = lo; i < hi; i++) {
		const struct srtp_rx_rec *r = &rec[i];
		const uint32_t roc0 = x->roc;
		const uint16_t s_l0 = x->s_l;
		const uint8_t set0 = x->set;
		uint64_t ix;
		int diff;

		if (r->stage == SRTP_RX_NOHDR) {
			if (err)
				err[i] = r->res;
			continue;
		}
		if (!x->set) {
			x->s_l = r->seq;
			x->set = 1;
		}
		diff = (int)r->seq - (int)x->s_l;
		if (diff > 32768) {
			if (err)
				err[i] = ETIMEDOUT;
			continue;
		}
		if (r->stage != SRTP_RX_IX)
			goto void_verdict;
		if (diff <= -32768) {
			x->roc++;
			x->s_l = 0;
		}
		ix = get_index(x->roc, x->s_l, r->seq);
		if (mode == RXF_EXACT) {
			if (ix != r->ix)
				goto void_verdict;
		}
		else if (mode == RXF_REL) {
			const int64_t v = (int64_t)x->roc - 1;
			if (v < *vmin)
				*vmin = v;
			if (!*hasD) {
				*D = r->ix - ix;
				*hasD = 1;
			}
			else if (r->ix - ix != *D) {
				goto void_verdict;
			}
		}
		if (r->res != 0 && r->res != EALREADY) {
			if (err)
				err[i] = r->res;        /* tag verdict: ROC bump stays */
			continue;
		}
		/* a replay verdict the fold changes voids the packet's side
		 * effects as well: HMAC suites return EALREADY before the
		 * decrypt with pos at the payload (srtp.c:355-368), GCM leaves
		 * pos there (:413-422), success restores it (:429).  Check
		 * the window on a copy so the state stays the one before it */
		{
			struct replay tmp = x->rp;
			const int ok = replay_check(&tmp, ix);
			if (ok != (r->res == 0))
				goto void_verdict;
			x->rp = tmp;
			if (!ok) {
				if (err)
					err[i] = EALREADY;
				continue;
			}
		}
		if (err)
			err[i] = 0;
		if (r->seq > x->s_l)
			x->s_l = r->seq;
		continue;
	void_verdict:
		x->roc = roc0;
		x->s_l = s_l0;
		x->set = set0;
		if (mode != RXF_WARM)
			return i;
	}
	return hi;
}

/*
 * The fold in parallel parts, as rx_walk_packed: part k > 0 guesses its
 * start state by a cold walk over the RXF_WARMN records before it (the
 * 64-packet window and s_l are re-established by a few hundred packets)
 * and folds with a relative ROC (RXF_R0: its indices never go below 0);
 * then, in order, each part's guess, index offset and lowest ROC are
 * checked against the previous part's true end state -- a right guess
 * makes its verdicts, its void position and its end state (shifted by
 * the ROC base) exact, because the window compares indices only by
 * difference while none wraps; a wrong one is folded again exactly.
 */
struct rxf {
	const struct srtp_rx_rec *rec;
	int32_t *err;
	size_t n;
	struct rxf_state st0;
	struct rxf_state guess[RXF_PARTS], end[RXF_PARTS];
	size_t stop[RXF_PARTS];
	uint64_t D[RXF_PARTS];
	int hasD[RXF_PARTS];
	int64_t vmin[RXF_PARTS];
};

static size_t rxf_lo(const struct rxf *q, size_t k)
{
	return q->n * k / RXF_PARTS;
}

static void rxf_part(void *arg, size_t k0, size_t k1)
{
	struct rxf *q = arg;
	size_t k;
	for (k = k0; k < k1; k++) {
		const size_t lo = rxf_lo(q, k), hi = rxf_lo(q, k + 1);
		struct rxf_state x = q->st0;
		if (!k) {
			q->stop[k] = rxf_walk(&x, q->rec, q->err, lo, hi,
					      RXF_EXACT, NULL, NULL, NULL);
			q->end[k] = x;
			continue;
		}
		memset(&x, 0, sizeof(x));
		x.roc = RXF_R0;
		(void)rxf_walk(&x, q->rec, NULL,
			       lo > RXF_WARMN ? lo - RXF_WARMN : 0, lo, RXF_WARM,
			       NULL, NULL, NULL);
		/* the part's relative ROC starts at RXF_R0 again */
		x.rp.lix -= (uint64_t)(x.roc - RXF_R0) << 16;
		x.roc = RXF_R0;
		q->guess[k] = x;
		q->vmin[k] = INT64_MAX;
		q->stop[k] = rxf_walk(&x, q->rec, q->err, lo, hi, RXF_REL,
				      &q->D[k], &q->hasD[k], &q->vmin[k]);
		q->end[k] = x;
	}
}

static int rxf_parallel(struct rxf_state *st, const struct srtp_rx_rec *rec,
			size_t n, int32_t *err, size_t *ndone)
{
	struct rxf *q = fi_calloc(1, sizeof(*q));
	size_t k;
	if (!q)
		return ENOMEM;
	q->rec = rec;
	q->err = err;
	q->n = n;
	q->st0 = *st;
	par_for(RXF_PARTS, 1, rxf_part, q);
	for (k = 0; k < RXF_PARTS; k++) {
		const size_t lo = rxf_lo(q, k), hi = rxf_lo(q, k + 1);
		if (k) {
			const struct rxf_state t = q->end[k - 1];
			const struct rxf_state *g = &q->guess[k];
			const int64_t base = (int64_t)t.roc - RXF_R0;
			const uint64_t B = (uint64_t)base << 16;
			const int right = t.set == g->set &&
				(!t.set || t.s_l == g->s_l) &&
				t.rp.bitmap == g->rp.bitmap &&
				t.rp.lix == g->rp.lix + B &&
				g->rp.lix < (1ull << 62) &&
				t.rp.lix < (1ull << 62) &&
				(!q->hasD[k] || q->D[k] == B) &&
				q->vmin[k] + base >= 0;
			if (right) {
				q->end[k].roc += (uint32_t)base;
				q->end[k].rp.lix += B;
			}
			else {
				struct rxf_state x = t;
				count(&g_cnt_rxw_redo, 1);
				q->stop[k] = rxf_walk(&x, rec, err, lo, hi,
						      RXF_EXACT, NULL, NULL, NULL);
				q->end[k] = x;
			}
		}
		if (q->stop[k] < hi) {
			*st = q->end[k];
			*ndone = q->stop[k];
			free(q);
			return 0;
		}
	}
	*st = q->end[RXF_PARTS - 1];
	*ndone = n;
	free(q);
	return 0;
}

int srtp_rx_fold(struct srtp_stream_state *st, enum srtp_suite suite,
		 const struct srtp_rx_rec *rec, size_t n, int32_t *err,
		 size_t *ndone)
{
	struct rxf_state x;
	int e = 0;

	/* every suite checks the replay window after its tag (srtp.c:362-368
	 * HMAC, 414-421 GCM), so suite is only validated */
	if (!st || !ndone || (n && (!rec || !err)) ||
	    (unsigned)suite > SRTP_AES_256_GCM)
		return EINVAL;
	x.rp.bitmap = st->replay_rtp_bitmap;
	x.rp.lix = st->replay_rtp_lix;
	x.roc = st->roc;
	x.s_l = st->s_l;
	x.set = st->s_l_set;
	if (n >= 65536 && !g_env.rxseq &&
	    (uint64_t)st->roc + n + RXF_R0 + 2 < 0x7fffffffull &&
	    st->replay_rtp_lix < (1ull << 62))
		e = rxf_parallel(&x, rec, n, err, ndone);
	else
		*ndone = rxf_walk(&x, rec, err, 0, n, RXF_EXACT, NULL, NULL,
				  NULL);
	if (e)
		return e;
	st->replay_rtp_bitmap = x.rp.bitmap;
	st->replay_rtp_lix = x.rp.lix;
	st->roc = x.roc;
	st->s_l = x.s_l;
	st->s_l_set = x.set;
	return 0;
}

