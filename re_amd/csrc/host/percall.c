/*
 * percall.c -- the per-packet calls of the unchanged re_srtp.h API
 * (srtp_encrypt / srtp_decrypt / srtcp_encrypt / srtcp_decrypt, one mbuf
 * per call: src/srtp/srtp.c:183-432, srtcp.c:31-287 of the reference)
 * from many threads, sharing GPU launches.
 */
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include "srtp_int.h"

/*
 * Per-packet calls from many threads (the unchanged re_srtp.h API: every
 * libre caller protects one mbuf per call, src/srtp/srtp.c:183-432)
 * share GPU launches: a calling thread queues its packet; if no thread is
 * running a batch it becomes the runner, takes everything queued (the
 * packets of other threads that arrived meanwhile) and runs it as one
 * multi-session batch per operation.  No timer and no waiting at low
 * load: a lone caller runs its packet at once.  A struct srtp is used by
 * one thread at a time (the reference's contract), so the packets of one
 * batch belong to distinct sessions, and each thread's calls stay in its
 * own order.
 *
 * Completion is per request: the runner marks each request done and wakes
 * only its owner (a futex on the request's state word; owners spin
 * briefly first), then hands the runner role to the owner of the first
 * request queued meanwhile -- no broadcast, so 64 callers do not convoy
 * through one mutex on every batch.
 */

enum { PC_QUEUED = 0, PC_DONE = 1, PC_RUN = 2, PC_SLEEP = 3 };

struct pc_req {
	struct pc_req *next;
	int op;
	struct srtp *s;
	struct mbuf *mb;
	int err;
	int state;              /* PC_*, atomic: the owner waits on it */
	int slot;               /* PC_RUN: the runner slot handed over */
	struct pc_req *list;    /* ... and the queue it runs (from this one) */
};

static pthread_mutex_t pc_lock = PTHREAD_MUTEX_INITIALIZER;
static struct pc_req *pc_head, *pc_tail;
static int pc_running;
static int pc_nq;               /* requests queued (under pc_lock) */

/* the owner learns v; a futex wake only if it went to sleep (PC_SLEEP) */
static void pc_wake(int *state, int v)
{
	if (__atomic_exchange_n(state, v, __ATOMIC_ACQ_REL) == PC_SLEEP)
		(void)syscall(SYS_futex, state, FUTEX_WAKE_PRIVATE, 1, NULL,
			      NULL, 0);
}

static int pc_wait(int *state)
{
	long spin;
	int v;
	/* a short spin, then sleep: many callers spinning on fewer cores
	 * would take the CPU from the runner and its helper */
	const long nspin = g_env.pcspin ? g_env.pcspin : 1000;
	for (spin = 0; spin < nspin; spin++) {
		v = __atomic_load_n(state, __ATOMIC_ACQUIRE);
		if (v != PC_QUEUED)
			return v;
		__builtin_ia32_pause();
	}
	for (;;) {
		int q = PC_QUEUED;
		if (!__atomic_compare_exchange_n(state, &q, PC_SLEEP, 0,
						 __ATOMIC_ACQ_REL,
						 __ATOMIC_ACQUIRE))
			return q;       /* DONE or RUN arrived */
		while ((v = __atomic_load_n(state, __ATOMIC_ACQUIRE)) ==
		       PC_SLEEP)
			(void)syscall(SYS_futex, state, FUTEX_WAIT_PRIVATE,
				      PC_SLEEP, NULL, NULL, 0);
		return v;
	}
}

/* one operation's requests of a list, as multi-session batches */
static void pc_run_op(struct pc_req *list, int op)
{
	enum { MAXB = 1024 };
	struct srtp *sv[MAXB];
	struct mbuf *mv[MAXB];
	struct pc_req *rq[MAXB];
	int ev[MAXB];
	struct pc_req *r = list;

	while (r) {
		size_t n = 0, i;
		int err;
		for (; r && n < MAXB; r = r->next) {
			if (r->op != op)
				continue;
			rq[n] = r;
			sv[n] = r->s;
			mv[n++] = r->mb;
		}
		if (!n)
			break;
		count(&g_cnt_pcbatch, 1);
		count(&g_cnt_pcpkts, n);
		table_rdlock();
		err = sess_host(sv, n);
		if (!err) {
			uint32_t *idx = fi_malloc(n * sizeof(*idx));
			if (!idx)
				err = ENOMEM;
			for (i = 0; !err && i < n; i++)
				idx[i] = (uint32_t)i;
			if (!err)
				err = run_mbufs_(op, sv, n, idx, mv, ev, n);
			free(idx);
		}
		if (err && n > 1) {
			/* a batch-level error (one session busy with another
			 * thread's asynchronous calls, an allocation): the
			 * failed batch changed nothing, so each request runs on
			 * its own and gets the result its own call would */
			for (i = 0; i < n; i++) {
				uint32_t zero = 0;
				int e = sess_host(&sv[i], 1);
				if (!e)
					e = run_mbufs_(op, &sv[i], 1, &zero, &mv[i],
						       &ev[i], 1);
				rq[i]->err = e ? e : ev[i];
			}
			table_unlock();
			continue;
		}
		table_unlock();
		for (i = 0; i < n; i++)
			rq[i]->err = err ? err : ev[i];
	}
}

/*
 * Runner slots: up to pcrunners (default PC_RUNNERS) runners at once, each
 * with its slot's workspace (HIP stream, pinned pools) and helper thread,
 * so the next list is planned and launched while the previous one is on
 * the GPU.  Concurrent lists hold distinct sessions too (a session's one
 * owner thread has one call in flight).
 *
 * A list usually mixes operations (callers alternate srtp_encrypt and
 * srtp_decrypt).  Lists the small kernel takes run as one launch
 * (pc_run_fused); otherwise each operation is its own batch, and the
 * batches of two operations run at once -- one on the slot's persistent
 * helper thread (its own workspace and HIP stream), the rest on the
 * runner -- instead of one GPU round trip after the other.
 */
/* runners 1..4 at 64 threads: 230, 278, 306, 326 K pairs/s
 * (profiles/r04_percall_runners.txt) */
enum { PC_SLOTS = 4, PC_RUNNERS = 4 };
/* a new runner's hold (srtp_gpu_tune pchold, us) ends early at this many
 * requests queued */
enum { PC_HOLD_N = 32 };

static struct pc_slot {
	struct ws *ws;
	int hok;                /* helper thread running */
	int hstate;             /* 0 idle, 1 posted, 2 done (futex word) */
	struct pc_req *hlist;
	int hop;
} pc_slots[PC_SLOTS];
static unsigned pc_slot_used;   /* under pc_lock */

static void *pc_helper(void *arg)
{
	struct pc_slot *sl = arg;
	for (;;) {
		/* one read gives both the check and the futex's expected
		 * value: a post (store 1 + wake) between two reads would
		 * otherwise leave the helper asleep on a word already 1 */
		int v;
		while ((v = __atomic_load_n(&sl->hstate, __ATOMIC_ACQUIRE)) != 1)
			(void)syscall(SYS_futex, &sl->hstate, FUTEX_WAIT_PRIVATE,
				      v, NULL, NULL, 0);
		pc_run_op(sl->hlist, sl->hop);
		__atomic_store_n(&sl->hstate, 2, __ATOMIC_RELEASE);
		(void)syscall(SYS_futex, &sl->hstate, FUTEX_WAKE_PRIVATE, 1,
			      NULL, NULL, 0);
	}
	return NULL;
}

/* the slot's helper, started on first use (only its runner calls this) */
static int pc_helper_ok(struct pc_slot *sl)
{
	if (!sl->hok) {
		pthread_t t;
		pthread_attr_t a;
		pthread_attr_init(&a);
		pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
		sl->hok = pthread_create(&t, &a, pc_helper, sl) == 0 ? 1 : -1;
		pthread_attr_destroy(&a);
	}
	return sl->hok > 0;
}

/*
 * A list mixing operations whose packets all fit the small kernel (<=
 * SGPU_SMALL_MAX bytes): every operation plans its first round
 * on the host and all of them run as ONE launch of the fused kernel (the
 * protect or unprotect body per job, by SJ_PROTECT) -- one GPU round trip
 * for the whole list instead of one per operation on two streams.  Later
 * rounds (a verdict that changes a plan) run per operation as usual.
 * Returns -1, with nothing changed, when the list does not qualify or a
 * batch-level error stopped it before any result (the caller then runs
 * the operations its usual way); else 0 with every request's result set.
 */
static int pc_run_fused(struct pc_req *list, unsigned ops)
{
	struct mbc cv[4];
	struct srtp **sv = NULL;
	struct mbuf **mv = NULL;
	struct pc_req **rq = NULL;
	int *ev = NULL;
	uint32_t *idx = NULL, mst[5], m = 0;
	size_t base[5], need[4], tot = 0, bytes = 0, i, k;
	int nc = 0, opk[4], err = 0, inited = 0, redo = 0;
	const uint64_t t0 = mono_ns();
	uint64_t t1 = t0;
	struct pc_req *r;
	struct sgpu_job *jh;
	uint8_t *vh;
	struct ws *w;

	if (g_env.nosmall || g_env.nofuse)
		return -1;
	/* per operation, in list order */
	base[0] = 0;
	for (k = 0; k < 4; k++) {
		size_t n = 0;
		if (!((ops >> k) & 1))
			continue;
		for (r = list; r; r = r->next)
			n += r->op == (int)k;
		opk[nc] = (int)k;
		base[nc + 1] = base[nc] + n;
		nc++;
	}
	tot = base[nc];
	if (!tot || tot > SGPU_COOP_MAX)
		return -1;
	sv = fi_malloc(tot * sizeof(*sv));
	mv = fi_malloc(tot * sizeof(*mv));
	rq = fi_malloc(tot * sizeof(*rq));
	ev = fi_malloc(tot * sizeof(*ev));
	idx = fi_malloc(tot * sizeof(*idx));
	if (!sv || !mv || !rq || !ev || !idx) {
		err = -1;
		goto out_free;
	}
	for (k = 0; k < (size_t)nc; k++) {
		i = base[k];
		for (r = list; r; r = r->next)
			if (r->op == opk[k]) {
				rq[i] = r;
				sv[i] = r->s;
				mv[i] = r->mb;
				idx[i] = (uint32_t)(i - base[k]);
				i++;
			}
	}

	table_rdlock();
	w = ws_get();
	err = w ? 0 : ENOMEM;
	for (k = 0; !err && k < (size_t)nc; k++)
		err = sess_host(sv + base[k], base[k + 1] - base[k]);
	for (k = 0; !err && k < (size_t)nc; k++) {
		const size_t b = base[k], n = base[k + 1] - b;
		inited = (int)k + 1;
		err = mbc_init(&cv[k], opk[k], sv + b, n, idx + b, mv + b,
			       ev + b, n);
	}
	/* round 0: every operation planned; the small kernel takes all? */
	for (k = 0; !err && k < (size_t)nc; k++) {
		need[k] = mbc_plan(&cv[k]);
		if (small_fits(&cv[k].E) == (size_t)-1)
			err = -1;
	}
	for (k = 0; !err && k < (size_t)nc; k++)
		bytes = mbc_offsets(&cv[k], bytes);
	if (!err)
		err = pool_reserve(w, &w->stage, bytes);
	if (!err)
		err = pool_reserve(w, &w->ctl, tot * (sizeof(struct sgpu_job) + 5));
	if (!err)
		err = idx_reserve(w, tot);
	if (err)
		goto out;
	jh = (struct sgpu_job *)w->ctl.h;
	for (k = 0; k < (size_t)nc; k++) {
		struct mbc *c = &cv[k];
		mbc_stage(c, w->stage.h);
		mst[k] = m;
		for (i = 0; i < c->n; i++) {
			const struct rec *rc = &c->E.rec[i];
			if (!rc->need_run)
				continue;
			jh[m] = rc->job;
			jh[m].off = c->soff[i];
			w->cls_idx[m++] = (uint32_t)i;
		}
	}
	mst[nc] = m;
	vh = w->ctl.h + (size_t)m * sizeof(struct sgpu_job);
	t1 = mono_ns();
	count(&g_ns_fused_prep, t1 - t0);
	if (m) {
		uint64_t tl;
		err = small_run(w, w->stage.h, bytes, jh, m, vh,
				(uint32_t *)(vh + m), 2, &tl);
		count(&g_cnt_small, 1);
		count(&g_ns_small_launch, tl);
		count(&g_ns_small_sync, mono_ns() - t1 - tl);
		t1 = mono_ns();
		if (err)
			goto out;
	}
	count(&g_cnt_pcbatch, 1);
	count(&g_cnt_pcpkts, tot);
	count(&g_cnt_pcfused, 1);
	for (k = 0; k < (size_t)nc; k++) {
		struct mbc *c = &cv[k];
		uint32_t q;
		if (!need[k]) {
			c->done = 1;
			continue;
		}
		for (q = mst[k]; q < mst[k + 1]; q++)
			collect_rec(&c->E.rec[w->cls_idx[q]], vh[q],
				    ((const uint32_t *)(vh + m))[q]);
		mbc_ran(c, w->stage.h);
	}
	/* later rounds reuse the staging memory: every operation's outputs
	 * aside first if any operation needs one */
	for (k = 0; k < (size_t)nc; k++)
		if (!cv[k].done && mbc_plan(&cv[k]))
			break;
	if (k < (size_t)nc)
		for (k = 0; k < (size_t)nc; k++)
			if (mbc_aside(&cv[k]))
				redo = 1;
	for (k = 0; k < (size_t)nc; k++) {
		struct mbc *c = &cv[k];
		const size_t b = base[k], n = base[k + 1] - b;
		int e = redo ? ENOMEM : 0;
		while (!e && !c->done)
			e = mbc_round(c, w);
		if (!e)
			e = mbc_finish(c);
		mbc_free(c, e);
		if (!e) {
			for (i = b; i < b + n; i++)
				rq[i]->err = ev[i];
			continue;
		}
		/* this operation as it found it: each request on its own,
		 * with the result its own call would get */
		for (i = b; i < b + n; i++) {
			uint32_t zero = 0;
			int e1 = sess_host(&sv[i], 1);
			if (!e1)
				e1 = run_mbufs_(opk[k], &sv[i], 1, &zero, &mv[i],
						&ev[i], 1);
			rq[i]->err = e1 ? e1 : ev[i];
		}
	}
	inited = 0;
	count(&g_ns_fused_post, mono_ns() - t1);
 out:
	/* nothing ran, or the launch failed: every operation as it was */
	for (k = 0; k < (size_t)inited; k++)
		mbc_free(&cv[k], 1);
	table_unlock();
	count(&g_ns_mbufs, mono_ns() - t0);
 out_free:
	free(sv);
	free(mv);
	free(rq);
	free(ev);
	free(idx);
	return err ? -1 : 0;
}

static void pc_run(struct pc_req *list, struct pc_slot *sl)
{
	unsigned ops = 0;
	int op, first = -1;
	struct pc_req *r;

	for (r = list; r; r = r->next)
		ops |= 1u << r->op;
	if ((ops & (ops - 1)) && pc_run_fused(list, ops) == 0)
		return;
	if ((ops & (ops - 1)) && pc_helper_ok(sl)) {
		/* the lowest operation to the slot's helper */
		first = __builtin_ctz(ops);
		sl->hlist = list;
		sl->hop = first;
		__atomic_store_n(&sl->hstate, 1, __ATOMIC_RELEASE);
		(void)syscall(SYS_futex, &sl->hstate, FUTEX_WAKE_PRIVATE, 1,
			      NULL, NULL, 0);
	}
	for (op = 0; op < 4; op++)
		if ((ops >> op) & 1 && op != first)
			pc_run_op(list, op);
	if (first >= 0) {
		int v;
		while ((v = __atomic_load_n(&sl->hstate, __ATOMIC_ACQUIRE)) != 2)
			(void)syscall(SYS_futex, &sl->hstate, FUTEX_WAIT_PRIVATE,
				      v, NULL, NULL, 0);
		__atomic_store_n(&sl->hstate, 0, __ATOMIC_RELAXED);
	}
}

static int one(int op, struct srtp *srtp, struct mbuf *mb)
{
	struct pc_req req;
	struct pc_slot *sl;
	int e = 0, err, run, busy, slot = 0, nrun;

	if (!srtp || !mb)
		return EINVAL;
	if (sess_busy(srtp))
		return EBUSY;   /* another thread's asynchronous call on it */
	if (g_env.nocombine || tk_pending()) {
		err = run_mbufs(op, srtp, &mb, &e, 1);
		return err ? err : e;
	}
	memset(&req, 0, sizeof(req));
	req.op = op;
	req.s = srtp;
	req.mb = mb;
	nrun = g_env.pcrunners > 0 ? (int)g_env.pcrunners : PC_RUNNERS;
	if (nrun > PC_SLOTS)
		nrun = PC_SLOTS;
	pthread_mutex_lock(&pc_lock);
	if (pc_tail)
		pc_tail->next = &req;
	else
		pc_head = &req;
	pc_tail = &req;
	pc_nq++;
	run = pc_running < nrun;
	busy = pc_running > 0;
	if (run) {
		/* a free slot: run the queue now (taken here, in the same
		 * critical section, so no hand-off can take this request) */
		pc_running++;
		slot = __builtin_ctz(~pc_slot_used);
		pc_slot_used |= 1u << slot;
		req.list = pc_head;
		pc_head = pc_tail = NULL;
		pc_nq = 0;
	}
	pthread_mutex_unlock(&pc_lock);
	if (run && busy && g_env.pchold > 0) {
		/* other runners are in flight, so other callers are active:
		 * hold the new launch a few us (or until PC_HOLD_N more
		 * requests queued) and take what arrived -- a launch of 10
		 * packets costs about what one of 30 does (the small kernel runs
		 * one packet per workgroup) */
		const uint64_t until = mono_ns() + (uint64_t)g_env.pchold * 1000u;
		struct pc_req *last = req.list;
		while (mono_ns() < until &&
		       __atomic_load_n(&pc_nq, __ATOMIC_RELAXED) < PC_HOLD_N)
			__builtin_ia32_pause();
		while (last->next)
			last = last->next;
		pthread_mutex_lock(&pc_lock);
		last->next = pc_head;
		pc_head = pc_tail = NULL;
		pc_nq = 0;
		pthread_mutex_unlock(&pc_lock);
	}
	if (!run && pc_wait(&req.state) == PC_DONE)
		return req.err;
	/* the runner (PC_RUN: slot and queue handed over): its queue on the
	 * slot's workspace, then the slot and the queue gathered meanwhile to
	 * that queue's first request (or the slot is freed) */
	slot = req.slot = run ? slot : req.slot;
	sl = &pc_slots[slot];
	if (!sl->ws)
		sl->ws = ws_new();      /* the slot is this thread's alone */
	{
		struct pc_req *list = req.list, *r, *nx, *next_runner;
		t_ws_use = sl->ws;      /* NULL: this thread's own */
		pc_run(list, sl);
		t_ws_use = NULL;
		/* the next batch first: hand the runner role on, then
		 * complete this one's callers */
		pthread_mutex_lock(&pc_lock);
		next_runner = pc_head;
		if (next_runner) {
			next_runner->slot = slot;
			next_runner->list = pc_head;
			pc_head = pc_tail = NULL;
			pc_nq = 0;
		}
		else {
			pc_running--;
			pc_slot_used &= ~(1u << slot);
		}
		pthread_mutex_unlock(&pc_lock);
		if (next_runner)
			pc_wake(&next_runner->state, PC_RUN);
		for (r = list; r; r = nx) {
			nx = r->next;   /* r may be gone once woken */
			if (r != &req)
				pc_wake(&r->state, PC_DONE);
		}
	}
	return req.err;
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

