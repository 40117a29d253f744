/*
 * srtp_int.h -- what the host translation units of the library share
 * (srtp.c: sessions, the planning engine and the mbuf front-end;
 * batch_host.c: host-planned device batches; batch_dev.c: device-planned
 * batches; batch_async.c: entry points and asynchronous tickets;
 * percall.c: the per-packet calls' shared launches; rxfold.c: the
 * cross-rank replay fold).  Internal: nothing here is exported (exports.map).
 */
#ifndef RE_AMD_SRTP_INT_H
#define RE_AMD_SRTP_INT_H

#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "re_mem.h"
#include "re_mbuf.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"
#include "../srtpgpu.h"
#include "fault.h"
#include "pool.h"

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
	uint32_t epoch;         /* fast path: call that last logged it */
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
	/* hot fields first: one cache line with stream 0 covers what the
	 * batch paths read per session (count, device slot, suite) */
	unsigned nstreams;
	uint32_t slot;          /* device session table slot */
	int suite;              /* enum srtp_suite */
	struct srtp_stream streams[SRTP_MAX_STREAMS];
	struct comp rtp, rtcp;
	int dev;
	uint32_t mp_epoch;      /* multi-session plan: call that gathered it
				   (detects sessv entries aliasing one
				   context) */
	int dres;               /* where stream 0's RTP state lives: DRES_* */
	uint64_t pend_p;        /* async: last pending single-stream call on
				   it (issuing thread's sequence number) */
	uint64_t pend_m;        /* ... last pending multi-session call */
	const struct tk_owner *pend_own; /* the thread that issued them */
};

struct tk_owner {
	uint64_t done;          /* sequence number of the last completed call */
};

struct srtp_env {
	int noplan;             /* RE_SRTP_NOPLAN: no device planners */
	int general;            /* RE_SRTP_GENERAL: general engine only */
	int perclass;           /* RE_SRTP_PERCLASS: one launch per class */
	int nolean;             /* RE_SRTP_NOLEAN: general CTR kernels for
				   device-planned single-key batches */
	int nocombine;          /* srtp_gpu_tune nocombine: per-packet calls
				   of different threads do not share launches */
	int nomk;               /* srtp_gpu_tune nomk: multi-session plans on
				   the general per-lane-key kernel */
	int splan;              /* srtp_gpu_tune splan: single-session RTP
				   batches through the per-stream planner */
	int nobucket;           /* srtp_gpu_tune nobucket: multi-session plans
				   by the counting grouping (plan_multi.hip),
				   not the bucket planner (plan_buckets.hip) */
	int mpradix;            /* srtp_gpu_tune mpradix: multi-session plans
				   group by the radix sort (not counting) */
	int nodevfold;          /* RE_SRTP_NODEVFOLD: forged packets in a
				   device-planned batch fold on the host */
	int nosmall;            /* RE_SRTP_NOSMALL: the per-packet path's small
				   CTR launches take the general kernels
				   with copies (not sgpu_run_small) */
	long pcrunners;         /* srtp_gpu_tune pcrunners: per-packet runners
				   at once (default PC_RUNNERS, at most
				   PC_SLOTS) */
	long pchold;            /* srtp_gpu_tune pchold: us a new per-packet
				   runner holds its launch while other
				   runners are in flight (percall.c) */
	int syncspin;           /* srtp_gpu_tune syncspin: a synchronous
				   one-stream call waits by spinning on its
				   post launch's completion word instead of a
				   stream synchronisation (A/B) */
	long pclinger;          /* srtp_gpu_tune pclinger: us a small-kernel
				   launch stays on the GPU after its batch,
				   taking the workspace's next batches from a
				   mailbox (0: off, one launch per batch) */
	long pcspin;            /* srtp_gpu_tune pcspin: pause loops a waiting
				   per-packet caller spins before it sleeps
				   (default 1000) */
	int rxseq;              /* srtp_gpu_tune rxseq: srtp_rx_index* and
				   srtp_rx_fold walk sequentially (A/B) */
	int smallsync;          /* srtp_gpu_tune smallsync: wait for a small
				   launch by a stream synchronisation, not
				   its completion word */
	int lplan;              /* srtp_gpu_tune lplan: single-stream AES-CM
				   batches planned by the one-launch planner
				   (k_lp_plan) in front of the lean kernel,
				   not inside the crypto launch (k_ctr_fused,
				   the default: measured 498 vs 490 GiB/s on
				   one box, profiles/r06/lplan_ab.txt) */
	int nopost;             /* srtp_gpu_tune nopost: single-stream plan
				   outs come back by a blit copy (and the
				   asynchronous gate by its own launch), not
				   by one k_plan_post launch (A/B) */
	int noplanfuse;         /* srtp_gpu_tune noplanfuse: single-stream
				   batches take the separate device planner
				   (k_parse + k_plan_*), not the plan inside
				   the crypto launch (k_ctr_fused.h) */
	long fzepoch;           /* srtp_gpu_tune fzepoch: the next fused
				   launch's look-back epoch (test hook) */
	int nofuse;             /* srtp_gpu_tune nofuse: the operations of a
				   shared per-packet launch run as separate
				   launches (helper thread), not one */
	int trace;              /* RE_SRTP_TRACE: per-call phase times */
	int times;              /* RE_SRTP_TIMES: multi-session phases */
	size_t chunk;           /* RE_SRTP_CHUNK: host-scan chunk */
	size_t par_min;         /* RE_SRTP_PAR_MIN: sessions per pool part */
};
extern struct srtp_env g_env;

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

struct pool {
	uint8_t *h;             /* pinned host */
	uint8_t *d;             /* device */
	size_t cap;
};

struct ulog {
	struct srtp *s;                 /* session entry: old nstreams */
	struct srtp_stream *st;         /* stream entry: old state */
	unsigned nstreams;
	struct srtp_stream old;
};

struct ulogv {
	struct ulog *v;
	size_t n, cap;
};

struct ws {
	void *stream;
	struct pool ctl;        /* jobs | verdict | save */
	struct pool stage;      /* host path: packet bytes */
	struct pool hdr;        /* device path: pos/end, parsed headers */
	uint32_t *cls_idx;
	size_t cls_cap;
	/* compact fast path */
	void *pstream;          /* header parse + D2H stream */
	struct pool up;         /* pos | end | sess (original values) */
	struct pool hd;         /* parsed headers */
	struct pool dsc;        /* descriptors | class lists */
	struct pool vs;         /* verdict | save | nfail */
	struct pool cm;         /* session -> comp index */
	struct pool pl;         /* device planner: out | scratch */
	struct pool es;         /* device API: original ends */
	struct pool ms;         /* multi-session plan: states in | out */
	struct pool mscr;       /* multi-session plan: device scratch */
	void **ev;              /* per-chunk parse events */
	void *upev;             /* multi-session plan: its state uploads done
				   (on the side stream w->stream) */
	size_t nev;
	struct ulogv ulog[1];   /* stream-state undo log */
	/* single-stream batches planned inside the crypto launch
	 * (dev_fused): ticket | pad | plan out x2 | look-back words */
	struct pool fz;
	uint8_t *fz_d;          /* fz.d the state below belongs to */
	uint32_t fz_tbase;      /* the next launch's first ticket */
	uint32_t fz_epoch;      /* the next launch's look-back epoch */
	uint32_t fz_par;        /* which plan out the next launch uses */
	/* the small kernel's completion word (small_wait) */
	uint32_t *sm_cnt;       /* device */
	uint32_t *sm_flag;      /* pinned host */
	uint32_t sm_seq;
	/* the lingering small kernel (srtp_gpu_tune pclinger): its mailbox
	 * (coherent pinned host), broadcast block (device), running */
	uint32_t *sy_word;      /* pinned: synchronous calls' completion
				   word (srtp_gpu_tune syncspin) */
	uint32_t sy_seq;
	struct sgpu_srv_mb *srv_mb;
	struct sgpu_srv_bc *srv_bc;
	int srv_on;
	/* multi-session batches of the bucket planner (plan_buckets.hip,
	 * batch_dev.c dev_bplanned_issue): its counters are zero between
	 * calls once bp.d has been zeroed (bp_d) */
	struct pool bp;
	uint8_t *bp_d;
};

struct mbc {
	int op, prot, snapped, done;
	struct engine E;
	struct mbuf **mbv;
	int *errv;
	size_t n, round;
	uint8_t **outp;         /* where packet i's GPU output lives */
	uint8_t *keep;          /* per-packet copies across rounds */
	uint32_t *soff;         /* staging offsets */
	size_t *koff;
};


/* where a session's stream-0 RTP state lives (struct srtp dres; srtp.c) */
enum { DRES_HOST = 0, DRES_BOTH = 1, DRES_DEV = 2, DRES_LISTED = 3 };
/* round_launch: the jobs to run, or the undo jobs of dirty records */
enum { SEL_RUN = 0, SEL_UNDO = 1 };

/* diagnostics counters (srtp_gpu_counter, srtp.c) */
extern uint64_t g_cnt_pcbatch, g_cnt_pcpkts, g_cnt_pcfused, g_cnt_rxw_redo;
extern uint64_t g_cnt_misses, g_cnt_folds, g_cnt_rejects, g_cnt_devfolds;
extern uint64_t g_cnt_splans, g_cnt_fused, g_cnt_gated;
extern uint64_t g_cnt_dplans, g_cnt_mplans, g_cnt_rplans, g_cnt_lbtimeout;
extern uint64_t g_cnt_lplans;
extern int g_fresh_multi;       /* srtp.c: the last first batch of a session
				   showed several SSRCs (see there) */
extern __thread struct tk_owner *t_own; /* srtp.c: this thread's async
					   completion counter */
extern __thread int t_noplan;   /* batch_host.c: a rejected device plan's
				   fallback runs without device planners */
extern uint64_t g_cnt_small, g_ns_small_launch, g_ns_small_sync, g_ns_mbufs;
extern uint64_t g_ns_fused_prep, g_ns_fused_post;
extern uint64_t g_cnt_sync_calls, g_ns_sync_issue, g_ns_sync_wait,
		g_ns_sync_finish;

static inline uint64_t mono_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static inline void count(uint64_t *c, uint64_t v)
{
	__atomic_add_fetch(c, v, __ATOMIC_RELAXED);
}

/* srtp.c */
int gpu_ready(void);
void table_rdlock(void);
void table_unlock(void);
int sess_busy(const struct srtp *s);
int sess_host(struct srtp **sessv, size_t nsess);
int tk_pending(void);
void parse_rtp(struct pinfo *pi, const uint8_t *buf);
uint64_t get_index(uint32_t roc, uint16_t s_l, uint16_t seq);
int replay_check(struct replay *r, uint64_t ix);
extern __thread struct ws *t_ws_use;
struct ws *ws_new(void);
struct ws *ws_get(void);
int pool_reserve(struct ws *w, struct pool *p, size_t bytes);
int idx_reserve(struct ws *w, size_t n);
size_t small_fits(const struct engine *E);
void collect_rec(struct rec *r, uint8_t v, uint32_t save);
void srv_stop(struct ws *w);
int small_run(struct ws *w, uint8_t *arena, uint64_t asz,
	      const struct sgpu_job *jobs, uint32_t m, uint8_t *vh,
	      uint32_t *sv, int prot, uint64_t *t_launch);
int mbc_init(struct mbc *c, int op, struct srtp **sessv, size_t nsess,
	     const uint32_t *sidx, struct mbuf **mbv, int *errv, size_t n);
size_t mbc_plan(struct mbc *c);
int mbc_aside(struct mbc *c);
size_t mbc_offsets(struct mbc *c, size_t base);
void mbc_stage(struct mbc *c, uint8_t *stage);
void mbc_ran(struct mbc *c, uint8_t *stage);
int mbc_round(struct mbc *c, struct ws *w);
int mbc_finish(struct mbc *c);
void mbc_free(struct mbc *c, int err);
int run_mbufs_(int op, struct srtp **sessv, size_t nsess,
	       const uint32_t *sidx, struct mbuf **mbv, int *errv, size_t n);
int run_mbufs(int op, struct srtp *srtp, struct mbuf **mbv, int *errv,
	      size_t n);


/* one device-planned batch between its launches and its completion
 * (the synchronous calls and the asynchronous tickets share it) */
struct dcall {
	int op;
	struct srtp **sessv;
	size_t nsess;
	struct srtp_batch_dev d;
	struct ws *w;
	const uint32_t *pred;   /* gate word of the pending call before */
	uint32_t *gate;         /* this call's gate word (chained) or NULL */
	struct sgpu_plan_in in; /* single stream: the plan input */
	size_t foff;            /* ... fold area in w->pl */
	uint32_t nup;           /* many sessions: states uploaded */
	uint64_t pend, done;    /* async: sequence numbers (mpg) */
	double t[3];
	uint32_t pfail;         /* finish: the rejected plan's SPF_* bits */
	struct sgpu_splan_in sin; /* several streams: the plan input */
	int devfold;            /* fold queued on the device */
	uint32_t spin;          /* synchronous: the post's completion word
				   value to wait for (0: the stream) */
	int radix;              /* ... grouped by the radix sort */
	int fused;              /* single stream planned inside the crypto
				   launch (fz_issue / fz_finish), 2: by the
				   one-launch planner (lp_issue / lp_finish) */
	struct sgpu_fused fz;   /* ... its launch */
	int bucket;             /* many sessions: the bucket planner */
	struct sgpu_bplan bp;   /* ... its launches */
};

/* srtp.c */
struct tk_owner *tk_me(void);
void env_init(void);
int stream_get(struct srtp_stream **sp, struct srtp *s, uint32_t ssrc);
uint32_t buf_grow(uint32_t size, uint32_t need);
int cap_short(const struct pinfo *pi, const struct comp *c, int rtcp);
void snap_take(struct engine *E);
void snap_restore(struct engine *E);
size_t plan_all(struct engine *E);
int engine_init(struct engine *E, int op, size_t n,
		       struct srtp **sessv, size_t nsess, const uint32_t *sidx);
void engine_free(struct engine *E);
int rec_dirty(const struct rec *r);
int round_launch(struct ws *w, struct engine *E, int sel,
			uint8_t *arena_d, uint64_t asz, const uint32_t *joff,
			int prot, uint32_t *pm, void *stream);
int round_fetch(struct ws *w, uint32_t m, void *stream);
void round_collect(struct ws *w, struct engine *E, uint32_t m);

/* batch_host.c */
double now_ms(void);
struct replay plan_replay(const struct replay *r0,
				 const uint64_t *tail_ix, size_t n);
void plan_in(struct sgpu_plan_in *in, const struct srtp *s,
		    uint32_t n, int prot, uint32_t T, uint32_t need);
void plan_apply(struct srtp *s, const struct sgpu_plan_out *po,
		       int prot, size_t n, struct srtp_stream *old);
void plan_unapply(struct srtp *s, unsigned nstreams0,
			 const struct srtp_stream *old);
int mplan_gather_res(struct srtp **sessv, size_t nsess,
			    struct sgpu_sstate *st, uint32_t *cm,
			    uint8_t *need, uint32_t *nup, uint64_t pend,
			    uint64_t done);
int run_classes(uint8_t *arena, uint64_t asz, struct sgpu_compact C,
		       const struct comp *c0, struct sgpu_plan_out *po_d,
		       int prot, void *stream);
int run_batch(int op, struct srtp **sessv, size_t nsess,
		     struct srtp_batch *b);

/* batch_dev.c */
int dev_planned_issue(struct dcall *k);
int dev_planned_finish(struct dcall *k);
int dev_planned(int op, struct srtp *s, struct srtp_batch_dev *d,
		       uint32_t *pfail);
int dev_splanned_issue(struct dcall *k);
int dev_splanned_finish(struct dcall *k);
int dev_splanned(int op, struct srtp *s, struct srtp_batch_dev *d);
int dev_planned_rtcp(int op, struct srtp *s, struct srtp_batch_dev *d);
int dev_mplanned_issue(struct dcall *k);
int dev_mplanned_finish(struct dcall *k);
int dev_mplanned_(int op, struct srtp **sessv, size_t nsess,
			 struct srtp_batch_dev *d, int radix, uint32_t *pfail);
int dev_mplanned(int op, struct srtp **sessv, size_t nsess,
			struct srtp_batch_dev *d);

/* batch_async.c */
void tk_drain(void);

#endif
