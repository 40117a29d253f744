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
 *
 * This file: sessions and streams, the per-packet planners, the planning
 * engine and its GPU rounds, and the mbuf front-end (srtp_encrypt /
 * srtp_decrypt and their batches of mbufs).  The device-resident batches
 * are in batch_host.c (host-planned), batch_dev.c (device-planned) and
 * batch_async.c (entry points, asynchronous tickets).
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


/*
 * Completion counter of one thread's asynchronous calls, readable by every
 * thread: a session with calls of thread A pending is busy for thread B
 * until A has completed them (srtp_batch_wait or any later entry point
 * of A), and B's calls on it return EBUSY meanwhile (re_srtp_batch.h).
 * Allocated on a thread's first asynchronous call and never freed
 * (sessions may name it after the thread has exited).
 */

__thread struct tk_owner *t_own;

struct tk_owner *tk_me(void)
{
	if (!t_own)
		t_own = fi_calloc(1, sizeof(*t_own));
	return t_own;
}

/* another thread's asynchronous call on s is still pending */
int sess_busy(const struct srtp *s)
{
	const struct tk_owner *o = s->pend_own;
	uint64_t p;
	if (!o || o == t_own)
		return 0;
	p = s->pend_p > s->pend_m ? s->pend_p : s->pend_m;
	return __atomic_load_n(&o->done, __ATOMIC_ACQUIRE) < p;
}

/*
 * Resident state (sgpu_sst_*): multi-session device batches keep each
 * session's RTP stream-0 state in HBM across calls.  DRES_BOTH: host and
 * device copies agree (a new session, no stream); DRES_DEV: the device
 * copy is newer (after a multi-session device batch); DRES_HOST: the host
 * copy is newer.  Host-side paths call sess_host() first.
 */

/* ------------------------------------------------------------------ */
/* tuning / diagnostics switches, read once (not per batch)             */

struct srtp_env g_env;
static pthread_once_t g_env_once = PTHREAD_ONCE_INIT;

static void env_read(void)
{
	const char *e;
	long v;
	g_env.noplan = getenv("RE_SRTP_NOPLAN") != NULL;
	g_env.general = getenv("RE_SRTP_GENERAL") != NULL;
	g_env.perclass = getenv("RE_SRTP_PERCLASS") != NULL;
	g_env.nolean = getenv("RE_SRTP_NOLEAN") != NULL;
	g_env.nodevfold = getenv("RE_SRTP_NODEVFOLD") != NULL;
	g_env.trace = getenv("RE_SRTP_TRACE") != NULL;
	g_env.nosmall = getenv("RE_SRTP_NOSMALL") != NULL;
	g_env.times = getenv("RE_SRTP_TIMES") != NULL;
	g_env.noplanfuse = getenv("RE_SRTP_NOPLANFUSE") != NULL;
	if (getenv("RE_SRTP_NOCOOP"))
		sgpu_set_coop(0);
	e = getenv("RE_SRTP_CHUNK");
	v = e ? atol(e) : 0;
	g_env.chunk = v >= 64 ? (size_t)v : (size_t)1 << 18;
	e = getenv("RE_SRTP_PAR_MIN");
	v = e ? atol(e) : 0;
	g_env.par_min = v > 0 ? (size_t)v : 4096;
}

void env_init(void)
{
	pthread_once(&g_env_once, env_read);
}

/* diagnostics counters (srtp_gpu_counter) */
uint64_t g_cnt_misses;   /* MAC/tag speculation misses */
uint64_t g_cnt_folds;    /* batches re-run to fold verdicts */
uint64_t g_cnt_rejects;  /* device plans rejected */
uint64_t g_cnt_devfolds; /* verdicts folded on the device */
uint64_t g_cnt_splans;   /* per-stream device plans accepted */
uint64_t g_cnt_fused;    /* batches planned inside the crypto launch
				   (dev_fused), accepted */
uint64_t g_cnt_dplans;   /* single-stream planner launches (k_plan_*,
				   GCM and noplanfuse), accepted */
uint64_t g_cnt_mplans;   /* multi-session device plans accepted */
uint64_t g_cnt_rplans;   /* SRTCP device plans (k_plan_rtcp) accepted */
uint64_t g_cnt_lplans;   /* single-stream batches planned by the
				   one-launch planner (k_lp_plan), accepted */
uint64_t g_cnt_lbtimeout; /* fused launches rejected by a look-back
				   wait past its bound (SPF_SLOW) */
/* a session's first batch (no stream yet) goes to the per-stream planner
 * while the last first batch planned showed several SSRCs: a one-stream
 * plan for it is rejected at completion and the batch planned again, a
 * second parse, plan and launch behind a host synchronisation.  Set by
 * that rejection, cleared by a first batch of one SSRC (the per-stream
 * plan is right for either, the one-stream plan only for one). */
int g_fresh_multi;
uint64_t g_cnt_pcbatch;  /* shared launches of per-packet calls */
uint64_t g_cnt_pcpkts;   /* ... and the packets they carried */
uint64_t g_cnt_rxw_redo; /* srtp_rx_index*: parts walked again */
uint64_t g_cnt_pcfused;  /* ... of which several operations in one
				   small launch (pc_run_fused) */
uint64_t g_cnt_gated;    /* asynchronous calls gated behind one the
				   host completed, re-run when waited for */
/* the per-packet path's small launches and where their time goes (ns):
 * the host work of run_mbufs_, the launch call, the synchronisation */
uint64_t g_cnt_small, g_ns_small_launch, g_ns_small_sync, g_ns_mbufs;
/* pc_run_fused: host time before the launch and after the sync (ns) */
uint64_t g_ns_fused_prep, g_ns_fused_post;
/* synchronous one-stream device calls (dev_fused): host time to issue,
 * waiting for the stream, completing (ns) */
uint64_t g_cnt_sync_calls, g_ns_sync_issue, g_ns_sync_wait, g_ns_sync_finish;

/* fault injection (srtp_gpu_tune "fail_grow", like the reference's
 * mem_threshold_set, src/mem/mem.c:45): the k-th workspace growth from
 * now fails with ENOMEM */
static long g_fail_grow;
/* fault.h: the k-th allocation from now fails (srtp_gpu_tune "fail_alloc") */
long re_amd_fail_alloc;
/* live mem_* blocks of the standalone allocator (mem.c; absent when libre
 * provides mem_*, LIBRE=1) */
extern size_t re_amd_mem_live(void) __attribute__((weak));
static uint32_t slots_live(void);


uint64_t srtp_gpu_counter(const char *name)
{
	if (!name)
		return 0;
	if (!strcmp(name, "misses"))
		return __atomic_load_n(&g_cnt_misses, __ATOMIC_RELAXED);
	if (!strcmp(name, "folds"))
		return __atomic_load_n(&g_cnt_folds, __ATOMIC_RELAXED);
	if (!strcmp(name, "rejects"))
		return __atomic_load_n(&g_cnt_rejects, __ATOMIC_RELAXED);
	if (!strcmp(name, "devfolds"))
		return __atomic_load_n(&g_cnt_devfolds, __ATOMIC_RELAXED);
	if (!strcmp(name, "splans"))
		return __atomic_load_n(&g_cnt_splans, __ATOMIC_RELAXED);
	if (!strcmp(name, "fused"))
		return __atomic_load_n(&g_cnt_fused, __ATOMIC_RELAXED);
	if (!strcmp(name, "lplans"))
		return __atomic_load_n(&g_cnt_lplans, __ATOMIC_RELAXED);
	if (!strcmp(name, "dplans"))
		return __atomic_load_n(&g_cnt_dplans, __ATOMIC_RELAXED);
	if (!strcmp(name, "mplans"))
		return __atomic_load_n(&g_cnt_mplans, __ATOMIC_RELAXED);
	if (!strcmp(name, "rplans"))
		return __atomic_load_n(&g_cnt_rplans, __ATOMIC_RELAXED);
	if (!strcmp(name, "lbtimeouts"))
		return __atomic_load_n(&g_cnt_lbtimeout, __ATOMIC_RELAXED);
	if (!strcmp(name, "pcbatches"))
		return __atomic_load_n(&g_cnt_pcbatch, __ATOMIC_RELAXED);
	if (!strcmp(name, "pcpackets"))
		return __atomic_load_n(&g_cnt_pcpkts, __ATOMIC_RELAXED);
	if (!strcmp(name, "rxw_redos"))
		return __atomic_load_n(&g_cnt_rxw_redo, __ATOMIC_RELAXED);
	if (!strcmp(name, "pcfused"))
		return __atomic_load_n(&g_cnt_pcfused, __ATOMIC_RELAXED);
	if (!strcmp(name, "gated"))
		return __atomic_load_n(&g_cnt_gated, __ATOMIC_RELAXED);
	if (!strcmp(name, "small_launches"))
		return __atomic_load_n(&g_cnt_small, __ATOMIC_RELAXED);
	if (!strcmp(name, "small_ns_launch"))
		return __atomic_load_n(&g_ns_small_launch, __ATOMIC_RELAXED);
	if (!strcmp(name, "small_ns_sync"))
		return __atomic_load_n(&g_ns_small_sync, __ATOMIC_RELAXED);
	if (!strcmp(name, "fused_ns_prep"))
		return __atomic_load_n(&g_ns_fused_prep, __ATOMIC_RELAXED);
	if (!strcmp(name, "fused_ns_post"))
		return __atomic_load_n(&g_ns_fused_post, __ATOMIC_RELAXED);
	if (!strcmp(name, "sync_calls"))
		return __atomic_load_n(&g_cnt_sync_calls, __ATOMIC_RELAXED);
	if (!strcmp(name, "sync_ns_issue"))
		return __atomic_load_n(&g_ns_sync_issue, __ATOMIC_RELAXED);
	if (!strcmp(name, "sync_ns_wait"))
		return __atomic_load_n(&g_ns_sync_wait, __ATOMIC_RELAXED);
	if (!strcmp(name, "sync_ns_finish"))
		return __atomic_load_n(&g_ns_sync_finish, __ATOMIC_RELAXED);
	if (!strcmp(name, "mbufs_ns"))
		return __atomic_load_n(&g_ns_mbufs, __ATOMIC_RELAXED);
	if (!strcmp(name, "freshmulti"))
		return (uint64_t)__atomic_load_n(&g_fresh_multi, __ATOMIC_RELAXED);
	if (!strcmp(name, "prof_voided"))
		return sgpu_prof_voided();
	if (!strcmp(name, "fail_alloc"))
		return (uint64_t)__atomic_load_n(&re_amd_fail_alloc,
						 __ATOMIC_RELAXED);
	if (!strcmp(name, "mem_live"))
		return re_amd_mem_live ? re_amd_mem_live() : 0;
	if (!strcmp(name, "slots_live"))
		return slots_live();
	return 0;
}

int srtp_gpu_tune(const char *name, long value)
{
	env_init();
	if (!name)
		return EINVAL;
	if (!strcmp(name, "noplan"))
		g_env.noplan = value > 0;
	else if (!strcmp(name, "general"))
		g_env.general = value > 0;
	else if (!strcmp(name, "perclass"))
		g_env.perclass = value > 0;
	else if (!strcmp(name, "nolean"))
		g_env.nolean = value > 0;
	else if (!strcmp(name, "nodevfold"))
		g_env.nodevfold = value > 0;
	else if (!strcmp(name, "splan"))
		g_env.splan = value > 0;
	else if (!strcmp(name, "nomk"))
		g_env.nomk = value > 0;
	else if (!strcmp(name, "nobucket"))
		g_env.nobucket = value > 0;
	else if (!strcmp(name, "mpradix"))
		g_env.mpradix = value > 0;
	else if (!strcmp(name, "nocoop"))
		sgpu_set_coop(value <= 0);
	else if (!strcmp(name, "nocombine"))
		g_env.nocombine = value > 0;
	else if (!strcmp(name, "nosmall"))
		g_env.nosmall = value > 0;
	else if (!strcmp(name, "lplan"))
		g_env.lplan = value > 0;
	else if (!strcmp(name, "nopost"))
		g_env.nopost = value > 0;
	else if (!strcmp(name, "bpexp"))
		sgpu_bplan_set_exp(value > 0 && value <= SGPU_BP_CAPMAX ?
				   (uint32_t)value : 0u);
	else if (!strcmp(name, "noplanfuse"))
		g_env.noplanfuse = value > 0;
	else if (!strcmp(name, "fzepoch"))
		/* test hook: the calling thread's next fused launch uses this
		 * look-back epoch (tests/test_gpu_fused.py: the wrap) */
		__atomic_store_n(&g_env.fzepoch, value > 0 ? value : 0,
				 __ATOMIC_RELAXED);
	else if (!strcmp(name, "nofuse"))
		g_env.nofuse = value > 0;
	else if (!strcmp(name, "smallsync"))
		g_env.smallsync = value > 0;
	else if (!strcmp(name, "rxseq"))
		g_env.rxseq = value > 0;
	else if (!strcmp(name, "freshmulti"))
		__atomic_store_n(&g_fresh_multi, value > 0, __ATOMIC_RELAXED);
	else if (!strcmp(name, "pcrunners"))
		g_env.pcrunners = value > 0 ? value : 0;
	else if (!strcmp(name, "pchold"))
		g_env.pchold = value > 0 ? value : 0;
	else if (!strcmp(name, "syncspin"))
		g_env.syncspin = value > 0;
	else if (!strcmp(name, "pclinger"))
		g_env.pclinger = value > 0 ? (value < 10000 ? value : 10000) : 0;
	else if (!strcmp(name, "pcspin"))
		g_env.pcspin = value > 0 ? value : 0;
	else if (!strcmp(name, "trace"))
		g_env.trace = value > 0;
	else if (!strcmp(name, "times"))
		g_env.times = value > 0;
	else if (!strcmp(name, "chunk"))
		g_env.chunk = value >= 64 ? (size_t)value : (size_t)1 << 18;
	else if (!strcmp(name, "par_min"))
		g_env.par_min = value > 0 ? (size_t)value : 4096;
	else if (!strcmp(name, "fail_grow"))
		__atomic_store_n(&g_fail_grow, value > 0 ? value : 0,
				 __ATOMIC_RELAXED);
	else if (!strcmp(name, "fail_alloc"))
		__atomic_store_n(&re_amd_fail_alloc, value > 0 ? value : 0,
				 __ATOMIC_RELAXED);
	else
		return EINVAL;
	return 0;
}

/* ------------------------------------------------------------------ */
/* device table slots                                                  */

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
/*
 * The device session table may move when it grows (sgpu_table_reserve).
 * Batch calls hold it read-locked for their whole duration (each call
 * synchronises its stream before returning, so no kernel of it still reads
 * the table afterwards); a growing allocation takes it write-locked.
 * Lock order: g_table_rw, then g_lock.
 */
static pthread_rwlock_t g_table_rw = PTHREAD_RWLOCK_INITIALIZER;
static uint32_t *g_free;
static uint32_t g_nfree, g_free_cap, g_next_slot;
static int g_gpu_state;         /* 0 unknown, 1 ok, -1 unavailable */

int gpu_ready(void)
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
	int err, held = 0;
	/* growth moves the table: only under the write lock (re-checked
	 * under g_lock, another allocation may have taken slots meanwhile) */
	for (;;) {
		pthread_mutex_lock(&g_lock);
		if (held || (uint64_t)g_next_slot + n <= sgpu_table_capacity())
			break;
		pthread_mutex_unlock(&g_lock);
		pthread_rwlock_wrlock(&g_table_rw);
		held = 1;
	}
	err = 0;
	/* the free list can hold every slot ever handed out, so slot_put
	 * never allocates (and never loses a slot) */
	if ((uint64_t)g_next_slot + n > g_free_cap) {
		uint64_t nc = g_free_cap ? g_free_cap : 256;
		uint32_t *nf;
		while (nc < (uint64_t)g_next_slot + n)
			nc *= 2;
		nf = nc <= UINT32_MAX ? fi_realloc(g_free, nc * sizeof(*nf))
				      : NULL;
		if (nf) {
			g_free = nf;
			g_free_cap = (uint32_t)nc;
		}
		else
			err = ENOMEM;
	}
	if (!err) {
		const uint32_t next0 = g_next_slot, nfree0 = g_nfree;
		for (i = 0; i < n; i++)
			slots[i] = g_nfree ? g_free[--g_nfree]
					   : g_next_slot++;
		err = sgpu_table_reserve(g_next_slot);
		if (err) {
			g_next_slot = next0;    /* nothing handed out */
			g_nfree = nfree0;
		}
	}
	pthread_mutex_unlock(&g_lock);
	if (held)
		pthread_rwlock_unlock(&g_table_rw);
	return err;
}

void table_rdlock(void)
{
	env_init();
	pthread_rwlock_rdlock(&g_table_rw);
}

void table_unlock(void)
{
	pthread_rwlock_unlock(&g_table_rw);
}

/* device table slots held by live contexts (leak checks) */
static uint32_t slots_live(void)
{
	uint32_t n;
	pthread_mutex_lock(&g_lock);
	n = g_next_slot - g_nfree;
	pthread_mutex_unlock(&g_lock);
	return n;
}

static void slot_put(uint32_t s)
{
	pthread_mutex_lock(&g_lock);
	if (g_nfree < g_free_cap)       /* always: slots_get sized it */
		g_free[g_nfree++] = s;
	pthread_mutex_unlock(&g_lock);
}

/* ------------------------------------------------------------------ */
/* srtp_alloc (srtp.c:88-180)                                          */

int tk_pending(void);

static void destructor(void *arg)
{
	struct srtp *srtp = arg;
	tk_drain();     /* a pending call of this thread may still use it */
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
	/* this thread's pending calls hold the table (growth waits for
	 * them) */
	tk_drain();

	req = fi_calloc(n ? n : 1, sizeof(*req));
	slots = fi_calloc(n ? n : 1, sizeof(*slots));
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
		struct srtp *s = fi_mem_zalloc(sizeof(*s), destructor);
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
		s->dres = DRES_BOTH;    /* sgpu_setup_sessions zeroed it */
		s->suite = (int)suite;
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
int stream_get(struct srtp_stream **sp, struct srtp *s, uint32_t ssrc)
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
int replay_check(struct replay *r, uint64_t ix)
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
uint64_t get_index(uint32_t roc, uint16_t s_l, uint16_t seq)
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



uint32_t buf_grow(uint32_t size, uint32_t need)
{
	/* mbuf_write_mem growth (src/mbuf/mbuf.c:244-252) */
	if (need > size) {
		uint32_t d = size ? size * 2 : 512;
		size = need > d ? need : d;
	}
	return size;
}

/* RTP header parse over host bytes (rtp.c:88-137) */
void parse_rtp(struct pinfo *pi, const uint8_t *buf)
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
int cap_short(const struct pinfo *pi, const struct comp *c, int rtcp)
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
		size = buf_grow(size, end + 16);
		end += 16;
		r->ext_end = end;
	}
	if (c->has_hmac) {
		r->job.flags |= SJ_HMAC | SJ_TRAILER;
		r->job.a_len = end - start;
		r->job.trailer = st->roc;
		r->job.tag_off = end - start;
		size = buf_grow(size, end + 4);
		size = buf_grow(size, end + c->tag_len);
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
		size = buf_grow(size, end + 16);
		end += 16;
	}
	eword = ep << 31 | st->rtcp_index;
	r->job.flags |= SJ_STORE_TRAIL;
	r->job.t_off = end - start;
	r->job.trailer = eword;
	size = buf_grow(size, end + 4);
	end += 4;
	if (c->has_hmac) {
		r->job.flags |= SJ_HMAC | SJ_TRAILER;
		r->job.a_len = end - 4 - start;
		r->job.tag_off = end - start;
		size = buf_grow(size, end + c->tag_len);
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


void snap_take(struct engine *E)
{
	size_t i;
	for (i = 0; i < E->nuniq; i++)
		E->snap[i] = *E->uniq[i];
}

void snap_restore(struct engine *E)
{
	size_t i;
	for (i = 0; i < E->nuniq; i++)
		*E->uniq[i] = E->snap[i];
}

size_t plan_all(struct engine *E)
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

int engine_init(struct engine *E, int op, size_t n,
		       struct srtp **sessv, size_t nsess, const uint32_t *sidx)
{
	size_t i;
	memset(E, 0, sizeof(*E));
	E->op = op;
	E->n = n;
	E->sess = fi_malloc((n ? n : 1) * sizeof(*E->sess));
	E->pi = fi_calloc(n ? n : 1, sizeof(*E->pi));
	E->rec = fi_calloc(n ? n : 1, sizeof(*E->rec));
	E->uniq = fi_malloc((nsess ? nsess : 1) * sizeof(*E->uniq));
	E->snap = fi_malloc((nsess ? nsess : 1) * sizeof(*E->snap));
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
		uint8_t *used = fi_calloc(nsess ? nsess : 1, 1);
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

void engine_free(struct engine *E)
{
	free(E->sess);
	free(E->pi);
	free(E->rec);
	free(E->uniq);
	free(E->snap);
}

/* ---- GPU rounds ----------------------------------------------------- */







static __thread struct ws *t_ws;

struct ws *ws_new(void)
{
	struct ws *w = fi_calloc(1, sizeof(*w));
	if (!w)
		return NULL;
	w->stream = sgpu_stream_create();
	if (!w->stream) {
		free(w);
		return NULL;
	}
	return w;
}

/* a per-packet runner's slot workspace while it runs (pc_slot_ws) */
__thread struct ws *t_ws_use;

struct ws *ws_get(void)
{
	if (t_ws_use)
		return t_ws_use;
	if (!t_ws)
		t_ws = ws_new();
	return t_ws;
}

/*
 * Launch the small kernel and wait for it by its completion word: the
 * host spins on the pinned word the last workgroup stores (system scope,
 * after every workgroup's writes) instead of a stream synchronisation,
 * checking the stream for an error now and then.  Without the word (its
 * allocation failed) a plain synchronisation.
 */
/* after a failed small launch: the workgroup count (0 between launches)
 * may be left part-way, so it is zeroed again on the idle stream before the
 * workspace's next launch counts on it -- or, when the stream does not
 * synchronise cleanly (the fault case) or the zeroing fails, the pair is
 * dropped and the next small_run allocates and zeroes a fresh one */
static int small_reset(struct ws *w, int err)
{
	srv_stop(w);
	if (!w->sm_cnt)
		return err;
	if (!sgpu_stream_sync(w->stream) &&
	    !sgpu_memset(w->sm_cnt, 0, 4, w->stream))
		return err;
	sgpu_free(w->sm_cnt);
	sgpu_host_free(w->sm_flag);
	w->sm_cnt = w->sm_flag = NULL;
	return err;
}

/*
 * The lingering small kernel (srtp_gpu_tune pclinger; struct sgpu_srv_mb):
 * a batch is posted into the workspace's mailbox; the kernel on the GPU
 * since an earlier batch takes it, or -- when none is there, or it left
 * (gone) before taking it -- a new launch does.  Exactly one launch takes
 * each batch: a kernel that stores gone has completed everything it took
 * and takes nothing after, and a new launch runs behind it on the stream.
 */
enum { SRV_GRID = 64, SRV_LIFE_US = 20000 };

static int srv_launch(struct ws *w)
{
	int err;
	w->srv_mb->stop = 0;
	__atomic_store_n(&w->srv_mb->gone, 0, __ATOMIC_RELEASE);
	err = sgpu_memset(w->srv_bc, 0, sizeof(*w->srv_bc), w->stream);
	if (!err)
		err = sgpu_run_small_srv(w->srv_mb, w->srv_bc, SRV_GRID,
					 (uint32_t)g_env.pclinger, SRV_LIFE_US,
					 w->sm_cnt, w->sm_flag, w->stream);
	w->srv_on = !err;
	return err;
}

/* before other work is queued on the workspace's stream: the lingering
 * kernel (idle: the thread that owns the workspace waited for its last
 * batch) is asked to stop and waited for */
void srv_stop(struct ws *w)
{
	unsigned long k;
	if (!w->srv_on)
		return;
	__atomic_store_n(&w->srv_mb->stop, 1u, __ATOMIC_RELEASE);
	for (k = 1; !__atomic_load_n(&w->srv_mb->gone, __ATOMIC_ACQUIRE); k++) {
		if (k & 1023) {
			__builtin_ia32_pause();
			continue;
		}
		if (sgpu_stream_query(w->stream) != EAGAIN)
			break;  /* not running (a fault): nothing to wait for */
	}
	w->srv_on = 0;
}

/* the server's mailbox and broadcast block, once per workspace */
static int srv_ready(struct ws *w)
{
	if (w->srv_mb)
		return 1;
	w->srv_mb = sgpu_host_alloc_coherent(sizeof(*w->srv_mb));
	w->srv_bc = fi_sgpu_malloc(sizeof(*w->srv_bc));
	if (!w->srv_mb || !w->srv_bc) {
		sgpu_host_free(w->srv_mb);
		sgpu_free(w->srv_bc);
		w->srv_mb = NULL;
		w->srv_bc = NULL;
		return 0;
	}
	memset(w->srv_mb, 0, sizeof(*w->srv_mb));
	return 1;
}

int small_run(struct ws *w, uint8_t *arena, uint64_t asz,
		     const struct sgpu_job *jobs, uint32_t m, uint8_t *vh,
		     uint32_t *sv, int prot, uint64_t *t_launch)
{
	const uint64_t t0 = mono_ns();
	unsigned long k;
	uint32_t seq;
	int err, srv;

	if (!w->sm_flag && !g_env.smallsync) {
		w->sm_cnt = fi_sgpu_malloc(4);
		w->sm_flag = fi_sgpu_host_alloc(4);
		if (w->sm_cnt && w->sm_flag &&
		    !sgpu_memset(w->sm_cnt, 0, 4, w->stream)) {
			*w->sm_flag = 0;
		}
		else {
			sgpu_free(w->sm_cnt);
			sgpu_host_free(w->sm_flag);
			w->sm_cnt = w->sm_flag = NULL;
		}
	}
	seq = ++w->sm_seq ? w->sm_seq : ++w->sm_seq;   /* never 0 */
	srv = g_env.pclinger > 0 && w->sm_flag && !g_env.smallsync &&
	      srv_ready(w);
	if (srv) {
		struct sgpu_srv_mb *mb = w->srv_mb;
		mb->njobs = m;
		mb->mode = (uint32_t)prot;
		mb->arena = (uint64_t)(uintptr_t)arena;
		mb->asz = asz;
		mb->jobs = (uint64_t)(uintptr_t)jobs;
		mb->verdict = (uint64_t)(uintptr_t)vh;
		mb->save = (uint64_t)(uintptr_t)sv;
		mb->comps = (uint64_t)(uintptr_t)sgpu_table_ptr();
		__atomic_store_n(&mb->post, seq, __ATOMIC_RELEASE);
		err = w->srv_on ? 0 : srv_launch(w);
		*t_launch = mono_ns() - t0;
		if (err)
			return small_reset(w, err);
	}
	else {
		uint32_t *flag = g_env.smallsync ? NULL : w->sm_flag;
		srv_stop(w);
		err = sgpu_run_small(arena, asz, jobs, m, vh, sv, prot,
				     w->sm_cnt, flag, seq, w->stream);
		*t_launch = mono_ns() - t0;
		if (err)
			return small_reset(w, err);
		if (!flag)
			return sgpu_stream_sync(w->stream);
	}
	for (k = 1;; k++) {
		int q;
		if (__atomic_load_n(w->sm_flag, __ATOMIC_ACQUIRE) == seq)
			return 0;
		if (srv && __atomic_load_n(&w->srv_mb->gone, __ATOMIC_ACQUIRE)) {
			/* the lingering kernel left before it took this batch
			 * (it completes what it takes before it leaves) */
			if (__atomic_load_n(w->sm_flag, __ATOMIC_ACQUIRE) == seq)
				return 0;
			err = srv_launch(w);
			if (err)
				return small_reset(w, err);
			continue;
		}
		if (k & 1023) {
			__builtin_ia32_pause();
			continue;
		}
		q = sgpu_stream_query(w->stream);
		if (q == EAGAIN)
			continue;
		if (__atomic_load_n(w->sm_flag, __ATOMIC_ACQUIRE) == seq)
			return 0;
		if (srv && __atomic_load_n(&w->srv_mb->gone, __ATOMIC_ACQUIRE))
			continue;       /* left meanwhile: launched again above */
		/* done without its word: a fault */
		return small_reset(w, q ? q : EIO);
	}
}

int pool_reserve(struct ws *w, struct pool *p, size_t bytes)
{
	size_t c;
	if (bytes <= p->cap)
		return 0;
	if (__atomic_load_n(&g_fail_grow, __ATOMIC_RELAXED) > 0 &&
	    __atomic_sub_fetch(&g_fail_grow, 1, __ATOMIC_RELAXED) == 0)
		return ENOMEM;
	c = bytes + bytes / 2 + 4096;
	srv_stop(w);
	sgpu_stream_sync(w->stream);
	sgpu_host_free(p->h);
	sgpu_free(p->d);
	p->h = fi_sgpu_host_alloc(c);
	p->d = fi_sgpu_malloc(c);
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

int idx_reserve(struct ws *w, size_t n)
{
	if (n > w->cls_cap) {
		size_t c = n + n / 2 + 64;
		uint32_t *ix = fi_realloc(w->cls_idx, c * sizeof(*ix));
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


/*
 * Device arenas are modified in place: a packet whose previous run no
 * longer stands -- it must run again with a different job, or the folded
 * verdicts left it with no job at all (e.g. ETIMEDOUT once an earlier
 * packet proved forged) -- is restored to its input bytes first.
 */
int rec_dirty(const struct rec *r)
{
	return r->ran && (r->need_run || !r->has_job);
}

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
int round_launch(struct ws *w, struct engine *E, int sel,
			uint8_t *arena_d, uint64_t asz, const uint32_t *joff,
			int prot, uint32_t *pm, void *stream)
{
	uint32_t cnt[16] = {0}, start[17], k, m = 0;
	size_t i, need = 0;
	struct sgpu_job *jh, *jd;
	uint8_t *vd;
	int err;

	for (i = 0; i < E->n; i++) {
		const struct rec *r = &E->rec[i];
		struct sgpu_job u;
		if (sel == SEL_RUN ? r->need_run : (rec_dirty(r) && undo_job(r, &u)))
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
			if (!(rec_dirty(r) && undo_job(r, &u)))
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
			if (!(rec_dirty(r) && undo_job(r, &u)))
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
	err = sgpu_memcpy_h2d(jd, jh, m * sizeof(struct sgpu_job), stream);
	if (err)
		return err;
	for (k = 0; k < 16; k++) {
		uint32_t a = start[k], b = start[k + 1];
		if (a == b)
			continue;
		err = sgpu_run_class(arena_d, asz, jd + a, b - a, vd + a,
				     (uint32_t *)(vd + m) + a, (k >> 3) & 1,
				     (k >> 2) & 1 ? 14 : 10, (int)(k & 3),
				     sel == SEL_RUN ? prot : 0, stream);
		if (err)
			return err;
	}
	*pm = m;
	return 0;
}

/* D2H of verdicts + saved tag words for the m jobs just launched */
int round_fetch(struct ws *w, uint32_t m, void *stream)
{
	size_t off = (size_t)m * sizeof(struct sgpu_job);
	if (!m)
		return 0;
	return sgpu_memcpy_d2h(w->ctl.h + off, w->ctl.d + off, (size_t)m * 5,
			       stream);
}

void collect_rec(struct rec *r, uint8_t v, uint32_t save)
{
	r->ran = 1;
	r->ran_job = r->job;
	r->vd = v;
	if (r->job.flags & SJ_ROC_AT_TAG)
		r->save = save;
}

void round_collect(struct ws *w, struct engine *E, uint32_t m)
{
	const uint8_t *v = w->ctl.h + (size_t)m * sizeof(struct sgpu_job);
	const uint32_t *sv = (const uint32_t *)(v + m);
	uint32_t k;
	for (k = 0; k < m; k++)
		collect_rec(&E->rec[w->cls_idx[k]], v[k], sv[k]);
}

/* #jobs of a planned round if the small kernel can take all of them,
 * else (size_t)-1 */
size_t small_fits(const struct engine *E)
{
	size_t i, need = 0;
	for (i = 0; i < E->n; i++) {
		const struct rec *r = &E->rec[i];
		if (!r->need_run)
			continue;
		if ((r->job.flags & SJ_UNDO) ||
		    r->ext_end - E->pi[i].start > SGPU_SMALL_MAX ||
		    r->in_end - E->pi[i].start > SGPU_SMALL_MAX)
			return (size_t)-1;
		need++;
	}
	return need;
}

/*
 * The per-packet path's round (few packets, every suite): the
 * staged packets and the jobs stay in pinned host memory and one fused
 * kernel reads and writes them there (sgpu_run_small, small.hip) -- no
 * copies; the verdicts land where round_collect reads them.  0 with *pm
 * jobs, errno, or -1: not eligible (an undo job, a packet past
 * SGPU_SMALL_MAX, more than SGPU_COOP_MAX jobs) -- nothing launched.
 */
static int round_small(struct ws *w, struct engine *E, uint64_t asz,
		       const uint32_t *joff, int prot, uint32_t *pm,
		       void *stream)
{
	struct sgpu_job *jh;
	uint8_t *vh;
	size_t i, need = 0;
	uint32_t m = 0;
	int err;

	*pm = 0;
	if (g_env.nosmall)
		return -1;
	need = small_fits(E);
	if (need == (size_t)-1)
		return -1;
	if (!need)
		return 0;
	if (need > SGPU_COOP_MAX)
		return -1;
	err = pool_reserve(w, &w->ctl, need * (sizeof(struct sgpu_job) + 5));
	if (!err)
		err = idx_reserve(w, need);
	if (err)
		return err;
	jh = (struct sgpu_job *)w->ctl.h;
	for (i = 0; i < E->n; i++) {
		const struct rec *r = &E->rec[i];
		if (!r->need_run)
			continue;
		jh[m] = r->job;
		jh[m].off = joff[i];
		w->cls_idx[m] = (uint32_t)i;
		m++;
	}
	vh = w->ctl.h + (size_t)m * sizeof(struct sgpu_job);
	(void)stream;
	{
		uint64_t tl;
		const uint64_t t0 = mono_ns();
		err = small_run(w, w->stage.h, asz, jh, m, vh,
				(uint32_t *)(vh + m), prot, &tl);
		count(&g_cnt_small, 1);
		count(&g_ns_small_launch, tl);
		count(&g_ns_small_sync, mono_ns() - t0 - tl);
	}
	if (!err)
		*pm = m;
	return err;
}

/* ---- host-resident front-end (mbufs) -------------------------------- */

/*
 * Bring the host copy of every session's state up to date before a
 * host-side path reads or changes it: sessions whose device copy is newer
 * (DRES_DEV) are read back in one transfer; all end up DRES_HOST (the
 * path may change them).  Needs the table read lock.
 */
int sess_host(struct srtp **sessv, size_t nsess)
{
	struct srtp **lst = NULL;
	uint32_t *slots = NULL;
	struct sgpu_sstate *st = NULL;
	size_t k, m = 0;
	int err = 0;

	for (k = 0; k < nsess; k++) {
		if (sessv[k] && sess_busy(sessv[k]))
			return EBUSY;
		if (sessv[k] && sessv[k]->dres == DRES_DEV)
			m++;
	}
	if (m) {
		lst = fi_malloc(m * sizeof(*lst));
		slots = fi_malloc(m * sizeof(*slots));
		st = fi_malloc(m * sizeof(*st));
		if (!lst || !slots || !st) {
			err = ENOMEM;
			goto out;
		}
		m = 0;
		for (k = 0; k < nsess; k++) {
			struct srtp *s = sessv[k];
			if (!s || s->dres != DRES_DEV)
				continue;
			s->dres = DRES_LISTED;          /* aliases: once */
			lst[m] = s;
			slots[m++] = s->slot;
		}
		err = sgpu_sst_read(slots, (uint32_t)m, st);
		for (k = 0; k < m; k++) {
			struct srtp *s = lst[k];
			struct srtp_stream *x;
			if (err) {
				s->dres = DRES_DEV;
				continue;
			}
			if (st[k].flags & SST_EXISTS) {
				if (!s->nstreams) {
					memset(&s->streams[0], 0,
					       sizeof(s->streams[0]));
					s->nstreams = 1;
				}
				x = &s->streams[0];
				x->ssrc = st[k].ssrc;
				x->roc = st[k].roc;
				x->s_l = (uint16_t)st[k].s_l;
				x->s_l_set = (st[k].flags & SST_SL_SET) ? 1 : 0;
				x->replay_rtp.lix = st[k].lix;
				x->replay_rtp.bitmap = st[k].bitmap;
			}
			s->dres = DRES_HOST;
		}
	}
 out:
	if (!err)
		for (k = 0; k < nsess; k++)
			if (sessv[k])
				sessv[k]->dres = DRES_HOST;
	free(lst);
	free(slots);
	free(st);
	return err;
}

/*
 * One operation's packets through the GPU rounds: plan on the host (the
 * reference's sequential semantics), stage the packets that need a run,
 * run them, collect the verdicts; a verdict that changes a later packet's
 * plan (a forged packet, a replay) makes another round from the snapshot.
 * run_mbufs_core drives one operation; pc_run_fused drives the first round
 * of several operations as one launch.
 */

int mbc_init(struct mbc *c, int op, struct srtp **sessv, size_t nsess,
		    const uint32_t *sidx, struct mbuf **mbv, int *errv,
		    size_t n)
{
	size_t i;
	int err;

	memset(c, 0, sizeof(*c));
	c->op = op;
	c->prot = op == OP_RTP_ENC || op == OP_RTCP_ENC;
	c->mbv = mbv;
	c->errv = errv;
	c->n = n;
	if (!sessv || !mbv)
		return EINVAL;
	for (i = 0; i < n; i++)
		if (!mbv[i])
			return EINVAL;
	err = engine_init(&c->E, op, n, sessv, nsess, sidx);
	if (err)
		return err;
	c->outp = fi_calloc(n ? n : 1, sizeof(*c->outp));
	c->soff = fi_calloc(n ? n : 1, sizeof(*c->soff));
	c->koff = fi_calloc(n ? n : 1, sizeof(*c->koff));
	if (!c->outp || !c->soff || !c->koff)
		return ENOMEM;
	for (i = 0; i < n; i++) {
		struct mbuf *mb = mbv[i];
		struct pinfo *pi = &c->E.pi[i];
		pi->start = (uint32_t)mb->pos;
		pi->end = (uint32_t)mb->end;
		pi->size = (uint32_t)mb->size;
		if (op == OP_RTP_ENC || op == OP_RTP_DEC)
			parse_rtp(pi, mb->buf);
		else
			parse_rtcp(pi, mb->buf);
	}
	snap_take(&c->E);
	c->snapped = 1;
	return 0;
}

/* the plan of the next round from the snapshot: #packets to run */
size_t mbc_plan(struct mbc *c)
{
	snap_restore(&c->E);
	return plan_all(&c->E);
}

/* staging is about to be reused: move the outputs of earlier rounds aside
 * (from round 1 on; idempotent) */
int mbc_aside(struct mbc *c)
{
	const struct engine *E = &c->E;
	size_t i;

	if (c->round == 0)
		return 0;
	if (!c->keep) {
		size_t tot = 0;
		for (i = 0; i < c->n; i++)
			if (c->outp[i]) {
				c->koff[i] = tot;
				tot += E->rec[i].ext_end - E->pi[i].start;
			}
		c->keep = fi_malloc(tot ? tot : 1);
		if (!c->keep)
			return ENOMEM;
	}
	for (i = 0; i < c->n; i++)
		if (c->outp[i] && c->outp[i] != c->keep + c->koff[i]) {
			memcpy(c->keep + c->koff[i], c->outp[i],
			       E->rec[i].ext_end - E->pi[i].start);
			c->outp[i] = c->keep + c->koff[i];
		}
	return 0;
}

/* stage the packets that need a run at 16-B aligned offsets from base */
size_t mbc_offsets(struct mbc *c, size_t base)
{
	const struct engine *E = &c->E;
	size_t i, bytes = base;
	for (i = 0; i < c->n; i++) {
		const struct rec *r = &E->rec[i];
		if (!r->need_run)
			continue;
		c->soff[i] = (uint32_t)bytes;
		bytes += ((r->ext_end - E->pi[i].start) + 31u) & ~15u;
	}
	return bytes;
}

void mbc_stage(struct mbc *c, uint8_t *stage)
{
	struct engine *E = &c->E;
	size_t i;
	for (i = 0; i < c->n; i++) {
		struct rec *r = &E->rec[i];
		if (!r->need_run)
			continue;
		memcpy(stage + c->soff[i], c->mbv[i]->buf + E->pi[i].start,
		       r->in_end - E->pi[i].start);
		/* job offsets are relative to the packet start */
		r->job.off = E->pi[i].start;
	}
}

void mbc_ran(struct mbc *c, uint8_t *stage)
{
	size_t i;
	for (i = 0; i < c->n; i++)
		if (c->E.rec[i].need_run)
			c->outp[i] = stage + c->soff[i];
	c->round++;
}

/* one round of one operation; c->done once nothing is left to run */
int mbc_round(struct mbc *c, struct ws *w)
{
	struct engine *E = &c->E;
	size_t need, bytes;
	uint32_t m;
	int err, rs;

	need = mbc_plan(c);
	if (!need) {
		c->done = 1;
		return 0;
	}
	if (c->round > c->n + 2)
		return EIO;
	err = mbc_aside(c);
	if (err)
		return err;
	bytes = mbc_offsets(c, 0);
	err = pool_reserve(w, &w->stage, bytes);
	if (err)
		return err;
	mbc_stage(c, w->stage.h);
	/* few packets: the fused kernel over the pinned staging memory
	 * itself, launched and waited for */
	rs = round_small(w, E, bytes, c->soff, c->prot, &m, w->stream);
	if (rs > 0)
		return rs;
	if (rs == 0) {
		round_collect(w, E, m);
		mbc_ran(c, w->stage.h);
		return 0;
	}
	srv_stop(w);
	err = sgpu_memcpy_h2d(w->stage.d, w->stage.h, bytes, w->stream);
	if (!err)
		err = round_launch(w, E, SEL_RUN, w->stage.d, bytes, c->soff,
				   c->prot, &m, w->stream);
	if (!err)
		err = round_fetch(w, m, w->stream);
	if (!err)
		err = sgpu_memcpy_d2h(w->stage.h, w->stage.d, bytes, w->stream);
	if (!err)
		err = sgpu_stream_sync(w->stream);
	if (err)
		return err;
	round_collect(w, E, m);
	mbc_ran(c, w->stage.h);
	return 0;
}

/* the results into the caller's mbufs */
int mbc_finish(struct mbc *c)
{
	const struct engine *E = &c->E;
	size_t i;
	int err;
	/* mbuf size growth (same policy) first: a failed resize leaves
	 * every mbuf's window and bytes, and the stream states, as before */
	for (i = 0; i < c->n; i++) {
		if (E->rec[i].size_o > c->mbv[i]->size) {
			err = mbuf_resize(c->mbv[i], E->rec[i].size_o);
			if (err)
				return err;
		}
	}
	/* unpack: bytes, pos/end, errno */
	for (i = 0; i < c->n; i++) {
		const struct rec *r = &E->rec[i];
		struct mbuf *mb = c->mbv[i];
		const struct pinfo *pi = &E->pi[i];
		if (r->has_job && c->outp[i])
			memcpy(mb->buf + pi->start, c->outp[i],
			       r->ext_end - pi->start);
		mb->pos = r->pos_o;
		mb->end = r->end_o;
		if (c->errv)
			c->errv[i] = r->err;
	}
	return 0;
}

void mbc_free(struct mbc *c, int err)
{
	/* a failed call leaves the stream states as it found them */
	if (err && c->snapped)
		snap_restore(&c->E);
	free(c->outp);
	free(c->keep);
	free(c->soff);
	free(c->koff);
	engine_free(&c->E);
}

static int run_mbufs_core(int op, struct srtp **sessv, size_t nsess,
			  const uint32_t *sidx, struct mbuf **mbv, int *errv,
			  size_t n)
{
	struct mbc c;
	struct ws *w;
	int err = mbc_init(&c, op, sessv, nsess, sidx, mbv, errv, n);

	if (!err) {
		w = ws_get();
		if (!w)
			err = ENOMEM;
		while (!err && !c.done)
			err = mbc_round(&c, w);
		if (!err)
			err = mbc_finish(&c);
	}
	mbc_free(&c, err);
	return err;
}

int run_mbufs_(int op, struct srtp **sessv, size_t nsess,
		      const uint32_t *sidx, struct mbuf **mbv, int *errv,
		      size_t n)
{
	const uint64_t t0 = mono_ns();
	const int err = run_mbufs_core(op, sessv, nsess, sidx, mbv, errv, n);
	count(&g_ns_mbufs, mono_ns() - t0);
	return err;
}

int run_mbufs(int op, struct srtp *srtp, struct mbuf **mbv, int *errv,
		     size_t n)
{
	int err;
	if (!srtp)
		return EINVAL;
	tk_drain();
	table_rdlock();
	err = sess_host(&srtp, 1);
	if (!err)
		err = run_mbufs_(op, &srtp, 1, NULL, mbv, errv, n);
	table_unlock();
	return err;
}
