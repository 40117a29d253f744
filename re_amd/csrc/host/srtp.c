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

static __thread struct tk_owner *t_own;

static struct tk_owner *tk_me(void)
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
enum { DRES_HOST = 0, DRES_BOTH = 1, DRES_DEV = 2, DRES_LISTED = 3 };

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

static void env_init(void)
{
	pthread_once(&g_env_once, env_read);
}

/* diagnostics counters (srtp_gpu_counter) */
static uint64_t g_cnt_misses;   /* MAC/tag speculation misses */
static uint64_t g_cnt_folds;    /* batches re-run to fold verdicts */
static uint64_t g_cnt_rejects;  /* device plans rejected */
static uint64_t g_cnt_devfolds; /* verdicts folded on the device */
static uint64_t g_cnt_splans;   /* per-stream device plans accepted */
static uint64_t g_cnt_fused;    /* batches planned inside the crypto launch
				   (dev_fused), accepted */
/* a session's first batch (no stream yet) goes to the per-stream planner
 * while the last first batch planned showed several SSRCs: a one-stream
 * plan for it is rejected at completion and the batch planned again, a
 * second parse, plan and launch behind a host synchronisation.  Set by
 * that rejection, cleared by a first batch of one SSRC (the per-stream
 * plan is right for either, the one-stream plan only for one). */
static int g_fresh_multi;
uint64_t g_cnt_pcbatch;  /* shared launches of per-packet calls */
uint64_t g_cnt_pcpkts;   /* ... and the packets they carried */
uint64_t g_cnt_rxw_redo; /* srtp_rx_index*: parts walked again */
uint64_t g_cnt_pcfused;  /* ... of which several operations in one
				   small launch (pc_run_fused) */
static uint64_t g_cnt_gated;    /* asynchronous calls gated behind one the
				   host completed, re-run when waited for */
/* the per-packet path's small launches and where their time goes (ns):
 * the host work of run_mbufs_, the launch call, the synchronisation */
uint64_t g_cnt_small, g_ns_small_launch, g_ns_small_sync, g_ns_mbufs;
/* pc_run_fused: host time before the launch and after the sync (ns) */
uint64_t g_ns_fused_prep, g_ns_fused_post;

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
	else if (!strcmp(name, "mpradix"))
		g_env.mpradix = value > 0;
	else if (!strcmp(name, "nocoop"))
		sgpu_set_coop(value <= 0);
	else if (!strcmp(name, "nocombine"))
		g_env.nocombine = value > 0;
	else if (!strcmp(name, "nosmall"))
		g_env.nosmall = value > 0;
	else if (!strcmp(name, "noplanfuse"))
		g_env.noplanfuse = value > 0;
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

static void tk_drain(void);
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

static void engine_free(struct engine *E)
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
 * workspace's next launch counts on it */
static int small_reset(struct ws *w, int err)
{
	if (w->sm_cnt && !sgpu_stream_sync(w->stream))
		(void)sgpu_memset(w->sm_cnt, 0, 4, w->stream);
	return err;
}

int small_run(struct ws *w, uint8_t *arena, uint64_t asz,
		     const struct sgpu_job *jobs, uint32_t m, uint8_t *vh,
		     uint32_t *sv, int prot, uint64_t *t_launch)
{
	const uint64_t t0 = mono_ns();
	unsigned long k;
	uint32_t seq;
	int err;

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
	{
		uint32_t *flag = g_env.smallsync ? NULL : w->sm_flag;
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
		if (k & 1023) {
			__builtin_ia32_pause();
			continue;
		}
		q = sgpu_stream_query(w->stream);
		if (q == EAGAIN)
			continue;
		if (__atomic_load_n(w->sm_flag, __ATOMIC_ACQUIRE) == seq)
			return 0;
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

enum { SEL_RUN = 0, SEL_UNDO = 1 };

/*
 * Device arenas are modified in place: a packet whose previous run no
 * longer stands -- it must run again with a different job, or the folded
 * verdicts left it with no job at all (e.g. ETIMEDOUT once an earlier
 * packet proved forged) -- is restored to its input bytes first.
 */
static int dirty(const struct rec *r)
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
static int round_launch(struct ws *w, struct engine *E, int sel,
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
		if (sel == SEL_RUN ? r->need_run : (dirty(r) && undo_job(r, &u)))
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
			if (!(dirty(r) && undo_job(r, &u)))
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
			if (!(dirty(r) && undo_job(r, &u)))
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
static int round_fetch(struct ws *w, uint32_t m, void *stream)
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

static void round_collect(struct ws *w, struct engine *E, uint32_t m)
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

/* ---- device-resident front-end ---------------------------------------- */

static int run_batch_general(int op, struct srtp **sessv, size_t nsess,
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
	int err, snapped = 0;

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
	/* the caller's stream; NULL is the default (null) stream, which
	 * orders this call after the caller's prior default-stream work */
	stream = b->stream;

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
		err = sgpu_parse_headers(b->arena, b->arena_size,
					 (const uint32_t *)w->hdr.d,
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
	snapped = 1;
	for (round = 0;; round++) {
		size_t need;
		uint32_t m = 0, mu = 0;

		size_t ndirty = 0;

		snap_restore(&E);
		need = plan_all(&E);
		for (i = 0; i < n; i++)
			if (dirty(&E.rec[i]))
				ndirty++;
		if (!need && !ndirty)
			break;
		if (round > n + 2) {
			err = EIO;
			goto out;
		}
		if (ndirty) {
			/* restore tag words overwritten by SJ_ROC_AT_TAG and
			 * re-apply keystreams of packets that must re-run */
			size_t nr = 0;
			uint32_t *wo, *wv;
			for (i = 0; i < n; i++) {
				const struct rec *r = &E.rec[i];
				if (dirty(r) && (r->ran_job.flags & SJ_ROC_AT_TAG))
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
					if (dirty(r) &&
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
					   b->arena_size, NULL, 0, &mu, stream);
			if (!err)
				err = sgpu_stream_sync(stream);
			if (err)
				goto out;
			/* restored packets without a job are back to input */
			for (i = 0; i < n; i++)
				if (E.rec[i].ran && !E.rec[i].has_job)
					E.rec[i].ran = 0;
			if (!need)
				break;
		}
		err = round_launch(w, &E, SEL_RUN, b->arena, b->arena_size,
				   NULL, prot, &m, stream);
		if (!err)
			err = round_fetch(w, m, stream);
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
	if (err && snapped)
		snap_restore(&E);
	engine_free(&E);
	return err;
}

/* ---- device-resident fast path (RTP, compact descriptors) -------------- */
/*
 * The general engine above materialises a 48-byte job per packet and a
 * full planning record.  For srtp_encrypt_batch / srtp_decrypt_batch the
 * host's share is only the sequential state machine (stream lookup, ROC,
 * s_l, index, replay window -- srtp.c:183-285, 288-432), so this path runs
 * exactly that over the parsed headers and emits one 8-byte descriptor per
 * packet (srtpgpu.h SD_*); the kernel derives the job on the device.  The
 * batch is cut into chunks so the host scan of chunk k+1 overlaps the GPU
 * crypto of chunk k.
 *
 * Unprotect speculates that every MAC/tag verifies (verdict-dependent
 * outcomes: srtp.c:360-368, 404-421).  The kernels count misses; on a
 * miss the whole call is undone -- arena bytes restored on the device,
 * stream states from the undo log, pos/end from the staged copies -- and
 * re-run through the general engine, which folds the verdicts exactly.
 */

static uint32_t g_epoch;
static __thread int t_noplan;   /* fallback of a rejected device plan */

static int ulog_push(struct ulogv *L, struct srtp *s, struct srtp_stream *st)
{
	struct ulog *u;
	if (L->n == L->cap) {
		size_t nc = L->cap ? 2 * L->cap : 256;
		struct ulog *nu = fi_realloc(L->v, nc * sizeof(*nu));
		if (!nu)
			return ENOMEM;
		L->v = nu;
		L->cap = nc;
	}
	u = &L->v[L->n++];
	u->s = s;
	u->st = st;
	if (s)
		u->nstreams = s->nstreams;
	if (st)
		u->old = *st;
	return 0;
}

static void ulog_undo(struct ulogv *L)
{
	while (L->n) {
		struct ulog *u = &L->v[--L->n];
		if (u->st)
			*u->st = u->old;
		else
			u->s->nstreams = u->nstreams;
	}
}

/* stream_get (stream.c:29-84) with an undo log entry on first touch */
static int fs_stream(struct ulogv *w, struct srtp *s, uint32_t ssrc,
		     uint32_t epoch, int log, struct srtp_stream **sp)
{
	unsigned i;
	for (i = 0; i < s->nstreams; i++) {
		struct srtp_stream *st = &s->streams[i];
		if (st->ssrc != ssrc)
			continue;
		if (log && st->epoch != epoch) {
			if (ulog_push(w, NULL, st))
				return ENOMEM;
			st->epoch = epoch;
		}
		*sp = st;
		return 0;
	}
	if (s->nstreams >= SRTP_MAX_STREAMS)
		return ENOSR;
	if (log && ulog_push(w, s, NULL))
		return ENOMEM;
	memset(&s->streams[s->nstreams], 0, sizeof(s->streams[0]));
	s->streams[s->nstreams].ssrc = ssrc;
	s->streams[s->nstreams].epoch = epoch;
	*sp = &s->streams[s->nstreams++];
	return 0;
}

struct fscan {
	struct ulogv *log_v;            /* stream-state undo log */
	struct srtp **sessv;
	const uint32_t *sidx;
	const struct sgpu_hdr *hd;     /* pinned */
	uint64_t *desc;                /* pinned */
	uint32_t *pos, *end;           /* caller arrays: in -> out */
	const uint32_t *cap;
	int32_t *err;
	uint32_t epoch;
	int log;
	int mode;
	uint32_t tag_len;
	int nomem;
	/* current stream, its state held in `cur` (flushed on a switch) */
	struct srtp *ls;
	uint32_t lssrc;
	struct srtp_stream *lst;
	struct srtp_stream cur;
};

static inline void fs_flush(struct fscan *F)
{
	if (F->lst)
		*F->lst = F->cur;
}

/* the stream of (s, ssrc) as F->cur; NULL with *err on ENOSR/ENOMEM */
static inline struct srtp_stream *fs_get(struct fscan *F, struct srtp *s,
					 uint32_t ssrc, int *err)
{
	struct srtp_stream *st;
	if (s == F->ls && ssrc == F->lssrc && F->lst)
		return &F->cur;
	fs_flush(F);
	F->lst = NULL;
	F->ls = NULL;
	*err = fs_stream(F->log_v, s, ssrc, F->epoch, F->log, &st);
	if (*err) {
		if (*err == ENOMEM)
			F->nomem = 1;
		return NULL;
	}
	F->ls = s;
	F->lssrc = ssrc;
	F->lst = st;
	F->cur = *st;
	return &F->cur;
}

static inline void fs_none(struct fscan *F, size_t i, int err, uint32_t pos)
{
	F->desc[i] = 0;
	F->err[i] = err;
	F->pos[i] = pos;
}

#define PF_DIST 24

/* srtp_encrypt (srtp.c:183-285) over packets [a, b); per-class counts */
static void scan_enc(struct fscan *F, size_t a, size_t b, uint32_t cnt[4])
{
	const uint32_t grow_by = F->mode == SGPU_MODE_GCM ? 16u : F->tag_len;
	const uint32_t need = F->mode == SGPU_MODE_GCM ? 16u
			      : (F->tag_len > 4 ? F->tag_len : 4u);
	const struct sgpu_hdr *__restrict hd = F->hd;
	uint64_t *__restrict desc = F->desc;
	uint32_t *__restrict pos = F->pos, *__restrict endv = F->end;
	const uint32_t *__restrict cap = F->cap;
	int32_t *__restrict errv = F->err;
	const uint32_t *__restrict sidx = F->sidx;
	size_t i;
	for (i = a; i < b; i++) {
		/* many sessions: their states are scattered; prefetch the
		 * one PF_DIST packets ahead */
		if (sidx && i + PF_DIST < b)
			__builtin_prefetch(F->sessv[sidx[i + PF_DIST]], 1, 1);
		struct srtp *s = F->sessv[sidx ? sidx[i] : 0];
		const struct sgpu_hdr h = hd[i];
		const uint32_t start = pos[i], end = endv[i];
		struct srtp_stream *st;
		const uint16_t seq = h.seq;
		int err = 0;
		if (h.hdr_len == UINT32_MAX) {
			fs_none(F, i, EBADMSG, start + h.err_pos);
			continue;
		}
		st = fs_get(F, s, h.ssrc, &err);
		if (!st) {
			fs_none(F, i, err, start + h.hdr_len);
			continue;
		}
		if (!st->s_l_set) {
			st->s_l = seq;
			st->s_l_set = 1;
		}
		if ((uint64_t)end + need > cap[i]) {
			fs_none(F, i, ENOMEM, start + h.hdr_len);
			continue;
		}
		if ((int)seq - (int)st->s_l <= -32768) {
			st->roc++;
			st->s_l = 0;
		}
		desc[i] = sgpu_desc(65536ULL * st->roc + seq, SD_RUN | SD_CIPHER);
		if (seq > st->s_l)
			st->s_l = seq;
		errv[i] = 0;
		endv[i] = end + grow_by;
		cnt[(h.hdr_len >> 2) & 3]++;
	}
	fs_flush(F);
}

/* srtp_decrypt (srtp.c:288-432) over packets [a, b), speculating that
 * every MAC/tag verifies */
static void scan_dec(struct fscan *F, size_t a, size_t b, uint32_t cnt[4])
{
	const int hmac = F->mode == SGPU_MODE_CTR;
	const uint32_t T = hmac ? F->tag_len : 16u;
	const struct sgpu_hdr *__restrict hd = F->hd;
	uint64_t *__restrict desc = F->desc;
	uint32_t *__restrict pos = F->pos, *__restrict endv = F->end;
	int32_t *__restrict errv = F->err;
	const uint32_t *__restrict sidx = F->sidx;
	size_t i;
	for (i = a; i < b; i++) {
		/* many sessions: their states are scattered; prefetch the
		 * one PF_DIST packets ahead */
		if (sidx && i + PF_DIST < b)
			__builtin_prefetch(F->sessv[sidx[i + PF_DIST]], 1, 1);
		struct srtp *s = F->sessv[sidx ? sidx[i] : 0];
		const struct sgpu_hdr h = hd[i];
		const uint32_t start = pos[i], end = endv[i];
		struct srtp_stream *st;
		const uint16_t seq = h.seq;
		uint32_t pld, fl = SD_RUN;
		int32_t v;
		uint64_t ix;
		int diff, err = 0;
		if (h.hdr_len == UINT32_MAX) {
			fs_none(F, i, EBADMSG, start + h.err_pos);
			continue;
		}
		pld = start + h.hdr_len;
		st = fs_get(F, s, h.ssrc, &err);
		if (!st) {
			fs_none(F, i, err, pld);
			continue;
		}
		if (!st->s_l_set) {
			st->s_l = seq;
			st->s_l_set = 1;
		}
		diff = (int)seq - (int)st->s_l;
		if (diff > 32768) {
			fs_none(F, i, ETIMEDOUT, pld);
			continue;
		}
		if (diff <= -32768) {
			st->roc++;
			st->s_l = 0;
		}
		/* misc.c:22-41 */
		if (st->s_l < 32768)
			v = ((int)seq - (int)st->s_l > 32768) ?
				(int32_t)(st->roc - 1) : (int32_t)st->roc;
		else
			v = ((int)st->s_l - 32768 > seq) ?
				(int32_t)(st->roc + 1) : (int32_t)st->roc;
		ix = seq + (uint64_t)(int64_t)v * 65536ull;
		if ((uint32_t)v != st->roc)
			fl |= (uint32_t)v + 1u == st->roc ? SD_ROC_P1 : SD_ROC_M1;
		if (end - pld < T) {
			fs_none(F, i, EBADMSG, pld);
			continue;
		}
		endv[i] = end - T;
		/* replay (replay.c:32-62), checked after a verified MAC
		 * (srtp.c:367) or tag (srtp.c:421) -- speculated verified */
		if (!replay_check(&st->replay_rtp, ix)) {
			desc[i] = sgpu_desc(ix, hmac ? fl : fl | SD_CIPHER);
			errv[i] = EALREADY;
			pos[i] = pld;
			cnt[hmac ? (h.hdr_len >> 2) & 3 : 0]++;
			continue;
		}
		desc[i] = sgpu_desc(ix, fl | SD_CIPHER);
		if (seq > st->s_l)
			st->s_l = seq;
		errv[i] = 0;
		cnt[hmac ? (h.hdr_len >> 2) & 3 : 0]++;
	}
	fs_flush(F);
}

struct flaunch {
	uint32_t base, n, shift, has_idx;
};

static double now_ms(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static size_t fast_chunk(void)
{
	return g_env.chunk;
}

/* replay state after the planned batch: the last <= 65 indices suffice
 * (every index is new and increasing, so older bits have shifted out) */
static struct replay plan_replay(const struct replay *r0,
				 const uint64_t *tail_ix, size_t n)
{
	struct replay r = *r0;
	size_t k, m = n < SGPU_PLAN_TAIL ? n : SGPU_PLAN_TAIL;
	if (n > SGPU_PLAN_TAIL) {
		r.lix = tail_ix[0];
		r.bitmap = 1;
		k = 1;
	}
	else {
		k = 0;
	}
	for (; k < m; k++)
		(void)replay_check(&r, tail_ix[k]);
	return r;
}

/* planner input from the session's (single) stream */
static void plan_in(struct sgpu_plan_in *in, const struct srtp *s,
		    uint32_t n, int prot, uint32_t T, uint32_t need)
{
	const struct srtp_stream *st0 = s->nstreams ? &s->streams[0] : NULL;
	memset(in, 0, sizeof(*in));
	in->n = n;
	in->prot = (uint32_t)prot;
	in->fresh = !st0 || !st0->s_l_set;
	in->ssrc_any = !st0;
	in->ssrc = st0 ? st0->ssrc : 0;
	in->roc = st0 ? st0->roc : 0;
	in->s_l = st0 ? st0->s_l : 0;
	in->lix = st0 ? st0->replay_rtp.lix : 0;
	in->bitmap = st0 ? st0->replay_rtp.bitmap : 0;
	in->tag = T;
	in->need = need;
	in->maxlen = SGPU_CACHED_MAX(s->rtp.mode);
}

/* stream state after an accepted device plan (old state kept for undo) */
static void plan_apply(struct srtp *s, const struct sgpu_plan_out *po,
		       int prot, size_t n, struct srtp_stream *old)
{
	struct srtp_stream *st;
	if (s->nstreams)
		*old = s->streams[0];
	else {
		memset(&s->streams[0], 0, sizeof(s->streams[0]));
		s->streams[0].ssrc = po->ssrc0;
		s->nstreams = 1;
	}
	st = &s->streams[0];
	st->s_l_set = 1;
	st->roc += po->wraps;
	st->s_l = (uint16_t)po->s_l_last;
	if (!prot)
		st->replay_rtp = plan_replay(&st->replay_rtp, po->tail_ix, n);
}

static void plan_unapply(struct srtp *s, unsigned nstreams0,
			 const struct srtp_stream *old)
{
	if (nstreams0)
		s->streams[0] = *old;
	s->nstreams = nstreams0;
}

/* ---- multi-session device plan ----------------------------------------- */

/* session passes run on the host pool from this many sessions per part
 * (RE_SRTP_PAR_MIN overrides: tests drive the pool with few sessions) */
static size_t mplan_par(void)
{
	return g_env.par_min;
}

struct mpg {
	struct srtp **sessv;
	struct sgpu_sstate *st;
	const struct sgpu_sstate *o;
	uint32_t *cm;
	int suite, prot;
	uint32_t epoch;         /* this call (alias detection) */
	atomic_int bad;
	uint8_t *need;          /* resident: st[k] is to be uploaded */
	atomic_uint nup;        /* ... how many */
	uint64_t pend, done;    /* async: this call's sequence number, the
				   thread's last completed one */
	const struct tk_owner *own;     /* ... and the issuing thread */
};

static void mplan_gather_part(void *arg, size_t a, size_t b)
{
	struct mpg *g = arg;
	size_t k;
	for (k = a; k < b; k++) {
		const struct srtp *s = g->sessv[k];
		struct sgpu_sstate *st = &g->st[k];
		if (k + 16 < b)
			__builtin_prefetch(g->sessv[k + 16], 0, 1);
		if (s->nstreams > 1 || s->suite != g->suite) {
			atomic_store(&g->bad, 1);
			return;
		}
		/* two sessv entries naming one context would plan the same
		 * stream as two independent segments: not plannable (the
		 * host engines work through the pointers) */
		if (__atomic_exchange_n(&((struct srtp *)s)->mp_epoch, g->epoch,
					__ATOMIC_RELAXED) == g->epoch) {
			atomic_store(&g->bad, 1);
			return;
		}
		if (g->cm)
			g->cm[k] = 2u * s->slot;        /* comp[0] = RTP */
		/* another thread's pending call: not plannable here (the
		 * host paths behind a rejected plan return EBUSY) */
		if (s->pend_own && s->pend_own != g->own && sess_busy(s)) {
			atomic_store(&g->bad, 1);
			return;
		}
		if (g->pend) {
			/* a pending single-stream call plans from host state
			 * this call cannot see yet */
			if (s->pend_own == g->own && s->pend_p > g->done) {
				atomic_store(&g->bad, 1);
				return;
			}
			((struct srtp *)s)->pend_m = g->pend;
			((struct srtp *)s)->pend_own = g->own;
		}
		if (g->need) {
			/* resident states: upload only what the host changed
			 * since the device last held it */
			if (s->dres == DRES_HOST) {
				g->need[k] = 1;
				atomic_fetch_add(&g->nup, 1);
			}
			else {
				g->need[k] = 0;
				((struct srtp *)s)->dres = DRES_DEV;
				continue;
			}
		}
		memset(st, 0, sizeof(*st));
		if (s->nstreams) {
			const struct srtp_stream *x = &s->streams[0];
			st->ssrc = x->ssrc;
			st->roc = x->roc;
			st->s_l = x->s_l;
			st->flags = SST_EXISTS | (x->s_l_set ? SST_SL_SET : 0);
			st->lix = x->replay_rtp.lix;
			st->bitmap = x->replay_rtp.bitmap;
		}
	}
}

/* session states in (pinned) -> device; -1 if some session has 2+ streams */
static int mplan_gather(struct srtp **sessv, size_t nsess,
			struct sgpu_sstate *st, uint32_t *cm)
{
	struct mpg g = {sessv, st, NULL, cm, sessv[0]->suite, 0, 0, 0, NULL,
			0, 0, 0, t_own};
	do {
		g.epoch = __atomic_add_fetch(&g_epoch, 1, __ATOMIC_RELAXED);
	} while (!g.epoch);
	par_for(nsess, mplan_par(), mplan_gather_part, &g);
	return atomic_load(&g.bad) ? -1 : 0;
}

/*
 * The same pass for resident states: sessions whose device copy is
 * current are only mapped (and marked DRES_DEV); host-newer ones are
 * copied to st[k] with need[k] = 1 for sgpu_sst_load.  *nup = how many.
 * -1: not plannable (the caller uploads nothing: need[] is ignored and
 * the marks are undone).
 */
static int mplan_gather_res(struct srtp **sessv, size_t nsess,
			    struct sgpu_sstate *st, uint32_t *cm,
			    uint8_t *need, uint32_t *nup, uint64_t pend,
			    uint64_t done)
{
	struct mpg g = {sessv, st, NULL, cm, sessv[0]->suite, 0, 0, 0, need,
			0, pend, done, t_own};
	size_t k;
	do {
		g.epoch = __atomic_add_fetch(&g_epoch, 1, __ATOMIC_RELAXED);
	} while (!g.epoch);
	par_for(nsess, mplan_par(), mplan_gather_part, &g);
	*nup = atomic_load(&g.nup);
	if (atomic_load(&g.bad)) {
		/* the device copies of sessions marked DEV here were current
		 * already (DRES_BOTH or DRES_DEV): DEV is still true */
		return -1;
	}
	if (*nup)
		for (k = 0; k < nsess; k++)
			if (need[k])
				sessv[k]->dres = DRES_DEV;
	return 0;
}

static void mplan_apply_part(void *arg, size_t a, size_t b)
{
	struct mpg *g = arg;
	const struct sgpu_sstate *o = g->o;
	size_t k;
	for (k = a; k < b; k++) {
		struct srtp *s;
		struct srtp_stream *x;
		if (k + 16 < b && (o[k + 16].flags & SST_TOUCHED))
			__builtin_prefetch(g->sessv[k + 16], 1, 1);
		if (!(o[k].flags & SST_TOUCHED))
			continue;
		s = g->sessv[k];
		if (!s->nstreams) {
			memset(&s->streams[0], 0, sizeof(s->streams[0]));
			s->nstreams = 1;
		}
		x = &s->streams[0];
		x->ssrc = o[k].ssrc;
		x->roc = o[k].roc;
		x->s_l = (uint16_t)o[k].s_l;
		x->s_l_set = 1;
		if (!g->prot) {
			x->replay_rtp.lix = o[k].lix;
			x->replay_rtp.bitmap = o[k].bitmap;
		}
	}
}

/* device results -> sessions (touched ones only) */
static void mplan_apply(struct srtp **sessv, size_t nsess,
			const struct sgpu_sstate *o, int prot)
{
	struct mpg g = {sessv, NULL, o, NULL, 0, prot, 0, 0, NULL, 0, 0, 0,
			t_own};
	par_for(nsess, mplan_par(), mplan_apply_part, &g);
}

/* undo mplan_apply from the gathered pre-call states */
static void mplan_unapply(struct srtp **sessv, size_t nsess, struct ws *w)
{
	const struct sgpu_sstate *in = (const struct sgpu_sstate *)w->ms.h;
	const struct sgpu_sstate *o = in + nsess;
	size_t k;
	for (k = 0; k < nsess; k++) {
		struct srtp *s;
		struct srtp_stream *x;
		if (!(o[k].flags & SST_TOUCHED))
			continue;
		s = sessv[k];
		if (!(in[k].flags & SST_EXISTS)) {
			s->nstreams = 0;
			continue;
		}
		x = &s->streams[0];
		x->roc = in[k].roc;
		x->s_l = (uint16_t)in[k].s_l;
		x->s_l_set = (in[k].flags & SST_SL_SET) ? 1 : 0;
		x->replay_rtp.lix = in[k].lix;
		x->replay_rtp.bitmap = in[k].bitmap;
	}
}

/*
 * The compact crypto launches of a device-planned batch.  GCM: one launch
 * guarded by po->fail.  AES-CM: the header class (SHIFT) is only known on
 * the device, so one k_ctr_hmac_any launch picks it from po->skip[0..3];
 * undo passes (rare) keep one guarded launch per class.
 */
static int run_classes(uint8_t *arena, uint64_t asz, struct sgpu_compact C,
		       const struct comp *c0, struct sgpu_plan_out *po_d,
		       int prot, void *stream)
{
	int q, err = 0;

	if (c0->mode == SGPU_MODE_GCM) {
		C.guard = &po_d->fail;
		return sgpu_run_compact(arena, asz, &C, c0->mode, (int)c0->nr,
					0, prot, stream);
	}
	if (!C.undo && !g_env.perclass) {
		C.guard = po_d->skip;
		/* one key and the planner's packet shape: lean kernels;
		 * per-lane keys (multi-session plan): their per-lane form */
		if (C.uniform == 1 && !g_env.nolean)
			C.uniform = 2;
		else if (!C.uniform && C.sess && !g_env.nolean &&
			 !g_env.nomk)
			C.uniform = 3;
		return sgpu_run_compact(arena, asz, &C, c0->mode, (int)c0->nr,
					-1, prot, stream);
	}
	for (q = 0; q < 4 && !err; q++) {
		C.guard = &po_d->skip[q];
		err = sgpu_run_compact(arena, asz, &C, c0->mode, (int)c0->nr,
				       q, prot, stream);
	}
	return err;
}

/*
 * Returns 0 (planned and launched; *nfailp holds the speculation misses,
 * fl/nfl the launches), an errno, -1 (not eligible: nothing done) or -2
 * (plan rejected: headers parsed on the device and downloaded to w->hd.h,
 * windows/sessions staged in w->up, nothing else modified).
 */
static int run_mplanned(int op, struct srtp **sessv, size_t nsess,
			struct srtp_batch *b, struct ws *w, void *stream,
			const struct comp *c0, uint32_t T,
			struct flaunch *fl, size_t *nfl, uint32_t *nfailp)
{
	const int prot = op == OP_RTP_ENC;
	const size_t n = b->n;
	const int gcm = c0->mode == SGPU_MODE_GCM;
	const int nclass = gcm ? 1 : 4;
	const uint32_t need = prot ? (gcm ? 16u : (T > 4 ? T : 4u)) : 0u;
	struct sgpu_plan_out *po = (struct sgpu_plan_out *)w->pl.h;
	struct sgpu_plan_out *po_d = (struct sgpu_plan_out *)w->pl.d;
	uint32_t *up_h = (uint32_t *)w->up.h, *up_d = (uint32_t *)w->up.d;
	struct sgpu_hdr *hd_d = (struct sgpu_hdr *)w->hd.d;
	uint64_t *desc_d = (uint64_t *)w->dsc.d;
	uint32_t *nfail_d = (uint32_t *)w->vs.d;
	uint32_t *save_d = (uint32_t *)(w->vs.d + 64);
	uint8_t *vd_d = w->vs.d + 64 + n * 4;
	struct sgpu_sstate *sin_h, *sin_d, *sout_h, *sout_d;
	uint32_t *order_d;
	struct sgpu_mplan_in in;
	size_t scr, i;
	uint32_t bits = 1;
	int err, capok = 1, q;

	while (bits < 32 && ((size_t)1 << bits) < nsess)
		bits++;
	/* the original windows first: the caller restores them from up_h on
	 * any error below (run_fast's `touched`) */
	memcpy(up_h, b->pos, n * 4);
	memcpy(up_h + n, b->end, n * 4);
	memcpy(up_h + 2 * n, b->sess, n * 4);
	scr = sgpu_mplan_scratch((uint32_t)n, (uint32_t)nsess);
	err = pool_reserve(w, &w->ms, nsess * 2 * sizeof(struct sgpu_sstate));
	if (!err)   /* scratch, then the launch order (n words) */
		err = pool_reserve(w, &w->mscr, scr + n * 4);
	if (err)
		return err;
	sin_h = (struct sgpu_sstate *)w->ms.h;
	sin_d = (struct sgpu_sstate *)w->ms.d;
	sout_h = sin_h + nsess;
	sout_d = sin_d + nsess;
	if (mplan_gather(sessv, nsess, sin_h, NULL))
		return -1;
	order_d = (uint32_t *)(w->mscr.d + scr);

	memset(&in, 0, sizeof(in));
	in.n = (uint32_t)n;
	in.nsess = (uint32_t)nsess;
	in.prot = (uint32_t)prot;
	in.tag = T;
	in.need = need;
	in.maxlen = SGPU_CACHED_MAX(c0->mode);
	in.key_bits = bits;
	err = sgpu_memcpy_h2d(w->cm.d, w->cm.h, nsess * 4, stream);
	if (!err)
		err = sgpu_memcpy_h2d(sin_d, sin_h,
				      nsess * sizeof(struct sgpu_sstate), stream);
	if (!err && !prot)
		err = sgpu_memset(nfail_d, 0, 4, stream);
	if (!err)
		err = sgpu_memcpy_h2d(up_d, up_h, n * 12, stream);
	if (!err)
		err = sgpu_parse_headers(b->arena, b->arena_size, up_d,
					 up_d + n, hd_d, NULL, (uint32_t)n, 0,
					 stream);
	if (!err)
		err = sgpu_mplan_rtp(&in, hd_d, up_d, up_d + n, NULL,
				     b->arena_size, up_d + 2 * n, sin_d, sout_d,
				     desc_d, w->mscr.d, scr, po_d, order_d,
				     stream);
	if (err)
		return err;
	if (prot)
		for (i = 0; i < n; i++)
			capok &= (uint64_t)b->end[i] + need <= b->cap[i];
	if (!err && capok) {
		struct sgpu_compact C = {
			up_d, up_d + n, hd_d, desc_d, up_d + 2 * n,
			(const uint32_t *)w->cm.d, order_d, 0, (uint32_t)n,
			vd_d, save_d, nfail_d, 0, 0, NULL, 0, NULL};
		err = run_classes(b->arena, b->arena_size, C, c0,
				  po_d, prot, stream);
	}
	if (!err)
		err = sgpu_memcpy_d2h(po, po_d, sizeof(*po), stream);
	if (!err)
		err = sgpu_memcpy_d2h(sout_h, sout_d,
				      nsess * sizeof(struct sgpu_sstate), stream);
	if (!err && !prot && capok)
		err = sgpu_memcpy_d2h(nfailp, nfail_d, 4, stream);
	if (err)
		return err;
	if (capok) {
		if (prot)
			for (i = 0; i < n; i++)
				b->end[i] += T;
		else
			for (i = 0; i < n; i++)
				b->end[i] -= T;
		memset(b->err, 0, n * sizeof(*b->err));
	}
	err = sgpu_stream_sync(stream);
	if (err)
		return err;
	if (g_env.trace)
		fprintf(stderr, "re_srtp mplan %s n=%zu nsess=%zu: fail 0x%x "
			"cap %d\n", prot ? "enc" : "dec", n, nsess, po->fail,
			capok);
	if (!po->fail && capok) {
		mplan_apply(sessv, nsess, sout_h, prot);
		for (q = 0; q < nclass; q++)
			fl[(*nfl)++] = (struct flaunch){0, (uint32_t)n,
							(uint32_t)q, 0};
		return 0;
	}
	if (capok)
		memcpy(b->end, up_h + n, n * 4);
	*nfailp = 0;
	err = sgpu_memcpy_d2h(w->hd.h, hd_d, n * sizeof(*hd_d), stream);
	if (!err && !prot)
		err = sgpu_memset(nfail_d, 0, 4, stream);
	return err ? err : -2;
}

/*
 * Returns 0 / errno like run_batch, or -1 when the batch is not eligible
 * (nothing touched: caller runs the general engine).
 */
static int run_fast(int op, struct srtp **sessv, size_t nsess,
		    struct srtp_batch *b)
{
	const int prot = op == OP_RTP_ENC;
	const size_t n = b->n, CH = fast_chunk();
	const size_t nch = (n + CH - 1) / CH;
	const struct comp *c0 = &sessv[0]->rtp;
	const uint32_t T = c0->mode == SGPU_MODE_GCM ? 16u : c0->tag_len;
	struct fscan FT[1];
	struct flaunch *fl = NULL;
	size_t nfl = 0, i, k;
	uint32_t *up_h, *up_d, *cm_h;
	struct sgpu_hdr *hd_d;
	uint64_t *desc_d;
	uint32_t *idx_h, *idx_d;
	uint8_t *vd_d;
	uint32_t *save_d, *nfail_d, nfail = 0;
	void *stream, *entry_ev = NULL;
	struct ws *w;
	int err = 0, parsed = 0, planned = 0;
	int touched = 0;        /* up_h holds every original window */
	void *pst;
	/* planned path: stream state before the call (undo) */
	struct srtp *ps = sessv[0];
	unsigned ps_n = ps->nstreams;
	struct srtp_stream ps_old;
	const int trace = g_env.trace;
	double t0 = trace ? now_ms() : 0, t1 = 0, t2 = 0, tscan = 0, twait = 0;

	if (n == 0)
		return -1;
	/* RTP contexts derive from the suite alone (srtp.c:101-153) */
	for (k = 0; k < nsess; k++) {
		if (k + 16 < nsess)
			__builtin_prefetch(sessv[k + 16], 0, 1);
		if (sessv[k]->suite != sessv[0]->suite)
			return -1;
	}
	w = ws_get();
	if (!w)
		return ENOMEM;
	w->ulog[0].n = 0;
	if (!w->pstream) {
		w->pstream = sgpu_stream_create();
		if (!w->pstream)
			return EIO;
	}
	/* the caller's stream; NULL is the default (null) stream, which
	 * orders this call after the caller's prior default-stream work */
	stream = b->stream;
	pst = w->pstream;

	err = pool_reserve(w, &w->up, n * 12);
	if (!err)
		err = pool_reserve(w, &w->hd, n * sizeof(struct sgpu_hdr));
	if (!err)
		err = pool_reserve(w, &w->dsc, n * 12);
	if (!err)
		err = pool_reserve(w, &w->vs, n * 5 + 64);
	if (!err)
		err = pool_reserve(w, &w->cm, nsess * 4);
	if (!err)
		err = pool_reserve(w, &w->pl, sizeof(struct sgpu_plan_out) +
				   (n / 256 + 8) * 4);
	if (err)
		return err;
	if (w->nev < nch) {
		void **ne = fi_realloc(w->ev, nch * sizeof(*ne));
		if (!ne)
			return ENOMEM;
		w->ev = ne;
		while (w->nev < nch) {
			w->ev[w->nev] = sgpu_event_create();
			if (!w->ev[w->nev])
				return EIO;
			w->nev++;
		}
	}
	fl = fi_malloc(4 * nch * sizeof(*fl) + 4 * sizeof(*fl));
	if (!fl)
		return ENOMEM;

	up_h = (uint32_t *)w->up.h;
	up_d = (uint32_t *)w->up.d;
	hd_d = (struct sgpu_hdr *)w->hd.d;
	desc_d = (uint64_t *)w->dsc.d;
	idx_h = (uint32_t *)(w->dsc.h + n * 8);
	idx_d = (uint32_t *)(w->dsc.d + n * 8);
	nfail_d = (uint32_t *)(w->vs.d);
	save_d = (uint32_t *)(w->vs.d + 64);
	vd_d = w->vs.d + 64 + n * 4;
	cm_h = (uint32_t *)w->cm.h;
	for (k = 0; k < nsess; k++)
		cm_h[k] = 2u * sessv[k]->slot;          /* comp[0] = RTP */


	/* 0b. many sessions, at most one stream each: plan on the device
	 *     (stable sort by session + per-session speculation); host work
	 *     is O(sessions): gather the states, apply the results. */
	if (b->sess && nsess > 1 && !t_noplan && !g_env.noplan) {
		int r = run_mplanned(op, sessv, nsess, b, w, stream, c0, T, fl,
				     &nfl, &nfail);
		touched = r != -1;
		if (r == 0) {
			planned = 2;
			if (trace)
				t1 = t2 = now_ms();
			goto checked;
		}
		if (r > 0) {
			err = r;
			goto out;
		}
		if (r == -2) {
			/* plan rejected after parsing: headers are on the
			 * device (and host), the scan path takes over */
			parsed = 1;
			pst = stream;
		}
	}

	/* 0. one stream: plan on the device (speculative scan, verified).
	 *    Everything is queued on one stream with a single sync: the
	 *    crypto launches are guarded on the device by the plan's verdict
	 *    (sgpu_plan_out.skip), so a rejected plan modifies nothing. */
	if (nsess == 1 && ps->nstreams <= 1 && !t_noplan &&
	    !g_env.noplan) {
		struct sgpu_plan_in in;
		struct sgpu_plan_out *po = (struct sgpu_plan_out *)w->pl.h;
		struct sgpu_plan_out *po_d = (struct sgpu_plan_out *)w->pl.d;
		uint32_t *scr = (uint32_t *)(w->pl.d + sizeof(*po));
		const uint32_t need = prot ? (c0->mode == SGPU_MODE_GCM ? 16u :
				      (T > 4 ? T : 4u)) : 0u;
		int capok = 1, q;
		/* CTR kernels are specialised per header shift class (one
		 * launch runs, the others exit on their guard); GCM is not */
		const int gcm = c0->mode == SGPU_MODE_GCM;
		const int nclass = gcm ? 1 : 4;

		plan_in(&in, ps, (uint32_t)n, prot, T, need);
		memcpy(up_h, b->pos, n * 4);
		memcpy(up_h + n, b->end, n * 4);
		touched = 1;
		err = sgpu_memcpy_h2d(w->cm.d, cm_h, 4, stream);
		if (!err && !prot)
			err = sgpu_memset(nfail_d, 0, 4, stream);
		if (!err)
			err = sgpu_memcpy_h2d(up_d, up_h, n * 8, stream);
		if (!err)
			err = sgpu_parse_headers(b->arena, b->arena_size, up_d,
						 up_d + n, hd_d, NULL,
						 (uint32_t)n, 0, stream);
		if (!err)
			err = sgpu_plan_rtp(&in, hd_d, up_d, up_d + n, NULL,
					    b->arena_size, desc_d, scr, po_d,
					    stream);
		if (err)
			goto out;
		/* device arenas cannot grow (cap_short), checked while the
		 * GPU plans */
		if (prot)
			for (i = 0; i < n; i++)
				capok &= (uint64_t)b->end[i] + need <= b->cap[i];
		if (!err && capok) {
			struct sgpu_compact C = {
				up_d, up_d + n, hd_d, desc_d, NULL,
				(const uint32_t *)w->cm.d, NULL, 0,
				(uint32_t)n, vd_d, save_d, nfail_d, 0, 1, NULL, 0, NULL};
			err = run_classes(b->arena, b->arena_size, C, c0,
					  po_d, prot, stream);
		}
		if (!err)
			err = sgpu_memcpy_d2h(po, po_d, sizeof(*po), stream);
		if (!err && !prot && capok)
			err = sgpu_memcpy_d2h(&nfail, nfail_d, 4, stream);
		if (err)
			goto out;
		/* per-packet results, speculatively, while the GPU runs */
		if (capok) {
			if (prot)
				for (i = 0; i < n; i++)
					b->end[i] += T;
			else
				for (i = 0; i < n; i++)
					b->end[i] -= T;
			memset(b->err, 0, n * sizeof(*b->err));
		}
		err = sgpu_stream_sync(stream);
		if (err)
			goto out;
		parsed = 1;
		if (trace)
			fprintf(stderr, "re_srtp plan %s n=%zu: fail 0x%x "
				"wraps %u cap %d (%.3f ms)\n", prot ? "enc" :
				"dec", n, po->fail, po->wraps, capok,
				now_ms() - t0);
		if (!po->fail && capok) {
			plan_apply(ps, po, prot, n, &ps_old);
			for (q = 0; q < nclass; q++)
				fl[nfl++] = (struct flaunch){0, (uint32_t)n,
							     (uint32_t)q, 0};
			planned = 1;
			if (trace)
				t1 = t2 = now_ms();
			goto checked;
		}
		if (capok)
			memcpy(b->end, up_h + n, n * 4);
		/* not plannable: headers down for the host scan */
		pst = stream;
		err = sgpu_memcpy_d2h(w->hd.h, hd_d, n * sizeof(*hd_d), stream);
		if (!err && !prot)
			err = sgpu_memset(nfail_d, 0, 4, stream);
		if (err)
			goto out;
	}

	/* 1. parse stream: staged windows up, headers parsed, back down,
	 *    chunk by chunk (ordered after the caller's prior work) */
	if (!parsed) {
		entry_ev = w->ev[0];
		/* the parse stream starts after the caller's prior work */
		err = sgpu_event_record(entry_ev, stream);
		if (!err)
			err = sgpu_stream_wait(w->pstream, entry_ev);
		if (!err)
			err = sgpu_memcpy_h2d(w->cm.d, cm_h, nsess * 4,
					      w->pstream);
		if (!err && !prot)
			err = sgpu_memset(nfail_d, 0, 4, w->pstream);
		if (err)
			goto out;
	}
	else {
		err = sgpu_memcpy_h2d(w->cm.d, cm_h, nsess * 4, stream);
		if (err)
			goto out;
	}
	for (k = 0; k < nch && !err; k++) {
		const size_t a = k * CH, e = a + CH < n ? a + CH : n;
		if (parsed) {
			err = sgpu_event_record(w->ev[k], pst);
			continue;
		}
		memcpy(up_h + a, b->pos + a, (e - a) * 4);
		memcpy(up_h + n + a, b->end + a, (e - a) * 4);
		err = sgpu_memcpy_h2d(up_d + a, up_h + a, (e - a) * 4,
				      w->pstream);
		if (!err)
			err = sgpu_memcpy_h2d(up_d + n + a, up_h + n + a,
					      (e - a) * 4, w->pstream);
		if (!err && b->sess) {
			memcpy(up_h + 2 * n + a, b->sess + a, (e - a) * 4);
			err = sgpu_memcpy_h2d(up_d + 2 * n + a,
					      up_h + 2 * n + a, (e - a) * 4,
					      w->pstream);
		}
		if (!err)
			err = sgpu_parse_headers(b->arena, b->arena_size,
						 up_d + a,
						 up_d + n + a, hd_d + a, NULL,
						 (uint32_t)(e - a), 0,
						 w->pstream);
		if (!err)
			err = sgpu_memcpy_d2h(w->hd.h + a * sizeof(*hd_d),
					      hd_d + a, (e - a) * sizeof(*hd_d),
					      w->pstream);
		if (!err)
			err = sgpu_event_record(w->ev[k], w->pstream);
	}
	if (err)
		goto out;
	touched = 1;
	if (parsed && b->sess) {
		memcpy(up_h + 2 * n, b->sess, n * 4);
		err = sgpu_memcpy_h2d(up_d + 2 * n, up_h + 2 * n, n * 4,
				      stream);
		if (err)
			goto out;
	}

	/* 2. sequential scan per chunk, crypto launched behind it */
	if (trace)
		t1 = now_ms();
	memset(FT, 0, sizeof(FT));
	FT[0].sessv = sessv;
	FT[0].sidx = b->sess;
	FT[0].hd = (const struct sgpu_hdr *)w->hd.h;
	FT[0].desc = (uint64_t *)w->dsc.h;
	FT[0].pos = b->pos;
	FT[0].end = b->end;
	FT[0].cap = b->cap;
	FT[0].err = b->err;
	FT[0].epoch = __atomic_add_fetch(&g_epoch, 1, __ATOMIC_RELAXED);
	/* every first touch of a stream is logged (undo on a miss or a
	 * failed call) */
	FT[0].log = 1;
	FT[0].mode = c0->mode;
	FT[0].tag_len = c0->tag_len;
	FT[0].log_v = &w->ulog[0];
	w->ulog[0].n = 0;
	for (k = 0; k < nch && !err; k++) {
		const size_t a = k * CH, e = a + CH < n ? a + CH : n;
		uint32_t cnt[4] = {0, 0, 0, 0}, nz = 0, sh = 0, q;
		double ta = trace ? now_ms() : 0, tb = 0;
		err = sgpu_event_sync(w->ev[k]);
		if (err)
			break;
		if (trace)
			tb = now_ms();
		if (prot)
			scan_enc(&FT[0], a, e, cnt);
		else
			scan_dec(&FT[0], a, e, cnt);
		if (FT[0].nomem)
			err = ENOMEM;
		if (trace) {
			twait += tb - ta;
			tscan += now_ms() - tb;
		}
		if (err)
			break;
		for (q = 0; q < 4; q++)
			if (cnt[q]) {
				nz++;
				sh = q;
			}
		err = sgpu_memcpy_h2d(desc_d + a, FT[0].desc + a, (e - a) * 8,
				      stream);
		if (err || !nz)
			continue;
		if (nz == 1) {
			fl[nfl++] = (struct flaunch){(uint32_t)a,
						     (uint32_t)(e - a), sh, 0};
		}
		else {
			/* mixed header-length classes: class lists */
			uint32_t st[4], o = (uint32_t)a;
			for (q = 0; q < 4; q++) {
				st[q] = o;
				o += cnt[q];
			}
			for (i = a; i < e; i++)
				if (FT[0].desc[i])
					idx_h[st[(FT[0].hd[i].hdr_len >> 2) & 3]++]
						= (uint32_t)i;
			o = (uint32_t)a;
			for (q = 0; q < 4; q++) {
				if (cnt[q])
					fl[nfl++] = (struct flaunch){o, cnt[q],
								     q, 1};
				o += cnt[q];
			}
			err = sgpu_memcpy_h2d(idx_d + a, idx_h + a,
					      (o - a) * 4, stream);
		}
		for (q = nfl - (nz == 1 ? 1 : nz); q < nfl && !err; q++) {
			struct sgpu_compact C = {
				up_d, up_d + n, hd_d, desc_d,
				b->sess ? up_d + 2 * n : NULL,
				(const uint32_t *)w->cm.d,
				fl[q].has_idx ? idx_d : NULL, fl[q].base,
				fl[q].n, vd_d, save_d, nfail_d, 0, nsess == 1,
				NULL, 0, NULL};
			err = sgpu_run_compact(b->arena, b->arena_size, &C,
					       c0->mode, (int)c0->nr,
					       (int)fl[q].shift, prot, stream);
		}
	}
	if (trace)
		t2 = now_ms();
	if (!err && !prot)
		err = sgpu_memcpy_d2h(&nfail, nfail_d, 4, stream);
	if (!err)
		err = sgpu_stream_sync(stream);
 checked:
	if (trace)
		fprintf(stderr, "re_srtp fast %s n=%zu%s: stage %.3f ms, "
			"parse-wait %.3f, scan %.3f, launch %.3f, tail %.3f, "
			"total %.3f\n", prot ? "enc" : "dec", n,
			planned ? " (device-planned)" : "", t1 - t0, twait,
			tscan, t2 - t1 - twait - tscan, now_ms() - t2,
			now_ms() - t0);
	if (err)
		goto out;
	if (nfail) {
		count(&g_cnt_misses, nfail);
		count(&g_cnt_folds, 1);
		/* speculation missed: undo and fold exactly */
		for (k = 0; k < nfl && !err; k++) {
			struct sgpu_compact C = {
				up_d, up_d + n, hd_d, desc_d,
				b->sess ? up_d + 2 * n : NULL,
				(const uint32_t *)w->cm.d,
				fl[k].has_idx ? idx_d : NULL, fl[k].base,
				fl[k].n, vd_d, save_d, nfail_d, 1, nsess == 1,
				!planned ? NULL :
				c0->mode == SGPU_MODE_GCM ?
				&((struct sgpu_plan_out *)w->pl.d)->fail :
				&((struct sgpu_plan_out *)w->pl.d)->
					  skip[fl[k].shift], 0, NULL};
			C.uniform = planned != 2 && nsess == 1;
			err = sgpu_run_compact(b->arena, b->arena_size, &C,
					       c0->mode, (int)c0->nr,
					       (int)fl[k].shift, prot, stream);
		}
		if (!err)
			err = sgpu_stream_sync(stream);
		if (err)
			goto out;
		if (planned == 1)
			plan_unapply(ps, ps_n, &ps_old);
		else if (planned == 2)
			mplan_unapply(sessv, nsess, w);
		ulog_undo(&w->ulog[0]);
		memcpy(b->pos, up_h, n * 4);
		memcpy(b->end, up_h + n, n * 4);
		free(fl);
		return run_batch_general(op, sessv, nsess, b);
	}
 out:
	if (err > 0 && touched) {
		/* a failed call leaves the stream states and windows as it
		 * found them (the arena may be partly processed: EIO) */
		if (planned == 1)
			plan_unapply(ps, ps_n, &ps_old);
		else if (planned == 2)
			mplan_unapply(sessv, nsess, w);
		ulog_undo(&w->ulog[0]);
		memcpy(b->pos, up_h, n * 4);
		memcpy(b->end, up_h + n, n * 4);
	}
	free(fl);
	return err;
}

static int run_batch(int op, struct srtp **sessv, size_t nsess,
		     struct srtp_batch *b)
{
	size_t i;
	uint32_t lim = UINT32_MAX;
	int r, big = 0;
	if ((op == OP_RTP_ENC || op == OP_RTP_DEC) && sessv && nsess && b &&
	    b->arena && b->pos && b->end && b->cap && b->err &&
	    b->n <= UINT32_MAX / 4 && b->arena_size <= UINT32_MAX &&
	    !g_env.general) {
		for (i = 0; i < nsess; i++) {
			if (!sessv[i])
				return EINVAL;
			if (SGPU_CACHED_MAX(sessv[i]->rtp.mode) < lim)
				lim = SGPU_CACHED_MAX(sessv[i]->rtp.mode);
		}
		for (i = 0; i < b->n; i++) {
			if ((b->pos[i] & 3) || b->end[i] > b->cap[i] ||
			    b->cap[i] > b->arena_size ||
			    b->pos[i] > b->end[i] ||
			    (b->sess && b->sess[i] >= nsess))
				return EINVAL;
			/* the compact kernels cache the counter block for
			 * packets under SGPU_CACHED_MAX (kern_common.h) */
			if (b->end[i] - b->pos[i] >= lim)
				big = 1;
		}
		r = big ? -1 : run_fast(op, sessv, nsess, b);
		if (r >= 0)
			return r;
	}
	return run_batch_general(op, sessv, nsess, b);
}

/* ---- fully device-resident batches ------------------------------------ */

static int run_batch(int op, struct srtp **sessv, size_t nsess,
		     struct srtp_batch *b);

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
	int radix;              /* ... grouped by the radix sort */
	int fused;              /* single stream planned inside the crypto
				   launch (fz_issue / fz_finish) */
	struct sgpu_fused fz;   /* ... its launch */
};

/* single-stream RTP batch planned and processed on the device: the
 * launches (no host synchronisation) */
static int fz_issue(struct dcall *k, int sync);
static int fz_finish(struct dcall *k, int sync);

static int dev_planned_issue(struct dcall *k)
{
	if (k->sessv[0]->rtp.mode == SGPU_MODE_CTR && !g_env.noplanfuse) {
		k->fused = 1;
		return fz_issue(k, 0);
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
			save_d, nfail_d, 0, 1, NULL, 0, flist_d};
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
static int dev_planned_finish(struct dcall *k)
{
	if (k->fused)
		return fz_finish(k, 0);
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
			save_d, nfail_d, 1, 1, NULL, 0, NULL};
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
	if (w->fz_d != fz || w->fz_epoch == 0 || w->fz_epoch > 0xffffu) {
		/* a new pool (or the look-back epoch wrapped): counters,
		 * plan outs and look-back words from zero */
		err = sgpu_memset(fz, 0, w->fz.cap, stream);
		if (err)
			return err;
		w->fz_d = fz;
		w->fz_epoch = 1;
		w->fz_tbase = 0;
		w->fz_par = 0;
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
	k->devfold = !sync && !prot && !g_env.nodevfold;
	if (!sync) {
		/* queued behind the launch: forged packets' ciphertext and the
		 * verdict fold (unprotect), the gate word of the next chained
		 * call (set if this call must be completed on the host) */
		struct sgpu_fold_out *fo_d =
			(struct sgpu_fold_out *)(fz + poff + FZ_FO_OFF);
		uint32_t *fscr = (uint32_t *)(w->pl.d + 64);
		if (k->devfold) {
			err = sgpu_fused_refix(d->arena, d->arena_size, F,
					       (int)c0->nr, stream);
			if (!err)
				err = sgpu_fold_rtp(1, &F->out->nfail, &F->in,
						    F->hdr, F->desc, F->verdict,
						    F->es, d->pos, d->end, d->err,
						    0, fscr, fo_d, stream);
		}
		if (!err && k->gate)
			err = sgpu_plan_finish(&F->out->fail, NULL, NULL, NULL, 0,
					       0, &F->out->nfail, k->gate, NULL,
					       k->devfold ? &fo_d->fail : NULL,
					       stream);
		if (!err && k->devfold)
			err = sgpu_fold_rtp(2, &F->out->nfail, &F->in, F->hdr,
					    F->desc, F->verdict, F->es, d->pos,
					    d->end, d->err, 0, fscr, fo_d,
					    stream);
	}
	if (!err)
		err = sgpu_memcpy_d2h(w->fz.h + poff, F->out,
				      k->devfold ? FZ_SLOT
						 : sizeof(struct sgpu_plan_out),
				      stream);
	return err;
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
		if (po->fail & SPF_BAD)
			w->fz_d = NULL; /* ticket / look-back state from zero */
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
	if (sync && !g_env.nodevfold) {
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
	err = fz_issue(&k, 1);
	if (!err)
		err = sgpu_stream_sync(d->stream);
	if (err)
		return err;
	err = fz_finish(&k, 1);
	*pfail = k.pfail;
	return err;
}

/* synchronous: -1 not plannable (nothing modified; *pfail: why, 0 for a
 * forged packet the host must fold), else 0 / errno */
static int dev_planned(int op, struct srtp *s, struct srtp_batch_dev *d,
		       uint32_t *pfail)
{
	struct dcall k;
	int err;
	if (s->rtp.mode == SGPU_MODE_CTR && !g_env.noplanfuse)
		return dev_fused(op, s, d, pfail);
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
static int dev_splanned_issue(struct dcall *k)
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
			save_d, nfail_d, 0, 1, NULL, 0, NULL};
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
static int dev_splanned_finish(struct dcall *k)
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
			NULL, 0, NULL};
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
static int dev_splanned(int op, struct srtp *s, struct srtp_batch_dev *d)
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

/*
 * Single-stream SRTCP batch planned and processed on the device (the
 * SRTCP counterpart of dev_planned): k_parse (with the E || index words),
 * k_plan_rtcp, the compact crypto launch, the per-packet results; one host
 * synchronisation.  -1: not plannable or a forged packet (undone), else 0
 * / errno.
 */
static int dev_planned_rtcp(int op, struct srtp *s, struct srtp_batch_dev *d)
{
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
			gcm ? &po_d->fail : &po_d->skip[2], 1, NULL};
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
			gcm ? &po_d->fail : &po_d->skip[2], 1, NULL};
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

static int dev_mplanned_issue(struct dcall *k)
{
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
			!prot && !gcm && !g_env.nodevfold ? flist_d : NULL};
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
static int dev_mplanned_finish(struct dcall *k)
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
			save_d, nfail_d, 1, 0, NULL, 0, NULL};
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
static int dev_mplanned_(int op, struct srtp **sessv, size_t nsess,
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
static int dev_mplanned(int op, struct srtp **sessv, size_t nsess,
			struct srtp_batch_dev *d)
{
	uint32_t pf = 0;
	int r = dev_mplanned_(op, sessv, nsess, d, g_env.mpradix, &pf);
	if (r == -1 && (pf & SPF_SEG) && !g_env.mpradix)
		r = dev_mplanned_(op, sessv, nsess, d, 1, &pf);
	return r;
}

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
static void tk_drain(void)
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
