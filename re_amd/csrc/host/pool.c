/*
 * pool.c -- a small persistent worker pool for the host passes over many
 * sessions (multi-session batches gather and apply one stream state per
 * session: 64K sessions are 64K cold heap objects, a memory-latency-bound
 * pointer chase that parallelises across cores).
 *
 * par_for(n, min_per, fn, arg) splits [0, n) into contiguous parts, runs
 * them on the calling thread plus up to RE_SRTP_THREADS-1 workers
 * (default 8) and returns when every part is done.  Thread k takes part k
 * first (gather and apply of one batch then touch the same sessions from
 * the same core), then steals unclaimed parts.  Calls are serialised; a
 * pool without workers runs fn(arg, 0, n) inline.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include "pool.h"

#define POOL_MAX 32

static pthread_mutex_t p_call = PTHREAD_MUTEX_INITIALIZER;
static pthread_mutex_t p_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t p_wake = PTHREAD_COND_INITIALIZER;
static pthread_once_t p_once = PTHREAD_ONCE_INIT;
static int p_nthr;                      /* workers started */
static long p_spin = 5000;              /* pause loops before sleeping */
/* job parameters: written by par_for under p_lock while no worker is
 * inside a job (p_active == 0), read by workers that entered under
 * p_lock with the current generation */
static unsigned long p_gen;
static par_fn p_fn;
static void *p_arg;
static size_t p_n, p_parts;
static atomic_ulong p_pub;              /* p_gen, readable unlocked */
static atomic_int p_active;             /* workers inside a job */
static _Atomic unsigned long p_claim[POOL_MAX + 1];  /* gen per part */
static atomic_size_t p_done;            /* parts finished */

static void run_part(unsigned long gen, size_t k)
{
	unsigned long v = atomic_load(&p_claim[k]);
	if (v == gen || !atomic_compare_exchange_strong(&p_claim[k], &v, gen))
		return;
	p_fn(p_arg, p_n * k / p_parts, p_n * (k + 1) / p_parts);
	atomic_fetch_add(&p_done, 1);
}

static void run_parts(unsigned long gen, size_t id)
{
	size_t k;
	if (id < p_parts)
		run_part(gen, id);
	for (k = 0; k < p_parts; k++)
		run_part(gen, k);
}

static void *worker(void *arg)
{
	const size_t id = (size_t)arg;
	unsigned long seen = 0;
	for (;;) {
		/* spin a little before sleeping: batches come back to back */
		long spin;
		for (spin = 0; spin < p_spin && atomic_load(&p_pub) == seen;
		     spin++)
			__builtin_ia32_pause();
		pthread_mutex_lock(&p_lock);
		while (p_gen == seen)
			pthread_cond_wait(&p_wake, &p_lock);
		seen = p_gen;
		atomic_fetch_add(&p_active, 1);
		pthread_mutex_unlock(&p_lock);
		run_parts(seen, id);
		atomic_fetch_sub(&p_active, 1);
	}
	return NULL;
}

static void pool_start(void)
{
	const char *e = getenv("RE_SRTP_THREADS");
	const char *sp = getenv("RE_SRTP_SPIN");
	long want = e ? atol(e) : 8;
	int i;
	if (sp)
		p_spin = atol(sp);
	if (want > POOL_MAX)
		want = POOL_MAX;
	for (i = 0; i + 1 < want; i++) {
		pthread_t t;
		pthread_attr_t a;
		int r;
		pthread_attr_init(&a);
		pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
		r = pthread_create(&t, &a, worker, (void *)(size_t)(i + 1));
		pthread_attr_destroy(&a);
		if (r)
			break;
		p_nthr++;
	}
}

void par_for(size_t n, size_t min_per, par_fn fn, void *arg)
{
	size_t parts;
	pthread_once(&p_once, pool_start);
	parts = min_per ? n / min_per : n;
	if (parts > (size_t)p_nthr + 1)
		parts = (size_t)p_nthr + 1;
	if (parts <= 1) {
		fn(arg, 0, n);
		return;
	}
	pthread_mutex_lock(&p_call);
	pthread_mutex_lock(&p_lock);
	/* a straggler of the previous job may still be scanning its parts */
	while (atomic_load(&p_active))
		__builtin_ia32_pause();
	p_fn = fn;
	p_arg = arg;
	p_n = n;
	p_parts = parts;
	atomic_store(&p_done, 0);
	p_gen++;
	atomic_store(&p_pub, p_gen);
	pthread_cond_broadcast(&p_wake);
	pthread_mutex_unlock(&p_lock);
	run_parts(p_gen, 0);
	while (atomic_load(&p_done) < parts)
		__builtin_ia32_pause();
	pthread_mutex_unlock(&p_call);
}
