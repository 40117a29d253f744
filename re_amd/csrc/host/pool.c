/*
 * pool.c -- a small persistent worker pool for the host passes over many
 * sessions (multi-session batches gather and apply one stream state per
 * session: 64K sessions are 64K cold heap objects, a memory-latency-bound
 * pointer chase that parallelises across cores).
 *
 * par_for(n, fn, arg) splits [0, n) into contiguous ranges, runs them on
 * the calling thread plus up to RE_SRTP_THREADS-1 workers (default 8) and
 * returns when every range is done.  Calls are serialised by a mutex; a
 * pool that cannot start degrades to running fn(arg, 0, n) inline.
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
static unsigned long p_gen;             /* job generation */
static par_fn p_fn;
static void *p_arg;
static size_t p_n, p_parts;
/* (generation << 32) | next part: a worker that wakes late for an old
 * generation cannot claim a part of the current one */
static _Atomic unsigned long long p_claim;
static atomic_size_t p_done;            /* parts finished */

static void run_parts(unsigned long gen)
{
	unsigned long long v = atomic_load(&p_claim);
	for (;;) {
		size_t k;
		if ((v >> 32) != (gen & 0xffffffffull) ||
		    (v & 0xffffffffull) >= p_parts)
			return;
		if (!atomic_compare_exchange_weak(&p_claim, &v, v + 1))
			continue;
		k = (size_t)(v & 0xffffffffull);
		p_fn(p_arg, p_n * k / p_parts, p_n * (k + 1) / p_parts);
		atomic_fetch_add(&p_done, 1);
		v = atomic_load(&p_claim);
	}
}

static void *worker(void *unused)
{
	unsigned long seen = 0;
	(void)unused;
	for (;;) {
		pthread_mutex_lock(&p_lock);
		while (p_gen == seen)
			pthread_cond_wait(&p_wake, &p_lock);
		seen = p_gen;
		pthread_mutex_unlock(&p_lock);
		run_parts(seen);
	}
	return NULL;
}

static void pool_start(void)
{
	const char *e = getenv("RE_SRTP_THREADS");
	long want = e ? atol(e) : 8;
	int i;
	if (want > POOL_MAX)
		want = POOL_MAX;
	for (i = 0; i + 1 < want; i++) {
		pthread_t t;
		pthread_attr_t a;
		pthread_attr_init(&a);
		pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
		if (pthread_create(&t, &a, worker, NULL)) {
			pthread_attr_destroy(&a);
			break;
		}
		pthread_attr_destroy(&a);
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
	p_fn = fn;
	p_arg = arg;
	p_n = n;
	p_parts = parts;
	atomic_store(&p_done, 0);
	p_gen++;
	atomic_store(&p_claim, (unsigned long long)(p_gen & 0xffffffffull)
				       << 32);
	pthread_cond_broadcast(&p_wake);
	pthread_mutex_unlock(&p_lock);
	run_parts(p_gen);
	while (atomic_load(&p_done) < parts)
		;
	pthread_mutex_unlock(&p_call);
}
