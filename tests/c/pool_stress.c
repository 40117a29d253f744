/*
 * pool_stress.c -- the host worker pool (re_amd/csrc/host/pool.c) under
 * ThreadSanitizer / AddressSanitizer (tests/test_san_cpu.py builds it with
 * gcc -fsanitize=...).  T caller threads issue par_for jobs back to back
 * (calls serialise on the pool; workers steal parts), each job writing
 * disjoint slices of its caller's array, as the multi-session gather and
 * apply passes do; then every element is checked.  Exit 0 = all correct.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "pool.h"

#define T 4
#define N 5000
#define ROUNDS 200

struct job {
	unsigned *v;
	unsigned round;
};

static void body(void *arg, size_t a, size_t b)
{
	struct job *j = arg;
	size_t i;
	for (i = a; i < b; i++)
		j->v[i] += (unsigned)i ^ j->round;
}

static void *caller(void *arg)
{
	unsigned *v = calloc(N, sizeof(*v));
	size_t r, i;
	long bad = 0;
	(void)arg;
	for (r = 0; r < ROUNDS; r++) {
		struct job j = {v, (unsigned)r};
		par_for(N, 1 + r % 300, body, &j);
	}
	for (i = 0; i < N; i++) {
		unsigned want = 0;
		for (r = 0; r < ROUNDS; r++)
			want += (unsigned)i ^ (unsigned)r;
		bad += v[i] != want;
	}
	free(v);
	return (void *)bad;
}

int main(void)
{
	pthread_t t[T];
	long bad = 0;
	int k;
	for (k = 0; k < T; k++)
		pthread_create(&t[k], NULL, caller, NULL);
	for (k = 0; k < T; k++) {
		void *r;
		pthread_join(t[k], &r);
		bad += (long)r;
	}
	printf("pool_stress: %ld wrong\n", bad);
	return bad != 0;
}
