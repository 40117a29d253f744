/*
 * ref_bench.c -- CPU baseline (TEST INFRASTRUCTURE ONLY).
 *
 * Times the reference src/srtp (compiled from /root/reference sources by
 * oracle/Makefile, OpenSSL backend) on a bounded sample of the bench
 * workload: protect+unprotect pairs of RTP packets, one struct srtp per
 * thread (the reference context is single-threaded, include/re_srtp.h).
 *
 *   ref_bench <suite> <pkt_len> <npkts_per_thread> <threads> [nsessions]
 *
 * Prints one JSON line: {"pairs":N,"seconds":T,"mpairs_s":..,"gib_s":..}
 * GiB/s = N*L/(t_protect+t_unprotect) as in SURVEY.md 8(d).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>
#include <re.h>
#include <openssl/crypto.h>

struct job {
	int suite;
	size_t len;
	size_t npkts;
	int nsess;
	int mixed;
	unsigned seed;
	size_t bytes;
	int errs;
	double sec;
};

static pthread_barrier_t bar;

static double now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static const size_t keylen[6]  = {16, 16, 32, 32, 16, 32};
static const size_t saltlen[6] = {14, 14, 14, 14, 12, 12};

static uint64_t xs(uint64_t *s)
{
	*s ^= *s >> 12; *s ^= *s << 25; *s ^= *s >> 27;
	return *s * 0x2545F4914F6CDD1Dull;
}

static void *worker(void *arg)
{
	struct job *j = arg;
	struct srtp **tx, **rx;
	uint32_t *cnt;          /* per-session packet ordinal (seq) */
	struct mbuf *mb = mbuf_alloc(2048);
	uint64_t s = 0xC0FFEEull + j->seed;
	uint8_t key[46];
	size_t i;
	int k;

	tx = calloc((size_t)j->nsess, sizeof(*tx));
	rx = calloc((size_t)j->nsess, sizeof(*rx));
	cnt = calloc((size_t)j->nsess, sizeof(*cnt));
	for (k = 0; k < j->nsess; k++) {
		size_t b;
		for (b = 0; b < sizeof(key); b++)
			key[b] = (uint8_t)xs(&s);
		srtp_alloc(&tx[k], j->suite, key,
			   keylen[j->suite] + saltlen[j->suite], 0);
		srtp_alloc(&rx[k], j->suite, key,
			   keylen[j->suite] + saltlen[j->suite], 0);
	}

	pthread_barrier_wait(&bar);
	j->sec = now();
	for (i = 0; i < j->npkts; i++) {
		int sess = j->nsess > 1 ? (int)(xs(&s) % (uint64_t)j->nsess)
				        : 0;
		size_t len = j->mixed ? ((xs(&s) & 1) ? 1400 : 200) : j->len;
		/* every session sends seq 65000, 65001, ... (workload.py) */
		uint16_t seq = (uint16_t)(65000 + cnt[sess]++);
		uint8_t *p = mb->buf;
		size_t b;

		p[0] = 0x80; p[1] = 0;
		p[2] = seq >> 8; p[3] = seq & 0xff;
		memset(p + 4, 0, 4);
		p[8] = 0x01; p[9] = 0x02; p[10] = 0x03; p[11] = (uint8_t)sess;
		for (b = 12; b < len; b += 8) {
			uint64_t v = xs(&s);
			memcpy(p + b, &v, 8);
		}
		mb->pos = 0;
		mb->end = len;
		j->errs += srtp_encrypt(tx[sess], mb) != 0;
		mb->pos = 0;
		j->errs += srtp_decrypt(rx[sess], mb) != 0;
		j->bytes += len;
	}
	j->sec = now() - j->sec;

	for (k = 0; k < j->nsess; k++) {
		mem_deref(tx[k]);
		mem_deref(rx[k]);
	}
	free(tx);
	free(rx);
	free(cnt);
	mem_deref(mb);
	return NULL;
}

int main(int argc, char **argv)
{
	struct job *jobs;
	pthread_t *th;
	int suite, threads, nsess, t, errs = 0;
	size_t len, npkts, bytes = 0;
	double sec;

	if (argc < 5) {
		fprintf(stderr, "usage: %s suite len npkts threads [nsess]\n",
			argv[0]);
		return 2;
	}
	suite = atoi(argv[1]);
	len = (size_t)atol(argv[2]);
	npkts = (size_t)atol(argv[3]);
	threads = atoi(argv[4]);
	nsess = argc > 5 ? atoi(argv[5]) : 1;

	jobs = calloc((size_t)threads, sizeof(*jobs));
	th = calloc((size_t)threads, sizeof(*th));

	pthread_barrier_init(&bar, NULL, (unsigned)threads);
	for (t = 0; t < threads; t++) {
		jobs[t].suite = suite;
		jobs[t].len = len;
		jobs[t].mixed = len == 0;
		jobs[t].npkts = npkts;
		jobs[t].nsess = nsess;
		jobs[t].seed = (unsigned)t;
		pthread_create(&th[t], NULL, worker, &jobs[t]);
	}
	for (t = 0; t < threads; t++) {
		pthread_join(th[t], NULL);
		bytes += jobs[t].bytes;
		errs += jobs[t].errs;
	}
	/* timed region = slowest thread's packet loop (setup excluded) */
	sec = 0;
	for (t = 0; t < threads; t++)
		if (jobs[t].sec > sec)
			sec = jobs[t].sec;

	printf("{\"pairs\":%zu,\"seconds\":%.6f,\"mpairs_s\":%.6f,"
	       "\"gib_s\":%.6f,\"threads\":%d,\"errors\":%d,"
	       "\"openssl\":\"%s\"}\n",
	       npkts * (size_t)threads, sec,
	       (double)(npkts * (size_t)threads) / sec / 1e6,
	       (double)bytes / sec / (1024.0 * 1024 * 1024), threads, errs,
	       OpenSSL_version(OPENSSL_VERSION));
	return 0;
}
