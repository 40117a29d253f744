/*
 * percall.c -- the per-packet drop-in path, measured (bench.py --percall).
 *
 * Every existing libre/baresip caller protects and unprotects one mbuf per
 * call (the reference API, src/srtp/srtp.c:183-432; baresip's SRTP media
 * helper calls it from the UDP helper chain, one datagram at a time).
 * This program times exactly that through libre_srtp_amd.so: srtp_encrypt
 * then srtp_decrypt of one 1200-byte RTP packet per call
 * (AES_CM_128_HMAC_SHA1_80, seq from 65000), per-call latency percentiles
 * and the single-thread rate, then T threads with a context pair each
 * (struct srtp is single-threaded, like the reference's).  Every packet's
 * round trip is checked.
 *
 *   percall <calls per thread> <threads...>   -> one JSON line
 *   (PERCALL_SUITE=<enum srtp_suite>, PERCALL_TUNE=name=value,...)
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "re_mbuf.h"
#include "re_mem.h"
#include "re_srtp.h"
#include "re_srtp_batch.h"

static double now_us(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

static int cmpd(const void *a, const void *b)
{
	const double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

struct job {
	long calls;
	int id;
	double *lat_e, *lat_d;          /* or NULL */
	long errors;
	double t0, t1;
};

/* the suite under test: PERCALL_SUITE = enum srtp_suite value (default
 * AES_CM_128_HMAC_SHA1_80); master key + salt lengths per suite */
static enum srtp_suite g_suite = SRTP_AES_CM_128_HMAC_SHA1_80;

static size_t key_len(enum srtp_suite s)
{
	switch (s) {
	case SRTP_AES_128_GCM:          return 16 + 12;
	case SRTP_AES_256_GCM:          return 32 + 12;
	case SRTP_AES_256_CM_HMAC_SHA1_32:
	case SRTP_AES_256_CM_HMAC_SHA1_80: return 32 + 14;
	default:                        return 16 + 14;
	}
}

static void *run(void *arg)
{
	struct job *j = arg;
	uint8_t key[46], pkt[1200];
	struct srtp *tx = NULL, *rx = NULL;
	struct mbuf *mb = mbuf_alloc(1400);
	long i;
	int k;

	for (k = 0; k < 46; k++)
		key[k] = (uint8_t)(17 * k + j->id);
	if (!mb || srtp_alloc(&tx, g_suite, key, key_len(g_suite), 0) ||
	    srtp_alloc(&rx, g_suite, key, key_len(g_suite), 0)) {
		j->errors = -1;
		return NULL;
	}
	for (k = 12; k < 1200; k++)
		pkt[k] = (uint8_t)(k * 7 + j->id);
	pkt[0] = 0x80;
	pkt[1] = 0;
	pkt[8] = 0x0B; pkt[9] = 0xAD; pkt[10] = 0xCA; pkt[11] = (uint8_t)j->id;
	j->t0 = now_us();
	for (i = 0; i < j->calls; i++) {
		const uint16_t seq = (uint16_t)(65000 + i);
		double a, b, c;
		pkt[2] = (uint8_t)(seq >> 8);
		pkt[3] = (uint8_t)seq;
		pkt[4] = (uint8_t)(i >> 24); pkt[5] = (uint8_t)(i >> 16);
		pkt[6] = (uint8_t)(i >> 8); pkt[7] = (uint8_t)i;
		mb->pos = 0;
		mb->end = 0;
		memcpy(mb->buf, pkt, sizeof(pkt));
		mb->end = sizeof(pkt);
		a = now_us();
		if (srtp_encrypt(tx, mb))
			j->errors++;
		b = now_us();
		mb->pos = 0;
		if (srtp_decrypt(rx, mb))
			j->errors++;
		c = now_us();
		if (mb->end != sizeof(pkt) || memcmp(mb->buf, pkt, sizeof(pkt)))
			j->errors++;
		if (j->lat_e) {
			j->lat_e[i] = b - a;
			j->lat_d[i] = c - b;
		}
	}
	j->t1 = now_us();
	mem_deref(tx);
	mem_deref(rx);
	mem_deref(mb);
	return NULL;
}

static double pct(double *v, long n, double p)
{
	return v[(long)(p * (n - 1))];
}

int main(int argc, char **argv)
{
	const long calls = argc > 1 ? atol(argv[1]) : 20000;
	if (getenv("PERCALL_SUITE"))
		g_suite = (enum srtp_suite)atoi(getenv("PERCALL_SUITE"));
	if (getenv("PERCALL_TUNE")) {
		/* A/B knobs: "name=value,name=value" (srtp_gpu_tune) */
		char *spec = strdup(getenv("PERCALL_TUNE")), *tok, *sp = NULL;
		for (tok = strtok_r(spec, ",", &sp); tok;
		     tok = strtok_r(NULL, ",", &sp)) {
			char *eq = strchr(tok, '=');
			if (eq)
				*eq = 0;
			if (srtp_gpu_tune(tok, eq ? atol(eq + 1) : 1)) {
				fprintf(stderr, "percall: bad knob %s\n", tok);
				return 2;
			}
		}
		free(spec);
	}
	struct job j0;
	int a;

	/* single thread, latency per call */
	memset(&j0, 0, sizeof(j0));
	j0.calls = calls;
	j0.lat_e = calloc(calls, sizeof(double));
	j0.lat_d = calloc(calls, sizeof(double));
	{       /* warm up: workspaces, table, code objects */
		struct job w = {200, 99, NULL, NULL, 0, 0, 0};
		run(&w);
	}
	const uint64_t c0 = srtp_gpu_counter("small_launches"),
		       l0 = srtp_gpu_counter("small_ns_launch"),
		       s0 = srtp_gpu_counter("small_ns_sync"),
		       m0 = srtp_gpu_counter("mbufs_ns");
	run(&j0);
	const double nl = (double)(srtp_gpu_counter("small_launches") - c0);
	const double us_launch = nl ? (srtp_gpu_counter("small_ns_launch") -
				       l0) / nl / 1e3 : 0;
	const double us_sync = nl ? (srtp_gpu_counter("small_ns_sync") - s0) /
				    nl / 1e3 : 0;
	const double us_mbufs = (srtp_gpu_counter("mbufs_ns") - m0) /
				(2.0 * calls) / 1e3;
	if (j0.errors) {
		fprintf(stderr, "percall: %ld errors (%s)\n", j0.errors,
			srtp_gpu_error());
		return 1;
	}
	qsort(j0.lat_e, calls, sizeof(double), cmpd);
	qsort(j0.lat_d, calls, sizeof(double), cmpd);
	printf("{\"calls\":%ld,\"pkt_len\":1200,"
	       "\"suite\":\"%s\","
	       "\"encrypt_us\":{\"p50\":%.2f,\"p99\":%.2f,\"min\":%.2f},"
	       "\"decrypt_us\":{\"p50\":%.2f,\"p99\":%.2f,\"min\":%.2f},"
	       "\"pairs_per_s_1thread\":%.0f,"
	       "\"per_call_us\":{\"run_mbufs\":%.2f,\"small_launch\":%.2f,"
	       "\"small_sync\":%.2f},\"threads\":[",
	       calls, srtp_suite_name(g_suite),
	       pct(j0.lat_e, calls, 0.5), pct(j0.lat_e, calls, 0.99),
	       j0.lat_e[0], pct(j0.lat_d, calls, 0.5),
	       pct(j0.lat_d, calls, 0.99), j0.lat_d[0],
	       calls / ((j0.t1 - j0.t0) * 1e-6), us_mbufs, us_launch, us_sync);
	for (a = 2; a < argc; a++) {
		const int T = atoi(argv[a]);
		struct job *js = calloc(T, sizeof(*js));
		pthread_t *th = calloc(T, sizeof(*th));
		double t0 = 1e300, t1 = 0;
		long err = 0;
		int t;
		const uint64_t b0 = srtp_gpu_counter("pcbatches"),
			       p0 = srtp_gpu_counter("pcpackets"),
			       f0 = srtp_gpu_counter("pcfused"),
			       sl0 = srtp_gpu_counter("small_launches"),
			       sy0 = srtp_gpu_counter("small_ns_sync"),
			       fp0 = srtp_gpu_counter("fused_ns_prep"),
			       fq0 = srtp_gpu_counter("fused_ns_post"),
			       mb0 = srtp_gpu_counter("mbufs_ns");
		for (t = 0; t < T; t++) {
			js[t].calls = calls / 4 > 1000 ? calls / 4 : 1000;
			js[t].id = t;
			pthread_create(&th[t], NULL, run, &js[t]);
		}
		for (t = 0; t < T; t++) {
			pthread_join(th[t], NULL);
			t0 = js[t].t0 < t0 ? js[t].t0 : t0;
			t1 = js[t].t1 > t1 ? js[t].t1 : t1;
			err += js[t].errors;
		}
		const double nb = (double)(srtp_gpu_counter("pcbatches") - b0);
		/* the launches' own time (run_mbufs_: host plan, launch,
		 * sync, unpack) against the wall time per launch */
		printf("%s{\"threads\":%d,\"pairs_per_s\":%.0f,\"errors\":%ld,"
		       "\"packets_per_launch\":%.1f,\"us_per_launch\":%.1f,"
		       "\"wall_us_per_launch\":%.1f,\"fused_frac\":%.2f,"
		       "\"small_sync_us\":%.1f,\"fused_prep_us\":%.1f,"
		       "\"fused_post_us\":%.1f}",
		       a > 2 ? "," : "", T, T * js[0].calls / ((t1 - t0) * 1e-6),
		       err, nb ? (srtp_gpu_counter("pcpackets") - p0) / nb : 0,
		       nb ? (srtp_gpu_counter("mbufs_ns") - mb0) / nb / 1e3 : 0,
		       nb ? (t1 - t0) / nb : 0,
		       nb ? (srtp_gpu_counter("pcfused") - f0) / nb : 0,
		       srtp_gpu_counter("small_launches") > sl0 ?
		       (srtp_gpu_counter("small_ns_sync") - sy0) / 1e3 /
		       (double)(srtp_gpu_counter("small_launches") - sl0) : 0,
		       srtp_gpu_counter("pcfused") > f0 ?
		       (srtp_gpu_counter("fused_ns_prep") - fp0) / 1e3 /
		       (double)(srtp_gpu_counter("pcfused") - f0) : 0,
		       srtp_gpu_counter("pcfused") > f0 ?
		       (srtp_gpu_counter("fused_ns_post") - fq0) / 1e3 /
		       (double)(srtp_gpu_counter("pcfused") - f0) : 0);
		free(js);
		free(th);
	}
	printf("]}\n");
	return 0;
}
