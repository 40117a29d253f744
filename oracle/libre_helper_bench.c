/*
 * libre_helper_bench.c -- one libre re_main thread receiving SRTP over
 * loopback (MEASUREMENT / TEST INFRASTRUCTURE, never part of the product).
 *
 * VERDICT r4 "next" 5: what a single-threaded libre application gains
 * from the batched GPU helper on libre's UDP helper chain, and at what
 * added latency.  libre's event loop and UDP layer come from
 * oracle/_ref/libre_net.so (the reference src/main, src/udp, ... compiled
 * by oracle/Makefile); a sender thread blasts config-2 SRTP datagrams
 * (1200-B RTP, AES_CM_128_HMAC_SHA1_80, one SSRC, seq from 65000; payload
 * word 0 = the packet's number, protected beforehand by the reference
 * src/srtp) from a plain socket, paced at a target rate, stamping each
 * send; the socket's receive handler stamps each plaintext it gets.
 * Modes:
 *   none  no SRTP helper (libre's own receive path, the ceiling);
 *   ref   the reference srtp_decrypt() per datagram on a udp helper
 *         (/root/reference/src/udp/udp.c:830-860 udp_register_helper --
 *         how an SRTP media transform sits on libre's chain);
 *   gpu   the product's batched helper (include/re_srtp_libre.h,
 *         re_amd/lib/libre_srtp_amd_libre.so, dlopened), `batch`
 *         datagrams per GPU call or `flush_ms` after the first.
 * Prints one JSON line: sent, received, dropped, lost, delivered pkt/s and
 * GiB/s, latency percentiles (send to handler, us, over the packets after
 * the first tenth), the re_main thread's CPU seconds per 1M packets.
 *
 *   helper_bench <none|ref|gpu> <npkts> <rate pkt/s, 0 = flat out>
 *                [batch flush_ms]
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <re.h>

#define LEN 1200
#define SLOT 1280
#define SSRC 0x01020304u
#define S0 65000u

static uint8_t *g_pkt;                  /* protected datagrams */
static uint32_t *g_plen;
static size_t g_n;
static double g_rate;
static uint64_t *g_t_send, *g_t_recv;
static volatile int g_sender_done;
static uint16_t g_port;
static size_t g_got, g_drop;
static uint64_t g_last_recv;
static struct tmr g_tmr;

static uint64_t now_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static void *sender(void *arg)
{
	struct sockaddr_in dst;
	int fd = socket(AF_INET, SOCK_DGRAM, 0);
	const uint64_t t0 = now_ns() + 20000000ull;     /* receiver ready */
	(void)arg;
	memset(&dst, 0, sizeof(dst));
	dst.sin_family = AF_INET;
	dst.sin_port = htons(g_port);
	dst.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
	while (now_ns() < t0)
		;
	for (size_t i = 0; i < g_n; i++) {
		if (g_rate > 0) {
			const uint64_t due = t0 + (uint64_t)((double)i * 1e9 /
							     g_rate);
			while (now_ns() < due)
				;
		}
		g_t_send[i] = now_ns();
		(void)sendto(fd, g_pkt + i * SLOT, g_plen[i], 0,
			     (struct sockaddr *)&dst, sizeof(dst));
	}
	close(fd);
	g_sender_done = 1;
	return NULL;
}

static int g_plain;                     /* mode none: SRTP as received */

static void recv_h(const struct sa *src, struct mbuf *mb, void *arg)
{
	uint32_t i;
	(void)src;
	(void)arg;
	if (g_plain) {
		/* the RTP timestamp (160 per packet) of the unprotected
		 * header */
		const uint8_t *b = mb->buf + mb->pos;
		if (mbuf_get_left(mb) < 12)
			return;
		i = ((uint32_t)b[4] << 24 | (uint32_t)b[5] << 16 |
		     (uint32_t)b[6] << 8 | b[7]) / 160u;
	}
	else {
		/* payload word 0 of the plaintext (srtp_decrypt leaves pos at
		 * the packet start, srtp.c:429) */
		if (mbuf_get_left(mb) < 16)
			return;
		memcpy(&i, mb->buf + mb->pos + 12, 4);
	}
	if (i < g_n && !g_t_recv[i]) {
		g_t_recv[i] = g_last_recv = now_ns();
		g_got++;
	}
	if (g_got == g_n)
		re_cancel();
}

/* the end of the run: every packet in, or 300 ms without one after the
 * sender finished */
static void watch(void *arg)
{
	(void)arg;
	if (g_sender_done && now_ns() - g_last_recv > 300000000ull) {
		re_cancel();
		return;
	}
	tmr_start(&g_tmr, 10, watch, NULL);
}

#ifdef HELPER_REF
/* the reference per-datagram transform on the helper chain: srtp_decrypt
 * (src/srtp/srtp.c:288-432); a failing datagram is dropped */
static bool ref_recv(struct sa *src, struct mbuf *mb, void *arg)
{
	(void)src;
	if (srtp_decrypt(arg, mb)) {
		g_drop++;
		return true;
	}
	return false;
}
#endif

static int cmp64(const void *a, const void *b)
{
	const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
	return x < y ? -1 : x > y;
}

int main(int argc, char **argv)
{
	const char *mode = argc > 1 ? argv[1] : "ref";
	const size_t batch = argc > 4 ? (size_t)atol(argv[4]) : 256;
	const unsigned flush = argc > 5 ? (unsigned)atoi(argv[5]) : 1;
	uint8_t key[30];
	struct srtp *tx = NULL, *rx = NULL;
	struct udp_sock *us = NULL;
	struct sa laddr, local;
	pthread_t th;
	struct rusage ru0, ru1;
	void *helper = NULL, *lib = NULL;
	struct udp_helper *uh = NULL;
	uint64_t t_start;
	int err;

	g_n = argc > 2 ? (size_t)atol(argv[2]) : 200000;
	g_rate = argc > 3 ? atof(argv[3]) : 0;
	g_pkt = calloc(g_n, SLOT);
	g_plen = calloc(g_n, 4);
	g_t_send = calloc(g_n, 8);
	g_t_recv = calloc(g_n, 8);
	if (!g_pkt || !g_plen || !g_t_send || !g_t_recv)
		return 1;
	for (size_t k = 0; k < sizeof(key); k++)
		key[k] = (uint8_t)(0x35 + 7 * k);
	if (libre_init())
		return 1;

	/* the datagrams, protected by the reference src/srtp linked into
	 * this program (the sender's side is not measured); the receiving
	 * context: the reference's (ref) or the product's (gpu: the LIBRE=1
	 * library dlopened, its srtp_alloc through the C-ABI) */
	g_plain = !strcmp(mode, "none");
	{
		if (srtp_alloc(&tx, SRTP_AES_CM_128_HMAC_SHA1_80, key, 30, 0) ||
		    srtp_alloc(&rx, SRTP_AES_CM_128_HMAC_SHA1_80, key, 30, 0)) {
			fprintf(stderr, "srtp_alloc failed\n");
			return 1;
		}
#ifndef HELPER_REF
		if (!strcmp(mode, "gpu")) {
			int (*alloc_)(struct srtp **, enum srtp_suite,
				      const uint8_t *, size_t, int);
			lib = dlopen(getenv("RE_SRTP_LIBRE_LIB") ?
				     getenv("RE_SRTP_LIBRE_LIB") :
				     "re_amd/lib/libre_srtp_amd_libre.so",
				     RTLD_NOW | RTLD_LOCAL);
			if (!lib) {
				fprintf(stderr, "dlopen: %s\n", dlerror());
				return 1;
			}
			alloc_ = (int (*)(struct srtp **, enum srtp_suite,
					  const uint8_t *, size_t, int))
				dlsym(lib, "srtp_alloc");
			rx = NULL;
			if (!alloc_ || alloc_(&rx, SRTP_AES_CM_128_HMAC_SHA1_80,
					      key, 30, 0)) {
				fprintf(stderr, "product srtp_alloc failed\n");
				return 1;
			}
		}
#endif
		struct mbuf *mb = mbuf_alloc(SLOT);
		for (size_t i = 0; i < g_n; i++) {
			const uint16_t seq = (uint16_t)(S0 + i);
			const uint32_t ts = (uint32_t)(160u * i);
			uint8_t h[12] = {0x80, 0, (uint8_t)(seq >> 8),
					 (uint8_t)seq, (uint8_t)(ts >> 24),
					 (uint8_t)(ts >> 16), (uint8_t)(ts >> 8),
					 (uint8_t)ts, (uint8_t)(SSRC >> 24),
					 (uint8_t)(SSRC >> 16), (uint8_t)(SSRC >> 8),
					 (uint8_t)SSRC};
			uint32_t word = (uint32_t)i;
			mbuf_rewind(mb);
			(void)mbuf_write_mem(mb, h, 12);
			(void)mbuf_write_mem(mb, (uint8_t *)&word, 4);
			for (size_t k = 16; k < LEN; k++)
				(void)mbuf_write_u8(mb, (uint8_t)(i * 31 + k));
			mb->pos = 0;
			if (srtp_encrypt(tx, mb)) {
				fprintf(stderr, "protect %zu failed\n", i);
				return 1;
			}
			memcpy(g_pkt + i * SLOT, mb->buf, mb->end);
			g_plen[i] = (uint32_t)mb->end;
		}
		mem_deref(mb);
	}

	(void)sa_set_str(&laddr, "127.0.0.1", 0);
	err = udp_listen(&us, &laddr, recv_h, NULL);
	if (!err)
		err = udp_sockbuf_set(us, 16 << 20);
	if (!err)
		err = udp_local_get(us, &local);
	if (err) {
		fprintf(stderr, "udp: %d\n", err);
		return 1;
	}
	g_port = sa_port(&local);
	if (!strcmp(mode, "gpu")) {
#ifndef HELPER_REF
		int (*ha)(void **, struct udp_sock *, int, struct srtp *,
			  struct srtp *, size_t, size_t, unsigned) =
			(int (*)(void **, struct udp_sock *, int, struct srtp *,
				 struct srtp *, size_t, size_t, unsigned))
			dlsym(lib, "srtp_udp_helper_alloc");
		err = ha ? ha(&helper, us, 0, rx, NULL, batch, SLOT, flush)
			 : ENOSYS;
#else
		err = ENOSYS;
#endif
	}
	else if (!strcmp(mode, "ref")) {
#ifdef HELPER_REF
		err = udp_register_helper(&uh, us, 0, NULL, ref_recv, rx);
#else
		err = ENOSYS;
#endif
	}
	if (err) {
		fprintf(stderr, "helper: %d\n", err);
		return 1;
	}

	g_last_recv = now_ns();
	tmr_init(&g_tmr);
	tmr_start(&g_tmr, 10, watch, NULL);
	getrusage(RUSAGE_THREAD, &ru0);
	t_start = now_ns();
	pthread_create(&th, NULL, sender, NULL);
	(void)re_main(NULL);
	getrusage(RUSAGE_THREAD, &ru1);
	pthread_join(th, NULL);
	tmr_cancel(&g_tmr);

	{
		/* latency over the steady state: the packets after the first
		 * tenth (the first GPU calls allocate their workspaces) */
		uint64_t *lat = calloc(g_n, 8), first = UINT64_MAX;
		size_t m = 0, mall = 0;
		for (size_t i = 0; i < g_n; i++) {
			if (g_t_send[i] && g_t_send[i] < first)
				first = g_t_send[i];
			if (g_t_recv[i]) {
				mall++;
				if (i >= g_n / 10)
					lat[m++] = g_t_recv[i] - g_t_send[i];
			}
		}
		qsort(lat, m, 8, cmp64);
		const double el = (double)(g_last_recv - first) * 1e-9;
		const double cpu = (double)(ru1.ru_utime.tv_sec -
					    ru0.ru_utime.tv_sec) +
			(double)(ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec) *
			1e-6 + (double)(ru1.ru_stime.tv_sec -
					ru0.ru_stime.tv_sec) +
			(double)(ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec) *
			1e-6;
		printf("{\"mode\":\"%s\",\"npkts\":%zu,\"rate\":%.0f,"
		       "\"batch\":%zu,\"flush_ms\":%u,\"received\":%zu,"
		       "\"dropped\":%zu,\"lost\":%zu,\"elapsed_s\":%.4f,"
		       "\"pkt_s\":%.0f,\"gib_s\":%.4f,"
		       "\"lat_us\":{\"p50\":%.1f,\"p90\":%.1f,\"p99\":%.1f,"
		       "\"max\":%.1f},\"loop_cpu_s_per_1M\":%.3f,"
		       "\"wall_s\":%.3f}\n",
		       mode, g_n, g_rate, batch, flush, g_got, g_drop,
		       g_n - g_got - g_drop, el, mall / (el > 0 ? el : 1),
		       mall * (double)LEN / (el > 0 ? el : 1) / (1 << 30),
		       m ? lat[m / 2] * 1e-3 : 0, m ? lat[m * 9 / 10] * 1e-3 : 0,
		       m ? lat[m * 99 / 100] * 1e-3 : 0,
		       m ? lat[m - 1] * 1e-3 : 0,
		       mall ? cpu / mall * 1e6 : 0,
		       (now_ns() - t_start) * 1e-9);
		free(lat);
	}
	mem_deref(helper);
	mem_deref(uh);
	mem_deref(us);
	return 0;
}
