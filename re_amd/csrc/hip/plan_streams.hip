/*
 * plan_streams.hip -- device planning of a single-session RTP batch whose
 * packets belong to up to SRTP_MAX_STREAMS (8) streams of that session
 * (one struct srtp, several SSRCs: stream.c:16-17, 29-67).
 *
 * The reference runs one sequential state machine per stream (srtp_encrypt
 * srtp.c:203-215, 279-280; srtp_decrypt srtp.c:310-321, 426-427;
 * srtp_get_index misc.c:22-41; srtp_replay_check replay.c:32-62) and finds
 * or creates the stream by SSRC on every packet (stream_get_seq,
 * stream.c:87-109; a 9th SSRC is ENOSR).  Streams are independent, so the
 * single-stream speculation of srtp_kernels.hip (k_plan_*) holds per
 * stream: packet i of stream k is assumed to see s_l = seq of the previous
 * packet of stream k, ROC rollovers are prefix-summed per stream, and every
 * assumption is verified.  No sort: the previous packet of the same stream
 * is found with one ballot per stream inside a wave and per-stream prefix
 * maxima across waves and blocks.
 *
 *   k_sp_ssrc   per block: the distinct SSRCs in first-appearance order,
 *               with their first and last packet index
 *   k_sp_merge  one workgroup: the session's stream table after the batch
 *               (known streams, then new SSRCs by first appearance -- the
 *               order stream_new appends them), and per block and stream
 *               the last packet index of the blocks before it
 *   k_sp_count  per packet: stream, previous packet of the stream, the s_l
 *               it sees, rollover, every check of k_plan_count; per block
 *               and stream: rollovers and packets
 *   k_sp_scan   one workgroup: exclusive per-stream prefix sums over blocks
 *   k_sp_desc   per packet: ROC, index, replay check against the previous
 *               packet of the stream, descriptor; per stream: the tail of
 *               indices for the final replay window and the final s_l
 *   k_sp_final  launch guards of the crypto kernels
 *
 * Any verification miss (or a 9th stream) sets out->base.fail: the host
 * then plans sequentially and the guarded launches do nothing.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include "../srtpgpu.h"

#define SP_BLOCK 1024
#define SP_WAVES (SP_BLOCK / 64)
#define SP_K SGPU_SP_MAX
#define SP_SCAN 1024
#define SP_H 16                 /* per-block SSRC hash slots */

/* the blocks' distinct SSRCs: SP_H hash slots per block, stored slot-major
 * (structure of arrays, nb words per row: consecutive blocks coalesce):
 * rows [0, SP_H) SSRC, [SP_H, 2 SP_H) first packet (~0: empty slot),
 * [2 SP_H, 3 SP_H) last packet */
#define SP_BL_SSRC(bl, nb, j, b)  (bl)[(size_t)(j) * (nb) + (b)]
#define SP_BL_FIRST(bl, nb, j, b) (bl)[(size_t)(SP_H + (j)) * (nb) + (b)]
#define SP_BL_LAST(bl, nb, j, b)  (bl)[(size_t)(2 * SP_H + (j)) * (nb) + (b)]

__device__ __forceinline__ uint64_t sp_desc(uint64_t ix, uint32_t flags)
{
	return (ix & 0xffffull) | ((uint64_t)(uint32_t)(ix >> 16) << 16) |
	       ((uint64_t)flags << 48);
}

/* srtp_get_index (misc.c:22-41), including the int wrap of roc +- 1 */
__device__ __forceinline__ int32_t sp_v(uint32_t roc, uint32_t s_l,
					uint32_t seq)
{
	if (s_l < 32768)
		return ((int)seq - (int)s_l > 32768) ? (int32_t)(roc - 1)
						     : (int32_t)roc;
	return ((int)s_l - 32768 > (int)seq) ? (int32_t)(roc + 1)
					     : (int32_t)roc;
}

/* ROC rollover seen by a packet (srtp.c:208-213, 318-321) */
__device__ __forceinline__ bool sp_wrap(uint32_t seq, uint32_t sb)
{
	return (int)seq - (int)sb <= -32768;
}

__device__ __forceinline__ int32_t sp_top(uint64_t m)
{
	return 63 - __clzll((long long)m);
}

__global__ void __launch_bounds__(SP_BLOCK)
k_sp_ssrc(const struct sgpu_hdr *hdr, uint32_t n, uint32_t *bl,
	  struct sgpu_splan_out *out)
{
	__shared__ unsigned long long hkey[SP_H];
	__shared__ uint32_t hfirst[SP_H], hlast[SP_H], hn;
	const uint32_t i = blockIdx.x * SP_BLOCK + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	const uint32_t base = blockIdx.x * SP_BLOCK + wv * 64u;
	if (threadIdx.x < SP_H) {
		hkey[threadIdx.x] = 0;
		hfirst[threadIdx.x] = ~0u;
		hlast[threadIdx.x] = 0;
	}
	if (threadIdx.x == 0)
		hn = 0;
	bool valid = false;
	uint32_t ssrc = 0;
	if (i < n) {
		const struct sgpu_hdr h = hdr[i];
		if (h.hdr_len == 0xffffffffu)
			atomicOr(&out->base.fail, (uint32_t)SPF_PARSE);
		else {
			valid = true;
			ssrc = h.ssrc;
		}
	}
	__syncthreads();
	/* the wave's distinct SSRCs (one ballot each) into the block's LDS
	 * hash set: first and last packet per SSRC */
	uint64_t pend = __ballot(valid);
	bool over = false;
	while (pend) {
		const int ld = __ffsll((long long)pend) - 1;
		const uint32_t s = (uint32_t)__shfl((int)ssrc, ld);
		const uint64_t m = __ballot(valid && ssrc == s);
		if (lane == 0) {
			const unsigned long long key = 1ull << 32 | s;
			uint32_t j = (s * 0x9E3779B1u) >> 28, q;
			for (q = 0; q < SP_H; q++, j = (j + 1) & (SP_H - 1)) {
				const unsigned long long o =
					atomicCAS(&hkey[j], 0ull, key);
				if (o == 0ull || o == key) {
					if (o == 0ull)
						atomicAdd(&hn, 1u);
					atomicMin(&hfirst[j], base + (uint32_t)ld);
					atomicMax(&hlast[j], base + (uint32_t)sp_top(m));
					break;
				}
			}
			if (q == SP_H)
				over = true;
		}
		pend &= ~m;
	}
	if (over)
		atomicOr(&out->base.fail, (uint32_t)SPF_SSRC);
	__syncthreads();
	if (threadIdx.x == 0 && hn > SP_K)
		atomicOr(&out->base.fail, (uint32_t)SPF_SSRC);
	const uint32_t t = threadIdx.x, nb = gridDim.x, b = blockIdx.x;
	if (t < SP_H)
		SP_BL_SSRC(bl, nb, t, b) = (uint32_t)hkey[t];
	else if (t < 2 * SP_H)
		SP_BL_FIRST(bl, nb, t - SP_H, b) = hfirst[t - SP_H];
	else if (t < 3 * SP_H)
		SP_BL_LAST(bl, nb, t - 2 * SP_H, b) = hlast[t - 2 * SP_H];
}

/* block-wide exclusive scans over SP_SCAN threads of the per-thread
 * values part[0..SP_K)[t] in LDS (in place), by wave shuffles and then the
 * wave totals; tot[q] = the block total.  Slot loops stay rolled: the
 * values live in LDS, not in register arrays (no scratch). */
__device__ __forceinline__ void sp_scan_max(int32_t (*part)[SP_SCAN],
					    int32_t *tot)
{
	__shared__ int32_t wt[SP_SCAN / 64][SP_K];
	const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
#pragma unroll 1
	for (uint32_t q = 0; q < SP_K; q++) {
		int32_t v = part[q][t];
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const int32_t y = __shfl_up(v, d);
			if ((int)lane >= d)
				v = max(v, y);
		}
		const int32_t ex = __shfl_up(v, 1);
		if (lane == 63)
			wt[wv][q] = v;
		part[q][t] = lane ? ex : -1;
	}
	__syncthreads();
#pragma unroll 1
	for (uint32_t q = 0; q < SP_K; q++) {
		int32_t pre = -1, all = -1;
		for (uint32_t w = 0; w < SP_SCAN / 64; w++) {
			const int32_t v = wt[w][q];
			if (w < wv)
				pre = max(pre, v);
			all = max(all, v);
		}
		part[q][t] = max(part[q][t], pre);
		if (t == 0)
			tot[q] = all;
	}
	__syncthreads();
}

__device__ __forceinline__ void sp_scan_add(uint2 (*part)[SP_SCAN], uint2 *tot)
{
	__shared__ uint2 wt[SP_SCAN / 64][SP_K];
	const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
#pragma unroll 1
	for (uint32_t q = 0; q < SP_K; q++) {
		uint32_t a = part[q][t].x, b = part[q][t].y;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const uint32_t ya = __shfl_up(a, d), yb = __shfl_up(b, d);
			if ((int)lane >= d) {
				a += ya;
				b += yb;
			}
		}
		const uint32_t ea = __shfl_up(a, 1), eb = __shfl_up(b, 1);
		if (lane == 63)
			wt[wv][q] = make_uint2(a, b);
		part[q][t] = lane ? make_uint2(ea, eb) : make_uint2(0, 0);
	}
	__syncthreads();
#pragma unroll 1
	for (uint32_t q = 0; q < SP_K; q++) {
		uint2 pre = make_uint2(0, 0), all = make_uint2(0, 0);
		for (uint32_t w = 0; w < SP_SCAN / 64; w++) {
			const uint2 v = wt[w][q];
			if (w < wv) {
				pre.x += v.x;
				pre.y += v.y;
			}
			all.x += v.x;
			all.y += v.y;
		}
		part[q][t].x += pre.x;
		part[q][t].y += pre.y;
		if (t == 0)
			tot[q] = all;
	}
	__syncthreads();
}

/* slot of SSRC s in the table (SP_K: none) */
__device__ __forceinline__ uint32_t sp_slot(const uint32_t *tab, uint32_t nt,
					    uint32_t s)
{
	uint32_t k = SP_K;
	for (uint32_t q = 0; q < nt; q++)
		if (tab[q] == s)
			k = q;
	return k;
}

__global__ void __launch_bounds__(SP_SCAN)
k_sp_merge(const struct sgpu_splan_in in, const uint32_t *bl, uint32_t nb,
	   int32_t *bprev, struct sgpu_splan_out *out)
{
	__shared__ uint32_t tab[SP_K];
	__shared__ uint32_t ntab;
	/* new SSRCs of the batch: LDS hash set with the first packet of each */
	__shared__ unsigned long long hkey[SP_H];
	__shared__ uint32_t hfirst[SP_H], over;
	const uint32_t t = threadIdx.x;
	const uint32_t per = (nb + SP_SCAN - 1) / SP_SCAN;
	const uint32_t a = t * per, e = min(a + per, nb);
#pragma unroll
	for (uint32_t q = 0; q < SP_K; q++)
		if (t == q)
			tab[q] = q < in.nst ? in.st[q].ssrc : 0u;
	if (t < SP_H) {
		hkey[t] = 0;
		hfirst[t] = ~0u;
	}
	if (t == 0) {
		ntab = in.nst < SP_K ? in.nst : SP_K;
		over = 0;
	}
	__syncthreads();
	const uint32_t nt0 = ntab;
	for (uint32_t b = a; b < e; b++) {
		for (uint32_t j = 0; j < SP_H; j++) {
			const uint32_t f = SP_BL_FIRST(bl, nb, j, b);
			if (f == ~0u)
				continue;
			const uint32_t s = SP_BL_SSRC(bl, nb, j, b);
			if (sp_slot(tab, nt0, s) < SP_K)
				continue;
			const unsigned long long key = 1ull << 32 | s;
			uint32_t h = (s * 0x9E3779B1u) >> 28, q;
			for (q = 0; q < SP_H; q++, h = (h + 1) & (SP_H - 1)) {
				const unsigned long long o =
					atomicCAS(&hkey[h], 0ull, key);
				if (o == 0ull || o == key) {
					atomicMin(&hfirst[h], f);
					break;
				}
			}
			if (q == SP_H)
				over = 1;
		}
	}
	__syncthreads();
	/* append them by first appearance (stream_new order): entry j's rank
	 * is the number of entries that appear before it */
	if (t < SP_H && hfirst[t] != ~0u) {
		uint32_t r = 0;
		for (uint32_t q = 0; q < SP_H; q++)
			r += hfirst[q] < hfirst[t];
		if (nt0 + r < SP_K)
			tab[nt0 + r] = (uint32_t)hkey[t];
		else
			over = 1;       /* a 9th stream: ENOSR on the host */
		atomicAdd(&ntab, 1u);
	}
	__syncthreads();
	if (t == 0 && over)
		atomicOr(&out->base.fail, (uint32_t)SPF_SSRC);
	const uint32_t nt = min(ntab, (uint32_t)SP_K);
	/* per stream: the last packet of each thread's blocks, then the
	 * exclusive prefix maximum over the threads (blocks in order) */
	__shared__ int32_t part[SP_K][SP_SCAN];
	__shared__ int32_t tot[SP_K];
#pragma unroll 1
	for (uint32_t q = 0; q < SP_K; q++)
		part[q][t] = -1;
	for (uint32_t b = a; b < e; b++) {
		for (uint32_t j = 0; j < SP_H; j++) {
			if (SP_BL_FIRST(bl, nb, j, b) == ~0u)
				continue;
			const uint32_t k = sp_slot(tab, nt, SP_BL_SSRC(bl, nb, j, b));
			if (k < SP_K)
				part[k][t] = max(part[k][t],
						 (int32_t)SP_BL_LAST(bl, nb, j, b));
		}
	}
	sp_scan_max(part, tot);
	for (uint32_t b = a; b < e; b++) {
#pragma unroll 1
		for (uint32_t q = 0; q < SP_K; q++)
			bprev[q * nb + b] = part[q][t];
		for (uint32_t j = 0; j < SP_H; j++) {
			if (SP_BL_FIRST(bl, nb, j, b) == ~0u)
				continue;
			const uint32_t k = sp_slot(tab, nt, SP_BL_SSRC(bl, nb, j, b));
			if (k < SP_K)
				part[k][t] = max(part[k][t],
						 (int32_t)SP_BL_LAST(bl, nb, j, b));
		}
	}
	if (t < SP_K) {
		out->ssrc[t] = tab[t];
		out->last[t] = tot[t];
	}
	if (t == 0)
		out->nst = nt;
}

/* the stream table and the pre-batch states, staged in LDS */
struct sp_lds {
	uint32_t tab[SP_K];
	int32_t last[SP_K];
	struct sgpu_sstate st[SP_K];
	uint32_t nt, nst;
};

__device__ __forceinline__ void sp_stage(const struct sgpu_splan_in &in,
					 const struct sgpu_splan_out *out,
					 struct sp_lds &L)
{
	const uint32_t t = threadIdx.x;
	if (t < SP_K) {
		L.tab[t] = out->ssrc[t];
		L.last[t] = out->last[t];
	}
#pragma unroll
	for (uint32_t q = 0; q < SP_K; q++)
		if (t == 32 + q)
			L.st[q] = in.st[q];
	if (t == 0) {
		L.nt = out->nst;
		L.nst = in.nst;
	}
	__syncthreads();
}

/* s_l the packet of stream k sees when no earlier packet of the batch
 * belongs to stream k: the stored one, or its own seq for a new stream or
 * one whose s_l is not set yet (stream_get_seq, stream.c:99-103) */
__device__ __forceinline__ uint32_t sp_sb0(const struct sp_lds &L,
					   uint32_t k, uint32_t seq)
{
	if (k >= L.nst || !(L.st[k].flags & SST_SL_SET))
		return seq;
	return L.st[k].s_l;
}

__global__ void __launch_bounds__(SP_BLOCK)
k_sp_count(const struct sgpu_splan_in in, const struct sgpu_hdr *hdr,
	   const uint32_t *pos, const uint32_t *end, const uint32_t *cap,
	   uint64_t asz, const int32_t *bprev, uint32_t *rec, int32_t *prv,
	   uint32_t *bcnt, struct sgpu_splan_out *out)
{
	__shared__ struct sp_lds L;
	__shared__ int32_t wlast[SP_WAVES][SP_K];
	__shared__ uint32_t wcnt[SP_WAVES][SP_K];
	sp_stage(in, out, L);
	const uint32_t i = blockIdx.x * SP_BLOCK + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	const uint32_t base = blockIdx.x * SP_BLOCK + wv * 64u;
	struct sgpu_hdr h = {0, 0, 0, 0xffffffffu};
	uint32_t k = SP_K, f = 0;
	if (i < in.n) {
		h = hdr[i];
		if (h.hdr_len == 0xffffffffu)
			f |= SPF_PARSE;
		else {
#pragma unroll
			for (uint32_t q = 0; q < SP_K; q++)
				if (q < L.nt && L.tab[q] == h.ssrc)
					k = q;
			if (k == SP_K)
				f |= SPF_SSRC;
		}
	}
	uint64_t mine = 0;
#pragma unroll
	for (uint32_t q = 0; q < SP_K; q++) {
		const uint64_t b = __ballot(k == q);
		if (k == q)
			mine = b;
		if (lane == 0)
			wlast[wv][q] = b ? (int32_t)base + sp_top(b) : -1;
	}
	__syncthreads();
	/* the previous packet of the same stream */
	int32_t p = -1;
	if (k < SP_K) {
		const uint64_t lt = mine & ((1ull << lane) - 1ull);
		if (lt) {
			p = (int32_t)base + sp_top(lt);
		}
		else {
			for (int w = (int)wv - 1; w >= 0 && p < 0; w--)
				p = wlast[w][k];
			if (p < 0)
				p = bprev[k * gridDim.x + blockIdx.x];
		}
	}
	bool wrap = false;
	if (k < SP_K) {
		const uint32_t seq = h.seq;
		const uint32_t sb = p >= 0 ? (uint32_t)hdr[p].seq : sp_sb0(L, k, seq);
		const uint32_t hl0 = hdr[0].hdr_len;
		if (hl0 == 0xffffffffu)
			f |= SPF_PARSE;
		else if (((h.hdr_len ^ hl0) >> 2) & 3u)
			f |= SPF_CLASS;
		if (!in.prot && end[i] - pos[i] - h.hdr_len < in.tag)
			f |= SPF_PARSE;
		if (!in.prot && (int)seq - (int)sb > 32768)
			f |= SPF_TIMEOUT;
		wrap = sp_wrap(seq, sb);
		/* the next packet of the stream sees s_l = seq only if this one
		 * left it so */
		if ((int32_t)i != L.last[k] && !wrap && seq < sb)
			f |= SPF_ORDER;
		rec[i] = sb | (wrap ? 1u << 16 : 0u) | k << 17;
		prv[i] = p;
	}
	else if (i < in.n) {
		rec[i] = (uint32_t)SP_K << 17;  /* unplanned (the plan fails) */
		prv[i] = -1;
	}
	if (i < in.n) {
		if (end[i] - pos[i] >= in.maxlen)
			f |= SPF_SIZE;
		if ((pos[i] & 3u) || pos[i] > end[i] || end[i] > asz ||
		    (cap && (end[i] > cap[i] || cap[i] > asz)))
			f |= SPF_BAD;
		if (in.prot && cap &&
		    (uint64_t)end[i] + in.need > (uint64_t)cap[i])
			f |= SPF_CAP;
		if (i == 0)
			out->base.hl0 = h.hdr_len;
		if (f)
			atomicOr(&out->base.fail, f);
	}
	const uint64_t wm = __ballot(wrap);
#pragma unroll
	for (uint32_t q = 0; q < SP_K; q++) {
		const uint64_t b = __ballot(k == q);
		if (lane == 0)
			wcnt[wv][q] = (uint32_t)__popcll(b & wm) |
				      (uint32_t)__popcll(b) << 16;
	}
	__syncthreads();
	if (threadIdx.x < SP_K) {
		uint32_t s = 0;
		for (uint32_t w = 0; w < SP_WAVES; w++)
			s += wcnt[w][threadIdx.x];
		bcnt[threadIdx.x * gridDim.x + blockIdx.x] = s;
	}
}

/* exclusive per-stream prefix sums of the block counts (one workgroup):
 * bpre[b][k] = (rollovers, packets) of stream k in the blocks before b */
__global__ void __launch_bounds__(SP_SCAN)
k_sp_scan(const uint32_t *bcnt, uint32_t nb, uint2 *bpre,
	  struct sgpu_splan_out *out)
{
	const uint32_t t = threadIdx.x;
	const uint32_t per = (nb + SP_SCAN - 1) / SP_SCAN;
	const uint32_t a = t * per, e = min(a + per, nb);
	__shared__ uint2 part[SP_K][SP_SCAN];
	__shared__ uint2 tot[SP_K];
#pragma unroll 1
	for (uint32_t q = 0; q < SP_K; q++)
		part[q][t] = make_uint2(0, 0);
	for (uint32_t b = a; b < e; b++) {
#pragma unroll 1
		for (uint32_t q = 0; q < SP_K; q++) {
			const uint32_t v = bcnt[q * nb + b];
			part[q][t].x += v & 0xffffu;
			part[q][t].y += v >> 16;
		}
	}
	sp_scan_add(part, tot);
	for (uint32_t b = a; b < e; b++) {
#pragma unroll 1
		for (uint32_t q = 0; q < SP_K; q++) {
			const uint32_t v = bcnt[q * nb + b];
			bpre[q * nb + b] = part[q][t];
			part[q][t].x += v & 0xffffu;
			part[q][t].y += v >> 16;
		}
	}
	if (t < SP_K) {
		out->wraps[t] = tot[t].x;
		out->cnt[t] = tot[t].y;
	}
}

__global__ void __launch_bounds__(SP_BLOCK)
k_sp_desc(const struct sgpu_splan_in in, const struct sgpu_hdr *hdr,
	  const uint32_t *rec, const int32_t *prv, const uint2 *bpre,
	  uint64_t *desc, struct sgpu_splan_out *out)
{
	__shared__ struct sp_lds L;
	__shared__ uint32_t wc[SP_WAVES][SP_K];
	__shared__ uint32_t cnt[SP_K];
	/* a plan already rejected: nothing behind it runs */
	if (out->base.fail)
		return;
	if (threadIdx.x < SP_K)
		cnt[threadIdx.x] = out->cnt[threadIdx.x];
	sp_stage(in, out, L);
	const uint32_t i = blockIdx.x * SP_BLOCK + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	uint32_t k = SP_K, sb = 0;
	bool wrap = false;
	if (i < in.n) {
		const uint32_t r = rec[i];
		k = r >> 17;
		sb = r & 0xffffu;
		wrap = (r >> 16) & 1u;
		if (k >= SP_K)          /* unplanned packet (the plan failed) */
			k = SP_K;
	}
	const uint64_t wm = __ballot(wrap);
	uint64_t mine = 0;
#pragma unroll
	for (uint32_t q = 0; q < SP_K; q++) {
		const uint64_t b = __ballot(k == q);
		if (k == q)
			mine = b;
		if (lane == 0)
			wc[wv][q] = (uint32_t)__popcll(b & wm) |
				    (uint32_t)__popcll(b) << 16;
	}
	__syncthreads();
	if (k >= SP_K)
		return;
	const uint64_t lt = mine & ((1ull << lane) - 1ull);
	const uint2 bp = bpre[k * gridDim.x + blockIdx.x];
	uint32_t wb = bp.x + (uint32_t)__popcll(lt & wm);
	uint32_t ord = bp.y + (uint32_t)__popcll(lt);
	for (uint32_t w = 0; w < wv; w++) {
		wb += wc[w][k] & 0xffffu;
		ord += wc[w][k] >> 16;
	}
	const struct sgpu_sstate S = L.st[k];
	const bool known = k < L.nst;
	const uint32_t seq = hdr[i].seq;
	/* ROC after this packet's own rollover */
	const uint32_t roc = (known ? S.roc : 0u) + wb + (wrap ? 1u : 0u);
	uint64_t ix;
	uint32_t fl = SD_RUN | SD_CIPHER;
	if (in.prot) {
		ix = 65536ull * roc + seq;              /* srtp.c:215 */
	}
	else {
		const int32_t v = sp_v(roc, wrap ? 0u : sb, seq);
		ix = seq + (uint64_t)(int64_t)v * 65536ull;
		if ((uint32_t)v != roc)
			fl |= (uint32_t)v + 1u == roc ? SD_ROC_P1 : SD_ROC_M1;
		const uint64_t lix = known ? S.lix : 0ull;
		const uint64_t bm = known ? S.bitmap : 0ull;
		/* replay: every packet of the stream new (replay.c:32-62) */
		const int32_t p = prv[i];
		bool ok;
		if (p < 0) {
			if (ix > lix) {
				ok = true;
			}
			else {
				const uint64_t d = lix - ix;
				ok = d < 64 && !(bm & (1ull << d));
			}
		}
		else {
			const uint32_t pr = rec[p];
			const uint32_t psb = pr & 0xffffu;
			const bool pw = (pr >> 16) & 1u;
			const uint32_t pseq = hdr[p].seq;
			const uint32_t proc = roc - (wrap ? 1u : 0u);
			const int32_t pv = sp_v(proc, pw ? 0u : psb, pseq);
			const uint64_t pix = pseq + (uint64_t)(int64_t)pv * 65536ull;
			/* above the pre-batch window too (see k_plan_desc) */
			ok = ix > pix && ix > lix;
		}
		if (!ok)
			atomicOr(&out->base.fail, (uint32_t)SPF_REPLAY);
	}
	desc[i] = sp_desc(ix, fl);
	const uint32_t C = cnt[k];
	const uint32_t t0 = C > SGPU_PLAN_TAIL ? C - SGPU_PLAN_TAIL : 0u;
	if (ord >= t0 && ord - t0 < SGPU_PLAN_TAIL)
		out->tail_ix[k][ord - t0] = ix;
	if ((int32_t)i == L.last[k])
		out->s_l_last[k] = wrap ? seq : (seq > sb ? seq : sb);
}

__global__ void k_sp_final(struct sgpu_splan_out *out)
{
	if (threadIdx.x < 4)
		out->base.skip[threadIdx.x] =
			out->base.fail ||
			(((out->base.hl0 >> 2) & 3u) != threadIdx.x);
}

static size_t sp_al(size_t x)
{
	return (x + 255) & ~(size_t)255;
}

extern "C" size_t sgpu_splan_scratch(uint32_t n)
{
	const size_t nb = (n + SP_BLOCK - 1) / SP_BLOCK;
	return sp_al(nb * 3 * SP_H * 4) +              /* bl */
	       sp_al(nb * SP_K * 4) +                  /* bprev */
	       sp_al(nb * SP_K * 4) +                  /* bcnt */
	       sp_al(nb * SP_K * 8) +                  /* bpre */
	       sp_al((size_t)n * 4) * 2;               /* rec, prv */
}

extern "C" int sgpu_splan_rtp(const struct sgpu_splan_in *in,
			      const struct sgpu_hdr *hdr, const uint32_t *pos,
			      const uint32_t *end, const uint32_t *cap,
			      uint64_t arena_size, uint64_t *desc,
			      void *scratch, size_t scratch_bytes,
			      struct sgpu_splan_out *out, void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t n = in->n;
	const uint32_t nb = (n + SP_BLOCK - 1) / SP_BLOCK;
	if (!n || in->nst > SP_K || scratch_bytes < sgpu_splan_scratch(n))
		return EINVAL;
	uint8_t *p = (uint8_t *)scratch;
	uint32_t *bl = (uint32_t *)p;
	p += sp_al((size_t)nb * 3 * SP_H * 4);
	int32_t *bprev = (int32_t *)p;
	p += sp_al((size_t)nb * SP_K * 4);
	uint32_t *bcnt = (uint32_t *)p;
	p += sp_al((size_t)nb * SP_K * 4);
	uint2 *bpre = (uint2 *)p;
	p += sp_al((size_t)nb * SP_K * 8);
	uint32_t *rec = (uint32_t *)p;
	p += sp_al((size_t)n * 4);
	int32_t *prv = (int32_t *)p;
	if (!in->zeroed) {
		hipError_t e = hipMemsetAsync(out, 0, sizeof(*out), st);
		if (e != hipSuccess)
			return EIO;
	}
	hipLaunchKernelGGL(k_sp_ssrc, dim3(nb), dim3(SP_BLOCK), 0, st, hdr, n,
			   bl, out);
	hipLaunchKernelGGL(k_sp_merge, dim3(1), dim3(SP_SCAN), 0, st, *in,
			   (const uint32_t *)bl, nb, bprev, out);
	hipLaunchKernelGGL(k_sp_count, dim3(nb), dim3(SP_BLOCK), 0, st, *in,
			   hdr, pos, end, cap, arena_size,
			   (const int32_t *)bprev, rec, prv, bcnt, out);
	hipLaunchKernelGGL(k_sp_scan, dim3(1), dim3(SP_SCAN), 0, st,
			   (const uint32_t *)bcnt, nb, bpre, out);
	hipLaunchKernelGGL(k_sp_desc, dim3(nb), dim3(SP_BLOCK), 0, st, *in,
			   hdr, (const uint32_t *)rec, (const int32_t *)prv,
			   (const uint2 *)bpre, desc, out);
	hipLaunchKernelGGL(k_sp_final, dim3(1), dim3(64), 0, st, out);
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
