/*
 * plan_multi.hip -- device planning of multi-session RTP batches.
 *
 * The host's sequential state machine (srtp_encrypt srtp.c:203-213,
 * 279-280; srtp_decrypt srtp.c:310-321, 426-427; srtp_get_index
 * misc.c:22-41; srtp_replay_check replay.c:32-62) runs per stream, and
 * streams of different sessions are independent.  Here:
 *   1. packets are stably grouped by session, so each session's packets
 *      form one segment in array order: up to 65536 sessions by a counting
 *      pass (per-session counts, one scan, an unstable scatter, then each
 *      packet's rank among its session's packets by index -- a session
 *      with more than SGPU_MP_SEGMAX packets fails the plan with SPF_SEG
 *      and the host re-plans with the radix sort), else (or in.radix) by a
 *      hipCUB LSD radix sort of the session index (values = packet index);
 *   2. inside a segment packet k is assumed to see s_l = seq of packet
 *      k-1 (the session's stored s_l for the first), ROC rollovers are
 *      prefix-summed, and every assumption is verified exactly as in the
 *      single-stream planner (srtp_kernels.hip k_plan_*);
 *   3. each touched session's final stream state is written out.
 * Any verification miss sets out->fail: the host then plans sequentially
 * and nothing launched behind the plan (guarded on out->skip[]) runs.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <errno.h>
#include <stdio.h>
#include "../srtpgpu.h"

#ifndef EAUTH
#define EAUTH 217               /* include/re_types.h:215-217 */
#endif

#define MP_BLOCK 256

__device__ __forceinline__ uint64_t mp_desc(uint64_t ix, uint32_t flags)
{
	return (ix & 0xffffull) | ((uint64_t)(uint32_t)(ix >> 16) << 16) |
	       ((uint64_t)flags << 48);
}

/* misc.c:22-41, including the int wrap of roc +- 1 */
__device__ __forceinline__ int32_t mp_v(uint32_t roc, uint32_t s_l,
					uint32_t seq)
{
	if (s_l < 32768)
		return ((int)seq - (int)s_l > 32768) ? (int32_t)(roc - 1)
						     : (int32_t)roc;
	return ((int)s_l - 32768 > (int)seq) ? (int32_t)(roc + 1)
					     : (int32_t)roc;
}

__device__ __forceinline__ bool mp_wrap(uint32_t seq, uint32_t sb)
{
	return (int)seq - (int)sb <= -32768;
}

struct mp_ctx {
	const uint32_t *key;            /* sorted session index */
	const uint32_t *val;            /* sorted packet index */
	const struct sgpu_hdr *hdr;
	const struct sgpu_sstate *st;
	uint32_t n;
	/* seq and SSRC in sorted order, written by k_mp_count: the later
	 * passes read neighbours contiguously instead of through val[] */
	uint32_t *sseq, *sssrc;
};

/* s_l seen by sorted position k of the segment starting at f */
__device__ __forceinline__ uint32_t mp_sb(const mp_ctx &c, uint32_t k,
					  uint32_t f)
{
	if (k == f) {
		const struct sgpu_sstate &S = c.st[c.key[k]];
		return (S.flags & SST_SL_SET) ? S.s_l : c.sseq[k];
	}
	return c.sseq[k - 1];
}

__device__ __forceinline__ bool mp_first(const mp_ctx &c, uint32_t k)
{
	return k == 0 || c.key[k - 1] != c.key[k];
}

/* sort input: identity values, and the session keys clamped -- an index
 * >= nsess fails the plan (SPF_BAD) and is sorted as session nsess-1, so
 * every later table access (st, segf, segl) stays in bounds */
template <typename K>
__global__ void k_mp_iota(uint32_t *v, const uint32_t *sess, K *kin,
			  uint32_t n, uint32_t nsess, struct sgpu_plan_out *out,
			  uint32_t *segl)
{
	const uint32_t i = blockIdx.x * MP_BLOCK + threadIdx.x;
	/* segment ends start as "none" (k_mp_mark fills the touched ones) */
	for (uint32_t k = i; k < nsess; k += gridDim.x * MP_BLOCK)
		segl[k] = 0xffffffffu;
	if (i < n) {
		const uint32_t s = sess[i];
		if (s >= nsess)
			atomicOr(&out->fail, (uint32_t)SPF_BAD);
		v[i] = i;
		kin[i] = (K)(s < nsess ? s : nsess - 1u);
	}
}

/* ---- counting grouping (sessions <= 65536) ---------------------------- */

/* per packet: its (clamped) session's count, the unstable slot in it;
 * MP_HPER packets per thread, their atomics in flight together */
#ifndef MP_HPER
#define MP_HPER 4
#endif
__global__ void k_mp_hist(const uint32_t *sess, uint32_t *cnt,
			  uint32_t *slot, uint32_t n, uint32_t nsess,
			  struct sgpu_plan_out *out)
{
	const uint32_t i0 = blockIdx.x * (MP_BLOCK * MP_HPER) + threadIdx.x;
	uint32_t s[MP_HPER], r[MP_HPER];
	bool bad = false;
#pragma unroll
	for (int j = 0; j < MP_HPER; j++) {
		const uint32_t i = i0 + j * MP_BLOCK;
		s[j] = i < n ? sess[i] : 0u;
		if (s[j] >= nsess) {
			bad = true;
			s[j] = nsess - 1u;
		}
	}
#pragma unroll
	for (int j = 0; j < MP_HPER; j++)
		r[j] = i0 + j * MP_BLOCK < n ? atomicAdd(&cnt[s[j]], 1u) : 0u;
#pragma unroll
	for (int j = 0; j < MP_HPER; j++)
		if (i0 + j * MP_BLOCK < n)
			slot[i0 + j * MP_BLOCK] = r[j];
	if (bad)
		atomicOr(&out->fail, (uint32_t)SPF_BAD);
}

/* segment bounds from the counts, two launches over 1024-session tiles:
 * k_mp_tscan leaves each tile's exclusive prefix in segf and its total
 * in tsum (SPF_SEG above SGPU_MP_SEGMAX); k_mp_toff adds the tiles
 * before it and turns the counts in segl into last positions ("none" for
 * an empty segment) */
__global__ void __launch_bounds__(1024)
k_mp_tscan(uint32_t *segf, const uint32_t *segl, uint32_t *tsum,
	   uint32_t nsess, struct sgpu_plan_out *out)
{
	__shared__ uint32_t wsum[16];
	const uint32_t k = blockIdx.x * 1024u + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	const uint32_t c = k < nsess ? segl[k] : 0u;
	if (c > SGPU_MP_SEGMAX)
		atomicOr(&out->fail, (uint32_t)SPF_SEG);
	uint32_t v = c;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t u = (uint32_t)__shfl_up((int)v, d);
		if (lane >= (uint32_t)d)
			v += u;
	}
	if (lane == 63)
		wsum[wv] = v;
	__syncthreads();
	uint32_t pre = 0;
	for (uint32_t q = 0; q < wv; q++)
		pre += wsum[q];
	if (k < nsess)
		segf[k] = pre + v - c;
	if (threadIdx.x == 1023)
		tsum[blockIdx.x] = pre + v;
}

__global__ void __launch_bounds__(1024)
k_mp_toff(uint32_t *segf, uint32_t *segl, const uint32_t *tsum,
	  uint32_t nsess)
{
	__shared__ uint32_t base;
	const uint32_t k = blockIdx.x * 1024u + threadIdx.x;
	if (threadIdx.x < 64) {
		uint32_t v = threadIdx.x < blockIdx.x ? tsum[threadIdx.x] : 0u;
		for (int d = 32; d > 0; d >>= 1)
			v += (uint32_t)__shfl_xor((int)v, d);
		if (threadIdx.x == 0)
			base = v;
	}
	__syncthreads();
	if (k >= nsess)
		return;
	const uint32_t c = segl[k], f = segf[k] + base;
	segf[k] = f;
	segl[k] = c ? f + c - 1u : 0xffffffffu;
}

__global__ void k_mp_cscatter(const uint32_t *sess, const uint32_t *slot,
			      const uint32_t *segf, uint32_t *tmp, uint32_t n,
			      uint32_t nsess)
{
	const uint32_t i = blockIdx.x * MP_BLOCK + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t s = sess[i] < nsess ? sess[i] : nsess - 1u;
	tmp[segf[s] + slot[i]] = i;
}

/* stable order: the packet at unstable position q goes to its segment
 * start + the number of its session's packets with a smaller index (a
 * segment is read by the lanes that hold it: broadcast loads) */
__global__ void k_mp_crank(const uint32_t *sess, const uint32_t *tmp,
			   const uint32_t *segf, const uint32_t *segl,
			   uint32_t *key, uint32_t *val, uint32_t n,
			   uint32_t nsess)
{
	const uint32_t q = blockIdx.x * MP_BLOCK + threadIdx.x;
	if (q >= n)
		return;
	const uint32_t i = tmp[q];
	const uint32_t s = sess[i] < nsess ? sess[i] : nsess - 1u;
	const uint32_t f = segf[s], l = segl[s];
	if (l - f >= SGPU_MP_SEGMAX) {
		/* SPF_SEG: the plan is not used, but the planner passes
		 * still read a permutation */
		key[q] = s;
		val[q] = i;
		return;
	}
	uint32_t r = 0;
	for (uint32_t k = f; k <= l; k++)
		r += tmp[k] < i ? 1u : 0u;
	key[f + r] = s;
	val[f + r] = i;
}

/* sorted 16-bit keys -> the 32-bit key array the planner passes read */
__global__ void k_mp_widen(const uint16_t *k16, uint32_t *k32, uint32_t n)
{
	const uint32_t i = blockIdx.x * MP_BLOCK + threadIdx.x;
	if (i < n)
		k32[i] = k16[i];
}

__global__ void __launch_bounds__(MP_BLOCK)
k_mp_count(const struct sgpu_mplan_in in, mp_ctx c, const uint32_t *pos,
	   const uint32_t *end, const uint32_t *cap, uint64_t asz,
	   uint32_t *bcnt, struct sgpu_plan_out *out)
{
	const uint32_t k = blockIdx.x * MP_BLOCK + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u;
	bool wrap = false;
	uint32_t f = 0;
	/* the previous sorted position's header: from the lane below, a
	 * gather only at lane 0 */
	struct sgpu_hdr h = {0, 0, 0, 0};
	if (k < in.n)
		h = c.hdr[c.val[k]];
	uint32_t pseq = (uint32_t)__shfl_up((int)h.seq, 1);
	uint32_t pssrc = (uint32_t)__shfl_up((int)h.ssrc, 1);
	if (lane == 0 && k > 0 && k < in.n) {
		const struct sgpu_hdr hp = c.hdr[c.val[k - 1]];
		pseq = hp.seq;
		pssrc = hp.ssrc;
	}
	if (k < in.n) {
		const uint32_t i = c.val[k], s = c.key[k];
		const bool first = mp_first(c, k);
		const bool last = k + 1 == in.n || c.key[k + 1] != s;
		const uint32_t hl0 = c.hdr[0].hdr_len;
		c.sseq[k] = h.seq;
		c.sssrc[k] = h.ssrc;
		const struct sgpu_sstate S = c.st[s];
		const uint32_t seq = h.seq;
		const uint32_t sb = first ? ((S.flags & SST_SL_SET) ? S.s_l : seq)
					  : pseq;
		if (s >= in.nsess)
			f |= SPF_BAD;
		if (h.hdr_len == 0xffffffffu || hl0 == 0xffffffffu)
			f |= SPF_PARSE;
		else if (((h.hdr_len ^ hl0) >> 2) & 3u)
			f |= SPF_CLASS;
		/* one SSRC per session: the stored one, or the segment's */
		if (first ? ((S.flags & SST_EXISTS) && h.ssrc != S.ssrc)
			  : h.ssrc != pssrc)
			f |= SPF_SSRC;
		if (!in.prot && (int)seq - (int)sb > 32768)
			f |= SPF_TIMEOUT;
		/* the window checks: made by the parse prologue (coalesced,
		 * in.wchk, folded in by k_mp_scan) or here (gathers) */
		if (!in.wchk) {
			if (!in.prot && h.hdr_len != 0xffffffffu &&
			    end[i] - pos[i] - h.hdr_len < in.tag)
				f |= SPF_PARSE;
			if (end[i] - pos[i] >= in.maxlen)
				f |= SPF_SIZE;
			if ((pos[i] & 3u) || pos[i] > end[i] || end[i] > asz ||
			    (cap && (end[i] > cap[i] || cap[i] > asz)))
				f |= SPF_BAD;
			if (in.prot && cap &&
			    (uint64_t)end[i] + in.need > (uint64_t)cap[i])
				f |= SPF_CAP;
		}
		wrap = mp_wrap(seq, sb);
		if (!last && !wrap && seq < sb)
			f |= SPF_ORDER;
		if (k == 0)
			out->hl0 = hl0;
		if (f)
			atomicOr(&out->fail, f);
	}
	const int cnt = __syncthreads_count(wrap);
	if (threadIdx.x == 0)
		bcnt[blockIdx.x] = (uint32_t)cnt;
}

/* exclusive scan of the per-block wrap counts (one workgroup) */
__global__ void __launch_bounds__(1024)
k_mp_scan(uint32_t *bcnt, uint32_t nb, const uint32_t *wchk,
	  struct sgpu_plan_out *out)
{
	__shared__ uint32_t part[1024];
	const uint32_t per = (nb + 1023u) / 1024u;
	const uint32_t a = threadIdx.x * per;
	uint32_t sum = 0, f = 0;
	for (uint32_t k = a; k < a + per && k < nb; k++) {
		sum += bcnt[k];
		if (wchk)
			f |= wchk[k];
	}
	if (f)
		atomicOr(&out->fail, f);
	part[threadIdx.x] = sum;
	__syncthreads();
	for (uint32_t d = 1; d < 1024; d <<= 1) {
		uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
		__syncthreads();
		part[threadIdx.x] += v;
		__syncthreads();
	}
	uint32_t run = part[threadIdx.x] - sum;
	for (uint32_t k = a; k < a + per && k < nb; k++) {
		const uint32_t v = bcnt[k];
		bcnt[k] = run;
		run += v;
	}
}

/* per position: exclusive wrap prefix; per session: segment bounds */
__global__ void __launch_bounds__(MP_BLOCK)
k_mp_mark(mp_ctx c, const uint32_t *bpre, uint32_t *pex, uint32_t *segf,
	  uint32_t *segl)
{
	__shared__ uint32_t wsum[MP_BLOCK / 64];
	const uint32_t k = blockIdx.x * MP_BLOCK + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	bool wrap = false, first = false, last = false;
	if (k < c.n) {
		first = mp_first(c, k);
		last = k + 1 == c.n || c.key[k + 1] != c.key[k];
		/* the segment start is only needed for k == f */
		const uint32_t sb = first ? mp_sb(c, k, k) : c.sseq[k - 1];
		wrap = mp_wrap(c.sseq[k], sb);
	}
	const uint64_t m = __ballot(wrap);
	if (lane == 0)
		wsum[wv] = (uint32_t)__popcll(m);
	__syncthreads();
	uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
	for (uint32_t q = 0; q < wv; q++)
		pre += wsum[q];
	if (k >= c.n)
		return;
	pex[k] = bpre[blockIdx.x] + pre;
	if (first)
		segf[c.key[k]] = k;
	if (last)
		segl[c.key[k]] = k;
}

/* exact index of sorted position k (segment start f) */
__device__ __forceinline__ uint64_t mp_ix(const mp_ctx &c,
					  const struct sgpu_mplan_in &in,
					  const uint32_t *pex, uint32_t k,
					  uint32_t f, uint32_t *flp,
					  uint32_t *rocp, bool *wrapp,
					  uint32_t *sbp)
{
	const struct sgpu_sstate &S = c.st[c.key[k]];
	const uint32_t seq = c.sseq[k];
	const uint32_t sb = mp_sb(c, k, f);
	const bool wrap = mp_wrap(seq, sb);
	const uint32_t fseq = c.sseq[f];
	const bool wf = mp_wrap(fseq, mp_sb(c, f, f));
	/* ROC after this packet's own rollover */
	const uint32_t roc = S.roc + (pex[k] + (wrap ? 1u : 0u)) -
			     (pex[f] + (wf ? 1u : 0u)) + (wf ? 1u : 0u);
	uint64_t ix;
	uint32_t fl = SD_RUN | SD_CIPHER;
	if (in.prot) {
		ix = 65536ull * roc + seq;                   /* srtp.c:215 */
	}
	else {
		const int32_t v = mp_v(roc, wrap ? 0u : sb, seq);
		ix = seq + (uint64_t)(int64_t)v * 65536ull;
		if ((uint32_t)v != roc)
			fl |= (uint32_t)v + 1u == roc ? SD_ROC_P1 : SD_ROC_M1;
	}
	if (flp)
		*flp = fl;
	if (rocp)
		*rocp = roc;
	if (wrapp)
		*wrapp = wrap;
	if (sbp)
		*sbp = sb;
	return ix;
}

__global__ void __launch_bounds__(MP_BLOCK)
k_mp_desc(const struct sgpu_mplan_in in, mp_ctx c, const uint32_t *pex,
	  const uint32_t *segf, uint64_t *desc, struct sgpu_plan_out *out)
{
	const uint32_t k = blockIdx.x * MP_BLOCK + threadIdx.x;
	if (k >= c.n)
		return;
	const uint32_t s = c.key[k], f = segf[s];
	uint32_t fl;
	const uint64_t ix = mp_ix(c, in, pex, k, f, &fl, NULL, NULL, NULL);
	if (!in.prot) {
		/* replay: every packet new (replay.c:32-62) */
		bool ok;
		if (k == f) {
			const struct sgpu_sstate &S = c.st[s];
			if (ix > S.lix)
				ok = true;
			else {
				const uint64_t d = S.lix - ix;
				ok = d < 64 && !(S.bitmap & (1ull << d));
			}
		}
		else {
			/* above the session's pre-batch lix as well (see
			 * k_plan_desc, srtp_kernels.hip) */
			ok = ix > mp_ix(c, in, pex, k - 1, f, NULL, NULL, NULL,
					NULL) && ix > c.st[s].lix;
		}
		if (!ok)
			atomicOr(&out->fail, (uint32_t)SPF_REPLAY);
	}
	desc[c.val[k]] = mp_desc(ix, fl);
}

/* final state of every touched session; launch guards */
__global__ void __launch_bounds__(MP_BLOCK)
k_mp_final(const struct sgpu_mplan_in in, mp_ctx c, const uint32_t *pex,
	   const uint32_t *segf, const uint32_t *segl,
	   struct sgpu_sstate *st_out, struct sgpu_plan_out *out)
{
	const uint32_t s = blockIdx.x * MP_BLOCK + threadIdx.x;
	if (s == 0)
		for (int q = 0; q < 4; q++)
			out->skip[q] = out->fail ||
				       (((out->hl0 >> 2) & 3u) != (uint32_t)q);
	if (s >= in.nsess)
		return;
	const struct sgpu_sstate S = c.st[s];
	struct sgpu_sstate o = S;
	o.flags &= ~SST_TOUCHED;
	const uint32_t l = segl[s];
	if (l == 0xffffffffu) {
		st_out[s] = o;
		return;
	}
	const uint32_t f = segf[s];
	uint32_t roc, sb;
	bool wrap;
	(void)mp_ix(c, in, pex, l, f, NULL, &roc, &wrap, &sb);
	const uint32_t seq = c.sseq[l];
	o.ssrc = (S.flags & SST_EXISTS) ? S.ssrc : c.sssrc[f];
	o.roc = roc;
	o.s_l = wrap ? seq : (seq > sb ? seq : sb);
	o.flags = SST_EXISTS | SST_SL_SET | SST_TOUCHED;
	if (!in.prot) {
		/* replay fold over the last <= 65 indices (older bits have
		 * shifted out: every index is new and increasing) */
		uint64_t lix = S.lix, bm = S.bitmap;
		uint32_t k = f;
		if (l - f + 1 > 65) {
			k = l - 64;
			lix = mp_ix(c, in, pex, k - 1, f, NULL, NULL, NULL,
				    NULL);
			bm = 1;
		}
		for (; k <= l; k++) {
			const uint64_t ix = mp_ix(c, in, pex, k, f, NULL, NULL,
						  NULL, NULL);
			if (ix > lix) {
				const uint64_t d = ix - lix;
				bm = d < 64 ? (bm << d) | 1ull : 1ull;
				lix = ix;
			}
			else {
				bm |= 1ull << (lix - ix);
			}
		}
		o.lix = lix;
		o.bitmap = bm;
	}
	st_out[s] = o;
}

/*
 * Launch order of the crypto kernels: packets grouped by descending number
 * of 64-byte chunks, so a wave's lanes carry packets of about the same
 * length -- with mixed 200/1400-B traffic (config 4) a wave otherwise runs
 * as long as its longest packet.  Only the grouping matters (any order
 * inside a group is a valid launch order), so this is a two-launch
 * counting sort: per-block LDS histograms folded into MP_OBINS global
 * counts, then each block scatters its packets behind a range reserved
 * with one global atomic per (block, bin).  Packets of >= MP_OBINS-1
 * chunks share the last group (the cached kernels take < 4032 B anyway).
 */
#define MP_OBINS 64
#define MP_OBLOCK 1024
#define MP_OPER 4

__device__ __forceinline__ uint32_t mp_obin(const uint32_t *pos,
					    const uint32_t *end, uint32_t i)
{
	const uint32_t L = end[i] >= pos[i] ? end[i] - pos[i] : 0u;
	const uint32_t ch = (L + 63u) >> 6;
	return (MP_OBINS - 1u) - (ch < MP_OBINS - 1u ? ch : MP_OBINS - 1u);
}

__global__ void __launch_bounds__(MP_OBLOCK)
k_mp_ocount(const uint32_t *pos, const uint32_t *end, uint32_t *ghist,
	    uint32_t n)
{
	__shared__ uint32_t h[MP_OBINS];
	const uint32_t t = threadIdx.x;
	if (t < MP_OBINS)
		h[t] = 0;
	__syncthreads();
	for (uint32_t j = 0; j < MP_OPER; j++) {
		const uint32_t i = blockIdx.x * (MP_OBLOCK * MP_OPER) +
				   j * MP_OBLOCK + t;
		if (i < n)
			atomicAdd(&h[mp_obin(pos, end, i)], 1u);
	}
	__syncthreads();
	if (t < MP_OBINS && h[t])
		atomicAdd(&ghist[t], h[t]);
}

__global__ void __launch_bounds__(MP_OBLOCK)
k_mp_oscatter(const uint32_t *pos, const uint32_t *end,
	      const uint32_t *ghist, uint32_t *gcur, uint32_t *order,
	      uint32_t n)
{
	__shared__ uint32_t h[MP_OBINS], base[MP_OBINS];
	const uint32_t t = threadIdx.x;
	uint32_t bin[MP_OPER], rank[MP_OPER];
	if (t < MP_OBINS)
		h[t] = 0;
	__syncthreads();
	for (uint32_t j = 0; j < MP_OPER; j++) {
		const uint32_t i = blockIdx.x * (MP_OBLOCK * MP_OPER) +
				   j * MP_OBLOCK + t;
		bin[j] = i < n ? mp_obin(pos, end, i) : 0u;
		rank[j] = i < n ? atomicAdd(&h[bin[j]], 1u) : 0u;
	}
	__syncthreads();
	if (t < MP_OBINS && h[t]) {
		uint32_t pre = 0;
		for (uint32_t q = 0; q < t; q++)
			pre += ghist[q];
		base[t] = pre + atomicAdd(&gcur[t], h[t]);
	}
	__syncthreads();
	for (uint32_t j = 0; j < MP_OPER; j++) {
		const uint32_t i = blockIdx.x * (MP_OBLOCK * MP_OPER) +
				   j * MP_OBLOCK + t;
		if (i < n)
			order[base[bin[j]] + rank[j]] = i;
	}
}

/*
 * Verdict fold of a multi-session unprotect (sgpu_mfold_rtp): the
 * single-stream fold (srtp_kernels.hip k_fold_*) per session segment of
 * the sorted order.  The planner speculated that every tag verifies; a
 * forged packet still bumps the ROC on a rollover but never sets s_l
 * (srtp.c:310-321, 342-359, 426-427), so the packets after it in its
 * segment may see another s_l than the plan assumed.  Packet k sees the
 * value left by the last "event" before it in its segment -- an authentic
 * packet (s_l = seq) or a rollover (s_l = 0 if forged) -- or the
 * session's stored s_l; the fold checks that every rollover decision,
 * ETIMEDOUT and index estimate is unchanged under it, and only then
 * writes the EAUTH results, each touched session's s_l and replay window.
 * The sort is still in the planner's scratch: val (sorted packet index),
 * sseq, segf / segl; the session of a sorted position is sess[val[k]].
 */
struct mf_ctx {
	const uint32_t *val, *sess, *sseq, *segf;
	const struct sgpu_sstate *st;
	const uint8_t *vd;
	uint32_t n, nsess;
	const uint32_t *nfail;  /* queued behind the crypto kernels: the
				   kernels' miss count (0: nothing to fold) */
};

__device__ __forceinline__ bool mf_idle(const mf_ctx &c)
{
	return c.nfail && *c.nfail == 0u;
}

__device__ __forceinline__ uint32_t mf_key(const mf_ctx &c, uint32_t k)
{
	const uint32_t s = c.sess[c.val[k]];
	return s < c.nsess ? s : c.nsess - 1u;
}

/* the s_l the segment starts from (stream_get_seq sets it to the first
 * packet's seq for a new stream, stream.c:87-109) */
__device__ __forceinline__ uint32_t mf_sl0(const mf_ctx &c, uint32_t s,
					   uint32_t f)
{
	const struct sgpu_sstate &S = c.st[s];
	return (S.flags & SST_SL_SET) ? S.s_l : c.sseq[f];
}

__device__ __forceinline__ bool mf_auth(const mf_ctx &c, uint32_t k)
{
	return (c.vd[c.val[k]] & SV_TAG_OK) != 0;
}

/* speculated s_l of position k (segment start f, session s) */
__device__ __forceinline__ uint32_t mf_sb(const mf_ctx &c, uint32_t k,
					  uint32_t f, uint32_t s)
{
	return k == f ? mf_sl0(c, s, f) : c.sseq[k - 1];
}

__device__ __forceinline__ bool mf_event(const mf_ctx &c, uint32_t k)
{
	const uint32_t s = mf_key(c, k), f = c.segf[s];
	return mf_auth(c, k) || mp_wrap(c.sseq[k], mf_sb(c, k, f, s));
}

/* true s_l after event position e (-1 or outside the segment: the
 * session's start value) */
__device__ __forceinline__ uint32_t mf_slv(const mf_ctx &c, int32_t e,
					   uint32_t f, uint32_t s)
{
	if (e < (int32_t)f)
		return mf_sl0(c, s, f);
	return mf_auth(c, (uint32_t)e) ? c.sseq[e] : 0u;
}

__global__ void __launch_bounds__(MP_BLOCK)
k_mf_count(mf_ctx c, int32_t *blast, struct sgpu_fold_out *out)
{
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		/* the verdict starts held (also when there is nothing to fold) */
		out->fail = 0;
		out->nok = 0;
		out->first_ok = 0xffffffffu;
		out->last_ok = 0xffffffffu;
		out->s_l = 0;
		out->pad = 0;
		out->lix = 0;
		out->bitmap = 0;
	}
	if (mf_idle(c))
		return;
	const uint32_t k = blockIdx.x * MP_BLOCK + threadIdx.x;
	int32_t last = (k < c.n && mf_event(c, k)) ? (int32_t)k : -1;
	for (int o = 32; o > 0; o >>= 1)
		last = max(last, __shfl_xor(last, o));
	__shared__ int32_t wl[MP_BLOCK / 64];
	if ((threadIdx.x & 63u) == 0)
		wl[threadIdx.x >> 6] = last;
	__syncthreads();
	if (threadIdx.x == 0) {
		int32_t m = -1;
		for (int w = 0; w < MP_BLOCK / 64; w++)
			m = max(m, wl[w]);
		blast[blockIdx.x] = m;
	}
}

/* exclusive prefix maximum of the block maxima (one workgroup) */
__global__ void __launch_bounds__(1024)
k_mf_scan(const int32_t *blast, int32_t *bprev, uint32_t nb,
	  const uint32_t *nfail)
{
	if (nfail && *nfail == 0u)
		return;
	__shared__ int32_t part[1024];
	const uint32_t per = (nb + 1023u) / 1024u;
	const uint32_t a = threadIdx.x * per;
	int32_t m = -1;
	for (uint32_t k = a; k < a + per && k < nb; k++)
		m = max(m, blast[k]);
	part[threadIdx.x] = m;
	__syncthreads();
	for (uint32_t d = 1; d < 1024; d <<= 1) {
		int32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : -1;
		__syncthreads();
		part[threadIdx.x] = max(part[threadIdx.x], v);
		__syncthreads();
	}
	int32_t run = threadIdx.x ? part[threadIdx.x - 1] : -1;
	for (uint32_t k = a; k < a + per && k < nb; k++) {
		bprev[k] = run;
		run = max(run, blast[k]);
	}
}

/* per sorted position: the speculation under the true s_l; at a
 * segment's last position, the session's s_l after the batch */
__global__ void __launch_bounds__(MP_BLOCK)
k_mf_check(mf_ctx c, const int32_t *bprev, struct sgpu_sstate *st_out,
	   struct sgpu_fold_out *out)
{
	__shared__ int32_t sc[MP_BLOCK];
	if (mf_idle(c))
		return;
	const uint32_t k = blockIdx.x * MP_BLOCK + threadIdx.x;
	const bool ev = k < c.n && mf_event(c, k);
	sc[threadIdx.x] = ev ? (int32_t)k : -1;
	__syncthreads();
	for (uint32_t d = 1; d < MP_BLOCK; d <<= 1) {
		int32_t v = threadIdx.x >= d ? sc[threadIdx.x - d] : -1;
		__syncthreads();
		sc[threadIdx.x] = max(sc[threadIdx.x], v);
		__syncthreads();
	}
	if (k >= c.n)
		return;
	const int32_t e = max(bprev[blockIdx.x],
			      threadIdx.x ? sc[threadIdx.x - 1] : -1);
	const uint32_t s = mf_key(c, k), f = c.segf[s];
	const uint32_t seq = c.sseq[k];
	const uint32_t sb = mf_sb(c, k, f, s);          /* speculated */
	const uint32_t sl = mf_slv(c, e, f, s);         /* true */
	const bool wrap = mp_wrap(seq, sb);
	bool bad = mp_wrap(seq, sl) != wrap ||
		   (int)seq - (int)sl > 32768;          /* ETIMEDOUT */
	if (!bad && !wrap) {
		/* same index estimate (misc.c:22-41) at any ROC */
		bad = mp_v(65536u, sl, seq) != mp_v(65536u, sb, seq);
		/* an authentic packet sets s_l = seq only if seq > s_l
		 * (srtp.c:426-427); the events assume it does */
		if (mf_auth(c, k) && seq < sl)
			bad = true;
	}
	if (bad)
		atomicOr(&out->fail, 1u);
	if (k + 1 == c.n || mf_key(c, k + 1) != s)
		st_out[s].s_l = mf_slv(c, ev ? (int32_t)k : e, f, s);
}

/* forged packets: EAUTH like srtp_decrypt (srtp.c:342-359, 404-411) */
__global__ void __launch_bounds__(MP_BLOCK)
k_mf_results(const uint8_t *vd, const struct sgpu_hdr *hdr,
	     const uint32_t *end0, uint32_t *pos, uint32_t *end, int32_t *err,
	     uint32_t n, int gcm, const struct sgpu_fold_out *out,
	     const uint32_t *nfail)
{
	const uint32_t i = blockIdx.x * MP_BLOCK + threadIdx.x;
	if ((nfail && *nfail == 0u) || i >= n || out->fail ||
	    (vd[i] & SV_TAG_OK))
		return;
	err[i] = EAUTH;
	pos[i] += hdr[i].hdr_len;
	if (gcm)
		end[i] = end0[i];
}

/* each touched session's replay window after the batch (replay.c:32-62):
 * the authentic packets of its segment, every index new and increasing,
 * so the window after the last authentic one j holds the authentic
 * packets j-63 .. j (and, close to the segment start, the stored window) */
__global__ void __launch_bounds__(MP_BLOCK)
k_mf_final(mf_ctx c, const uint32_t *segl, const uint64_t *desc,
	   struct sgpu_sstate *st_out, const struct sgpu_fold_out *out)
{
	const uint32_t s = blockIdx.x * MP_BLOCK + threadIdx.x;
	if (mf_idle(c) || s >= c.nsess || out->fail)
		return;
	const uint32_t l = segl[s];
	if (l == 0xffffffffu)
		return;
	const uint32_t f = c.segf[s];
	const struct sgpu_sstate &S = c.st[s];
	int32_t j = (int32_t)l;
	while (j >= (int32_t)f && !mf_auth(c, (uint32_t)j))
		j--;
	uint64_t lix = S.lix, bm = S.bitmap;
	if (j >= (int32_t)f) {
		uint32_t q = f;
		if ((uint32_t)j - f >= 64u) {
			q = (uint32_t)j - 63u;
			const uint64_t d = desc[c.val[q - 1]];
			lix = (d & 0xffffull) | ((d >> 16) & 0xffffffffull) << 16;
			bm = 0;
		}
		for (; q <= (uint32_t)j; q++) {
			if (!mf_auth(c, q))
				continue;
			const uint64_t d = desc[c.val[q]];
			const uint64_t ix = (d & 0xffffull) |
					    ((d >> 16) & 0xffffffffull) << 16;
			if (ix > lix) {
				const uint64_t dl = ix - lix;
				bm = dl < 64 ? (bm << dl) | 1ull : 1ull;
				lix = ix;
			}
			else {
				bm |= 1ull << (lix - ix);
			}
		}
	}
	st_out[s].lix = lix;
	st_out[s].bitmap = bm;
}

/* ---- host side ------------------------------------------------------ */

static size_t mp_align(size_t x)
{
	return (x + 255) & ~(size_t)255;
}

/* up to 65536 sessions the keys sort as uint16_t: rocPRIM then takes its
 * onesweep radix sort for more than 100K items (device_radix_sort.hpp:
 * 2-byte keys skip the merge-sort path, ~20 launches for 1M items) */
static size_t mp_cub_bytes(uint32_t n, uint32_t bits)
{
	size_t tb = 0, t16 = 0;
	(void)hipcub::DeviceRadixSort::SortPairs(
		(void *)NULL, tb, (const uint32_t *)NULL, (uint32_t *)NULL,
		(const uint32_t *)NULL, (uint32_t *)NULL, (int)n, 0,
		(int)bits);
	if (bits <= 16)
		(void)hipcub::DeviceRadixSort::SortPairs(
			(void *)NULL, t16, (const uint16_t *)NULL,
			(uint16_t *)NULL, (const uint32_t *)NULL,
			(uint32_t *)NULL, (int)n, 0, (int)bits);
	return tb > t16 ? tb : t16;
}

/* the counting grouping's counters: segl (see sgpu_mplan_rtp_phase),
 * followed by the launch-order bins: sgpu_mplan_counter_words(nsess)
 * words to zero */
extern "C" uint32_t sgpu_mplan_counter_words(uint32_t nsess)
{
	return (uint32_t)(mp_align((size_t)nsess * 4) / 4) + 2 * MP_OBINS;
}

extern "C" uint32_t *sgpu_mplan_counters(void *scratch, uint32_t n,
					 uint32_t nsess)
{
	const uint32_t nb = (n + MP_BLOCK - 1) / MP_BLOCK;
	return (uint32_t *)((uint8_t *)scratch + 6 * mp_align((size_t)n * 4) +
			    mp_align((size_t)nb * 4 + 64) +
			    mp_align((size_t)nsess * 4));
}

extern "C" size_t sgpu_mplan_scratch(uint32_t n, uint32_t nsess)
{
	const uint32_t nb = (n + MP_BLOCK - 1) / MP_BLOCK;
	/* the radix sort's temporary storage doubles as the counting
	 * grouping's launch-order bins (>= 512 B) */
	size_t tb = mp_align(mp_cub_bytes(n, 32));
	if (tb < 512)
		tb = 512;
	return 6 * mp_align((size_t)n * 4) + mp_align((size_t)nb * 4 + 64) +
	       2 * mp_align((size_t)nsess * 4) + tb;
}

extern "C" int sgpu_mplan_rtp(const struct sgpu_mplan_in *in,
			      const struct sgpu_hdr *hdr, const uint32_t *pos,
			      const uint32_t *end, const uint32_t *cap,
			      uint64_t arena_size, const uint32_t *sess,
			      const struct sgpu_sstate *st_in,
			      struct sgpu_sstate *st_out, uint64_t *desc,
			      void *scratch, size_t scratch_bytes,
			      struct sgpu_plan_out *out, uint32_t *order,
			      void *stream)
{
	int e = sgpu_mplan_rtp_phase(1, in, hdr, pos, end, cap, arena_size,
				     sess, st_in, st_out, desc, scratch,
				     scratch_bytes, out, order, stream);
	if (!e)
		e = sgpu_mplan_rtp_phase(2, in, hdr, pos, end, cap, arena_size,
					 sess, st_in, st_out, desc, scratch,
					 scratch_bytes, out, order, stream);
	return e;
}

extern "C" int sgpu_mplan_rtp_phase(int phase, const struct sgpu_mplan_in *in,
				    const struct sgpu_hdr *hdr,
				    const uint32_t *pos, const uint32_t *end,
				    const uint32_t *cap, uint64_t arena_size,
				    const uint32_t *sess,
				    const struct sgpu_sstate *st_in,
				    struct sgpu_sstate *st_out, uint64_t *desc,
				    void *scratch, size_t scratch_bytes,
				    struct sgpu_plan_out *out, uint32_t *order,
				    void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t n = in->n, nb = (n + MP_BLOCK - 1) / MP_BLOCK;
	uint8_t *p = (uint8_t *)scratch;
	uint32_t *kout = (uint32_t *)p;  p += mp_align((size_t)n * 4);
	uint32_t *vin = (uint32_t *)p;   p += mp_align((size_t)n * 4);
	uint32_t *vout = (uint32_t *)p;  p += mp_align((size_t)n * 4);
	uint32_t *pex = (uint32_t *)p;   p += mp_align((size_t)n * 4);
	uint32_t *sseq = (uint32_t *)p;  p += mp_align((size_t)n * 4);
	uint32_t *sssrc = (uint32_t *)p; p += mp_align((size_t)n * 4);
	uint32_t *bcnt = (uint32_t *)p;  p += mp_align((size_t)nb * 4 + 64);
	uint32_t *segf = (uint32_t *)p;  p += mp_align((size_t)in->nsess * 4);
	uint32_t *segl = (uint32_t *)p;  p += mp_align((size_t)in->nsess * 4);
	size_t tb = mp_cub_bytes(n, in->key_bits);
	if (!n || !in->nsess ||
	    (size_t)(p - (uint8_t *)scratch) + tb > scratch_bytes)
		return EINVAL;
	if (phase == 2)
		goto plan;
	if (!in->out_zeroed &&
	    hipMemsetAsync(out, 0, sizeof(*out), st) != hipSuccess)
		return EIO;
	if (in->nsess <= 65536 && !in->radix) {
		/* counting grouping: the counts in segl (zeroed by the parse
		 * prologue or here), unstable slots in vin, the unstable
		 * order in pex (free until k_mp_mark) */
		if (!in->cnt_zeroed &&
		    hipMemsetAsync(segl, 0, (size_t)in->nsess * 4, st) !=
		    hipSuccess)
			return EIO;
		const uint32_t nt = (in->nsess + 1023u) / 1024u;  /* <= 64 */
		hipLaunchKernelGGL(k_mp_hist,
				   dim3((n + MP_BLOCK * MP_HPER - 1) /
					(MP_BLOCK * MP_HPER)),
				   dim3(MP_BLOCK), 0, st, sess, segl, vin, n,
				   in->nsess, out);
		/* the tile totals in bcnt (free until k_mp_count) */
		hipLaunchKernelGGL(k_mp_tscan, dim3(nt), dim3(1024), 0, st, segf,
				   (const uint32_t *)segl, bcnt, in->nsess, out);
		hipLaunchKernelGGL(k_mp_toff, dim3(nt), dim3(1024), 0, st, segf,
				   segl, (const uint32_t *)bcnt, in->nsess);
		hipLaunchKernelGGL(k_mp_cscatter, dim3(nb), dim3(MP_BLOCK), 0,
				   st, sess, (const uint32_t *)vin,
				   (const uint32_t *)segf, pex, n, in->nsess);
		hipLaunchKernelGGL(k_mp_crank, dim3(nb), dim3(MP_BLOCK), 0, st,
				   sess, (const uint32_t *)pex,
				   (const uint32_t *)segf, (const uint32_t *)segl,
				   kout, vout, n, in->nsess);
	}
	/* pex is free until k_mp_mark (the clamped keys), sseq until
	 * k_mp_count (sorted 16-bit keys) */
	else if (in->nsess <= 65536 && in->key_bits <= 16) {
		uint16_t *k16 = (uint16_t *)pex, *o16 = (uint16_t *)sseq;
		hipLaunchKernelGGL(k_mp_iota<uint16_t>, dim3(nb), dim3(MP_BLOCK),
				   0, st, vin, sess, k16, n, in->nsess, out, segl);
		if (hipcub::DeviceRadixSort::SortPairs(p, tb, k16, o16, vin,
						       vout, (int)n, 0,
						       (int)in->key_bits,
						       st) != hipSuccess)
			return EIO;
		hipLaunchKernelGGL(k_mp_widen, dim3(nb), dim3(MP_BLOCK), 0, st,
				   (const uint16_t *)o16, kout, n);
	}
	else {
		hipLaunchKernelGGL(k_mp_iota<uint32_t>, dim3(nb), dim3(MP_BLOCK),
				   0, st, vin, sess, pex, n, in->nsess, out, segl);
		if (hipcub::DeviceRadixSort::SortPairs(p, tb, pex, kout, vin,
						       vout, (int)n, 0,
						       (int)in->key_bits,
						       st) != hipSuccess)
			return EIO;
	}
	if (phase == 1)
		return hipGetLastError() == hipSuccess ? 0 : EIO;
 plan:;
	mp_ctx c = {kout, vout, hdr, st_in, n, sseq, sssrc};
	hipLaunchKernelGGL(k_mp_count, dim3(nb), dim3(MP_BLOCK), 0, st, *in, c,
			   pos, end, cap, arena_size, bcnt, out);
	hipLaunchKernelGGL(k_mp_scan, dim3(1), dim3(1024), 0, st, bcnt, nb,
			   in->wchk, out);
	hipLaunchKernelGGL(k_mp_mark, dim3(nb), dim3(MP_BLOCK), 0, st, c,
			   (const uint32_t *)bcnt, pex, segf, segl);
	hipLaunchKernelGGL(k_mp_desc, dim3(nb), dim3(MP_BLOCK), 0, st, *in, c,
			   (const uint32_t *)pex, (const uint32_t *)segf, desc,
			   out);
	hipLaunchKernelGGL(k_mp_final,
			   dim3((in->nsess + MP_BLOCK - 1) / MP_BLOCK),
			   dim3(MP_BLOCK), 0, st, *in, c, (const uint32_t *)pex,
			   (const uint32_t *)segf, (const uint32_t *)segl,
			   st_out, out);
	if (order) {
		/* crypto launch order: bin counts and cursors right behind the
		 * counters, zeroed with them by the parse prologue (counting
		 * grouping: sgpu_mplan_counters, 64 + 64 words), else in pex
		 * and kout (free once k_mp_final has run, each >= 256 B) */
		const uint32_t ob = (n + MP_OBLOCK * MP_OPER - 1) /
				    (MP_OBLOCK * MP_OPER);
		uint32_t *ghist = pex, *gcur = kout;
		if (!in->radix && in->cnt_zeroed && in->nsess <= 65536) {
			ghist = (uint32_t *)p;
			gcur = ghist + MP_OBINS;
		}
		else if (hipMemsetAsync(pex, 0, MP_OBINS * 4, st) != hipSuccess ||
			 hipMemsetAsync(kout, 0, MP_OBINS * 4, st) != hipSuccess)
			return EIO;
		hipLaunchKernelGGL(k_mp_ocount, dim3(ob), dim3(MP_OBLOCK), 0,
				   st, pos, end, ghist, n);
		hipLaunchKernelGGL(k_mp_oscatter, dim3(ob), dim3(MP_OBLOCK), 0,
				   st, pos, end, (const uint32_t *)ghist, gcur,
				   order, n);
	}
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}

extern "C" size_t sgpu_mfold_scratch(uint32_t n)
{
	return 2 * ((size_t)(n + MP_BLOCK - 1) / MP_BLOCK + 2) * 4;
}

extern "C" int sgpu_mfold_rtp(int phase, const uint32_t *nfail,
			      const struct sgpu_mplan_in *in,
			      const struct sgpu_hdr *hdr, const uint32_t *sess,
			      const uint64_t *desc, const uint8_t *verdict,
			      const uint32_t *end0, uint32_t *pos,
			      uint32_t *end, int32_t *err, int gcm,
			      const struct sgpu_sstate *st_in,
			      struct sgpu_sstate *st_out, void *scratch,
			      size_t scratch_bytes, uint32_t *fscratch,
			      struct sgpu_fold_out *out, void *stream)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t n = in->n, nb = (n + MP_BLOCK - 1) / MP_BLOCK;
	uint8_t *p = (uint8_t *)scratch;
	/* the planner's scratch layout (sgpu_mplan_rtp_phase) */
	p += mp_align((size_t)n * 4);                                   /* kout */
	p += mp_align((size_t)n * 4);                                   /* vin */
	const uint32_t *vout = (const uint32_t *)p;  p += mp_align((size_t)n * 4);
	p += mp_align((size_t)n * 4);                                   /* pex */
	const uint32_t *sseq = (const uint32_t *)p;  p += mp_align((size_t)n * 4);
	p += mp_align((size_t)n * 4);                                   /* sssrc */
	p += mp_align((size_t)nb * 4 + 64);                             /* bcnt */
	const uint32_t *segf = (const uint32_t *)p;
	p += mp_align((size_t)in->nsess * 4);
	const uint32_t *segl = (const uint32_t *)p;
	p += mp_align((size_t)in->nsess * 4);
	if (!n || !in->nsess || (size_t)(p - (uint8_t *)scratch) > scratch_bytes)
		return EINVAL;
	int32_t *blast = (int32_t *)fscratch, *bprev = blast + nb + 2;
	mf_ctx c = {vout, sess, sseq, segf, st_in, verdict, n, in->nsess, nfail};
	if (phase != 2) {
		/* the verdict: out->fail (0 also when nothing is to fold) */
		hipLaunchKernelGGL(k_mf_count, dim3(nb), dim3(MP_BLOCK), 0, st,
				   c, blast, out);
		hipLaunchKernelGGL(k_mf_scan, dim3(1), dim3(1024), 0, st,
				   (const int32_t *)blast, bprev, nb, nfail);
		hipLaunchKernelGGL(k_mf_check, dim3(nb), dim3(MP_BLOCK), 0, st,
				   c, (const int32_t *)bprev, st_out, out);
	}
	if (phase != 1) {
		/* on a held fold: the forged packets' results (over those of
		 * sgpu_plan_finish) and the touched sessions' windows */
		hipLaunchKernelGGL(k_mf_results, dim3(nb), dim3(MP_BLOCK), 0,
				   st, verdict, hdr, end0, pos, end, err, n, gcm,
				   (const struct sgpu_fold_out *)out, nfail);
		hipLaunchKernelGGL(k_mf_final,
				   dim3((in->nsess + MP_BLOCK - 1) / MP_BLOCK),
				   dim3(MP_BLOCK), 0, st, c, segl, desc, st_out,
				   (const struct sgpu_fold_out *)out);
	}
	return hipGetLastError() == hipSuccess ? 0 : EIO;
}
