/*
 * plan_buckets.hip -- multi-session RTP batches planned on the device in
 * three launches around the crypto (srtpgpu.h struct sgpu_bplan).
 *
 * The reference keeps one sequential state machine per stream
 * (srtp_encrypt srtp.c:203-215, 279-280; srtp_decrypt srtp.c:310-321,
 * 426-427; srtp_get_index misc.c:22-41; srtp_replay_check replay.c:32-62),
 * and streams of different sessions are independent.  The counting
 * grouping of plan_multi.hip needs a global scan between its passes (17
 * launches per call with the plan and the launch order); here the sessions
 * are cut into buckets of 2^bshift consecutive ids, each with a fixed
 * region of `cap` entries, so a packet is placed in the launch that parses
 * it, and every later step of a session happens inside the one workgroup
 * that owns its bucket:
 *
 *   k_bp_scatter  per packet: parse + window checks (k_parse), end copy,
 *                 its slot in its bucket (LDS count per workgroup, one
 *                 global atomic per (workgroup, bucket) for the base)
 *   k_bp_plan     per bucket, in LDS: the sessions' resident states, the
 *                 entries grouped by session (counting) and ranked by
 *                 packet index inside each session, the single-stream
 *                 speculation per session segment (k_mp_count / desc /
 *                 final of plan_multi.hip), the launch order (length bins
 *                 in arrival order); each workgroup ORs a share of the
 *                 scatter's fail words into the plan out (no last-workgroup
 *                 ticket: its release fences cost ~40 us per call)
 *   k_bp_finish   results; the bucket workgroups re-zero the bucket and
 *                 bin counters and commit the touched states; with
 *                 speculation misses the verdict fold per bucket (k_mf_*
 *                 of plan_multi.hip) and, in the last workgroup, the
 *                 forged packets' EAUTH results and the commit
 *
 * A batch the buckets cannot hold (a bucket over cap, a session over
 * SGPU_BP_SEGMAX packets in it) fails with SPF_SEG and is re-planned by the
 * radix-sort grouping; any other failed check rejects the plan exactly as
 * the other planners do (nothing modified, the host plans).
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include "../srtpgpu.h"
#include "plan_common.h"

#ifndef EAUTH
#define EAUTH 217               /* include/re_types.h:215-217 */
#endif

#define BPB SGPU_BP_BLOCK
#define BP_IMASK 0x3ffffffu     /* entry: packet index | length bin << 26 */
#define BP_OBINS 64

/* ---- block-wide scans (1024 threads, 16 waves) ------------------------ */

__device__ __forceinline__ uint32_t bp_excl_sum(uint32_t v, uint32_t *wsum,
						uint32_t *total)
{
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	uint32_t x = v;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t u = (uint32_t)__shfl_up((int)x, d);
		if (lane >= (uint32_t)d)
			x += u;
	}
	if (lane == 63)
		wsum[wv] = x;
	__syncthreads();
	uint32_t pre = 0, tot = 0;
	for (uint32_t q = 0; q < BPB / 64u; q++) {
		const uint32_t w = wsum[q];
		pre += q < wv ? w : 0u;
		tot += w;
	}
	__syncthreads();
	if (total)
		*total = tot;
	return pre + x - v;
}

/* exclusive prefix maximum of v (-1: none) */
__device__ __forceinline__ int32_t bp_excl_max(int32_t v, int32_t *wmax)
{
	const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	int32_t x = v;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const int32_t u = __shfl_up(x, d);
		if (lane >= (uint32_t)d)
			x = max(x, u);
	}
	if (lane == 63)
		wmax[wv] = x;
	int32_t below = __shfl_up(x, 1);
	if (lane == 0)
		below = -1;
	__syncthreads();
	int32_t pre = -1;
	for (uint32_t q = 0; q < wv; q++)
		pre = max(pre, wmax[q]);
	__syncthreads();
	return max(pre, below);
}

/* the last-workgroup hand-off (cdna_hip_programming.md, the split-K
 * reducer recipe): every wave's stores drained, then one release fence and
 * one agent-scope ticket per workgroup; the workgroup drawing the last
 * ticket acquires before it reads the others' words */
__device__ __forceinline__ bool bp_last(uint32_t *ticket, uint32_t tbase,
					uint32_t nblk, uint32_t *flag)
{
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x == 0) {
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		const uint32_t t = __hip_atomic_fetch_add(ticket, 1u,
							  __ATOMIC_RELAXED,
							  __HIP_MEMORY_SCOPE_AGENT);
		*flag = (t - tbase) == nblk - 1u;
		if (*flag) {
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		}
	}
	__syncthreads();
	return *flag != 0;
}

static_assert(sizeof(struct sgpu_sstate) == 32 &&
	      offsetof(struct sgpu_sstate, flags) == 12,
	      "bp_ld/bp_st move the state as two 16-byte words");

__device__ __forceinline__ struct sgpu_sstate bp_ld(const struct sgpu_sstate *p)
{
	const uint4 a = ((const uint4 *)p)[0], b = ((const uint4 *)p)[1];
	struct sgpu_sstate s;
	s.ssrc = a.x; s.roc = a.y; s.s_l = a.z; s.flags = a.w;
	s.lix = (uint64_t)b.y << 32 | b.x;
	s.bitmap = (uint64_t)b.w << 32 | b.z;
	return s;
}

__device__ __forceinline__ void bp_st(struct sgpu_sstate *p,
				      const struct sgpu_sstate &s)
{
	((uint4 *)p)[0] = make_uint4(s.ssrc, s.roc, s.s_l, s.flags);
	((uint4 *)p)[1] = make_uint4((uint32_t)s.lix, (uint32_t)(s.lix >> 32),
				     (uint32_t)s.bitmap,
				     (uint32_t)(s.bitmap >> 32));
}

/* ---- 1: parse, checks, bucket scatter --------------------------------- */

__global__ void __launch_bounds__(BPB)
k_bp_scatter(const uint8_t *__restrict__ arena, uint64_t asz,
	     const struct sgpu_bplan P)
{
	__shared__ uint32_t hist[SGPU_BP_NBMAX], base[SGPU_BP_NBMAX];
	__shared__ uint32_t oh[BP_OBINS], ob[BP_OBINS];
	__shared__ uint32_t bf, hl0s;
	const uint32_t tid = threadIdx.x, nb = P.nb;
	for (uint32_t k = tid; k < nb; k += BPB)
		hist[k] = 0;
	if (tid < BP_OBINS)
		oh[tid] = 0;
	if (tid == 0) {
		bf = 0;
		/* packet 0's header: every packet's class is checked against
		 * it (k_mp_count's SPF_CLASS) */
		const uint32_t q = P.pos[0], qe = P.end[0];
		hl0s = parse_rtp_hdr(arena + q, q, (qe > q && qe <= asz) ?
						   qe - q : 0u).hdr_len;
		if (blockIdx.x == 0) {
			/* the call's outs: nothing else writes them before the
			 * plan kernel (the crypto launch's miss counter too) */
			*P.nfail = 0;
			P.out->fail = 0;
			P.out->wraps = 0;
			P.out->ssrc0 = 0;
			P.out->s_l_last = 0;
			P.out->nfail = 0;
			P.fo->fail = 0;
		}
	}
	uint32_t bk[SGPU_BP_PPT], rk[SGPU_BP_PPT], wd[SGPU_BP_PPT];
	uint32_t orank[SGPU_BP_PPT], wy[SGPU_BP_PPT], wz[SGPU_BP_PPT];
	uint32_t pv[SGPU_BP_PPT], ev[SGPU_BP_PPT], cv[SGPU_BP_PPT];
	uint32_t sv[SGPU_BP_PPT], w0[SGPU_BP_PPT], w2[SGPU_BP_PPT];
	uint32_t f = 0;
	const uint32_t i0 = blockIdx.x * (BPB * SGPU_BP_PPT) + tid;
	/* every window first, then every header's two words: all of a
	 * thread's loads in flight together */
#pragma unroll
	for (int j = 0; j < SGPU_BP_PPT; j++) {
		const uint32_t i = i0 + j * BPB;
		pv[j] = ev[j] = cv[j] = sv[j] = 0;
		if (i < P.n) {
			pv[j] = P.pos[i];
			ev[j] = P.end[i];
			cv[j] = P.capv ? P.capv[i] : 0u;
			sv[j] = P.sess[i];
		}
	}
#pragma unroll
	for (int j = 0; j < SGPU_BP_PPT; j++) {
		const uint32_t p = pv[j], e = ev[j];
		w0[j] = w2[j] = 0;
		/* the batch APIs' 4-byte aligned windows (parse_rtp_hdr's fast
		 * load); anything else parses byte by byte below */
		if (i0 + j * BPB < P.n && e > p && e <= asz && e - p >= 12 &&
		    !(p & 3u)) {
			w0[j] = *(const uint32_t *)(arena + p);
			w2[j] = *(const uint32_t *)(arena + p + 8);
		}
	}
	__syncthreads();
	const uint32_t hl0 = hl0s;
#pragma unroll
	for (int j = 0; j < SGPU_BP_PPT; j++) {
		const uint32_t i = i0 + j * BPB;
		bk[j] = 0xffffffffu;
		rk[j] = wd[j] = orank[j] = wy[j] = wz[j] = 0;
		if (i >= P.n)
			continue;
		const uint32_t p = pv[j], e = ev[j], c = cv[j];
		uint32_t s = sv[j];
		P.es[i] = e;
		/* a window outside the arena is never read */
		const uint32_t left = (e > p && e <= asz) ? e - p : 0u;
		struct sgpu_hdr h;
		const uint32_t b0 = w0[j] & 0xffu;
		if (left >= 12 && !(p & 3u) && !(b0 & 0x1fu)) {
			/* no CSRC, no extension: the header is the two words */
			h.seq = (uint16_t)((w0[j] >> 8 & 0xff00u) | (w0[j] >> 24));
			h.ssrc = __builtin_bswap32(w2[j]);
			h.err_pos = 0;
			h.hdr_len = 12;
		}
		else {
			h = parse_rtp_hdr(arena + p, p, left);
		}
		P.hdr[i] = h;
		if (i == 0) {
			/* the crypto launches' class guards (out->fail is their
			 * second guard word, final after the plan kernel) */
			P.out->hl0 = h.hdr_len;
			for (uint32_t q = 0; q < 4; q++)
				P.out->skip[q] = h.hdr_len == 0xffffffffu ||
						 ((h.hdr_len >> 2) & 3u) != q;
		}
		/* the window checks of k_mp_count (via k_parse_rtp_checked) */
		if (h.hdr_len == 0xffffffffu)
			f |= SPF_PARSE;
		else if (!P.prot && e - p - h.hdr_len < P.tag)
			f |= SPF_PARSE;
		if (e - p >= P.maxlen)
			f |= SPF_SIZE;
		if ((p & 3u) || p > e || e > asz ||
		    (P.capv && (e > c || c > asz)))
			f |= SPF_BAD;
		if (P.prot && P.capv && (uint64_t)e + P.need > (uint64_t)c)
			f |= SPF_CAP;
		if (s >= P.nsess) {
			f |= SPF_BAD;
			s = P.nsess - 1u;
		}
		if (hl0 == 0xffffffffu)
			f |= SPF_PARSE;
		else if (h.hdr_len != 0xffffffffu && ((h.hdr_len ^ hl0) >> 2) & 3u)
			f |= SPF_CLASS;
		/* the crypto launch order's class: descending 64-B chunks */
		const uint32_t L = e >= p ? e - p : 0u, ch = (L + 63u) >> 6;
		const uint32_t bin = (BP_OBINS - 1u) -
				     (ch < BP_OBINS - 1u ? ch : BP_OBINS - 1u);
		bk[j] = s >> P.bshift;
		rk[j] = atomicAdd(&hist[bk[j]], 1u);
		orank[j] = atomicAdd(&oh[bin], 1u);
		wd[j] = i | bin << 26;
		/* the plan kernel's whole view of the packet, so it gathers
		 * nothing: seq, session in bucket, SSRC */
		wy[j] = (uint32_t)h.seq | (s - (bk[j] << P.bshift)) << 16;
		wz[j] = h.ssrc;
	}
	if (blockIdx.x == 0 && tid == 0 && P.pred && *P.pred)
		f |= SPF_PRED;          /* sgpu_gate_pred */
	__syncthreads();
	for (uint32_t k = tid; k < nb; k += BPB)
		base[k] = hist[k] ? atomicAdd(&P.bcount[k], hist[k]) : 0u;
	if (tid < BP_OBINS)
		ob[tid] = oh[tid] ? atomicAdd(&P.obins[tid], oh[tid]) : 0u;
	__syncthreads();
#pragma unroll
	for (int j = 0; j < SGPU_BP_PPT; j++) {
		if (bk[j] == 0xffffffffu)
			continue;
		/* the packet's place in its length bin: the workgroup's packets
		 * stay together there, so a crypto wave reads neighbouring
		 * slots of the arena (arrival order, not bucket order: the
		 * bucket-major order measured 1.73 ms per launch against 0.98) */
		const uint32_t slot = base[bk[j]] + rk[j];
		if (slot < P.cap)
			P.tmp[(size_t)bk[j] * P.cap + slot] =
				make_uint4(wd[j], wy[j], wz[j],
					   ob[wd[j] >> 26] + orank[j]);
		else
			f |= SPF_SEG;   /* the bucket overflows: radix re-plan */
	}
	if (f)
		atomicOr(&bf, f);
	__syncthreads();
	if (tid == 0)
		P.afail[blockIdx.x] = bf;
}

/* ---- 2: per bucket, the plan ------------------------------------------ */

#define BP_EPT (SGPU_BP_CAPMAX / BPB)   /* entries per thread, at most */

struct BpPlanLds {
	uint32_t ent[SGPU_BP_CAPMAX];   /* entry word, arrival order in bucket */
	uint16_t sq[SGPU_BP_CAPMAX];    /* seq */
	uint16_t srt[SGPU_BP_CAPMAX];   /* rank in session, then: entries by
					   (session, packet index) */
	uint16_t un[SGPU_BP_CAPMAX];    /* entries by session (unstable) */
	uint16_t pw[SGPU_BP_CAPMAX];    /* rollovers up to and including
					   sorted position k */
	uint8_t sl[SGPU_BP_CAPMAX];     /* session in bucket */
	struct sgpu_sstate st[SGPU_BP_NSB];
	uint64_t lixl[SGPU_BP_NSB];     /* index of the segment's last packet */
	uint32_t cnt[SGPU_BP_NSB], start[SGPU_BP_NSB];
	uint32_t smin[SGPU_BP_NSB], smax[SGPU_BP_NSB];
	uint32_t sl0[SGPU_BP_NSB];      /* s_l the segment starts from */
	uint32_t rbase[SGPU_BP_NSB];    /* ROC of position k: rbase + pw[k] */
	uint32_t froc[SGPU_BP_NSB], fsl[SGPU_BP_NSB];   /* after the batch */
	uint32_t wlo[SGPU_BP_NSB], whi[SGPU_BP_NSB];    /* replay bits */
	uint32_t bb[BP_OBINS];
	uint32_t wsum[BPB / 64];
	uint32_t bf;
};

/* speculated s_l seen by sorted position k (its segment l starting at f):
 * the previous packet's seq, or the session's stored s_l (a new stream:
 * its first packet's seq, stream.c:87-109) */
__device__ __forceinline__ uint32_t bp_sb(const BpPlanLds &S, uint32_t k,
					  uint32_t f, uint32_t l)
{
	return k != f ? S.sq[S.srt[k - 1]] : S.sl0[l];
}

/* index of sorted position k (mp_ix of plan_multi.hip) */
__device__ __forceinline__ uint64_t bp_ix(const BpPlanLds &S, uint32_t prot,
					  uint32_t k, uint32_t f, uint32_t l,
					  uint32_t *flp, uint32_t *rocp,
					  bool *wrapp, uint32_t *sbp)
{
	const uint32_t seq = S.sq[S.srt[k]];
	const uint32_t sb = bp_sb(S, k, f, l);
	const bool wrap = plan_wrap(seq, sb);
	/* ROC after this packet's own rollover */
	const uint32_t roc = S.rbase[l] + S.pw[k];
	uint64_t ix;
	uint32_t fl = SD_RUN | SD_CIPHER;
	if (prot) {
		ix = 65536ull * roc + seq;                   /* srtp.c:215 */
	}
	else {
		const int32_t v = plan_v(roc, wrap ? 0u : sb, seq);
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

__global__ void __launch_bounds__(BPB)
k_bp_plan(const struct sgpu_bplan P)
{
	__shared__ BpPlanLds S;
	const uint32_t tid = threadIdx.x, b = blockIdx.x;
	const uint32_t s0 = b << P.bshift;
	const uint32_t ns = min(1u << P.bshift, P.nsess - s0);
	const uint32_t EPT = P.cap / BPB;
	uint32_t m = P.bcount[b];
	uint32_t f = 0;
	{
		/* the scatter workgroups' fail words, spread over the buckets
		 * (no workgroup waits for another) */
		const uint32_t na = (P.n + BPB * SGPU_BP_PPT - 1) /
				    (BPB * SGPU_BP_PPT);
		for (uint32_t k = b + tid * P.nb; k < na; k += BPB * P.nb)
			f |= P.afail[k];
	}
	if (m > P.cap) {
		f |= SPF_SEG;           /* (the scatter flagged it too) */
		m = 0;
	}
	/* the bucket's entries (EPT per thread, all in flight): index and
	 * length bin, seq and session, SSRC, place in the bin */
	uint4 ev4[BP_EPT];
#pragma unroll
	for (int j = 0; j < BP_EPT; j++) {
		const uint32_t k = tid + j * BPB;
		ev4[j] = k < m ? P.tmp[(size_t)b * P.cap + k]
			       : make_uint4(0, 0, 0, 0);
	}
	if (tid == 0)
		S.bf = 0;
	if (tid < BP_OBINS)
		S.bb[tid] = P.obins[tid];       /* the bins' totals */
	if (tid < ns) {
		/* the session's resident state (k_sst_load): the host's upload
		 * first where the device copy is stale */
		const uint32_t s = s0 + tid, slot = P.cm[s] >> 1;
		struct sgpu_sstate x;
		if (P.upneed && P.upneed[s]) {
			x = bp_ld(P.up + s);
			bp_st(P.sst + slot, x);
		}
		else {
			x = bp_ld(P.sst + slot);
		}
		S.st[tid] = x;
		S.cnt[tid] = 0;
		S.smin[tid] = 0xffffffffu;
		S.smax[tid] = 0;
		S.wlo[tid] = S.whi[tid] = 0;
	}
	__syncthreads();
	/* the entries: seq, session, rank in session (the header checks
	 * were the scatter's) */
#pragma unroll
	for (int j = 0; j < BP_EPT; j++) {
		const uint32_t k = tid + j * BPB;
		if (k >= m)
			continue;
		const uint32_t l = ev4[j].y >> 16;
		S.ent[k] = ev4[j].x;
		S.sq[k] = (uint16_t)ev4[j].y;
		S.sl[k] = (uint8_t)l;
		S.srt[k] = (uint16_t)atomicAdd(&S.cnt[l], 1u);
		atomicMin(&S.smin[l], ev4[j].z);
		atomicMax(&S.smax[l], ev4[j].z);
	}
	__syncthreads();
	/* segment starts (sessions, <= 256: wave 0) and the length bins'
	 * starts in the launch order (64: wave 1) */
	if (tid < 64) {
		uint32_t c4[4], v = 0;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t l = 4 * tid + q;
			c4[q] = l < ns ? S.cnt[l] : 0u;
			v += c4[q];
		}
		uint32_t x = v;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const uint32_t u = (uint32_t)__shfl_up((int)x, d);
			if (tid >= (uint32_t)d)
				x += u;
		}
		uint32_t run = x - v;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const uint32_t l = 4 * tid + q;
			if (l < SGPU_BP_NSB)
				S.start[l] = run;
			run += c4[q];
		}
	}
	else if (tid < 128) {
		const uint32_t lane = tid - 64, v = S.bb[lane];
		uint32_t x = v;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const uint32_t u = (uint32_t)__shfl_up((int)x, d);
			if (lane >= (uint32_t)d)
				x += u;
		}
		S.bb[lane] = x - v;
	}
	/* one SSRC per session: the stored one, or the segment's
	 * (k_mp_count's SPF_SSRC, order-free) */
	if (tid < ns && S.cnt[tid]) {
		const struct sgpu_sstate &x = S.st[tid];
		if (S.smin[tid] != S.smax[tid] ||
		    ((x.flags & SST_EXISTS) && S.smin[tid] != x.ssrc))
			f |= SPF_SSRC;
		if (S.cnt[tid] > SGPU_BP_SEGMAX)
			f |= SPF_SEG;
	}
	if (f)
		atomicOr(&S.bf, f);
	__syncthreads();
	const bool dead = S.bf != 0;    /* the plan fails: nothing more */
	if (!dead) {
		/* grouped by session; the crypto launch order (descending
		 * length bins, each scatter workgroup's packets together) */
#pragma unroll
		for (int j = 0; j < BP_EPT; j++) {
			const uint32_t k = tid + j * BPB;
			if (k >= m)
				continue;
			const uint32_t i = ev4[j].x & BP_IMASK;
			S.un[S.start[S.sl[k]] + S.srt[k]] = (uint16_t)k;
			P.order[S.bb[ev4[j].x >> 26] + ev4[j].w] = i;
		}
	}
	__syncthreads();
	if (!dead) {
		/* inside a session by packet index: the stable order the
		 * reference processes them in */
		for (uint32_t q = tid; q < m; q += BPB) {
			const uint32_t e = S.un[q], l = S.sl[e];
			const uint32_t f0 = S.start[l], c = S.cnt[l];
			const uint32_t ie = S.ent[e] & BP_IMASK;
			uint32_t r = 0;
			for (uint32_t t = f0; t < f0 + c; t++)
				r += (S.ent[S.un[t]] & BP_IMASK) < ie ? 1u : 0u;
			S.srt[f0 + r] = (uint16_t)e;
		}
	}
	__syncthreads();
	if (tid < ns && !dead)
		S.sl0[tid] = (S.st[tid].flags & SST_SL_SET) ? S.st[tid].s_l
			     : S.cnt[tid] ? S.sq[S.srt[S.start[tid]]] : 0u;
	__syncthreads();
	/* rollovers up to each sorted position (EPT consecutive positions per
	 * thread; the sum runs across segments, rbase takes it off) */
	uint32_t loc = 0, wbits = 0;
	if (!dead) {
		for (uint32_t j = 0; j < EPT; j++) {
			const uint32_t k = tid * EPT + j;
			if (k >= m)
				break;
			const uint32_t l = S.sl[S.srt[k]];
			const bool w = plan_wrap(S.sq[S.srt[k]],
						 bp_sb(S, k, S.start[l], l));
			wbits |= (w ? 1u : 0u) << j;
			loc += w ? 1u : 0u;
		}
	}
	{
		uint32_t run = bp_excl_sum(loc, S.wsum, NULL);
		if (!dead)
			for (uint32_t j = 0; j < EPT; j++) {
				const uint32_t k = tid * EPT + j;
				if (k >= m)
					break;
				run += (wbits >> j) & 1u;
				S.pw[k] = (uint16_t)run;
			}
	}
	__syncthreads();
	if (tid < ns && !dead && S.cnt[tid]) {
		/* roc(k) = stored ROC + rollovers of positions f..k */
		const uint32_t f0 = S.start[tid];
		const bool wf = plan_wrap(S.sq[S.srt[f0]], S.sl0[tid]);
		S.rbase[tid] = S.st[tid].roc - S.pw[f0] + (wf ? 1u : 0u);
	}
	__syncthreads();
	if (!dead) {
		/* per packet: the checks of k_mp_count that need the order,
		 * the index, the replay speculation, desc (k_mp_desc) */
		for (uint32_t k = tid; k < m; k += BPB) {
			const uint32_t e = S.srt[k], l = S.sl[e];
			const uint32_t f0 = S.start[l];
			const bool last = k + 1 == f0 + S.cnt[l];
			const uint32_t i = S.ent[e] & BP_IMASK;
			const uint32_t seq = S.sq[e];
			uint32_t fl, sb, roc;
			bool wrap;
			const uint64_t ix = bp_ix(S, P.prot, k, f0, l, &fl, &roc,
						  &wrap, &sb);
			if (!P.prot && (int)seq - (int)sb > 32768)
				f |= SPF_TIMEOUT;
			if (!last && !wrap && seq < sb)
				f |= SPF_ORDER;
			if (!P.prot) {
				/* replay: every packet new (replay.c:32-62),
				 * above the session's pre-batch lix as well */
				const struct sgpu_sstate &x = S.st[l];
				bool ok;
				if (k == f0) {
					if (ix > x.lix) {
						ok = true;
					}
					else {
						const uint64_t d = x.lix - ix;
						ok = d < 64 && !(x.bitmap & (1ull << d));
					}
				}
				else {
					ok = ix > bp_ix(S, 0, k - 1, f0, l, NULL, NULL,
							NULL, NULL) && ix > x.lix;
				}
				if (!ok)
					f |= SPF_REPLAY;
			}
			if (last) {
				/* the session after the batch (k_mp_final) */
				S.froc[l] = roc;
				S.fsl[l] = wrap ? seq : (seq > sb ? seq : sb);
				S.lixl[l] = ix;
			}
			P.desc[i] = d_desc(ix, fl);
			P.sorted[(size_t)b * P.cap + k] = i;
		}
	}
	__syncthreads();
	if (!dead && !P.prot) {
		/* the replay window after the batch (replay.c:32-62): every
		 * index is new and increasing (checked above), so it holds the
		 * batch's indices within 64 of the last one and the stored
		 * window shifted up to it -- each packet sets its own bit */
		for (uint32_t k = tid; k < m; k += BPB) {
			const uint32_t e = S.srt[k], l = S.sl[e];
			const uint32_t f0 = S.start[l];
			if (k + 64u < f0 + S.cnt[l])
				continue;       /* 64 or more packets before the
						   last: shifted out */
			const uint64_t top = S.lixl[l] > S.st[l].lix ?
					     S.lixl[l] : S.st[l].lix;
			const uint64_t d = top - bp_ix(S, 0, k, f0, l, NULL, NULL,
						       NULL, NULL);
			if (d < 32)
				atomicOr(&S.wlo[l], 1u << d);
			else if (d < 64)
				atomicOr(&S.whi[l], 1u << (d - 32));
		}
	}
	__syncthreads();
	/* every session's state after the batch */
	if (tid < ns) {
		const uint32_t s = s0 + tid, c = S.cnt[tid];
		struct sgpu_sstate o = S.st[tid];
		o.flags &= ~(uint32_t)SST_TOUCHED;
		if (c && !dead) {
			const struct sgpu_sstate &x = S.st[tid];
			o.ssrc = (x.flags & SST_EXISTS) ? x.ssrc : S.smin[tid];
			o.roc = S.froc[tid];
			o.s_l = S.fsl[tid];
			o.flags = SST_EXISTS | SST_SL_SET | SST_TOUCHED;
			if (!P.prot) {
				const uint64_t top = S.lixl[tid] > x.lix ?
						     S.lixl[tid] : x.lix;
				uint64_t bm = (uint64_t)S.whi[tid] << 32 | S.wlo[tid];
				if (top - x.lix < 64)
					bm |= x.bitmap << (top - x.lix);
				o.lix = top;
				o.bitmap = bm;
			}
			P.sseg[s] = S.start[tid] | c << 16;
		}
		else {
			P.sseg[s] = 0;
		}
		bp_st(P.sout + s, o);
	}
	if (f)
		atomicOr(&S.bf, f);
	__syncthreads();
	if (tid == 0 && S.bf)
		atomicOr(&P.out->fail, S.bf);
}

/* ---- 3: results, commit, verdict fold --------------------------------- */

struct BpFoldLds {
	uint32_t idx[SGPU_BP_CAPMAX];   /* packet of sorted position k */
	uint16_t sq[SGPU_BP_CAPMAX];
	int16_t ev[SGPU_BP_CAPMAX];     /* last event position <= k, or -1 */
	uint8_t au[SGPU_BP_CAPMAX];     /* tag verified */
	uint8_t sl[SGPU_BP_CAPMAX];     /* session in bucket */
	struct sgpu_sstate st[SGPU_BP_NSB];     /* before the batch */
	uint32_t f0[SGPU_BP_NSB], cnt[SGPU_BP_NSB];
	int32_t wmax[BPB / 64];
	uint32_t m, cf, flag, ff;
};

/* the s_l a segment starts from (stream_get_seq, stream.c:87-109) */
__device__ __forceinline__ uint32_t bf_sl0(const BpFoldLds &S, uint32_t l)
{
	return (S.st[l].flags & SST_SL_SET) ? S.st[l].s_l : S.sq[S.f0[l]];
}

/* speculated s_l of position k */
__device__ __forceinline__ uint32_t bf_sb(const BpFoldLds &S, uint32_t k,
					  uint32_t l)
{
	return k == S.f0[l] ? bf_sl0(S, l) : S.sq[k - 1];
}

/* true s_l after event position e (before the segment: its start) */
__device__ __forceinline__ uint32_t bf_slv(const BpFoldLds &S, int32_t e,
					   uint32_t l)
{
	if (e < (int32_t)S.f0[l])
		return bf_sl0(S, l);
	return S.au[e] ? S.sq[e] : 0u;
}

/* forged packet i: srtp_decrypt's EAUTH (srtp.c:342-359: HMAC, end at
 * the tag; 404-411: GCM, end as it was) */
__device__ __forceinline__ void bp_forged(const struct sgpu_bplan &P,
					  uint32_t i)
{
	P.err[i] = EAUTH;
	P.posw[i] += P.hdr[i].hdr_len;
	P.endw[i] = P.gcm ? P.es[i] : P.es[i] + (uint32_t)P.delta;
}

/* the call's outcome (plan out, fold out) to the caller's pinned mirror
 * with vector stores, once it is final: no blit copy behind the launch */
__device__ __forceinline__ void bp_post(const struct sgpu_bplan &P,
					uint32_t tid)
{
	if (!P.outh)
		return;
	const uint32_t *src = (const uint32_t *)P.out;
	for (uint32_t w = tid; w < P.outbytes / 4u; w += BPB)
		P.outh[w] = src[w];
}

__global__ void __launch_bounds__(BPB)
k_bp_finish(const struct sgpu_bplan P)
{
	__shared__ BpFoldLds S;
	const uint32_t tid = threadIdx.x;
	const uint32_t fail = P.out->fail;
	const uint32_t nf = *(volatile const uint32_t *)P.nfail;
	if (blockIdx.x >= P.nb) {
		/* per packet (coalesced): every authentic packet's results
		 * (k_plan_finish); forged ones wait for the fold */
		if (fail)
			return;
		const uint32_t i0 = (blockIdx.x - P.nb) * (BPB * SGPU_BP_PPT);
#pragma unroll
		for (int j = 0; j < SGPU_BP_PPT; j++) {
			const uint32_t i = i0 + j * BPB + tid;
			if (i >= P.n)
				break;
			if (P.prot || !nf || (P.verdict[i] & SV_TAG_OK)) {
				P.endw[i] = P.es[i] + (uint32_t)P.delta;
				P.err[i] = 0;
			}
		}
		return;
	}
	const uint32_t b = blockIdx.x;
	const uint32_t s0 = b << P.bshift;
	const uint32_t ns = min(1u << P.bshift, P.nsess - s0);
	const uint32_t EPT = P.cap / BPB;
	if (tid == 0) {
		S.cf = 0;
		S.m = 0;
		/* the scatter's counters back to zero for the next call (the
		 * plan kernel, their last reader, is done) */
		P.bcount[b] = 0;
	}
	if (b == 0 && tid < BP_OBINS)
		P.obins[tid] = 0;
	if (b == 0 && tid == 0 && (fail || !nf)) {
		/* nothing to fold: the call's outcome is known */
		struct sgpu_fold_out *fo = P.fo;
		fo->fail = 0;
		fo->nok = 0;
		fo->first_ok = 0xffffffffu;
		fo->last_ok = 0xffffffffu;
		fo->s_l = 0;
		fo->pad = 0;
		fo->lix = 0;
		fo->bitmap = 0;
		P.out->nfail = nf;
		if (P.gate)     /* sgpu_gate_set */
			*P.gate = fail ? 1u : 0u;
	}
	__syncthreads();
	if (b == 0 && (fail || !nf))
		bp_post(P, tid);
	if (fail || !nf) {
		/* every tag verified: the touched states replace the resident
		 * ones (k_sst_commit) */
		if (!fail && tid < ns) {
			const uint32_t s = s0 + tid;
			struct sgpu_sstate o = bp_ld(P.sout + s);
			if (o.flags & SST_TOUCHED) {
				o.flags &= ~(uint32_t)SST_TOUCHED;
				bp_st(P.sst + (P.cm[s] >> 1), o);
			}
		}
		return;
	}
	{
		/* the verdict fold of this bucket's sessions (k_mf_count /
		 * scan / check / final): a forged packet still bumps the ROC
		 * on a rollover but never sets s_l (srtp.c:310-321, 342-359,
		 * 426-427), so later packets of its session may see another
		 * s_l than the plan assumed */
		if (tid < ns) {
			const uint32_t s = s0 + tid, v = P.sseg[s];
			S.st[tid] = bp_ld(P.sst + (P.cm[s] >> 1));
			S.f0[tid] = v & 0xffffu;
			S.cnt[tid] = v >> 16;
			if (v >> 16)
				atomicMax(&S.m, (v & 0xffffu) + (v >> 16));
			for (uint32_t k = v & 0xffffu; k < (v & 0xffffu) + (v >> 16);
			     k++)
				S.sl[k] = (uint8_t)tid;
		}
		__syncthreads();
		const uint32_t m = S.m;
		for (uint32_t k = tid; k < m; k += BPB) {
			const uint32_t i = P.sorted[(size_t)b * P.cap + k];
			S.idx[k] = i;
			S.sq[k] = P.hdr[i].seq;
			S.au[k] = (P.verdict[i] & SV_TAG_OK) ? 1 : 0;
		}
		__syncthreads();
		/* events: an authentic packet (s_l = seq) or a rollover (s_l =
		 * 0 when forged); the last one at or before each position */
		int32_t loc = -1;
		for (uint32_t j = 0; j < EPT; j++) {
			const uint32_t k = tid * EPT + j;
			if (k >= m)
				break;
			const uint32_t l = S.sl[k];
			if (S.au[k] || plan_wrap(S.sq[k], bf_sb(S, k, l)))
				loc = (int32_t)k;
		}
		{
			int32_t run = bp_excl_max(loc, S.wmax);
			for (uint32_t j = 0; j < EPT; j++) {
				const uint32_t k = tid * EPT + j;
				if (k >= m)
					break;
				const uint32_t l = S.sl[k];
				if (S.au[k] || plan_wrap(S.sq[k], bf_sb(S, k, l)))
					run = (int32_t)k;
				S.ev[k] = (int16_t)run;
			}
		}
		__syncthreads();
		uint32_t cf = 0;
		for (uint32_t k = tid; k < m; k += BPB) {
			const uint32_t l = S.sl[k];
			const int32_t e = k ? S.ev[k - 1] : -1;
			const uint32_t seq = S.sq[k];
			const uint32_t sb = bf_sb(S, k, l);     /* speculated */
			const uint32_t sv = bf_slv(S, e, l);    /* true */
			const bool wrap = plan_wrap(seq, sb);
			bool bad = plan_wrap(seq, sv) != wrap ||
				   (int)seq - (int)sv > 32768;  /* ETIMEDOUT */
			if (!bad && !wrap) {
				/* the same index estimate (misc.c:22-41) */
				bad = plan_v(65536u, sv, seq) !=
				      plan_v(65536u, sb, seq);
				/* an authentic packet sets s_l = seq only if
				 * seq > s_l (srtp.c:426-427) */
				if (S.au[k] && seq < sv)
					bad = true;
			}
			if (bad)
				cf = 1;
		}
		if (P.nofold)
			cf = 1;         /* srtp_gpu_tune nodevfold */
		/* each touched session's s_l and replay window after the batch
		 * (the authentic packets only) */
		if (tid < ns && S.cnt[tid]) {
			const uint32_t s = s0 + tid, f0 = S.f0[tid];
			const uint32_t l = f0 + S.cnt[tid] - 1u;
			struct sgpu_sstate o = bp_ld(P.sout + s);
			o.s_l = bf_slv(S, S.ev[l], tid);
			const struct sgpu_sstate &x = S.st[tid];
			int32_t j = (int32_t)l;
			while (j >= (int32_t)f0 && !S.au[j])
				j--;
			uint64_t lix = x.lix, bm = x.bitmap;
			if (j >= (int32_t)f0) {
				uint32_t q = f0;
				if ((uint32_t)j - f0 >= 64u) {
					q = (uint32_t)j - 63u;
					const uint64_t d = P.desc[S.idx[q - 1]];
					lix = (d & 0xffffull) |
					      ((d >> 16) & 0xffffffffull) << 16;
					bm = 0;
				}
				for (; q <= (uint32_t)j; q++) {
					if (!S.au[q])
						continue;
					const uint64_t d = P.desc[S.idx[q]];
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
			o.lix = lix;
			o.bitmap = bm;
			bp_st(P.sout + s, o);
		}
		if (cf)
			atomicOr(&S.cf, 1u);
		__syncthreads();
		if (tid == 0 && S.cf)
			atomicOr(&P.fo->fail, 1u);
	}
	/* the last bucket workgroup: the fold's outcome (the ticket is taken
	 * only on this path, and reset by the last taker) */
	if (!bp_last(P.ticket, 0u, P.nb, &S.flag))
		return;
	if (tid == 0) {
		S.ff = __hip_atomic_load(&P.fo->fail, __ATOMIC_RELAXED,
					 __HIP_MEMORY_SCOPE_AGENT);
		*P.ticket = 0;
	}
	__syncthreads();
	{
		if (!S.ff) {
			/* the fold holds: the states and the forged packets'
			 * results (a fold that fails leaves all to the host) */
			for (uint32_t s = tid; s < P.nsess; s += BPB) {
				struct sgpu_sstate o = bp_ld(P.sout + s);
				if (o.flags & SST_TOUCHED) {
					o.flags &= ~(uint32_t)SST_TOUCHED;
					bp_st(P.sst + (P.cm[s] >> 1), o);
				}
			}
			if (P.flist) {
				for (uint32_t q = tid; q < nf; q += BPB)
					bp_forged(P, P.flist[q]);
			}
			else {
				for (uint32_t i = tid; i < P.n; i += BPB)
					if (!(P.verdict[i] & SV_TAG_OK))
						bp_forged(P, i);
			}
		}
	}
	if (tid == 0) {
		const uint32_t ff = S.ff;
		struct sgpu_fold_out *fo = P.fo;
		fo->fail = ff ? 1u : 0u;
		fo->nok = 0;
		fo->first_ok = 0xffffffffu;
		fo->last_ok = 0xffffffffu;
		fo->s_l = 0;
		fo->pad = 0;
		fo->lix = 0;
		fo->bitmap = 0;
		P.out->nfail = nf;
		if (P.gate)     /* sgpu_gate_set: completed here, or not */
			*P.gate = ff ? 1u : 0u;
	}
	__syncthreads();
	bp_post(P, tid);
}

/* ---- host side ------------------------------------------------------ */

static size_t bp_align(size_t x)
{
	return (x + 255) & ~(size_t)255;
}

/* srtp_gpu_tune bpexp (A/B): the expected entries per bucket the
 * geometry aims at instead of SGPU_BP_EXP (0: the default) */
static uint32_t g_bp_exp;

extern "C" void sgpu_bplan_set_exp(uint32_t e)
{
	__atomic_store_n(&g_bp_exp, e, __ATOMIC_RELAXED);
}

extern "C" int sgpu_bplan_geometry(uint32_t n, uint32_t nsess,
				   uint32_t *bshift, uint32_t *nb,
				   uint32_t *cap)
{
	if (n == 0 || n > SGPU_BP_NMAX || nsess < 2)
		return -1;
	const uint32_t ge = __atomic_load_n(&g_bp_exp, __ATOMIC_RELAXED);
	const uint64_t emax = ge ? ge : SGPU_BP_EXP;
	/* the most sessions per bucket (<= 256) that keep the expected
	 * entries per bucket <= SGPU_BP_EXP (a workgroup of 1024 lanes, ~two
	 * packets each, two workgroups per CU: one round over the chip at
	 * 64K sessions); the region holds twice the expected entries at most
	 * (a fuller bucket: SPF_SEG, the radix grouping); at most
	 * SGPU_BP_NBMAX buckets */
	for (int sh = 8; sh >= 0; sh--) {
		const uint64_t nbk = ((uint64_t)nsess + (1ull << sh) - 1) >> sh;
		const uint64_t exp = ((uint64_t)n << sh) / nsess + 1;
		if (nbk > SGPU_BP_NBMAX)
			return -1;      /* fewer sessions per bucket: more */
		if (exp > emax)
			continue;
		uint64_t c = 2 * exp + 1024;
		c = (c + BPB - 1) / BPB * BPB;
		if (c > SGPU_BP_CAPMAX)
			c = SGPU_BP_CAPMAX;
		*bshift = (uint32_t)sh;
		*nb = (uint32_t)nbk;
		*cap = (uint32_t)c;
		return 0;
	}
	return -1;
}

extern "C" size_t sgpu_bplan_scratch(uint32_t n, uint32_t nsess, uint32_t nb,
				     uint32_t cap)
{
	const size_t na = (n + BPB * SGPU_BP_PPT - 1) / (BPB * SGPU_BP_PPT);
	return bp_align((size_t)nb * cap * 16) +    /* tmp */
	       bp_align((size_t)nb * cap * 4) +     /* sorted */
	       bp_align(na * 4) +                    /* afail */
	       bp_align((size_t)nsess * 4) +         /* sseg */
	       bp_align((size_t)nsess * 32);         /* sout */
}

static int bp_check(const struct sgpu_bplan *b)
{
	if (!b->n || b->n > SGPU_BP_NMAX || b->nsess < 2 || !b->nb ||
	    b->nb > SGPU_BP_NBMAX || b->bshift > 8 || !b->cap ||
	    b->cap > SGPU_BP_CAPMAX || b->cap % BPB ||
	    ((uint64_t)b->nb << b->bshift) < b->nsess ||
	    ((uint64_t)(b->nb - 1) << b->bshift) >= b->nsess)
		return EINVAL;
	return 0;
}

static int bp_err(const char *what)
{
	const hipError_t e = hipGetLastError();
	if (e == hipSuccess)
		return 0;
	fprintf(stderr, "re_srtp: %s launch: %s\n", what, hipGetErrorString(e));
	return EIO;
}

extern "C" int sgpu_bplan_scatter(const uint8_t *arena, uint64_t arena_size,
				  const struct sgpu_bplan *b, void *stream)
{
	if (bp_check(b))
		return EINVAL;
	const uint32_t g = (b->n + BPB * SGPU_BP_PPT - 1) / (BPB * SGPU_BP_PPT);
	hipLaunchKernelGGL(k_bp_scatter, dim3(g), dim3(BPB), 0,
			   (hipStream_t)stream, arena, arena_size, *b);
	return bp_err("k_bp_scatter");
}

extern "C" int sgpu_bplan_plan(const struct sgpu_bplan *b, void *stream)
{
	if (bp_check(b))
		return EINVAL;
	hipLaunchKernelGGL(k_bp_plan, dim3(b->nb), dim3(BPB), 0,
			   (hipStream_t)stream, *b);
	return bp_err("k_bp_plan");
}

extern "C" int sgpu_bplan_finish(const struct sgpu_bplan *b, void *stream)
{
	if (bp_check(b))
		return EINVAL;
	const uint32_t g = (b->n + BPB * SGPU_BP_PPT - 1) / (BPB * SGPU_BP_PPT);
	hipLaunchKernelGGL(k_bp_finish, dim3(b->nb + g), dim3(BPB), 0,
			   (hipStream_t)stream, *b);
	return bp_err("k_bp_finish");
}
