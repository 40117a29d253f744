/*
 * k_ctr_fused.h -- single-stream AES-CM + HMAC-SHA1 batches planned inside
 * the crypto launch (BASELINE configs 2 and 5; srtpgpu.h struct sgpu_fused).
 *
 * The separate device planner (srtp_kernels.hip k_parse, k_plan_count /
 * scan / desc / final, k_plan_finish) reads every packet's header line once
 * more before the crypto launch reads it again, and costs ~60 us of launches
 * per 1M packets per direction.  Here each 1024-packet workgroup of the
 * lean kernel (k_ctr_fast.h, one packet per lane) plans its own packets:
 *
 *   1. ticket (atomic, so every workgroup before it is running or done);
 *   2. every lane loads its window and header (rtp_hdr_decode,
 *      rtp.c:88-137) -- in flight while the 128 KiB T4 image is filled --
 *      and makes the checks of k_plan_count (window, class, SSRC,
 *      ETIMEDOUT, order, size, room); the seqs of the two packets before
 *      the workgroup come from the arena;
 *   3. wave 0 publishes the workgroup's ROC rollover count and fail bits,
 *      then looks back over the workgroups before it, 64 at a time, to the
 *      nearest one that published its inclusive prefix (decoupled
 *      look-back), and publishes its own inclusive prefix;
 *   4. each lane forms its index and ROC exactly as k_plan_desc does
 *      (srtp.c:203-215 sender, misc.c:22-41 receiver, replay.c:32-62 over
 *      the batch), writes desc / hdr / end copy / results, then runs the
 *      lean kernel's per-packet body.
 *
 * Measured against the alternatives (profiles/r05_fused_ab.txt): K packets
 * per lane in a loop (one plan per CU) and waves taking 64-packet tickets
 * independently both lost more to the loop's register allocation (~120-300
 * VGPRs of spills against ~30-85) than they saved in planning latency.
 *
 * A workgroup with a failed check of its own or before it does no crypto
 * (desc = 0).  A check that fails anywhere sets out->fail
 * and the host undoes every processed packet (k_ctr_fused_undo) and plans
 * the batch on the host engine, as for a rejected separate plan.
 */
#pragma once
#include "k_ctr_fast.h"
#include "plan_common.h"

struct FArgs {
	KArgs a;
	struct sgpu_fused p;
};

#define FZ_BLOCK CTRF_BLOCK      /* packets per workgroup, one per lane */

struct FShared {
	uint32_t t;                     /* ticket: the workgroup's position */
	uint32_t fail;                  /* OR of its packets' SPF_* */
	uint32_t hl0, ssrc0, seq0;      /* packet 0 of the batch */
	uint32_t excl;                  /* rollovers before the workgroup */
	uint32_t xfail;                 /* fail bits of it and those before */
	uint32_t wsum[FZ_BLOCK / 64];   /* rollovers per wave */
	uint32_t seq[FZ_BLOCK + 2];     /* seq of packets base-2 .. base+B-1 */
};

/* SPF_* bits a look-back word carries (bits 32..45) */
#define FZ_FMASK 0x3fffu
static_assert((SPF_SLOW | SPF_SEG | SPF_PRED | 0x1ffu) <= FZ_FMASK, "fz_word");

__device__ __forceinline__ uint64_t fz_word(uint32_t epoch, uint32_t st,
					    uint32_t fail, uint32_t wraps)
{
	return (uint64_t)epoch << 48 | (uint64_t)st << 46 |
	       (uint64_t)(fail & FZ_FMASK) << 32 | wraps;
}

__device__ __forceinline__ void fz_store(unsigned long long *w, uint64_t v)
{
	__hip_atomic_store(w, (unsigned long long)v, __ATOMIC_RELAXED,
			   __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t fz_load(unsigned long long *w)
{
	return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += (uint32_t)__shfl_xor((int)v, o);
	return v;
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v |= (uint32_t)__shfl_xor((int)v, o);
	return v;
}

#ifdef FZ_WTIME
#define FZ_WTIME_MAX 4096u
#define FZ_WREC 24u
/* per ticket: [0] start (thread 0), [1] CU id, [2 + w] wave w's end,
 * [18 + k] thread 0 at the plan's k-th barrier */
__device__ uint64_t g_fzw[FZ_WREC * FZ_WTIME_MAX];
#define FZ_STAMP(k)                                                          \
	do {                                                                 \
		if (threadIdx.x == 0 && S.t < FZ_WTIME_MAX)                  \
			g_fzw[FZ_WREC * S.t + 18u + (k)] =                   \
				__builtin_amdgcn_s_memrealtime();            \
	} while (0)
#else
#define FZ_STAMP(k) do { } while (0)
#endif

/*
 * Steps 1-4 of the header comment for the calling workgroup (packets
 * base + tid).  Returns the header class (0..3) if the lane has a packet
 * to encrypt / decrypt (fp), -1 if it has none or the workgroup does
 * nothing.
 */
template <bool PROT>
__device__ __forceinline__ int fz_plan(const FArgs &fa, FShared &S,
				       uint8_t *smem, FastPkt &fp)
{
	const KArgs &a = fa.a;
	const struct sgpu_fused &P = fa.p;
	const struct sgpu_plan_in &in = P.in;
	const uint32_t tid = threadIdx.x, B = FZ_BLOCK;
	const uint32_t lane = tid & 63u, wv = tid >> 6;
	const uint64_t asz = a.asz;
	const uint32_t n = in.n;

	if (tid == 0) {
		S.t = atomicAdd(P.ticket, 1u) - P.tbase;
		S.fail = 0;
	}
	__syncthreads();
	FZ_STAMP(0);
	const uint32_t t = S.t;
	const uint32_t base = t * B, i = base + tid;
	const bool live = i < n;
	/* the window's loads, then the header's, fly while the T4 image is
	 * filled */
	uint32_t p = 0, e = 0, cp = 0;
	struct sgpu_hdr h;
	h.ssrc = 0; h.seq = 0; h.err_pos = 0; h.hdr_len = 0xffffffffu;
	if (live) {
		p = P.pos[i];
		e = P.end[i];
		cp = P.cap ? P.cap[i] : 0u;
		const uint32_t left = (e > p && e <= asz) ? e - p : 0u;
		h = parse_rtp_hdr(a.arena + p, p, left);
	}
	if (tid < 3) {
		if (tid == 0) {
			/* packet 0: every packet's class and SSRC are checked
			 * against it.  Workgroup 0 may already have moved end[0]
			 * by delta: a processed packet 0 parses to the same
			 * header either way (its length stays >= hl, + tag) */
			const uint32_t q = P.pos[0], qe = P.end[0];
			const uint32_t left = (qe > q && qe <= asz) ? qe - q : 0u;
			const struct sgpu_hdr h0 = parse_rtp_hdr(a.arena + q, q,
								 left);
			S.hl0 = h0.hdr_len;
			S.ssrc0 = h0.ssrc;
			S.seq0 = h0.seq;
			if (t == 0) {
				/* the next launch's counters; the context index
				 * for the launches behind this one */
				P.out_next->fail = 0;
				P.out_next->nfail = 0;
				if (P.cm_out)
					*P.cm_out = P.comp;
			}
		}
		else if (base >= tid) {
			/* seq of packet base - tid (bytes 2-3; a packet too
			 * short for a header failed its own workgroup's check,
			 * so this value then never matters) */
			const uint32_t q = P.pos[base - tid];
			uint32_t sv = 0;
			if ((uint64_t)q + 4u <= asz)
				sv = (uint32_t)a.arena[q + 2] << 8 | a.arena[q + 3];
			S.seq[2 - tid] = sv;
		}
	}
#ifndef FZ_FILL_LOOP
	static_assert(FZ_BLOCK == 1024, "tt4_fill_b1024");
	tt4_fill_b1024(smem, a.t0);
#else
	tt4_fill(smem, a.t0);
#endif
	FZ_STAMP(4);
	if (live) {
		P.hdr[i] = h;
		P.es[i] = e;
		S.seq[tid + 2] = h.seq;
	}
	__syncthreads();
	FZ_STAMP(1);

	/* k_plan_count's checks (srtp_kernels.hip) */
	const uint32_t hl0 = S.hl0;
	const uint32_t ssrc0 = in.ssrc_any ? S.ssrc0 : in.ssrc;
	const uint32_t s_l0 = in.fresh ? S.seq0 : in.s_l;       /* plan_sb(0) */
	const uint32_t seq = h.seq;
	uint32_t f = 0, sb = 0;
	bool wrap = false;
	if (live) {
		sb = i == 0 ? s_l0 : S.seq[tid + 1];
		const uint32_t L = e - p;
		if (h.hdr_len == 0xffffffffu || hl0 == 0xffffffffu)
			f |= SPF_PARSE;
		else if (((h.hdr_len ^ hl0) >> 2) & 3u)
			f |= SPF_CLASS;
		/* (an unparsable packet has no SSRC: SPF_PARSE alone, so the
		 * host does not try the per-stream planner for it) */
		if (h.ssrc != ssrc0 && h.hdr_len != 0xffffffffu)
			f |= SPF_SSRC;
		if (!PROT && h.hdr_len != 0xffffffffu && L - h.hdr_len < in.tag)
			f |= SPF_PARSE;
		if (!PROT && (int)seq - (int)sb > 32768)
			f |= SPF_TIMEOUT;
		if (L >= in.maxlen)
			f |= SPF_SIZE;
		if ((p & 3u) || p > e || e > asz ||
		    (P.cap && (e > cp || cp > asz)))
			f |= SPF_BAD;
		if (PROT && P.cap && (uint64_t)e + in.need > (uint64_t)cp)
			f |= SPF_CAP;
		wrap = plan_wrap(seq, sb);
		if (i + 1 < n && !wrap && seq < sb)
			f |= SPF_ORDER;
		if (i == 0) {
			P.out->ssrc0 = h.ssrc;
			P.out->hl0 = h.hdr_len;
		}
	}
	if (tid == 0 && in.pred && *in.pred)    /* sgpu_gate_pred */
		f |= SPF_PRED;
	if (f)
		atomicOr(&S.fail, f);
	const uint64_t m = __ballot(wrap);
	if (lane == 0)
		S.wsum[wv] = (uint32_t)__popcll(m);
	__syncthreads();
	FZ_STAMP(2);

	if (wv == 0) {
		/* step 3: aggregate, look-back, inclusive prefix */
		const uint32_t tot = wave_sum(lane < B / 64u ? S.wsum[lane] : 0u);
		const uint32_t lf = S.fail;
		uint32_t excl = 0, xf = 0;
		if (t != 0) {
			if (lane == 0)
				fz_store(&P.agg[t], fz_word(P.epoch, 1, lf, tot));
			int32_t j = (int32_t)t - 1;
			for (;;) {
				const int32_t k = j - (int32_t)lane;
				uint64_t w = 0;
				uint32_t st = 2;
				if (k >= 0) {
					/* every workgroup below t is running or
					 * done and publishes before it waits; the
					 * bound (2^18 polls of s_sleep 1, ~64
					 * clocks each: ~7 ms at 2.4 GHz) only
					 * turns a stalled predecessor or a broken
					 * ticket count into a rejected plan
					 * (SPF_SLOW: the host re-plans, resets
					 * the counters and counts it apart from
					 * a bad window, "lbtimeouts") instead of
					 * a wave that never ends */
					for (uint32_t spin = 0;; spin++) {
						w = fz_load(&P.agg[k]);
						st = (uint32_t)(w >> 46) & 3u;
						if ((uint32_t)(w >> 48) == P.epoch &&
						    st != 0)
							break;
						if (spin > (1u << 18)) {
							w = fz_word(0, 2, SPF_SLOW, 0);
							st = 2;
							break;
						}
						__builtin_amdgcn_s_sleep(1);
					}
				}
				const uint64_t inc = __ballot(st == 2);
				const uint32_t first = inc ?
					(uint32_t)__ffsll((long long)inc) - 1u : 64u;
				const bool take = lane <= first;
				excl += wave_sum(take ? (uint32_t)w : 0u);
				xf |= wave_or(take ? (uint32_t)(w >> 32) & FZ_FMASK
						   : 0u);
				if (inc)
					break;
				j -= 64;
			}
		}
		if (lane == 0) {
			fz_store(&P.agg[t], fz_word(P.epoch, 2, lf | xf,
						    excl + tot));
			S.excl = excl;
			S.xfail = lf | xf;
			if (lf | (xf & (SPF_BAD | SPF_SLOW)))
				atomicOr(&P.out->fail,
					 lf | (xf & (SPF_BAD | SPF_SLOW)));
		}
	}
	__syncthreads();
	FZ_STAMP(3);
	if (!live)
		return -1;
	if (S.xfail) {
		P.desc[i] = 0;          /* not processed */
		return -1;
	}

	/* step 4: k_plan_desc (srtp_kernels.hip) */
	uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
	for (uint32_t q = 0; q < wv; q++)
		pre += S.wsum[q];
	const uint32_t roc = in.roc + S.excl + pre + (wrap ? 1u : 0u);
	uint64_t ix;
	uint32_t fl = SD_RUN | SD_CIPHER;
	if (PROT) {
		ix = 65536ull * roc + seq;                      /* srtp.c:215 */
	}
	else {
		const int32_t v = plan_v(roc, wrap ? 0u : sb, seq);
		ix = seq + (uint64_t)(int64_t)v * 65536ull;
		if ((uint32_t)v != roc)
			fl |= (uint32_t)v + 1u == roc ? SD_ROC_P1 : SD_ROC_M1;
		bool ok;
		if (i == 0) {
			if (ix > in.lix)
				ok = true;
			else {
				const uint64_t d = in.lix - ix;
				ok = d < 64 && !(in.bitmap & (1ull << d));
			}
		}
		else {
			const uint32_t pseq = sb;       /* packet i-1's seq */
			const uint32_t psb = i == 1 ? s_l0 : S.seq[tid];
			const bool pw = plan_wrap(pseq, psb);
			const uint32_t proc = roc - (wrap ? 1u : 0u);
			const int32_t pv = plan_v(proc, pw ? 0u : psb, pseq);
			const uint64_t pix = pseq + (uint64_t)(int64_t)pv * 65536ull;
			ok = ix > pix && ix > in.lix;
		}
		if (!ok)
			atomicOr(&P.out->fail, (uint32_t)SPF_REPLAY);
	}
	P.desc[i] = d_desc(ix, fl);
	const uint32_t t0 = n > SGPU_PLAN_TAIL ? n - SGPU_PLAN_TAIL : 0u;
	if (i >= t0)
		P.out->tail_ix[i - t0] = ix;
	if (i + 1 == n) {
		P.out->s_l_last = wrap ? seq : (seq > sb ? seq : sb);
		P.out->wraps = roc - in.roc;
	}
	/* k_plan_finish's results */
	P.end[i] = e + (uint32_t)P.delta;
	P.err[i] = 0;
	fp.p = i;
	fp.off = p;
	fp.L = e - p;
	fp.hl = h.hdr_len;
	fp.ssrc = h.ssrc;
	fp.ixhi = (uint32_t)(ix >> 16);
	fp.ixlo = (uint32_t)(ix & 0xffffu);
	/* the trailer ROC (fast_pkt: ixhi +- the SD_ROC_* correction) */
	fp.roc = roc;
	/* (the class from the hl0 read above: switching on a second read of
	 * S.hl0 after the crypto's setup spilled ~90 more VGPRs) */
	return (int)((hl0 >> 2) & 3u);
}

/* sgpu_run_fused always launches FZ_BLOCK threads (one packet per lane,
 * both directions), so the attributes name FZ_BLOCK, not the lean
 * kernel's per-direction CTRF_BLK(PROT) (a build with CTRF_BLOCK_U below
 * CTRF_BLOCK would otherwise fail every fused unprotect launch) */
template <int NR, bool PROT>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, FZ_BLOCK)))
__attribute__((amdgpu_waves_per_eu(FZ_BLOCK / 256, 8)))
k_ctr_fused(const FArgs fa)
{
#ifdef FZ_WTIME
	uint64_t t_start = 0;
	if (threadIdx.x == 0)
		t_start = __builtin_amdgcn_s_memrealtime();
#endif
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	__shared__ FShared S;
	FastPkt f;
	const int cls = fz_plan<PROT>(fa, S, smem, f);
#ifdef FZ_WTIME
	if (threadIdx.x == 0 && S.t < FZ_WTIME_MAX) {
		uint32_t hw;
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
		g_fzw[FZ_WREC * S.t] = t_start;
		g_fzw[FZ_WREC * S.t + 1u] = hw;
	}
#endif
	if (cls < 0)
		return;
	const uint32_t ci = fa.p.comp;
	switch (cls) {
	case 0: ctr_fast_pkt<NR, 0, PROT>(fa.a, smem, f, ci); break;
	case 1: ctr_fast_pkt<NR, 1, PROT>(fa.a, smem, f, ci); break;
	case 2: ctr_fast_pkt<NR, 2, PROT>(fa.a, smem, f, ci); break;
	case 3: ctr_fast_pkt<NR, 3, PROT>(fa.a, smem, f, ci); break;
	default: break;
	}
	/* (no stamp after the crypto: a value kept live across its body
	 * costs the SGPRs that hold the round keys -- it spilled ~90 VGPRs) */
#ifdef FZ_WTIME
	/* A/B diagnostic build only (scripts/fz_wtime.py): each wave's end
	 * time, the ticket re-read from LDS, not kept live */
	if ((threadIdx.x & 63u) == 0) {
		const uint32_t t = S.t;
		if (t < FZ_WTIME_MAX)
			g_fzw[FZ_WREC * t + 2u + threadIdx.x / 64u] =
				__builtin_amdgcn_s_memrealtime();
	}
#endif
}

/*
 * The plan alone, as its own launch in front of the lean crypto kernels
 * (k_ctr_fast_any, guarded by skip[] and out->fail; k_gcmu, guarded by
 * out->fail): the one-launch single-stream planner (batch_dev.c lp_issue).
 * It writes what k_parse, k_plan_count / scan / desc / final and
 * k_plan_finish wrote (hdr, es, desc, the plan out, the results of every
 * packet planned) in one launch instead of six, and leaves the crypto
 * launch its full LDS and registers (the in-launch plan of k_ctr_fused
 * costs each crypto workgroup ~15 us of latency, four workgroups in turn
 * per CU).  The steps of fz_plan, with LP_PPT packets per lane: a
 * workgroup covers LP_PPT x 1024 packets (packet q = j * 1024 + lane id,
 * loads coalesced per j and all of a lane's in flight together), so a 1M
 * batch takes 256 tickets and one look-back chain of 256 instead of 1024.
 */
#ifndef LP_PPT
#define LP_PPT 4
#endif
#define LP_WG (FZ_BLOCK * LP_PPT)

struct LpShared {
	uint32_t t, fail, hl0, ssrc0, seq0, excl, xfail;
	uint32_t wsum[LP_PPT][FZ_BLOCK / 64];   /* rollovers per (round, wave) */
	uint32_t seq[LP_WG + 2];                /* packets base-2 .. */
};

template <bool PROT>
__global__ void __launch_bounds__(FZ_BLOCK)
k_lp_plan(const FArgs fa)
{
	__shared__ LpShared S;
	const KArgs &a = fa.a;
	const struct sgpu_fused &P = fa.p;
	const struct sgpu_plan_in &in = P.in;
	const uint32_t tid = threadIdx.x;
	const uint32_t lane = tid & 63u, wv = tid >> 6;
	const uint64_t asz = a.asz;
	const uint32_t n = in.n;

	if (tid == 0) {
		S.t = atomicAdd(P.ticket, 1u) - P.tbase;
		S.fail = 0;
	}
	__syncthreads();
	const uint32_t t = S.t;
	const uint32_t base = t * LP_WG;
	uint32_t pv[LP_PPT], ev[LP_PPT], cv[LP_PPT], w0[LP_PPT], w2[LP_PPT];
#pragma unroll
	for (int j = 0; j < LP_PPT; j++) {
		const uint32_t i = base + j * FZ_BLOCK + tid;
		pv[j] = ev[j] = cv[j] = 0;
		if (i < n) {
			pv[j] = P.pos[i];
			ev[j] = P.end[i];
			cv[j] = P.cap ? P.cap[i] : 0u;
		}
	}
#pragma unroll
	for (int j = 0; j < LP_PPT; j++) {
		const uint32_t p = pv[j], e = ev[j];
		w0[j] = w2[j] = 0;
		if (base + j * FZ_BLOCK + tid < n && e > p && e <= asz &&
		    e - p >= 12 && !(p & 3u)) {
			w0[j] = *(const uint32_t *)(a.arena + p);
			w2[j] = *(const uint32_t *)(a.arena + p + 8);
		}
	}
	if (tid < 3) {
		if (tid == 0) {
			/* packet 0: every packet's class and SSRC are checked
			 * against it */
			const uint32_t q = P.pos[0], qe = P.end[0];
			const uint32_t left = (qe > q && qe <= asz) ? qe - q : 0u;
			const struct sgpu_hdr h0 = parse_rtp_hdr(a.arena + q, q,
								 left);
			S.hl0 = h0.hdr_len;
			S.ssrc0 = h0.ssrc;
			S.seq0 = h0.seq;
			if (t == 0) {
				/* the next launch's counters; the context index
				 * and the class guards for the crypto launch */
				P.out_next->fail = 0;
				P.out_next->nfail = 0;
				if (P.cm_out)
					*P.cm_out = P.comp;
				for (uint32_t c = 0; c < 4; c++)
					P.out->skip[c] =
						h0.hdr_len == 0xffffffffu ||
						((h0.hdr_len >> 2) & 3u) != c;
			}
		}
		else if (base >= tid) {
			/* seq of packet base - tid (the workgroup before) */
			const uint32_t q = P.pos[base - tid];
			uint32_t sv = 0;
			if ((uint64_t)q + 4u <= asz)
				sv = (uint32_t)a.arena[q + 2] << 8 | a.arena[q + 3];
			S.seq[2 - tid] = sv;
		}
	}
	struct sgpu_hdr hv[LP_PPT];
#pragma unroll
	for (int j = 0; j < LP_PPT; j++) {
		const uint32_t i = base + j * FZ_BLOCK + tid;
		hv[j].ssrc = 0; hv[j].seq = 0; hv[j].err_pos = 0;
		hv[j].hdr_len = 0xffffffffu;
		if (i >= n)
			continue;
		const uint32_t p = pv[j], e = ev[j];
		const uint32_t left = (e > p && e <= asz) ? e - p : 0u;
		if (left >= 12 && !(p & 3u) && !(w0[j] & 0x1fu)) {
			/* no CSRC, no extension: the header is the two words */
			hv[j].seq = (uint16_t)((w0[j] >> 8 & 0xff00u) |
					       (w0[j] >> 24));
			hv[j].ssrc = __builtin_bswap32(w2[j]);
			hv[j].hdr_len = 12;
		}
		else {
			hv[j] = parse_rtp_hdr(a.arena + p, p, left);
		}
		P.hdr[i] = hv[j];
		P.es[i] = e;
		S.seq[2 + j * FZ_BLOCK + tid] = hv[j].seq;
	}
	__syncthreads();

	/* k_plan_count's checks (srtp_kernels.hip), as fz_plan */
	const uint32_t hl0 = S.hl0;
	const uint32_t ssrc0 = in.ssrc_any ? S.ssrc0 : in.ssrc;
	const uint32_t s_l0 = in.fresh ? S.seq0 : in.s_l;       /* plan_sb(0) */
	uint32_t f = 0;
	uint32_t sbv[LP_PPT];
	uint64_t wm[LP_PPT];
#pragma unroll
	for (int j = 0; j < LP_PPT; j++) {
		const uint32_t q = j * FZ_BLOCK + tid, i = base + q;
		const struct sgpu_hdr &h = hv[j];
		bool wrap = false;
		sbv[j] = 0;
		if (i < n) {
			const uint32_t p = pv[j], e = ev[j], cp = cv[j];
			const uint32_t seq = h.seq;
			const uint32_t sb = i == 0 ? s_l0 : S.seq[q + 1];
			const uint32_t L = e - p;
			sbv[j] = sb;
			if (h.hdr_len == 0xffffffffu || hl0 == 0xffffffffu)
				f |= SPF_PARSE;
			else if (((h.hdr_len ^ hl0) >> 2) & 3u)
				f |= SPF_CLASS;
			if (h.ssrc != ssrc0 && h.hdr_len != 0xffffffffu)
				f |= SPF_SSRC;
			if (!PROT && h.hdr_len != 0xffffffffu &&
			    L - h.hdr_len < in.tag)
				f |= SPF_PARSE;
			if (!PROT && (int)seq - (int)sb > 32768)
				f |= SPF_TIMEOUT;
			if (L >= in.maxlen)
				f |= SPF_SIZE;
			if ((p & 3u) || p > e || e > asz ||
			    (P.cap && (e > cp || cp > asz)))
				f |= SPF_BAD;
			if (PROT && P.cap && (uint64_t)e + in.need > (uint64_t)cp)
				f |= SPF_CAP;
			wrap = plan_wrap(seq, sb);
			if (i + 1 < n && !wrap && seq < sb)
				f |= SPF_ORDER;
			if (i == 0) {
				P.out->ssrc0 = h.ssrc;
				P.out->hl0 = h.hdr_len;
			}
		}
		wm[j] = __ballot(wrap);
		if (lane == 0)
			S.wsum[j][wv] = (uint32_t)__popcll(wm[j]);
	}
	if (tid == 0 && in.pred && *in.pred)    /* sgpu_gate_pred */
		f |= SPF_PRED;
	if (f)
		atomicOr(&S.fail, f);
	__syncthreads();

	if (wv == 0) {
		/* aggregate, look-back, inclusive prefix (fz_plan step 3) */
		uint32_t tot = 0;
#pragma unroll
		for (int j = 0; j < LP_PPT; j++)
			tot += wave_sum(lane < FZ_BLOCK / 64u ? S.wsum[j][lane] : 0u);
		const uint32_t lf = S.fail;
		uint32_t excl = 0, xf = 0;
		if (t != 0) {
			if (lane == 0)
				fz_store(&P.agg[t], fz_word(P.epoch, 1, lf, tot));
			int32_t jj = (int32_t)t - 1;
			for (;;) {
				const int32_t k = jj - (int32_t)lane;
				uint64_t w = 0;
				uint32_t st = 2;
				if (k >= 0) {
					for (uint32_t spin = 0;; spin++) {
						w = fz_load(&P.agg[k]);
						st = (uint32_t)(w >> 46) & 3u;
						if ((uint32_t)(w >> 48) == P.epoch &&
						    st != 0)
							break;
						if (spin > (1u << 18)) {
							w = fz_word(0, 2, SPF_SLOW, 0);
							st = 2;
							break;
						}
						__builtin_amdgcn_s_sleep(1);
					}
				}
				const uint64_t inc = __ballot(st == 2);
				const uint32_t first = inc ?
					(uint32_t)__ffsll((long long)inc) - 1u : 64u;
				const bool take = lane <= first;
				excl += wave_sum(take ? (uint32_t)w : 0u);
				xf |= wave_or(take ? (uint32_t)(w >> 32) & FZ_FMASK
						   : 0u);
				if (inc)
					break;
				jj -= 64;
			}
		}
		if (lane == 0) {
			fz_store(&P.agg[t], fz_word(P.epoch, 2, lf | xf,
						    excl + tot));
			S.excl = excl;
			S.xfail = lf | xf;
			if (lf | (xf & (SPF_BAD | SPF_SLOW)))
				atomicOr(&P.out->fail,
					 lf | (xf & (SPF_BAD | SPF_SLOW)));
		}
	}
	__syncthreads();
	const bool dead = S.xfail != 0;
	uint32_t pre = S.excl;
#pragma unroll
	for (int j = 0; j < LP_PPT; j++) {
		const uint32_t q = j * FZ_BLOCK + tid, i = base + q;
		uint32_t wpre = (uint32_t)__popcll(wm[j] & ((1ull << lane) - 1ull));
		for (uint32_t w = 0; w < wv; w++)
			wpre += S.wsum[j][w];
		const uint32_t rpre = pre + wpre;
		for (uint32_t w = 0; w < FZ_BLOCK / 64u; w++)
			pre += S.wsum[j][w];
		if (i >= n)
			continue;
		if (dead) {
			P.desc[i] = 0;          /* not planned */
			continue;
		}
		/* fz_plan step 4: k_plan_desc (srtp_kernels.hip) */
		const uint32_t seq = hv[j].seq, sb = sbv[j];
		const bool wrap = (wm[j] >> lane) & 1ull;
		const uint32_t roc = in.roc + rpre + (wrap ? 1u : 0u);
		uint64_t ix;
		uint32_t fl = SD_RUN | SD_CIPHER;
		if (PROT) {
			ix = 65536ull * roc + seq;                      /* srtp.c:215 */
		}
		else {
			const int32_t v = plan_v(roc, wrap ? 0u : sb, seq);
			ix = seq + (uint64_t)(int64_t)v * 65536ull;
			if ((uint32_t)v != roc)
				fl |= (uint32_t)v + 1u == roc ? SD_ROC_P1 : SD_ROC_M1;
			bool ok;
			if (i == 0) {
				if (ix > in.lix)
					ok = true;
				else {
					const uint64_t d = in.lix - ix;
					ok = d < 64 && !(in.bitmap & (1ull << d));
				}
			}
			else {
				const uint32_t pseq = sb;       /* packet i-1's seq */
				const uint32_t psb = i == 1 ? s_l0 : S.seq[q];
				const bool pw = plan_wrap(pseq, psb);
				const uint32_t proc = roc - (wrap ? 1u : 0u);
				const int32_t pv2 = plan_v(proc, pw ? 0u : psb, pseq);
				const uint64_t pix = pseq + (uint64_t)(int64_t)pv2 * 65536ull;
				ok = ix > pix && ix > in.lix;
			}
			if (!ok)
				atomicOr(&P.out->fail, (uint32_t)SPF_REPLAY);
		}
		P.desc[i] = d_desc(ix, fl);
		const uint32_t t0 = n > SGPU_PLAN_TAIL ? n - SGPU_PLAN_TAIL : 0u;
		if (i >= t0)
			P.out->tail_ix[i - t0] = ix;
		if (i + 1 == n) {
			P.out->s_l_last = wrap ? seq : (seq > sb ? seq : sb);
			P.out->wraps = roc - in.roc;
		}
		/* k_plan_finish's results (the host puts the ends back if the
		 * plan fails anywhere) */
		P.end[i] = ev[j] + (uint32_t)P.delta;
		P.err[i] = 0;
	}
}

/*
 * Undo of a rejected fused launch (or of a device fold that failed):
 * every processed packet (desc SD_RUN) back to its bytes before the call.
 * Protect: the keystream re-applied over [hl, L) (the tag written past L
 * is rewritten by the host engine's re-run).  Unprotect: over [hl, A),
 * A = L - tag, where still decrypted (SV_CIPHERED; k_ctr_refix_list
 * restored the forged ones), and the tag word the ROC was written over
 * (srtp.c:342-344) back from save.
 */
template <int NR, int SHIFT, bool PROT>
__device__ __forceinline__ void fz_undo_body(const FArgs &fa, uint8_t *smem)
{
	const KArgs &a = fa.a;
	const struct sgpu_fused &P = fa.p;
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	bool run = false, ciph = false;
	if (i < P.in.n && ((uint32_t)(P.desc[i] >> 48) & SD_RUN)) {
		run = true;
		ciph = PROT || (P.verdict[i] & SV_CIPHERED);
	}
	if (!__syncthreads_or(run))
		return;
	tt4_fill(smem, a.t0);
	__syncthreads();
	if (!run)
		return;
	const uint64_t d = P.desc[i];
	const uint32_t fl = (uint32_t)(d >> 48);
	FastPkt f;
	f.p = i;
	f.off = P.pos[i];
	f.L = P.es[i] - f.off;
	f.ssrc = P.hdr[i].ssrc;
	f.hl = P.hdr[i].hdr_len;
	f.ixhi = (uint32_t)(d >> 16);
	f.ixlo = (uint32_t)(d & 0xffffu);
	f.roc = f.ixhi + ((fl & SD_ROC_P1) ? 1u : 0u) -
		((fl & SD_ROC_M1) ? 1u : 0u);
	uint32_t rk[4 * (NR + 1)];
	const struct sgpu_comp *cp = fast_keys_at<NR>(a, P.comp, rk);
	const uint32_t lo = (threadIdx.x & 31u) * 4u;
	uint8_t *pkt = a.arena + f.off;
	const uint64_t pasz = a.asz - f.off;
	const uint32_t A = PROT ? f.L : f.L - cp->tag_len;
	if (ciph) {
		const int32_t cw4 = (int32_t)(f.hl >> 4);
		uint32_t iv[4];
		fast_iv(cp, f, iv);
		CtrKs<NR, true, true> C;
		C.init(smem, lo, rk, iv);
		uint32_t carry[4] = {0, 0, 0, 0};
		for (uint32_t k = 0; 64u * k < A; k++) {
			const uint32_t c0 = 64u * k;
			if (c0 + 64u <= f.hl)
				continue;
			uint32_t dd[16];
#pragma unroll
			for (int g = 0; g < 4; g++) {
				uint4 v = make_uint4(0, 0, 0, 0);
				if (c0 + 16u * g < A)
					v = ld16(pkt, pasz, c0 + 16u * g);
				dd[4 * g] = v.x; dd[4 * g + 1] = v.y;
				dd[4 * g + 2] = v.z; dd[4 * g + 3] = v.w;
			}
			tail_xor_store<NR, SHIFT>(smem, lo, rk, C,
						  (int32_t)(4 * k) - cw4, carry, dd,
						  pkt, c0, f.hl, A);
		}
	}
	if (!PROT) {
		const uint32_t v = P.save[i];
		pkt[A] = (uint8_t)v;
		pkt[A + 1] = (uint8_t)(v >> 8);
		pkt[A + 2] = (uint8_t)(v >> 16);
		pkt[A + 3] = (uint8_t)(v >> 24);
		P.verdict[i] &= (uint8_t)~SV_CIPHERED;
	}
}

template <int NR, bool PROT>
__global__ void
__attribute__((amdgpu_flat_work_group_size(1, CTRF_BLOCK)))
__attribute__((amdgpu_waves_per_eu(CTRF_BLOCK / 256, 8)))
k_ctr_fused_undo(const FArgs fa)
{
	__shared__ __attribute__((aligned(16))) uint8_t smem[TT4_BYTES];
	switch (fa.p.shift) {
	case 0: fz_undo_body<NR, 0, PROT>(fa, smem); break;
	case 1: fz_undo_body<NR, 1, PROT>(fa, smem); break;
	case 2: fz_undo_body<NR, 2, PROT>(fa, smem); break;
	case 3: fz_undo_body<NR, 3, PROT>(fa, smem); break;
	default: break;
	}
}
