/**
 * @file re_srtp_batch.h  Batched SRTP/SRTCP -- extension (no reference
 * counterpart; the reference API is one mbuf per call).
 *
 * Semantics: a batch of n packets gives exactly the results of n sequential
 * re_srtp.h calls in array order -- per-packet errno, the mbuf pos/end the
 * call would leave, the same bytes, and the same evolution of the ROC,
 * s_l, replay windows and SRTCP index (src/srtp/srtp.h:23-38).
 *
 * Two entry families:
 *   srtp_*_mbufs   host-resident packets (mbuf array), staged through
 *                  pinned memory; the end-to-end path (socket -> GPU ->
 *                  socket).  srtp_encrypt() etc. are this with n = 1.
 *   srtp_*_batch   device-resident arena: packet bytes already in HBM,
 *                  per-packet (pos, end, cap) windows, results in place.
 */
#ifndef RE_SRTP_BATCH_H
#define RE_SRTP_BATCH_H

#include "re_srtp.h"

#ifdef __cplusplus
extern "C" {
#endif

int srtp_encrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
		       size_t n);
int srtp_decrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
		       size_t n);
int srtcp_encrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
			size_t n);
int srtcp_decrypt_mbufs(struct srtp *srtp, struct mbuf **mbv, int *errv,
			size_t n);

/**
 * Device-resident batch.  arena is a device pointer (hipMalloc'ed); packet
 * i occupies arena[pos[i], end[i]) and may grow up to cap[i] (the mbuf
 * `size` analog: protect appends the tag there).  pos[i] must be a multiple
 * of 4.  pos/end/cap/err/sess are host arrays; pos/end are updated like
 * mbuf->pos/end.  sessv[sess[i]] is packet i's session (sess == NULL: all
 * packets use sessv[0]).  stream: hipStream_t or NULL (default stream).
 * Returns 0 if the batch ran (per-packet results in err[]), else an errno
 * (EINVAL for bad arguments, EIO for a HIP failure).
 */
struct srtp_batch {
	uint8_t *arena;
	size_t arena_size;
	uint32_t *pos;
	uint32_t *end;
	const uint32_t *cap;
	int32_t *err;
	const uint32_t *sess;
	size_t n;
	void *stream;
};

int srtp_encrypt_batch(struct srtp **sessv, size_t nsess,
		       struct srtp_batch *b);
int srtp_decrypt_batch(struct srtp **sessv, size_t nsess,
		       struct srtp_batch *b);
int srtcp_encrypt_batch(struct srtp **sessv, size_t nsess,
			struct srtp_batch *b);
int srtcp_decrypt_batch(struct srtp **sessv, size_t nsess,
			struct srtp_batch *b);

/**
 * Fully device-resident batch: like struct srtp_batch, but the per-packet
 * windows and results (pos, end, cap, err, sess) are device arrays too, so
 * a GPU-resident pipeline never moves per-packet data through the host.
 * Same per-packet semantics.  Single-stream RTP batches are planned on the
 * device (O(1) host work); other batches are staged through the host
 * engine transparently.
 */
struct srtp_batch_dev {
	uint8_t *arena;
	size_t arena_size;
	uint32_t *pos;          /* device, in/out */
	uint32_t *end;          /* device, in/out */
	const uint32_t *cap;    /* device */
	int32_t *err;           /* device, out */
	const uint32_t *sess;   /* device or NULL */
	size_t n;
	void *stream;
};

int srtp_encrypt_batch_dev(struct srtp **sessv, size_t nsess,
			   struct srtp_batch_dev *b);
int srtp_decrypt_batch_dev(struct srtp **sessv, size_t nsess,
			   struct srtp_batch_dev *b);
int srtcp_encrypt_batch_dev(struct srtp **sessv, size_t nsess,
			    struct srtp_batch_dev *b);
int srtcp_decrypt_batch_dev(struct srtp **sessv, size_t nsess,
			    struct srtp_batch_dev *b);

/**
 * Asynchronous device-resident RTP batches: the call is queued on
 * b->stream and returns without waiting for the GPU; srtp_batch_wait()
 * completes it and returns what srtp_*_batch_dev would have returned.
 * Calls issued one after another on the same stream run back to back on
 * the GPU (e.g. protect on one context set, then unprotect of the same
 * arena on another): each is planned against the states the calls
 * before it leave, and a call queued behind one that must be completed on
 * the host (a rejected device plan, a forged packet needing the host
 * fold) does nothing on the GPU and is re-run when waited for -- results
 * are always those of the synchronous calls in issue order.
 *
 * Until the ticket is waited for, sessv, the session contexts and the
 * device arrays in *b (b itself is copied) must stay valid and unused by
 * other calls; tickets are waited for on the issuing thread.  Any other
 * call of this API on that thread first completes its pending tickets
 * (their results stay in the tickets).  At most 4 calls are pending per
 * thread (a fifth completes the oldest first).  Returns 0 with *tp set
 * (the call may already have completed), or EINVAL / ENOMEM.
 *
 * A session with calls of one thread pending is busy for every other
 * thread until the issuing thread has completed them: calls of this API
 * from another thread that name it return (or, asynchronous, complete
 * with) EBUSY and change nothing.
 */
struct srtp_batch_ticket;

int srtp_encrypt_batch_dev_async(struct srtp **sessv, size_t nsess,
				 struct srtp_batch_dev *b,
				 struct srtp_batch_ticket **tp);
int srtp_decrypt_batch_dev_async(struct srtp **sessv, size_t nsess,
				 struct srtp_batch_dev *b,
				 struct srtp_batch_ticket **tp);

/** complete an asynchronous call: its result; frees the ticket */
int srtp_batch_wait(struct srtp_batch_ticket *t);

/**
 * Stream state export/import (checkpoint/resume and multi-GPU hand-off:
 * lets a second context continue an SSRC exactly where another left it).
 * Layout follows struct srtp_stream (src/srtp/srtp.h:29-38).
 */
struct srtp_stream_state {
	uint64_t replay_rtp_bitmap, replay_rtp_lix;
	uint64_t replay_rtcp_bitmap, replay_rtcp_lix;
	uint32_t ssrc;
	uint32_t roc;
	uint16_t s_l;
	uint8_t s_l_set;
	uint8_t pad;
	uint32_t rtcp_index;
};

int srtp_stream_export(const struct srtp *srtp, uint32_t ssrc,
		       struct srtp_stream_state *st);
int srtp_stream_import(struct srtp *srtp, const struct srtp_stream_state *st);

/**
 * Cross-rank replay fold of ONE SRTP stream whose unprotect was split
 * across ranks (no reference counterpart: the reference is
 * single-process).  Each rank unprotects its contiguous shard from an
 * assumed boundary state (srtp_stream_import), then records per packet
 * what its own receiver did (srtp_rx_index: 16 B per packet); the ranks
 * all-gather the records and srtp_rx_fold replays the reference receiver
 * over the whole stream in arrival order -- stream_get_seq's first-seq
 * rule (src/srtp/stream.c:87-109), ETIMEDOUT and the ROC bump before
 * authentication (src/srtp/srtp.c:313-321), the tag verdict, the replay
 * window after the tag (src/srtp/replay.c:32-62; srtp.c:362-368, 414-421) and
 * s_l on success only (srtp.c:426-427) -- so a packet replayed across a
 * shard boundary gets EALREADY exactly as one receiver would give it.
 */
enum srtp_rx_stage {
	SRTP_RX_NOHDR = 0,      /* failed before the stream step: res is final */
	SRTP_RX_NOIX = 1,       /* the rank gave ETIMEDOUT: no index computed */
	SRTP_RX_IX = 2,         /* the rank authenticated at index ix */
};

struct srtp_rx_rec {
	uint64_t ix;            /* 48-bit index the rank used (SRTP_RX_IX) */
	int32_t res;            /* the rank's result for the packet */
	uint16_t seq;
	uint8_t stage;          /* enum srtp_rx_stage */
	uint8_t pad;
};

/**
 * A rank's records: its packets arena[pos[i], end[i]) in arrival order (all
 * of SSRC st0->ssrc, else EINVAL), res[i] the results its
 * srtp_decrypt_batch* call returned, st0 the state the rank imported
 * before that call.  0 or EINVAL.
 */
int srtp_rx_index(const struct srtp_stream_state *st0, const uint8_t *arena,
		  const uint32_t *pos, const uint32_t *end,
		  const int32_t *res, size_t n, struct srtp_rx_rec *rec);

/**
 * The same for a rank whose arena, windows and results (the
 * srtp_decrypt_batch_dev outputs) are DEVICE memory: the headers are
 * parsed on the device, which packs seq, header verdict and result into
 * one 4-byte word per packet; those words come down (plus the 4-byte
 * results of a batch whose results fall outside 0..255, a second copy),
 * the arena does not; rec is host memory.  Queued on stream (hipStream_t, NULL: default)
 * and synchronised.  0 or EINVAL / ENOMEM / EIO / ENOSYS.
 */
int srtp_rx_index_dev(const struct srtp_stream_state *st0,
		      const uint8_t *arena, size_t arena_size,
		      const uint32_t *pos, const uint32_t *end,
		      const int32_t *res, size_t n, struct srtp_rx_rec *rec,
		      void *stream);

/**
 * Fold the gathered records of the whole stream from *st (the true state
 * before packet 0): err[i] = the reference receiver's result.  Stops at
 * the first packet whose true index differs from the one its rank
 * authenticated at (the rank's boundary state was wrong, so its verdict
 * is void), or whose replay verdict the whole stream's window changes
 * (0 <-> EALREADY: the rank's bytes, pos and end for it are then those of
 * the other outcome, src/srtp/srtp.c:355-368, 413-429): *ndone = that
 * packet's position and *st = the exact state before it -- re-run packets
 * ndone.. from *st (srtp_stream_import) on their received bytes.
 * *ndone == n when every verdict stands; *st is then the final state.
 * err[i] for i >= *ndone is unspecified.  0, EINVAL or ENOMEM.
 */
int srtp_rx_fold(struct srtp_stream_state *st, enum srtp_suite suite,
		 const struct srtp_rx_rec *rec, size_t n, int32_t *err,
		 size_t *ndone);

/** Batched session setup: n contexts in one GPU launch (key agility). */
int srtp_alloc_many(struct srtp **srtpv, size_t n, enum srtp_suite suite,
		    const uint8_t *keys, size_t key_bytes, int flags);

/**
 * Diagnostics / tuning knobs (defaults from the environment, read once:
 * RE_SRTP_NOPLAN, RE_SRTP_GENERAL, RE_SRTP_PERCLASS, RE_SRTP_NOLEAN,
 * RE_SRTP_NODEVFOLD, RE_SRTP_NOCOOP, RE_SRTP_TRACE,
 * RE_SRTP_TIMES, RE_SRTP_CHUNK, RE_SRTP_PAR_MIN).  name is one of
 * "noplan" (no device planners), "general" (general engine only),
 * "perclass" (one CTR launch per header class), "nolean" (the general
 * CTR kernels for device-planned batches), "nocoop" (small host-planned
 * CTR launches keep the cipher in the one-packet-per-lane kernel),
 * "lplan" (single-stream AES-CM batches planned by the one-launch planner
 * in front of the lean kernel instead of inside the crypto launch; GCM
 * batches always take the one-launch planner), "nopost" (single-stream
 * plan outs come back by a copy and the asynchronous gate word by a launch
 * of its own, instead of one post launch that does both),
 * "mpradix" (multi-session plans group packets by the radix sort),
 * "nobucket" (multi-session plans by the counting grouping of
 * plan_multi.hip instead of the bucket planner), "bpexp" (value: the
 * bucket planner's target of expected packets per bucket, 0 = default),
 * "syncspin" (a synchronous one-stream call waits on its post launch's
 * completion word instead of synchronising the stream; the stream may
 * then still run that launch's tail on return),
 * "pclinger" (value: us a per-packet small-kernel launch stays on the
 * GPU after its batch, taking the workspace's next batches from a pinned
 * mailbox; 0 = off, the default -- while it lingers, other streams mapped
 * to its hardware queue wait up to that long),
 * "nodevfold" (forged packets
 * of a device-planned batch fold on the host), "nocombine" (per-packet
 * calls of different threads do not share launches), "nosmall" (the
 * per-packet path's fused small kernel off), "nofuse" (the operations of
 * a shared per-packet launch run as one launch each), "smallsync" (a small
 * launch waited for by a stream synchronisation, not its completion
 * word), "pcrunners" (per-packet runners at once, 1-4, default 4),
 * "pcspin" (pause loops a waiting per-packet caller spins before it
 * sleeps, default 1000), "pchold" (us a new per-packet runner holds its
 * launch to gather more calls while other runners are in flight, default
 * 0), "noplanfuse" (single-stream AES-CM device batches take the separate
 * planner launches, not the plan inside the crypto launch), "fzepoch"
 * (test hook, process-wide and one-shot: the next fused launch of any
 * thread takes this look-back epoch, its look-back words zeroed first),
 * "rxseq" (srtp_rx_index* and srtp_rx_fold walk
 * in one sequential pass, not in parallel parts), "freshmulti" (the
 * planner's first-batch hint: 1 sends a session's first batch to the
 * per-stream planner, 0 to the one-stream plan; the library sets it when a
 * first batch showed several SSRCs and clears it when one showed one),
 * "trace", "times" (phase
 * timings on stderr), "chunk" (host-scan chunk, packets), "par_min"
 * (sessions per host-pool part); value 0 turns a switch off and restores
 * a size's built-in default.  Results never depend on them.  0 or EINVAL.
 */
int srtp_gpu_tune(const char *name, long value);

/**
 * Diagnostics counters since load: "misses" (packets whose MAC/tag
 * speculation failed -- forged or mis-planned), "folds" (batches re-run to
 * fold such verdicts exactly on the host), "devfolds" (batches whose
 * verdicts folded on the device, no re-run), "rejects" (device plans
 * rejected: the host planned instead), "splans" (per-stream device plans),
 * "pcbatches" / "pcpackets" (shared launches of per-packet calls and the
 * packets they carried), "pcfused" (those of them that ran several
 * operations as one launch), "gated" (asynchronous calls queued behind one
 * the host completed, re-run when waited for), "freshmulti" (the
 * first-batch hint, 0/1).  0 for an unknown name.
 */
uint64_t srtp_gpu_counter(const char *name);

/** last HIP-level error text (diagnostics) */
const char *srtp_gpu_error(void);

/**
 * Kernel timing (diagnostics, used by bench.py): when enabled, every
 * crypto kernel launch is bracketed by HIP events on its own stream.
 * srtp_gpu_prof_read() returns and resets, per kernel class
 * slot = protect*16 + gcm*8 + aes256*4 + shift, the summed device
 * milliseconds, launch count and packet count.
 */
void srtp_gpu_prof(int enable);
void srtp_gpu_prof_read(double ms[32], uint64_t launches[32],
			uint64_t jobs[32]);
/** the same, plus the kernel each slot's launches ran, as
 *  "name<rounds,protect>" (a trailing '+': launches of other kernels
 *  shared the slot) */
void srtp_gpu_prof_read_named(double ms[32], uint64_t launches[32],
			      uint64_t jobs[32], char names[32][48]);

#ifdef __cplusplus
}
#endif

#endif
