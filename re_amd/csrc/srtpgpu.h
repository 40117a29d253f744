/*
 * srtpgpu.h -- the thin C-ABI shim between the C host library and the HIP
 * kernels (re_amd/csrc/hip/srtp_kernels.hip).  Plain C types only.
 *
 * The host C code (re_amd/csrc/host/srtp.c) keeps every piece of SRTP
 * *state* (ROC, s_l, replay windows, SRTCP index, stream table -- exactly
 * the reference's struct srtp_stream, src/srtp/srtp.h:29-38) and turns each
 * packet into one `struct sgpu_job`.  The GPU does all *cipher and MAC*
 * arithmetic: AES-CTR keystream (src/aes/openssl/aes.c:136-171), AES-GCM
 * (aes.c:183-249), HMAC-SHA1 (src/hmac/openssl/hmac.c:78-95) and the session
 * key derivation (src/srtp/misc.c:44-73, srtp.c:33-72).
 */
#ifndef SRTPGPU_H
#define SRTPGPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-direction device crypto context (one per struct comp) -------- */
/* Built on the GPU by sgpu_setup_sessions(); never touched by the host.  */
enum {
	SGPU_MODE_CTR = 0,
	SGPU_MODE_GCM = 1,
};

struct sgpu_comp {              /* 640 bytes, 16-B aligned */
	uint32_t rk[60];        /* AES round keys, LE words of the byte
				   schedule; rounds 1..nr-1 stored rot16 */
	uint32_t nr;            /* 10 or 14 */
	uint32_t mode;          /* SGPU_MODE_* */
	uint32_t tag_len;       /* HMAC truncation (0 for GCM) */
	uint32_t flags;         /* bit0 has_aes, bit1 has_hmac */
	uint32_t k_s[4];        /* session salt k_s (14 B used), LE words */
	uint32_t ipad[5];       /* HMAC-SHA1 inner midstate */
	uint32_t opad[5];       /* HMAC-SHA1 outer midstate */
	uint32_t pad0[2];
	uint32_t htab[16][4];   /* GHASH 4-bit Shoup table (i * H) */
};

struct sgpu_session {           /* rtp = comp[0], rtcp = comp[1] */
	struct sgpu_comp comp[2];
};

/* input to the setup kernel (one per session) */
struct sgpu_keyreq {
	uint8_t master[48];     /* master key ‖ master salt */
	uint32_t cipher_bytes;  /* 16 or 32 */
	uint32_t salt_bytes;    /* 14 or 12 */
	uint32_t tag_len;       /* 4, 10 or 0 */
	uint32_t mode;          /* SGPU_MODE_* */
	uint32_t hash;          /* 1: HMAC-SHA1 suites */
	uint32_t rtcp_encrypted;/* !(flags & SRTP_UNENCRYPTED_SRTCP) */
	uint32_t pad[2];
};

/* ---- per-packet job (host -> device), 48 bytes ------------------------- */
enum {
	SJ_PROTECT      = 1u << 0,  /* 0 = unprotect */
	SJ_CIPHER       = 1u << 1,  /* apply keystream over [c_off,c_off+c_len) */
	SJ_HMAC         = 1u << 2,  /* HMAC-SHA1 over [0,a_len) ‖ trailer? */
	SJ_GCM          = 1u << 3,  /* AES-GCM (AAD [0,a_len) ‖ trailer?) */
	SJ_TRAILER      = 1u << 4,  /* append BE32(trailer) to the MAC/AAD input */
	SJ_STORE_TRAIL  = 1u << 5,  /* protect: store BE32(trailer) at t_off */
	SJ_CIPHER_IF_OK = 1u << 6,  /* unprotect HMAC: decrypt only if tag ok */
	SJ_ROC_AT_TAG   = 1u << 7,  /* unprotect HMAC: if tag ok write BE32(trailer)
				       at tag_off (srtp.c:342-344) */
	SJ_GCM_IV       = 1u << 8,  /* IV per srtp_iv_calc_gcm (misc.c:93-105) */
	SJ_UNDO         = 1u << 9,  /* re-apply keystream only (CTR involution) */
	SJ_SKIP         = 1u << 15, /* no GPU work (host-decided error) */
};

struct sgpu_job {
	uint32_t off;       /* packet start (mbuf start position) in arena */
	uint32_t comp;      /* index of sgpu_comp in the device table */
	uint32_t a_len;     /* HMAC message prefix / GCM AAD prefix, bytes */
	uint32_t c_off;     /* cipher region start, bytes from off (4-aligned) */
	uint32_t c_len;     /* cipher region length, bytes */
	uint32_t tag_off;   /* where the tag is written / read, from off */
	uint32_t t_off;     /* where SJ_STORE_TRAIL stores the trailer */
	uint32_t trailer;   /* ROC or E‖SRTCP-index (host order) */
	uint32_t ssrc;      /* for the IV */
	uint32_t ixhi;      /* (uint32_t)(ix >> 16) */
	uint32_t ixlo;      /* (uint16_t)ix */
	uint32_t flags;     /* SJ_* */
};

/* verdict bits returned per job (unprotect) */
enum {
	SV_TAG_OK   = 1u << 0,
	SV_CIPHERED = 1u << 1,
};

/* ---- shim entry points (implemented in srtp_kernels.hip) --------------- */
int   sgpu_init(void);                  /* 0, or ENODEV / ENOSYS */
const char *sgpu_last_error(void);

/* device session-context table: slots are allocated by the host */
int   sgpu_table_reserve(uint32_t nsessions);      /* grow capacity (moves
							   the table: callers
							   exclude batches) */
uint32_t sgpu_table_capacity(void);
int   sgpu_setup_sessions(const struct sgpu_keyreq *req, const uint32_t *slot,
			  uint32_t n);               /* KDF + key schedule */
uint64_t sgpu_table_device_ptr(void);

/* run one kernel class over jobs[0..njobs) of a device arena.  Every job
 * of a launch shares (mode, nr, shift = (c_off/4)&3, direction); verdict is
 * a device array (or NULL).  `stream` is a hipStream_t or NULL. */
#define SGPU_COOP_MAX 2048     /* general launches of at most this many jobs
				   run their cipher regions one packet per
				   workgroup (k_ctr_coop, k_gcm_coop) */
void  sgpu_set_coop(int on);
/* the per-packet path (few packets, CTR + HMAC-SHA1 suites): one fused
 * kernel, one packet per workgroup, over jobs, packets, verdicts and saved
 * words in PINNED HOST memory (sgpu_host_alloc: device-accessible), no
 * copies; packets of at most SGPU_SMALL_MAX bytes from their start.
 * prot: 0 unprotect, 1 protect, 2 per job (SJ_PROTECT).  done_flag (pinned
 * host word, or NULL): done_seq is stored there once every workgroup's
 * writes are visible; done_cnt: a device word, 0 between launches */
#define SGPU_SMALL_MAX 2048
int   sgpu_run_small(uint8_t *arena, uint64_t arena_size,
		     const struct sgpu_job *jobs, uint32_t njobs,
		     uint8_t *verdict, uint32_t *save, int prot,
		     uint32_t *done_cnt, uint32_t *done_flag,
		     uint32_t done_seq, void *stream);
/* The lingering form of that kernel (srtp_gpu_tune pclinger): one launch
 * serves successive batches posted through a mailbox in coherent pinned
 * host memory (sgpu_host_alloc_coherent); bc is a device block zeroed on
 * the stream before each launch.  The host writes a batch's arguments,
 * then post = its sequence number (never 0); the kernel stores it into
 * done_flag when the batch is complete.  The kernel exits when the last
 * batch is complete and it has been idle for linger_us (or stop is set,
 * or it has lived life_us), storing last = the batch it completed last and
 * gone = 1: a batch posted after that was not taken. */
struct sgpu_srv_mb {
	uint32_t post;                  /* host */
	uint32_t stop;                  /* host */
	uint32_t gone;                  /* device, at exit */
	uint32_t last;                  /* device, at exit */
	uint32_t njobs;                 /* host: the batch posted */
	uint32_t mode;                  /* 0 / 1 / 2 as sgpu_run_small's prot */
	uint64_t arena, asz, jobs, verdict, save, comps;
};
struct sgpu_srv_bc {
	uint32_t seq, done, njobs, mode;
	uint64_t arena, asz, jobs, verdict, save, comps;
};
int   sgpu_run_small_srv(struct sgpu_srv_mb *mb, struct sgpu_srv_bc *bc,
			 uint32_t grid, uint32_t linger_us, uint32_t life_us,
			 uint32_t *done_cnt, uint32_t *done_flag, void *stream);
const void *sgpu_table_ptr(void);
void *sgpu_host_alloc_coherent(size_t n);
int   sgpu_run_class(uint8_t *arena, uint64_t arena_size,
		     const struct sgpu_job *jobs, uint32_t njobs,
		     uint8_t *verdict, uint32_t *save, int mode, int nr,
		     int shift, int prot, void *stream);

/*
 * Compact RTP path.  The host's sequential pass emits one 8-byte
 * descriptor per packet; the kernel derives the rest of the job from the
 * packet window (pos/end), the header it parsed (sgpu_hdr) and the session
 * context -- exactly the fields plan_rtp_enc/plan_rtp_dec would set.
 *   bits  0..15  (uint16_t)ix
 *   bits 16..47  (uint32_t)(ix >> 16)
 *   bits 48..63  SD_* flags
 */
enum {
	SD_RUN      = 1u << 0,  /* packet has a GPU job (else host-decided) */
	SD_CIPHER   = 1u << 1,  /* apply the keystream (dec HMAC: if tag ok) */
	SD_ROC_M1   = 1u << 2,  /* trailer ROC = ixhi - 1 (receiver v=roc+1) */
	SD_ROC_P1   = 1u << 3,  /* trailer ROC = ixhi + 1 (receiver v=roc-1) */
};

static inline uint64_t sgpu_desc(uint64_t ix, uint32_t flags)
{
	return (ix & 0xffffull) | ((uint64_t)(uint32_t)(ix >> 16) << 16) |
	       ((uint64_t)flags << 48);
}

struct sgpu_hdr;

struct sgpu_compact {
	const uint32_t *pos;            /* packet start in arena (device) */
	const uint32_t *end;            /* packet end (device) */
	const struct sgpu_hdr *hdr;     /* parsed headers (device) */
	const uint64_t *desc;           /* descriptors (device) */
	const uint32_t *sess;           /* per-packet session index or NULL */
	const uint32_t *compmap;        /* session index -> sgpu_comp index */
	const uint32_t *idx;            /* packet list of this class, or NULL:
					   packets base .. base+n-1 */
	uint32_t base;
	uint32_t n;
	uint8_t *verdict;               /* [packet] SV_* (device) */
	uint32_t *save;                 /* [packet] tag word under the ROC */
	uint32_t *nfail;                /* +1 per speculation miss (device) */
	int undo;                       /* restore the pre-call bytes */
	int uniform;                    /* every packet: one session context;
					   2: and the device planner's shape
					   (SD_RUN | SD_CIPHER, [hl, A) --
					   the lean CTR kernels); 4: the same
					   for SRTCP (k_plan_rtcp, rtcp = 1) */
	const uint32_t *guard;          /* device word; nonzero: do nothing
					   (a rejected device plan) or NULL */
	int rtcp;                       /* SRTCP packets: descriptor = SRTCP
					   index | E << 31 (sgpu_rdesc) */
	uint32_t *flist;                /* lean unprotect: forged packets are
					   listed here (n words, device; slot =
					   the nfail count) and restored by a
					   packet-per-workgroup pass; NULL: a
					   full-grid pass finds them */
	const uint32_t *gfail;          /* or NULL: a second guard word (the
					   bucket planner's fail word, beside
					   the class guards in guard[]) */
};

/* SRTCP descriptor: bits 0..30 SRTCP index, bit 31 E, bits 48..63 SD_* */
static inline uint64_t sgpu_rdesc(uint32_t index, uint32_t e, uint32_t flags)
{
	return (uint64_t)(index & 0x7fffffffu) | ((uint64_t)(e & 1u) << 31) |
	       ((uint64_t)flags << 48);
}



/* launch the compact kernel of class (mode, nr, shift, prot) */
int   sgpu_run_compact(uint8_t *arena, uint64_t arena_size,
		       const struct sgpu_compact *c, int mode, int nr,
		       int shift, int prot, void *stream);

/*
 * Device-side planning of a single-stream RTP batch (the sequential state
 * machine of srtp.c:203-213/279-280 and 310-321/426-427, misc.c:22-41,
 * replay.c:32-62) as a speculative parallel scan: packet i is assumed to
 * see s_l = seq[i-1]; ROC wraps are prefix-summed; every assumption is
 * verified on the device.  out->fail != 0 means "plan on the host".
 */
struct sgpu_plan_in {
	uint32_t n;
	uint32_t prot;          /* 1 srtp_encrypt, 0 srtp_decrypt */
	uint32_t fresh;         /* s_l not set yet (first RTP packet) */
	uint32_t ssrc;          /* existing stream's SSRC (!fresh) */
	uint32_t roc;
	uint32_t s_l;
	uint64_t lix;           /* replay_rtp */
	uint64_t bitmap;
	uint32_t tag;           /* bytes the tag adds / removes */
	uint32_t ssrc_any;      /* no stream yet: take packet 0's SSRC */
	uint32_t need;          /* protect: tag room end + need <= cap */
	uint32_t maxlen;        /* packets of maxlen bytes or more: SPF_SIZE */
	uint32_t zeroed;        /* out already zeroed (sgpu_parse_prologue) */
	uint32_t pad;
	const uint32_t *pred;   /* async chain: the gate word of the call
				   before, or NULL (sgpu_gate_pred, folded
				   into the plan's first kernel) */
};

/* compact (counter-cached) kernels take packets shorter than this:
 * AES-CM caches rounds 1-2 for block indices < 256 (kern_common.h CtrKs,
 * CTR_B15), the single-key GCM kernel for counters < 256 (GCMU_B8) */
#define SGPU_CACHED_MAX_CTR (4096u - 64u)
#define SGPU_CACHED_MAX_GCM (4096u - 64u)
#define SGPU_CACHED_MAX(mode) \
	((mode) == SGPU_MODE_GCM ? SGPU_CACHED_MAX_GCM : SGPU_CACHED_MAX_CTR)

enum {
	SPF_PARSE   = 1u << 0,  /* EBADMSG / short packet */
	SPF_SSRC    = 1u << 1,  /* more than one SSRC */
	SPF_CLASS   = 1u << 2,  /* header lengths of different shift class */
	SPF_ORDER   = 1u << 3,  /* s_l speculation broken (reordering) */
	SPF_TIMEOUT = 1u << 4,  /* ETIMEDOUT */
	SPF_REPLAY  = 1u << 5,  /* index not strictly increasing */
	SPF_SIZE    = 1u << 6,  /* payload of 1 MiB or more */
	SPF_CAP     = 1u << 7,  /* protect: tag does not fit (ENOMEM) */
	SPF_BAD     = 1u << 8,  /* invalid window (pos/end/cap/arena) */
	SPF_PRED    = 1u << 9,  /* the chained call before did not complete
				   on the device (async batches) */
	SPF_SEG     = 1u << 10, /* multi-session counting grouping: a session
				   with more than SGPU_MP_SEGMAX packets (the
				   host re-plans with the radix sort) */
	SPF_SLOW    = 1u << 11, /* fused launch: a look-back wait ran past its
				   bound (a stalled predecessor, not a bad
				   window: counted as "lbtimeouts") */
};
#define SGPU_MP_SEGMAX 1024

/*
 * Chained asynchronous batches: a call queued behind a pending one on the
 * same stream is planned as failed (SPF_PRED, nothing modified) if the
 * earlier call's gate word is set, i.e. if that call must be completed on
 * the host; it is then re-run when waited for.
 *   pred: *fail |= SPF_PRED if *pred (launch after fail is zeroed, before
 *         the plan's guards are derived from it)
 *   set:  *gate = *fail || (nfail && *nfail)  (after the call's launches)
 */
int   sgpu_gate_pred(const uint32_t *pred, uint32_t *fail, void *stream);
int   sgpu_gate_set(const uint32_t *fail, const uint32_t *nfail,
		    uint32_t *gate, void *stream);

#define SGPU_PLAN_TAIL 65
struct sgpu_plan_out {
	uint32_t fail;          /* SPF_* */
	uint32_t wraps;         /* ROC increments over the batch */
	uint32_t ssrc0;
	uint32_t hl0;           /* header length of packet 0 */
	uint32_t s_l_last;      /* s_l after the last packet */
	uint32_t nfail;         /* the crypto launch's speculation misses
				   (copied here by sgpu_plan_finish) */
	uint32_t skip[4];       /* guard of the shift-class-s crypto launch:
				   fail || class(hl0) != s */
	uint64_t tail_ix[SGPU_PLAN_TAIL]; /* ix of the last min(n,65) packets */
};

/*
 * Single-stream AES-CM batch planned INSIDE its crypto launch
 * (k_ctr_fused.h): each workgroup parses its packets' headers, makes every
 * check of sgpu_plan_rtp, takes its ROC prefix from the workgroups before
 * it by a decoupled look-back over agg[] (ticket order, so each
 * predecessor is running or done), then encrypts / decrypts.  A workgroup
 * that sees a failed check (its own, or one published before it) does
 * nothing; out->fail != 0 after the launch means the batch must be undone
 * (sgpu_fused_undo: every packet whose desc has SD_RUN back to its bytes)
 * and planned on the host -- the same "a rejected plan modifies nothing"
 * as the separate planner.  Per packet the launch writes hdr, es (the end
 * before the call) and desc (0: not processed); processed packets also
 * end + delta, err = 0 and (unprotect) verdict / save / flist / nfail.
 * out (fail, nfail) must be zero at launch: the workgroup with ticket 0
 * zeroes out_next's for the workspace's next launch.  agg: one word per
 * workgroup (n / sgpu_fused_block()), (epoch << 48 | status << 46 |
 * fail << 32 | wraps); epoch 1..65535, the host zeroes agg when it wraps.
 * ticket: the workgroups take tbase, tbase + 1, ... (the next launch's
 * tbase: + f->ntickets).
 */
struct sgpu_fused {
	struct sgpu_plan_in in;
	const uint32_t *pos;
	uint32_t *end;
	const uint32_t *cap;            /* or NULL */
	int32_t *err;
	uint32_t *es;
	struct sgpu_hdr *hdr;
	uint64_t *desc;
	uint8_t *verdict;               /* unprotect */
	uint32_t *save;                 /* unprotect: tag word under the ROC */
	uint32_t *flist;                /* unprotect: forged packets */
	struct sgpu_plan_out *out;
	struct sgpu_plan_out *out_next;
	uint32_t *cm_out;               /* *cm_out = comp (for later launches) */
	unsigned long long *agg;
	uint32_t *ticket;
	uint32_t tbase;
	uint32_t epoch;
	uint32_t comp;                  /* the session's sgpu_comp index */
	int32_t delta;                  /* end change of a processed packet */
	uint32_t shift;                 /* undo: the batch's header class */
	uint32_t ntickets;              /* (out) tickets the launch takes (its
					   workgroups) -- the next tbase */
	uint64_t prof_id;               /* (out) its srtp_gpu_prof record */
};
unsigned sgpu_fused_block(void);        /* packets per workgroup */
/* the plan of sgpu_run_fused alone (k_lp_plan), for a lean crypto launch
 * behind it: the same outputs, plus out->skip[] (the class guards; the
 * crypto launch's second guard word is out->fail) and the results of
 * every packet planned; no byte of the arena is written */
int   sgpu_run_fzplan(uint8_t *arena, uint64_t arena_size,
		      struct sgpu_fused *f, void *stream);
int   sgpu_run_fused(uint8_t *arena, uint64_t arena_size,
		     struct sgpu_fused *f, int nr, void *stream);
/* after a rejected fused launch (f->shift = class of packet 0's header):
 * every processed packet back to its bytes before the call -- protect: the
 * keystream re-applied over [hl, L); unprotect: over [hl, L - tag) where
 * still decrypted (SV_CIPHERED), and the tag word under the ROC restored */
int   sgpu_fused_undo(uint8_t *arena, uint64_t arena_size,
		      const struct sgpu_fused *f, int nr, int prot,
		      void *stream);
/* unprotect with forged packets: their ciphertext back (the list the
 * launch filled, k_ctr_refix_list) -- before sgpu_fold_rtp */
int   sgpu_fused_refix(uint8_t *arena, uint64_t arena_size,
		       const struct sgpu_fused *f, int nr, void *stream);

/* plan n packets (hdr/pos/end/cap device arrays; cap may be NULL) into
 * desc (device); scratch holds >= n/256 + 2 words; out is a device
 * pointer.  out->fail is the guard of the launches that follow. */
int   sgpu_plan_rtp(const struct sgpu_plan_in *in, const struct sgpu_hdr *hdr,
		    const uint32_t *pos, const uint32_t *end, const uint32_t *cap,
		    uint64_t arena_size, uint64_t *desc, uint32_t *scratch,
		    struct sgpu_plan_out *out, void *stream);

/*
 * Multi-session device planning (many sessions with at most one RTP
 * stream each, e.g. 64K sessions x 1 SSRC): packets are stably sorted by
 * session on the device, every session's run of packets gets the
 * single-stream speculation above, and each touched session's final state
 * is returned (sgpu_sstate), so the host work is O(sessions).
 * order (device, n words, or NULL): the packets by descending length, the
 * launch order for the crypto kernels (equal work per wave).
 */
enum {
	SST_EXISTS  = 1u << 0,  /* stream 0 exists */
	SST_SL_SET  = 1u << 1,  /* s_l set */
	SST_TOUCHED = 1u << 2,  /* (out) the batch had packets for it */
};

struct sgpu_sstate {            /* 32 bytes */
	uint32_t ssrc;
	uint32_t roc;
	uint32_t s_l;
	uint32_t flags;         /* SST_* */
	uint64_t lix;           /* replay_rtp */
	uint64_t bitmap;
};

/*
 * Device planning of a single-session RTP batch over up to SGPU_SP_MAX
 * streams (SRTP_MAX_STREAMS SSRCs of one struct srtp, plan_streams.hip):
 * the speculation of sgpu_plan_rtp per stream, new SSRCs appended in
 * first-appearance order.  in->st[k] (k < nst): the session's streams in
 * table order (SST_EXISTS, SST_SL_SET, RTP replay).  Per stream k of
 * out->ssrc[0..nst): wraps, packets (cnt), final s_l (if cnt) and the
 * indices of its last min(cnt, 65) packets; out->base.fail / skip[] as in
 * sgpu_plan_out (nst > SGPU_SP_MAX: SPF_SSRC).
 */
#define SGPU_SP_MAX 8
struct sgpu_splan_in {
	uint32_t n;
	uint32_t prot;
	uint32_t tag;
	uint32_t need;
	uint32_t maxlen;
	uint32_t zeroed;        /* out already zeroed */
	uint32_t nst;           /* streams before the batch */
	uint32_t pad;
	struct sgpu_sstate st[SGPU_SP_MAX];
};
struct sgpu_splan_out {
	struct sgpu_plan_out base;      /* fail, hl0, skip[] */
	uint32_t nst;                   /* streams after the batch */
	uint32_t pad;
	uint32_t ssrc[SGPU_SP_MAX];
	uint32_t wraps[SGPU_SP_MAX];
	uint32_t cnt[SGPU_SP_MAX];
	uint32_t s_l_last[SGPU_SP_MAX];
	int32_t last[SGPU_SP_MAX];      /* last packet index of the stream */
	uint32_t pad2[2];
	uint64_t tail_ix[SGPU_SP_MAX][SGPU_PLAN_TAIL];
};
size_t sgpu_splan_scratch(uint32_t n);
int   sgpu_splan_rtp(const struct sgpu_splan_in *in,
		     const struct sgpu_hdr *hdr, const uint32_t *pos,
		     const uint32_t *end, const uint32_t *cap,
		     uint64_t arena_size, uint64_t *desc, void *scratch,
		     size_t scratch_bytes, struct sgpu_splan_out *out,
		     void *stream);


struct sgpu_mplan_in {
	uint32_t n;
	uint32_t nsess;
	uint32_t prot;
	uint32_t tag;
	uint32_t need;
	uint32_t key_bits;      /* bits of the session index */
	uint32_t maxlen;        /* packets of maxlen bytes or more: SPF_SIZE */
	uint32_t out_zeroed;    /* out already zeroed (sgpu_parse_prologue) */
	const uint32_t *wchk;   /* or NULL: the window checks (SPF_PARSE,
				   SIZE, BAD, CAP) were made by the parse
				   prologue, one word per 256-packet block
				   (sgpu_prologue.wchk) */
	uint32_t radix;         /* group by the radix sort (else, for up to
				   65536 sessions, the counting grouping) */
	uint32_t cnt_zeroed;    /* counting: its per-session counters
				   (sgpu_mplan_counters) already zeroed */
};

/* the counting grouping's per-session counters inside the scratch (the
 * parse prologue zeroes them: in.cnt_zeroed) */
uint32_t *sgpu_mplan_counters(void *scratch, uint32_t n, uint32_t nsess);
/* ... how many words from there the prologue zeroes (counters and the
 * crypto launch order's bins) */
uint32_t sgpu_mplan_counter_words(uint32_t nsess);

/* the same in two launch groups: phase 1 sorts the packets by session
 * (needs neither st_in nor the session map), phase 2 plans; the host
 * prepares the session states in between (same arguments to both) */
int   sgpu_mplan_rtp_phase(int phase, const struct sgpu_mplan_in *in,
			   const struct sgpu_hdr *hdr, const uint32_t *pos,
			   const uint32_t *end, const uint32_t *cap,
			   uint64_t arena_size, const uint32_t *sess,
			   const struct sgpu_sstate *st_in,
			   struct sgpu_sstate *st_out, uint64_t *desc,
			   void *scratch, size_t scratch_bytes,
			   struct sgpu_plan_out *out, uint32_t *order,
			   void *stream);

/*
 * Resident stream states: the device keeps one sgpu_sstate per table slot
 * (stream 0 of the session's RTP direction), zeroed by
 * sgpu_setup_sessions.  Multi-session device batches read and update it
 * in place, so session state does not cross PCIe per call; the host
 * reads it back (sgpu_sst_read) before any host-side path touches the
 * session.  cm: session index -> comp index (2 * slot), device.
 *   load:   st_in[k] = need && need[k] ? (table[slot] = up[k]) : table[slot]
 *   commit: table[slot] = st_out[k] (touched ones, SST_TOUCHED cleared)
 *           unless *fail or *nfail (device words, read when it runs)
 *   read:   out[i] = table[slot[i]] (host arrays, synchronous)
 */
int   sgpu_sst_load(const uint32_t *cm, const uint8_t *need,
		    const struct sgpu_sstate *up, uint32_t nsess,
		    struct sgpu_sstate *st_in, void *stream);
int   sgpu_sst_commit(const uint32_t *cm, const struct sgpu_sstate *st_out,
		      uint32_t nsess, const uint32_t *fail,
		      const uint32_t *nfail, void *stream);
int   sgpu_sst_read(const uint32_t *slot, uint32_t n,
		    struct sgpu_sstate *out);

/* device scratch needed by sgpu_mplan_rtp */
size_t sgpu_mplan_scratch(uint32_t n, uint32_t nsess);

int   sgpu_mplan_rtp(const struct sgpu_mplan_in *in,
		     const struct sgpu_hdr *hdr, const uint32_t *pos,
		     const uint32_t *end, const uint32_t *cap,
		     uint64_t arena_size, const uint32_t *sess,
		     const struct sgpu_sstate *st_in,
		     struct sgpu_sstate *st_out, uint64_t *desc,
		     void *scratch, size_t scratch_bytes,
		     struct sgpu_plan_out *out, uint32_t *order,
		     void *stream);

/*
 * Multi-session device planning in four launches (plan_buckets.hip): the
 * sessions are cut into nb buckets of 2^bshift consecutive session ids,
 * each bucket has a fixed region of cap entries, so no global scan is
 * needed before a packet is placed:
 *   sgpu_bplan_scatter  per packet: header parse (rtp_hdr_decode), window
 *                       checks, end copy; its bucket slot by an atomic per
 *                       (workgroup, bucket), the entry packed as
 *                       16-byte entry of everything the plan needs
 *                       (SPF_SEG past cap); its place in its length bin
 *                       likewise
 *   sgpu_bplan_plan     per bucket (one workgroup): the sessions' resident
 *                       states (+ uploads), the entries sorted by session
 *                       and packet index in LDS, the speculation of
 *                       sgpu_plan_rtp per session segment (srtp.c:203-215,
 *                       310-321, misc.c:22-41, replay.c:32-62), desc, the
 *                       crypto launch order (descending length bins, the
 *                       packets of a scatter workgroup together), each
 *                       session's state after the batch; its fail bits
 *                       and the scatter's into out->fail (the scatter's
 *                       first workgroup zeroed it, wrote hl0 and the
 *                       class guards skip[])
 *   (crypto, in `order`, guarded by skip[] and out->fail; unprotect CTR:
 *   the forged-packet restore)
 *   sgpu_bplan_finish   the results (end, err) per packet, the commit of
 *                       the touched sessions' states, the bucket and bin
 *                       counters back to zero; with speculation misses
 *                       the verdict fold per bucket (the fold of
 *                       sgpu_mfold_rtp), the last workgroup then writes
 *                       the forged packets' EAUTH results and commits --
 *                       or leaves everything for the host (fo->fail);
 *                       gate word, out->nfail
 * No workgroup waits for another except the fold's last one (a ticket,
 * taken only when there are misses).  bcount / obins / ticket must be zero
 * before the first launch of a workspace; every call leaves them so.
 */
#ifdef __HIPCC__
typedef uint4 uint4_t_;
#else
typedef struct { uint32_t x, y, z, w; } uint4_t_;
#endif
#define SGPU_BP_BLOCK 1024
#define SGPU_BP_PPT 4           /* scatter: packets per thread */
#define SGPU_BP_CAPMAX 4096     /* entries per bucket */
#define SGPU_BP_EXP 2100        /* expected entries per bucket, at most
				   (64K sessions x 1M packets: 128 sessions,
				   ~2049 entries in a 4096-entry region;
				   against 1088 -- 64 sessions, twice the
				   buckets -- the planner launches took 169
				   instead of 190 us per config-4 step,
				   profiles/r06/bucket_geometry_ab.txt) */
#define SGPU_BP_NSB 256         /* sessions per bucket, at most */
#define SGPU_BP_NBMAX 4096      /* buckets, at most */
#define SGPU_BP_NMAX (1u << 26) /* packets per call, at most */
#define SGPU_BP_SEGMAX 1024     /* packets of one session per bucket pass */
struct sgpu_bplan {
	uint32_t n, nsess, prot, tag, need, maxlen;
	uint32_t bshift, nb, cap;       /* bucket geometry */
	int32_t delta;                  /* end change of a processed packet */
	uint32_t gcm;
	uint32_t nofold;                /* misses are left to the host fold */
	const uint32_t *pos, *end, *capv, *sess;
	uint32_t *posw;                 /* = pos (EAUTH: pos += header) */
	uint32_t *endw;                 /* = end (results) */
	int32_t *err;
	uint32_t *es;                   /* end before the call */
	struct sgpu_hdr *hdr;
	uint64_t *desc;
	uint32_t *order;                /* crypto launch order (n) */
	uint4_t_ *tmp;                  /* nb x cap bucket entries: index |
					   bin << 26, seq | session in bucket
					   << 16, SSRC, place in the bin */
	uint32_t *sorted;               /* nb x cap: packet index by session */
	uint32_t *bcount;               /* nb: entries per bucket (zeroed) */
	uint32_t *obins;                /* 64: packets per length bin (zeroed) */
	uint32_t *ticket;               /* the fold's last-workgroup ticket
					   (zero between calls) */
	uint32_t *afail;                /* per scatter workgroup */
	uint32_t *sseg;                 /* per session: start | count << 16 */
	const uint32_t *cm;             /* session -> comp index (2 slot) */
	const uint8_t *upneed;          /* or NULL: upload up[s] first */
	const struct sgpu_sstate *up;
	struct sgpu_sstate *sst;        /* resident states by slot */
	struct sgpu_sstate *sout;       /* per session, after the batch */
	struct sgpu_plan_out *out;
	struct sgpu_fold_out *fo;
	const uint32_t *pred;           /* async chain: the call before's gate */
	uint32_t *gate;                 /* or NULL */
	uint32_t *nfail;                /* the crypto launch's miss counter
					   (zeroed by the scatter) */
	const uint8_t *verdict;
	const uint32_t *flist;          /* CTR: forged packets, or NULL */
	uint32_t *outh;                 /* or NULL: the call's outcome (the
					   outbytes from out, fo behind it) to
					   this pinned mirror by k_bp_finish */
	uint32_t outbytes;
};
/* the geometry's target of expected entries per bucket (0: SGPU_BP_EXP) */
void sgpu_bplan_set_exp(uint32_t e);
size_t sgpu_bplan_scratch(uint32_t n, uint32_t nsess, uint32_t nb,
			  uint32_t cap);
/* geometry for n packets over nsess sessions: 0 and bshift/nb/cap, or -1
 * (the bucket planner does not take the batch) */
int   sgpu_bplan_geometry(uint32_t n, uint32_t nsess, uint32_t *bshift,
			  uint32_t *nb, uint32_t *cap);
/* the resident state table (sgpu_sst_*) */
struct sgpu_sstate *sgpu_sst_table(void);
int   sgpu_bplan_scatter(const uint8_t *arena, uint64_t arena_size,
			 const struct sgpu_bplan *b, void *stream);
int   sgpu_bplan_plan(const struct sgpu_bplan *b, void *stream);
int   sgpu_bplan_finish(const struct sgpu_bplan *b, void *stream);

/*
 * Device-side planning of a single-stream SRTCP batch (srtcp_encrypt
 * srtcp.c:31-140, srtcp_decrypt srtcp.c:143-287): protect numbers the
 * packets rtcp_index + 1, + 2, ...; unprotect reads E || index from each
 * packet and, for the HMAC suites, speculates every index new and
 * increasing (replay_rtcp, replay.c:32-62) and every tag authentic.
 * out->fail != 0 means "plan on the host"; skip[2] guards the launches
 * (SRTCP's cipher region starts at byte 8: class 2).
 */
struct sgpu_rplan_in {
	uint32_t n;
	uint32_t prot;
	uint32_t ssrc_any;      /* no stream yet: take packet 0's SSRC */
	uint32_t ssrc;
	uint32_t rtcp_index;    /* stream's index (protect) */
	uint32_t tag;           /* HMAC tag length (0 for GCM) */
	uint32_t gcm;
	uint32_t hmac;          /* replay-checked (HMAC suites) */
	uint32_t encrypted;     /* E for protect (has_aes / encrypted) */
	uint32_t need;          /* protect: bytes appended */
	uint64_t lix, bitmap;   /* replay_rtcp */
	uint32_t maxlen;        /* packets of maxlen bytes or more: SPF_SIZE
				   (the counter-cached kernels' bound) */
	uint32_t pad;
};

/* the same plan in one launch with the header parse (k_rp_plan): per
 * packet hdr, es and desc (not the results: the workgroup after reads a
 * packet's end for the replay order -- sgpu_plan_results behind the
 * crypto launch writes them); out is the call's
 * plan out (fail, nfail zeroed by the launch before, through out_next),
 * out->fail the crypto launch's guard, out->nfail its miss counter;
 * *cm_out = comp */
struct sgpu_rfused {
	struct sgpu_rplan_in in;
	const uint32_t *pos;
	uint32_t *end;
	const uint32_t *cap;            /* or NULL */
	int32_t *err;
	uint32_t *es;
	struct sgpu_hdr *hdr;
	uint64_t *desc;
	struct sgpu_plan_out *out, *out_next;
	uint32_t *cm_out;
	uint32_t comp;
	int32_t delta;
};
int   sgpu_run_rpplan(const uint8_t *arena, uint64_t arena_size,
		      const struct sgpu_rfused *r, void *stream);

int   sgpu_plan_rtcp(const struct sgpu_rplan_in *in,
		     const struct sgpu_hdr *hdr, const uint32_t *eix,
		     const uint32_t *pos, const uint32_t *end,
		     const uint32_t *cap, uint64_t arena_size, uint64_t *desc,
		     struct sgpu_plan_out *out, void *stream);

/*
 * Verdict fold of a device-planned single-stream unprotect (srtp_decrypt,
 * srtp.c:288-432) on the device.  The plan assumed every tag authentic;
 * with the verdicts known, packet i really sees s_l = seq of the last
 * earlier packet that authenticated, or 0 after a later forged rollover
 * (the ROC is bumped before the MAC check, s_l updated only on success:
 * srtp.c:318-321, 426-427).  If every packet's rollover, ETIMEDOUT status
 * and index are unchanged under that s_l, the speculation's verdicts are
 * the reference's and the fold is exact: forged packets get EAUTH
 * (pos = payload, end = tag start; GCM: end untouched, srtp.c:404-411),
 * the stream's s_l and replay window follow the authentic packets only.
 * Otherwise out->fail is set and the host folds instead.
 */
struct sgpu_fold_out {
	uint32_t fail;          /* speculation inconsistent with the verdicts */
	uint32_t nok;           /* authentic packets */
	uint32_t first_ok;      /* index of the first authentic packet */
	uint32_t last_ok;       /* ... and of the last (0xffffffff: none) */
	uint32_t s_l;           /* s_l after the batch */
	uint32_t pad;
	uint64_t lix, bitmap;   /* replay_rtp after the batch */
};

/* scratch: >= 5 * (n / 256 + 2) words.  gcm: EAUTH leaves end as is.
 * Runs after the crypto kernels (verdict[] complete); results written
 * only if the fold holds (out->fail == 0).  phase 0: all; 1: the verdict
 * (out); 2: the forged packets' results.  nfail (device, may be NULL):
 * the kernels' miss count -- the fold does nothing when it is 0. */
int   sgpu_fold_rtp(int phase, const uint32_t *nfail,
		    const struct sgpu_plan_in *in, const struct sgpu_hdr *hdr,
		    const uint64_t *desc, const uint8_t *verdict,
		    const uint32_t *end0, uint32_t *pos, uint32_t *end,
		    int32_t *err, int gcm, uint32_t *scratch,
		    struct sgpu_fold_out *out, void *stream);

/* verdict fold of a multi-session unprotect planned by sgpu_mplan_rtp
 * (same scratch, still holding the sort): per session segment what
 * sgpu_fold_rtp does for one stream.  Writes the EAUTH results and the
 * touched sessions' s_l / replay window into st_out only if the fold holds
 * (out->fail == 0); fscratch: sgpu_mfold_scratch(n) bytes.  phase 0: all;
 * 1: the verdict only (out->fail); 2: results and windows.  nfail (device,
 * may be NULL): the crypto kernels' miss count -- queued behind them, the
 * fold does nothing when it is 0 (out->fail = 0). */
size_t sgpu_mfold_scratch(uint32_t n);
int   sgpu_mfold_rtp(int phase, const uint32_t *nfail,
		     const struct sgpu_mplan_in *in,
		     const struct sgpu_hdr *hdr, const uint32_t *sess,
		     const uint64_t *desc, const uint8_t *verdict,
		     const uint32_t *end0, uint32_t *pos, uint32_t *end,
		     int32_t *err, int gcm, const struct sgpu_sstate *st_in,
		     struct sgpu_sstate *st_out, void *scratch,
		     size_t scratch_bytes, uint32_t *fscratch,
		     struct sgpu_fold_out *out, void *stream);

/* guarded per-packet results of a device-planned batch (device arrays):
 * if *guard == 0: end[i] = end0[i] + delta, err[i] = 0 */
/* sgpu_plan_results, and in the same launch: *gate = *guard || *nfail
 * (sgpu_gate_set; gate may be NULL) and *nfail_out = *nfail (next to the
 * plan, so one copy brings both back; nfail_out may be NULL).  ffail
 * (may be NULL): the device fold's verdict word -- a miss then gates the
 * next call only if the fold failed: *gate = *guard || (*nfail && *ffail) */
int   sgpu_plan_finish(const uint32_t *guard, const uint32_t *end0,
		       uint32_t *end, int32_t *err, uint32_t n, int32_t delta,
		       const uint32_t *nfail, uint32_t *gate,
		       uint32_t *nfail_out, const uint32_t *ffail,
		       void *stream);
/* out (struct sgpu_plan_out, bytes of it) to pinned host memory with
 * vector stores; gate (or NULL) = out->fail || out->nfail; done (pinned
 * host word, or NULL) = seq after all of it */
int   sgpu_plan_post(const void *out, void *host, uint32_t bytes,
		     uint32_t *gate, uint32_t *done, uint32_t seq,
		     void *stream);
int   sgpu_plan_results(const uint32_t *guard, const uint32_t *end0,
			uint32_t *end, int32_t *err, uint32_t n, int32_t delta,
			void *stream);

/* store 4 raw bytes (LE word vals[i]) at arena + offs[i], any alignment
 * (restores tag bytes before a re-run) -- device arrays */
int   sgpu_store_words(uint8_t *arena, const uint32_t *offs,
		       const uint32_t *vals, uint32_t n, void *stream);

/* device-resident header parse: for each packet i, reads the RTP (or RTCP)
 * header at arena[pos[i]] bounded by end[i] and writes sgpu_hdr[i]. */
struct sgpu_hdr {               /* 12 bytes */
	uint32_t ssrc;
	uint16_t seq;
	uint16_t err_pos;   /* bytes consumed before an EBADMSG (0 if ok) */
	uint32_t hdr_len;   /* full RTP header length (0xffffffff on EBADMSG) */
};
/* eix (RTCP, optional): 3 words per packet, the BE word at end-4-tl for
 * tl = 0, 4, 10 (the E-bit/SRTCP-index word for each tag length). */
int   sgpu_parse_headers(const uint8_t *arena, uint64_t arena_size,
			 const uint32_t *pos, const uint32_t *end,
			 struct sgpu_hdr *out, uint32_t *eix, uint32_t n,
			 int rtcp, void *stream);
/* srtp_rx_index_dev: per packet seq | ok << 16 | (ssrc != ssrc0) << 17 |
 * (res outside 0..255) << 23 | (res & 255) << 24 */
int   sgpu_rx_pack(const struct sgpu_hdr *hd, const int32_t *res,
		   uint32_t ssrc0, uint32_t *out, uint32_t n, void *stream);

/* sgpu_parse_headers plus the per-call prologue of a device batch in the
 * same launch: end_copy[i] = end[i] (if set), z0[0..nz0) and z1[0..nz1)
 * zeroed, *cm_out = cm (if set) -- instead of separate copy/fill ops */
struct sgpu_prologue {
	uint32_t *end_copy;
	uint32_t *z0, *z1;
	uint32_t nz0, nz1;
	uint32_t *cm_out;
	uint32_t cm;
	/* wchk != NULL: per 256-packet block, the OR of each packet's
	 * window checks of the RTP planners (k_plan_count / k_mp_count:
	 * SPF_PARSE, SPF_SIZE, SPF_BAD, SPF_CAP), with these parameters */
	uint32_t *wchk;
	const uint32_t *cap;
	uint32_t prot, tag, need, maxlen;
	uint32_t *z2;           /* nz2 words zeroed by the whole grid */
	uint32_t nz2;
};
int   sgpu_parse_prologue(const uint8_t *arena, uint64_t arena_size,
			  const uint32_t *pos, const uint32_t *end,
			  struct sgpu_hdr *out, uint32_t *eix, uint32_t n,
			  int rtcp, const struct sgpu_prologue *pro,
			  void *stream);

/* kernel timing (HIP events recorded on the launch stream) */
void  sgpu_prof_enable(int on);
/* launches behind a rejected device plan (they did nothing), not counted
 * by sgpu_prof_read */
uint64_t sgpu_prof_voided(void);
/* ... and a fused launch the host found rejected (struct sgpu_fused
 * prof_id) */
void  sgpu_prof_void(uint64_t id);
/* RTCP compound decode (rtcp_walk.hip, include/re_rtcp_batch.h) */
struct rtcp_desc;
struct rtcp_item;
struct rtcp_enc_batch;
int sgpu_rtcp_walk(const uint8_t *arena, uint64_t arena_size,
		   const uint32_t *pos, const uint32_t *end, uint32_t n,
		   struct rtcp_desc *descv, uint32_t maxmsg, uint32_t *nmsg,
		   struct rtcp_item *itemv, uint32_t maxitem, uint32_t *nitem,
		   int32_t *err, uint32_t *stop, void *stream);
/* rtcp_encode.hip: the batch's packets into its arena (re_rtcp_batch.h) */
int sgpu_rtcp_encode(const struct rtcp_enc_batch *b);

#define SGPU_PROF_NAME 48
void  sgpu_prof_read(double *ms, uint64_t *launches, uint64_t *jobs,
		     char (*names)[SGPU_PROF_NAME]);

/* memory helpers (device / pinned host) */
void *sgpu_malloc(size_t n);
void  sgpu_free(void *p);
void *sgpu_host_alloc(size_t n);
void  sgpu_host_free(void *p);
int   sgpu_memcpy_h2d(void *dst, const void *src, size_t n, void *stream);
int   sgpu_memcpy_d2h(void *dst, const void *src, size_t n, void *stream);
int   sgpu_memcpy_d2d(void *dst, const void *src, size_t n, void *stream);
int   sgpu_memset(void *dst, int v, size_t n, void *stream);
int   sgpu_stream_sync(void *stream);
int   sgpu_stream_query(void *stream);  /* 0 done, EAGAIN, EIO */
int   sgpu_device_sync(void);
void *sgpu_stream_create(void);
void  sgpu_stream_destroy(void *s);
int   sgpu_set_device(int dev);
void *sgpu_event_create(void);
void  sgpu_event_destroy(void *ev);
int   sgpu_event_record(void *ev, void *stream);
int   sgpu_event_sync(void *ev);
int   sgpu_stream_wait(void *stream, void *ev);
int   sgpu_get_device(void);

#ifdef __cplusplus
}
#endif

#endif
