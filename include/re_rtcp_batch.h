/**
 * @file re_rtcp_batch.h  Batched RTCP compound decode and encode on the
 * GPU (extension).
 *
 * libre hands every received (and, with SRTP, srtcp_decrypt()ed) RTCP
 * compound packet to rtcp_recv_handler, which calls
 * `while (0 == rtcp_decode(&msg, mb))` (src/rtp/rtp.c:164) and dispatches
 * each message.  rtcp_decode_batch_dev() runs that loop for a whole batch
 * of packets resident in HBM -- typically the arena srtcp_decrypt_batch_dev
 * just unprotected -- and returns, instead of allocated struct rtcp_msg
 * objects, one fixed-size descriptor per decoded message with the fields a
 * dispatcher routes on.  The walk is the reference's byte for byte
 * (src/rtp/pkt.c:115-133, 337-551; rr.c, sdes.c, fb.c): each body parse
 * advances the cursor by what it reads, reads past the end yield 0 without
 * moving, padding is slurped to the message's next 32-bit boundary, and
 * the walk stops at the first call that fails.
 */
#ifndef RE_RTCP_BATCH_H
#define RE_RTCP_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/** one decoded RTCP message (20 bytes) */
struct rtcp_desc {
	uint32_t off;      /**< message start, bytes from the packet's pos   */
	uint32_t size;     /**< bytes rtcp_decode consumed (with padding)    */
	uint8_t  pt;       /**< packet type (enum rtcp_type)                  */
	uint8_t  count;    /**< header count / FMT field                      */
	uint16_t length;   /**< header length field, 32-bit words minus one   */
	uint32_t ssrc;     /**< the body's first SSRC: SR/RR sender, first
			        SDES chunk / BYE source (0 if count is 0), APP
			        src, FIR/NACK ssrc, RTPFB/PSFB packet sender,
			        XR ssrc; 0 for unknown types                  */
	uint32_t aux;      /**< SR: RTP timestamp; APP: name (big-endian
			        word); NACK: fsn << 16 | blp; RTPFB/PSFB:
			        media source; XR: block type << 16 | block
			        length; otherwise 0                            */
};

/**
 * Decode n RTCP compound packets, all arrays in device memory: packet i is
 * arena[pos[i], end[i]).  descv holds n * maxmsg descriptors (packet i's
 * from descv[i * maxmsg]); nmsg[i] = messages decoded (those beyond
 * maxmsg are counted, not written); err[i] = the errno of the rtcp_decode
 * call that ended the walk (EBADMSG -- also for a packet consumed exactly
 * to its end, like the reference loop; EINVAL for a window outside the
 * arena) and stop[i] the offset that call began at (== end - pos: the
 * whole packet decoded).  Queued on stream (hipStream_t, NULL: default);
 * no host synchronisation.  Returns 0 or EINVAL / EIO / ENOSYS (no GPU).
 */
int rtcp_decode_batch_dev(const uint8_t *arena, size_t arena_size,
			  const uint32_t *pos, const uint32_t *end, size_t n,
			  struct rtcp_desc *descv, uint32_t maxmsg,
			  uint32_t *nmsg, int32_t *err, uint32_t *stop,
			  void *stream);

/* ---- message contents ------------------------------------------------- */

/**
 * What rtcp_decode fills into struct rtcp_msg (include/re_rtp.h:205-280)
 * beyond the descriptor, as a list of fixed-size items per packet in
 * message order.  Variable-length data stays in the arena: an item gives
 * its offset (bytes from the packet's pos) and length, where the reference
 * copies it (sdes.c:134-137 item data, pkt.c:454 BYE reason, :476 APP
 * data) or references it (fb.c:119-156 TWCC chunks / deltas, :280-291
 * AFB).
 */
enum rtcp_item_kind {
	RTCP_ITEM_SR = 1,         /* v: ntp_sec, ntp_frac, rtp_ts, psent,
				     osent (pkt.c:383-388)                   */
	RTCP_ITEM_RB = 2,         /* report block (rr.c:55-72): v: ssrc,
				     fraction, lost (24 bits), last_seq,
				     jitter, lsr, dlsr                       */
	RTCP_ITEM_SDES_CHUNK = 3, /* v: src, items in the chunk (sdes.c)  */
	RTCP_ITEM_SDES = 4,       /* sub: type; v: length, data offset     */
	RTCP_ITEM_BYE_SRC = 5,    /* v: src                                */
	RTCP_ITEM_BYE_REASON = 6, /* v: length, offset                     */
	RTCP_ITEM_APP = 7,        /* sub: subtype (header count); v: src,
				     name (big-endian word), data offset,
				     data length                            */
	RTCP_ITEM_FIR = 8,        /* RFC 2032 FIR: v: ssrc                 */
	RTCP_ITEM_NACK = 9,       /* RFC 2032 NACK: v: ssrc, fsn, blp      */
	RTCP_ITEM_FB = 10,        /* RTPFB / PSFB header: sub: FMT; v:
				     ssrc_packet, ssrc_media, n (FCI
				     entries: length - 2, halved for FIR)    */
	RTCP_ITEM_GNACK = 11,     /* generic NACK FCI: v: pid, blp         */
	RTCP_ITEM_TWCC = 12,      /* v: seq, count, reftime, fbcount,
				     chunks offset, chunks length, deltas
				     length (the deltas follow the chunks)   */
	RTCP_ITEM_SLI = 13,       /* v: first, number, picid               */
	RTCP_ITEM_AFB = 14,       /* v: offset, length                     */
	RTCP_ITEM_PSFB_FIR = 15,  /* RFC 5104 FIR FCI: v: ssrc, seq_n      */
	RTCP_ITEM_XR = 16,        /* v: ssrc, block type, block length     */
	RTCP_ITEM_RRTR = 17,      /* v: ntp_msw, ntp_lsw                   */
	RTCP_ITEM_DLRR = 18,      /* v: ssrc, lrr, dlrr                    */
};

/** one decoded field group (32 bytes) */
struct rtcp_item {
	uint16_t msg;      /**< the message's index within its packet      */
	uint8_t  kind;     /**< enum rtcp_item_kind                         */
	uint8_t  sub;      /**< kind-specific (SDES type, APP subtype, FMT) */
	uint32_t v[7];
};

/**
 * rtcp_decode_batch_dev plus every message's contents: itemv holds
 * n * maxitem items (packet i's from itemv[i * maxitem]); nitem[i] =
 * items of the messages decoded (beyond maxitem counted, not written).
 * The items of the message whose decode failed are not reported (the
 * reference frees that message, pkt.c:540-551).  itemv / nitem may be
 * NULL (maxitem 0): then it is rtcp_decode_batch_dev.
 */
int rtcp_decode_full_batch_dev(const uint8_t *arena, size_t arena_size,
			       const uint32_t *pos, const uint32_t *end,
			       size_t n, struct rtcp_desc *descv,
			       uint32_t maxmsg, uint32_t *nmsg,
			       struct rtcp_item *itemv, uint32_t maxitem,
			       uint32_t *nitem, int32_t *err, uint32_t *stop,
			       void *stream);

/* ---- compound encode --------------------------------------------------- */

/**
 * One message of a compound packet to encode: what one rtcp_encode() call
 * (src/rtp/pkt.c:316, rtcp_vencode :136-313) appends, with the encode
 * handlers' output (rtcp_rr_encode rr.c:35, rtcp_sdes_encode sdes.c:36,
 * FB / XR handlers) given as data:
 *
 *   SR   (200)  w[0..5]: ssrc, ntp_sec, ntp_frac, rtp_ts, psent, osent;
 *               report blocks rbv[first .. first+num)
 *   RR   (201)  w[0]: ssrc; report blocks rbv[first .. first+num)
 *   SDES (202)  chunks chunkv[first .. first+num)
 *   BYE  (203)  sources srcv[first .. first+count); with
 *               RTCP_ENC_REASON the reason pool[off .. off+len)
 *   APP  (204)  w[0]: src, w[1]: name (big-endian bytes); data
 *               pool[off .. off+len) (len % 4: EBADMSG, pkt.c:199-203)
 *   FIR  (192)  w[0]: ssrc
 *   NACK (193)  w[0]: ssrc, w[1]: fsn, w[2]: blp
 *   RTPFB (205) / PSFB (206)  w[0]: ssrc_packet, w[1]: ssrc_media;
 *               FCI bytes pool[off .. off+len) (what the handler writes,
 *               e.g. rtcp_rtpfb_gnack_encode pid / blp pairs)
 *   XR   (207)  w[0]: ssrc; report block bytes pool[off .. off+len)
 *
 * count is the header count / FMT written as rtcp_hdr_encode does
 * (pkt.c:92: RTCP_VERSION << 6 | count, in one byte).  Every message is
 * padded with zeros to 32 bits and its length field is its size in words
 * minus one.
 */
enum { RTCP_ENC_REASON = 1 };

struct rtcp_enc_msg {                   /* 44 bytes */
	uint8_t  pt;
	uint8_t  count;
	uint16_t flags;                 /* RTCP_ENC_REASON */
	uint32_t w[6];
	uint32_t first, num;
	uint32_t off, len;
};

struct rtcp_enc_rb {                    /* rtcp_rr_encode (rr.c:35-51) */
	uint32_t ssrc;
	uint32_t fraction;              /* low 8 bits used */
	uint32_t lost;                  /* low 24 bits used */
	uint32_t last_seq, jitter, lsr, dlsr;
};

struct rtcp_enc_chunk {                 /* rtcp_sdes_encode (sdes.c:36-76) */
	uint32_t src;
	uint32_t first, num;            /* items itemv[first .. first+num):
					   none is EINVAL (sdes.c:42) */
};

struct rtcp_enc_sdes {                  /* one SDES item */
	uint8_t  type;
	uint8_t  pad;
	uint16_t len;                   /* > 255: EINVAL (sdes.c:57-60) */
	uint32_t off;                   /* value pool[off .. off+len) */
};

/** one batch (every pointer device memory) */
struct rtcp_enc_batch {
	uint8_t *arena;
	size_t arena_size;
	const uint32_t *pos;            /* packet i is written from pos[i] */
	uint32_t *end;                  /* out: pos[i] + encoded bytes */
	const uint32_t *cap;            /* room up to cap[i]: larger is ENOMEM
					   (an arena cannot grow like the
					   reference's mbuf) */
	const uint32_t *mfirst;         /* n + 1 entries: packet i is
					   msgv[mfirst[i] .. mfirst[i+1]) */
	const struct rtcp_enc_msg *msgv;
	const struct rtcp_enc_rb *rbv;
	const struct rtcp_enc_chunk *chunkv;
	const struct rtcp_enc_sdes *sdesv;
	const uint32_t *srcv;
	const uint8_t *pool;
	uint32_t nmsg, nrb, nchunk, nsdes, nsrc, pool_size;  /* array sizes */
	int32_t *err;                   /* per packet: 0, or the errno of the
					   first message that failed (EINVAL:
					   unknown type, an SDES chunk with no
					   items or an item over 255 bytes, a
					   reference outside its array;
					   EBADMSG: APP data not a multiple of
					   4; ENOMEM: over cap) -- nothing is
					   written for that packet and end[i]
					   stays pos[i] */
	size_t n;
	void *stream;                   /* hipStream_t; NULL: default */
};

/**
 * Encode n RTCP compound packets into the arena, each byte-exact with the
 * rtcp_encode() calls its messages describe appended to one mbuf from
 * pos[i].  Queued on b->stream, no host synchronisation: the arena can go
 * straight on to srtcp_encrypt_batch_dev with the same pos / end (leave
 * cap room for the SRTCP index and tag).  0 or EINVAL / EIO / ENOSYS.
 */
int rtcp_encode_batch_dev(const struct rtcp_enc_batch *b);

#ifdef __cplusplus
}
#endif

#endif
