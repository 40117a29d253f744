/**
 * @file re_rtcp_batch.h  Batched RTCP compound decode on the GPU
 * (extension).
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

#ifdef __cplusplus
}
#endif

#endif
