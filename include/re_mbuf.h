/**
 * @file re_mbuf.h  Packet buffer -- standalone subset, layout-identical to
 * libre's struct mbuf (baresip/re v4.10.0 include/re_mbuf.h:43-48).  When this
 * library is built inside libre, libre's own re_mbuf.h/mbuf.c are used.
 */
#ifndef RE_MBUF_H
#define RE_MBUF_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct mbuf {
	uint8_t *buf;   /**< Buffer memory      */
	size_t size;    /**< Size of buffer     */
	size_t pos;     /**< Position in buffer */
	size_t end;     /**< End of buffer      */
};

struct mbuf *mbuf_alloc(size_t size);
int      mbuf_resize(struct mbuf *mb, size_t size);
int      mbuf_write_mem(struct mbuf *mb, const uint8_t *buf, size_t size);
int      mbuf_write_u32(struct mbuf *mb, uint32_t v);
int      mbuf_read_mem(struct mbuf *mb, uint8_t *buf, size_t size);

static inline uint8_t *mbuf_buf(const struct mbuf *mb)
{
	return mb ? mb->buf + mb->pos : (uint8_t *)NULL;
}

static inline size_t mbuf_get_left(const struct mbuf *mb)
{
	return (mb && (mb->end > mb->pos)) ? (mb->end - mb->pos) : 0;
}

#ifdef __cplusplus
}
#endif

#endif
