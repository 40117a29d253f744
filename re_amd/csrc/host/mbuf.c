/*
 * mbuf.c -- standalone subset of libre's packet buffer with the same
 * growth rule as src/mbuf/mbuf.c:235-260 (MAX(needed, 2*size), 512 if
 * empty) so that `size` evolves exactly as in the reference.
 */
#include <errno.h>
#include <string.h>
#include "re_mem.h"
#include "re_mbuf.h"

enum { DEFAULT_SIZE = 512 };

static void mbuf_destructor(void *data)
{
	struct mbuf *mb = data;
	mem_deref(mb->buf);
}

struct mbuf *mbuf_alloc(size_t size)
{
	struct mbuf *mb = mem_zalloc(sizeof(*mb), mbuf_destructor);
	if (!mb)
		return NULL;
	if (mbuf_resize(mb, size ? size : DEFAULT_SIZE))
		return mem_deref(mb);
	return mb;
}

int mbuf_resize(struct mbuf *mb, size_t size)
{
	uint8_t *buf;
	if (!mb)
		return EINVAL;
	buf = mb->buf ? mem_realloc(mb->buf, size) : mem_alloc(size, NULL);
	if (!buf)
		return ENOMEM;
	mb->buf = buf;
	mb->size = size;
	return 0;
}

int mbuf_write_mem(struct mbuf *mb, const uint8_t *buf, size_t size)
{
	size_t rsize;
	if (!mb || !buf)
		return EINVAL;
	rsize = mb->pos + size;
	if (rsize > mb->size) {
		size_t dsize = mb->size ? mb->size * 2 : DEFAULT_SIZE;
		int err = mbuf_resize(mb, rsize > dsize ? rsize : dsize);
		if (err)
			return err;
	}
	memcpy(mb->buf + mb->pos, buf, size);
	mb->pos += size;
	if (mb->pos > mb->end)
		mb->end = mb->pos;
	return 0;
}

int mbuf_write_u32(struct mbuf *mb, uint32_t v)
{
	return mbuf_write_mem(mb, (const uint8_t *)&v, sizeof(v));
}

int mbuf_read_mem(struct mbuf *mb, uint8_t *buf, size_t size)
{
	if (!mb || !buf)
		return EINVAL;
	if (size > mbuf_get_left(mb))
		return EOVERFLOW;
	memcpy(buf, mb->buf + mb->pos, size);
	mb->pos += size;
	return 0;
}
