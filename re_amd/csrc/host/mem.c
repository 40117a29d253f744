/*
 * mem.c -- reference-counted allocator with destructors.  Standalone
 * stand-in for libre's src/mem (same contract as include/re_mem.h:23-34:
 * mem_zalloc/mem_ref/mem_deref, destructor runs when the last reference
 * is dropped).  Thread-safe reference counting.
 */
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "re_mem.h"

struct mem_hdr {
	size_t nrefs;
	mem_destroy_h *dh;
	size_t size;
	size_t pad;          /* keep the payload 32-byte aligned */
};

static size_t g_live;           /* live blocks (leak checks) */

size_t re_amd_mem_live(void)
{
	return __atomic_load_n(&g_live, __ATOMIC_RELAXED);
}

static struct mem_hdr *hdr_of(const void *p)
{
	return (struct mem_hdr *)((uint8_t *)(uintptr_t)p - sizeof(struct mem_hdr));
}

void *mem_alloc(size_t size, mem_destroy_h *dh)
{
	struct mem_hdr *m = malloc(sizeof(*m) + size);
	if (!m)
		return NULL;
	m->nrefs = 1;
	m->dh = dh;
	m->size = size;
	__atomic_add_fetch(&g_live, 1, __ATOMIC_RELAXED);
	return m + 1;
}

void *mem_zalloc(size_t size, mem_destroy_h *dh)
{
	void *p = mem_alloc(size, dh);
	if (p)
		memset(p, 0, size);
	return p;
}

void *mem_realloc(void *data, size_t size)
{
	struct mem_hdr *m, *m2;
	if (!data)
		return mem_alloc(size, NULL);
	m = hdr_of(data);
	m2 = realloc(m, sizeof(*m2) + size);
	if (!m2)
		return NULL;
	m2->size = size;
	return m2 + 1;
}

void *mem_ref(void *data)
{
	if (data)
		__atomic_add_fetch(&hdr_of(data)->nrefs, 1, __ATOMIC_RELAXED);
	return data;
}

void *mem_deref(void *data)
{
	struct mem_hdr *m;
	if (!data)
		return NULL;
	m = hdr_of(data);
	if (__atomic_sub_fetch(&m->nrefs, 1, __ATOMIC_ACQ_REL) > 0)
		return NULL;
	if (m->dh)
		m->dh(data);
	free(m);
	__atomic_sub_fetch(&g_live, 1, __ATOMIC_RELAXED);
	return NULL;
}

unsigned mem_nrefs(const void *data)
{
	return data ? (unsigned)__atomic_load_n(&hdr_of(data)->nrefs,
						__ATOMIC_RELAXED) : 0;
}
