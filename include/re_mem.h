/**
 * @file re_mem.h  Reference-counted memory -- standalone subset of libre's
 * include/re_mem.h:23-34 (mem_zalloc / mem_ref / mem_deref / mem_realloc).
 */
#ifndef RE_MEM_H
#define RE_MEM_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void (mem_destroy_h)(void *data);

void    *mem_alloc(size_t size, mem_destroy_h *dh);
void    *mem_zalloc(size_t size, mem_destroy_h *dh);
void    *mem_realloc(void *data, size_t size);
void    *mem_ref(void *data);
void    *mem_deref(void *data);
unsigned mem_nrefs(const void *data);

#ifdef __cplusplus
}
#endif

#endif
