/* pool.h -- persistent host worker pool (pool.c) */
#ifndef RE_AMD_POOL_H
#define RE_AMD_POOL_H
#include <stddef.h>

typedef void (*par_fn)(void *arg, size_t a, size_t b);

/* run fn over [0, n) in contiguous ranges of at least min_per items */
void par_for(size_t n, size_t min_per, par_fn fn, void *arg);

#endif
