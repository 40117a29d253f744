/*
 * fault.h -- allocation-failure injection for the host C, the counterpart
 * of the reference's mem_threshold_set (src/mem/mem.c) and its retest -o
 * sweep (test/test.c:468-560): srtp_gpu_tune("fail_alloc", k) makes the
 * k-th host or device allocation of the library from now on fail, once.
 * Every allocation site of srtp.c, keying.c and udp.c goes through these
 * wrappers; a failed one must leave the caller's state as it was
 * (tests/test_gpu_faults.py sweeps k over whole calls).
 */
#ifndef RE_AMD_FAULT_H
#define RE_AMD_FAULT_H
#include <stdlib.h>
#include "re_mem.h"
#include "../srtpgpu.h"

extern long re_amd_fail_alloc __attribute__((visibility("hidden")));

static inline int fi_fail(void)
{
	return __atomic_load_n(&re_amd_fail_alloc, __ATOMIC_RELAXED) > 0 &&
	       __atomic_sub_fetch(&re_amd_fail_alloc, 1, __ATOMIC_RELAXED) == 0;
}

#define fi_malloc(n)        (fi_fail() ? NULL : malloc(n))
#define fi_calloc(n, s)     (fi_fail() ? NULL : calloc((n), (s)))
#define fi_realloc(p, n)    (fi_fail() ? NULL : realloc((p), (n)))
#define fi_mem_zalloc(n, d) (fi_fail() ? NULL : mem_zalloc((n), (d)))
#define fi_sgpu_malloc(n)   (fi_fail() ? NULL : sgpu_malloc(n))
#define fi_sgpu_host_alloc(n) (fi_fail() ? NULL : sgpu_host_alloc(n))

#endif
