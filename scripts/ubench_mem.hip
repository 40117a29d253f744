/*
 * ubench_mem.hip -- HBM counter calibration for the crypto kernels' own
 * access patterns (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are
 * calibrated only for 16-B-per-lane streaming accesses).
 *
 * Arena: N packets of L bytes in S-byte slots (default 1M x 1200 in 1216,
 * the BASELINE config-2/3 layout).  Every kernel reads and rewrites the
 * same bytes of every packet (x ^= 1 on each word), so the byte count is
 * known: N * (bytes touched) read + the same written.  Patterns:
 *   stream     16 B per lane, consecutive lanes consecutive (reference)
 *   lane64     one packet per lane, 64-B chunks from the packet start
 *              (4 x 16-B loads/stores per chunk: k_gcmu / k_ctr_hmac
 *              without quad coalescing)
 *   quad64     four lanes move one packet's 64-B chunk (quad coalescing,
 *              the access pattern of quad_load / quad_store)
 *   lane64o12  lane64 from c_off = 12 (the round-1 k_gcmu units)
 *   quad64o12  quad64 from c_off = 12
 * Build: hipcc -O3 --offload-arch=gfx950 scripts/ubench_mem.hip -o ubench_mem
 * Run under rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE) --kernel-trace.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_stream(uint8_t *a, uint64_t n16)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n16)
		return;
	uint4 *p = (uint4 *)a + i;
	uint4 v = *p;
	v.x ^= 1; v.y ^= 1; v.z ^= 1; v.w ^= 1;
	*p = v;
}

/* one packet per lane: 64-B units from off0, nunit of them */
__global__ void k_lane64(uint8_t *a, uint32_t n, uint32_t slot, uint32_t off0,
			 uint32_t nunit)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	uint8_t *pkt = a + (uint64_t)i * slot + off0;
	for (uint32_t m = 0; m < nunit; m++) {
		uint4 d[4];
#pragma unroll
		for (int g = 0; g < 4; g++)
			d[g] = *(const uint4 *)(pkt + 64u * m + 16u * g);
#pragma unroll
		for (int g = 0; g < 4; g++) {
			d[g].x ^= 1; d[g].y ^= 1; d[g].z ^= 1; d[g].w ^= 1;
			*(uint4 *)(pkt + 64u * m + 16u * g) = d[g];
		}
	}
}

/* quad-coalesced: lane q of a quad moves quarter q of each quad member's
 * unit (the memory side of quad_load / quad_store) */
__global__ void k_quad64(uint8_t *a, uint32_t n, uint32_t slot, uint32_t off0,
			 uint32_t nunit)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t q = i & 3u, base = i & ~3u;
	for (uint32_t m = 0; m < nunit; m++) {
		uint4 d[4];
#pragma unroll
		for (int g = 0; g < 4; g++)
			d[g] = *(const uint4 *)(a + (uint64_t)(base + g) * slot +
						off0 + 64u * m + 16u * q);
#pragma unroll
		for (int g = 0; g < 4; g++) {
			d[g].x ^= 1; d[g].y ^= 1; d[g].z ^= 1; d[g].w ^= 1;
			*(uint4 *)(a + (uint64_t)(base + g) * slot + off0 +
				   64u * m + 16u * q) = d[g];
		}
	}
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
	const uint32_t slot = argc > 2 ? (uint32_t)atoi(argv[2]) : 1216u;
	const int reps = 5;
	uint8_t *a;
	const uint64_t bytes = (uint64_t)n * slot;
	CHK(hipMalloc(&a, bytes));
	CHK(hipMemset(a, 0, bytes));
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	struct { const char *name; int kind; uint32_t off0, nunit; } K[] = {
		{"stream", 0, 0, 0},
		{"lane64", 1, 0, 19},
		{"quad64", 2, 0, 19},
		{"lane64o12", 1, 12, 18},
		{"quad64o12", 2, 12, 18},
	};
	for (auto &k : K) {
		float best = 1e9f;
		for (int r = 0; r < reps; r++) {
			CHK(hipEventRecord(e0, 0));
			if (k.kind == 0)
				hipLaunchKernelGGL(k_stream, dim3((bytes / 16 + 255) / 256),
						   dim3(256), 0, 0, a, bytes / 16);
			else if (k.kind == 1)
				hipLaunchKernelGGL(k_lane64, dim3((n + 255) / 256),
						   dim3(256), 0, 0, a, n, slot,
						   k.off0, k.nunit);
			else
				hipLaunchKernelGGL(k_quad64, dim3((n + 255) / 256),
						   dim3(256), 0, 0, a, n, slot,
						   k.off0, k.nunit);
			CHK(hipGetLastError());
			CHK(hipEventRecord(e1, 0));
			CHK(hipEventSynchronize(e1));
			float ms;
			CHK(hipEventElapsedTime(&ms, e0, e1));
			if (ms < best)
				best = ms;
		}
		const double touched = k.kind == 0 ? (double)bytes :
				       (double)n * 64.0 * k.nunit;
		printf("%-10s best %.4f ms  bytes/dir %.3f GB  %.2f TB/s (r+w)\n",
		       k.name, best, touched / 1e9, 2 * touched / best / 1e9);
	}
	CHK(hipFree(a));
	return 0;
}
