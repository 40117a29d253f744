/*
 * ubench_launch.hip -- the per-packet path's fixed cost: one small launch
 * and its completion, measured four ways (median of 2000 round trips):
 *   sync   hipLaunchKernelGGL + hipStreamSynchronize
 *   query  the same, completion by spinning on hipStreamQuery
 *   flag   completion by spinning on a pinned host word the kernel's last
 *          workgroup stores (system-scope release) after its writes
 *   work   'flag' with 32 workgroups each reading and writing 1200 B of
 *          pinned host memory (the small kernel's traffic shape)
 * hipcc --offload-arch=gfx950 -O2 scripts/ubench_launch.hip -o /tmp/ul
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <algorithm>
#include <vector>

static double now_us()
{
	timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

__global__ void k_touch(uint32_t *buf, uint32_t nw, unsigned *cnt,
			volatile uint32_t *flag, uint32_t seq, int allfence)
{
	const uint32_t b = blockIdx.x;
	for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x)
		buf[b * nw + w] = seq + w;
	if (allfence)
		__threadfence_system();
	else
		__builtin_amdgcn_s_waitcnt(0);  /* the wave's stores done */
	__syncthreads();
	if (threadIdx.x == 0) {
		__threadfence_system();
		if (atomicAdd(cnt, 1u) + 1u == gridDim.x) {
			*cnt = 0;
			__hip_atomic_store((uint32_t *)flag, seq, __ATOMIC_RELEASE,
					   __HIP_MEMORY_SCOPE_SYSTEM);
		}
	}
}

static double median(std::vector<double> &v)
{
	std::sort(v.begin(), v.end());
	return v[v.size() / 2];
}

int main()
{
	hipStream_t s;
	uint32_t *hbuf, *flag;
	unsigned *cnt;
	const int N = 2000;
	hipStreamCreate(&s);
	hipHostMalloc((void **)&hbuf, 64 * 1200, hipHostMallocDefault);
	hipHostMalloc((void **)&flag, 64, hipHostMallocDefault);
	hipMalloc((void **)&cnt, 4);
	hipMemset(cnt, 0, 4);
	*flag = 0;
	const char *mode[5] = {"sync", "query", "flag", "work", "workall"};
	for (int m = 0; m < 5; m++) {
		std::vector<double> t;
		const uint32_t g = m >= 3 ? 32 : 1, nw = m >= 3 ? 300 : 0;
		long bad = 0;
		for (int i = 0; i < N + 100; i++) {
			const uint32_t seq = (uint32_t)(m * 100000 + i + 1);
			const double a = now_us();
			hipLaunchKernelGGL(k_touch, dim3(g), dim3(256), 0, s, hbuf,
					   nw, cnt, flag, seq, m == 4);
			if (m == 0) {
				hipStreamSynchronize(s);
			}
			else if (m == 1) {
				while (hipStreamQuery(s) == hipErrorNotReady)
					;
			}
			else {
				while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq)
					__builtin_ia32_pause();
			}
			const double b = now_us();
			/* every word the kernel stored is visible once the
			 * flag is */
			for (uint32_t k = 0; k < g * nw; k++)
				bad += hbuf[k] != seq + k % nw;
			if (i >= 100)
				t.push_back(b - a);
		}
		hipStreamSynchronize(s);
		printf("%-7s grid %2u: median %.2f us, p10 %.2f, stale words %ld\n",
		       mode[m], g, median(t), t[t.size() / 10], bad);
	}
	return 0;
}
