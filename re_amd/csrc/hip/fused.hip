/*
 * fused.hip -- instantiations of the single-stream plan + crypto kernels
 * (k_ctr_fused.h), a TU of their own so their four inlined class bodies
 * build in parallel with the other kernels.
 */
#include "k_ctr_fused.h"

typedef void (*kfn_f)(const FArgs);

/* undo: the undo kernel, else the plan + crypto kernel */
kfn_f sgpu_pick_fused(int nr, int prot, int undo)
{
	if (undo)
		return nr == 10 ? (prot ? k_ctr_fused_undo<10, true>
					: k_ctr_fused_undo<10, false>)
				: (prot ? k_ctr_fused_undo<14, true>
					: k_ctr_fused_undo<14, false>);
	return nr == 10 ? (prot ? k_ctr_fused<10, true> : k_ctr_fused<10, false>)
			: (prot ? k_ctr_fused<14, true> : k_ctr_fused<14, false>);
}

kfn_f sgpu_pick_fzplan(int prot)
{
	return prot ? k_lp_plan<true> : k_lp_plan<false>;
}

unsigned sgpu_lp_wg(void)
{
	return LP_WG;
}

#ifdef FZ_WTIME
/* the diagnostic stamps of the last launches (scripts/fz_wtime.py) */
extern "C" __attribute__((visibility("default"))) int
sgpu_fz_wtime(uint64_t *out, size_t n)
{
	if (n > FZ_WREC * FZ_WTIME_MAX)
		n = FZ_WREC * FZ_WTIME_MAX;
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fzw), n * 8, 0,
				   hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
