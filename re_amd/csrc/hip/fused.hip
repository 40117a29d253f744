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
