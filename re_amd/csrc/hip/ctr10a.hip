/*
 * ctr10a.hip -- AES-128-CM + HMAC-SHA1 any-class kernels (k_ctr_hmac_any,
 * see k_ctr.h); a TU of its own so the four inlined class bodies build in
 * parallel with the per-class instantiations.
 */
#include "k_ctr.h"

kfn_t sgpu_pick_ctr10_any(bool uni, int prot)
{
	return uni ? (prot ? k_ctr_hmac_any<10, true, true>
			   : k_ctr_hmac_any<10, false, true>)
		   : (prot ? k_ctr_hmac_any<10, true, false>
			   : k_ctr_hmac_any<10, false, false>);
}
