/*
 * ctr14a.hip -- AES-256-CM + HMAC-SHA1 any-class kernels (k_ctr_hmac_any,
 * see k_ctr.h); a TU of its own so the four inlined class bodies build in
 * parallel with the per-class instantiations.
 */
#include "k_ctr.h"

kfn_t sgpu_pick_ctr14_any(bool uni, int prot)
{
	return uni ? (prot ? k_ctr_hmac_any<14, true, true>
			   : k_ctr_hmac_any<14, false, true>)
		   : (prot ? k_ctr_hmac_any<14, true, false>
			   : k_ctr_hmac_any<14, false, false>);
}
