/*
 * ctr14.hip -- AES-256-CM + HMAC-SHA1 kernel instantiations (see k_ctr.h).
 */
#include "k_ctr.h"

/* small general launches: the cipher regions one packet per workgroup */
kfn_t sgpu_pick_ctr14_coop(int prot)
{
	return prot ? k_ctr_coop<14, true> : k_ctr_coop<14, false>;
}

kfn_t sgpu_pick_ctr14(bool compact, bool uni, int shift, int prot)
{
	if (shift < 0)
		return compact ? sgpu_pick_ctr14_any(uni, prot) : NULL;
#define PICK(C, U, S)                                                          \
	if (compact == C && uni == U && shift == S)                            \
		return prot ? k_ctr_hmac<14, S, true, C, U>                    \
			    : k_ctr_hmac<14, S, false, C, U>;
#define PICK4(C, U) PICK(C, U, 0) PICK(C, U, 1) PICK(C, U, 2) PICK(C, U, 3)
	PICK4(false, false)
	PICK4(true, false)
	PICK4(true, true)
#undef PICK4
#undef PICK
	return NULL;
}
