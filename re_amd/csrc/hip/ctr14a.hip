/*
 * ctr14a.hip -- AES-256-CM + HMAC-SHA1 any-class kernels (k_ctr_hmac_any,
 * see k_ctr.h); a TU of its own so the four inlined class bodies build in
 * parallel with the per-class instantiations.
 */
#include "k_ctr.h"
#include "k_ctr_fast.h"

kfn_t sgpu_pick_ctr14_any(bool uni, int prot)
{
	return uni ? (prot ? k_ctr_hmac_any<14, true, true>
			   : k_ctr_hmac_any<14, false, true>)
		   : (prot ? k_ctr_hmac_any<14, true, false>
			   : k_ctr_hmac_any<14, false, false>);
}

/* lean kernels of device-planned single-key batches (k_ctr_fast.h) */
kfn_t sgpu_pick_ctr14_fast(int prot, int refix)
{
	if (refix == 3)         /* multi-session: per-packet keys */
		return k_ctr_refix_list<14, true>;
	if (refix == 2)
		return k_ctr_refix_list<14>;
	if (refix)
		return k_ctr_fast_refix<14>;
	return prot ? k_ctr_fast_any<14, true> : k_ctr_fast_any<14, false>;
}

/* ... their single-key SRTCP form */
kfn_t sgpu_pick_ctr14_fast_rtcp(int prot)
{
	return prot ? k_ctr_fast_rtcp<14, true> : k_ctr_fast_rtcp<14, false>;
}

/* ... and their multi-session (per-lane key) form */
kfn_t sgpu_pick_ctr14_fast_mk(int prot)
{
	return prot ? k_ctr_fast_mk<14, true> : k_ctr_fast_mk<14, false>;
}
