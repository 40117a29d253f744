/*
 * ctr10a.hip -- AES-128-CM + HMAC-SHA1 any-class kernels (k_ctr_hmac_any,
 * see k_ctr.h); a TU of its own so the four inlined class bodies build in
 * parallel with the per-class instantiations.
 */
#include "k_ctr.h"
#include "k_ctr_fast.h"

kfn_t sgpu_pick_ctr10_any(bool uni, int prot)
{
	return uni ? (prot ? k_ctr_hmac_any<10, true, true>
			   : k_ctr_hmac_any<10, false, true>)
		   : (prot ? k_ctr_hmac_any<10, true, false>
			   : k_ctr_hmac_any<10, false, false>);
}

/* lean kernels of device-planned single-key batches (k_ctr_fast.h) */
kfn_t sgpu_pick_ctr10_fast(int prot, int refix)
{
	if (refix == 3)         /* multi-session: per-packet keys */
		return k_ctr_refix_list<10, true>;
	if (refix == 2)
		return k_ctr_refix_list<10>;
	if (refix)
		return k_ctr_fast_refix<10>;
	return prot ? k_ctr_fast_any<10, true> : k_ctr_fast_any<10, false>;
}

/* ... their single-key SRTCP form */
kfn_t sgpu_pick_ctr10_fast_rtcp(int prot)
{
	return prot ? k_ctr_fast_rtcp<10, true> : k_ctr_fast_rtcp<10, false>;
}

/* ... and their multi-session (per-lane key) form */
kfn_t sgpu_pick_ctr10_fast_mk(int prot)
{
	return prot ? k_ctr_fast_mk<10, true> : k_ctr_fast_mk<10, false>;
}

unsigned sgpu_ctr_fast_block(int prot)
{
	return CTRF_BLK(prot);
}

unsigned sgpu_ctr_fast_mk_block(void)
{
	return CTRF_MK_BLOCK;
}
