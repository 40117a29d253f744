/*
 * plan_common.h -- device helpers shared by the RTP planners
 * (srtp_kernels.hip k_parse / k_plan_*, and the fused plan + crypto kernel
 * k_ctr_fused.h): the RTP header parse and the index speculation rules.
 */
#pragma once
#include "kern_common.h"

/* one RTP header (rtp_hdr_decode, rtp.c:88-137) from a window of `left`
 * bytes at b (p: its arena offset, for the aligned fast load) */
__device__ __forceinline__ struct sgpu_hdr parse_rtp_hdr(const uint8_t *b,
							 uint32_t p,
							 uint32_t left)
{
	struct sgpu_hdr h;
	h.ssrc = 0; h.seq = 0; h.err_pos = 0; h.hdr_len = 0xffffffffu;
	if (left < 12)
		return h;
	uint32_t b0;
	if (!(p & 3u)) {
		const uint32_t w0 = *(const uint32_t *)b;
		const uint32_t w2 = *(const uint32_t *)(b + 8);
		b0 = w0 & 0xffu;
		h.seq = (uint16_t)((w0 >> 8 & 0xff00u) | (w0 >> 24));
		h.ssrc = __builtin_bswap32(w2);
	}
	else {
		b0 = b[0];
		h.seq = (uint16_t)(b[2] << 8 | b[3]);
		h.ssrc = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 |
			 (uint32_t)b[10] << 8 | b[11];
	}
	const uint32_t cc = b0 & 0x0fu, x = (b0 >> 4) & 1u;
	uint32_t hl = 12;
	if (left - hl < 4 * cc) {
		h.err_pos = (uint16_t)hl;
		return h;
	}
	hl += 4 * cc;
	if (x) {
		if (left - hl < 4) {
			h.err_pos = (uint16_t)hl;
			return h;
		}
		const uint32_t xl = (uint32_t)b[hl + 2] << 8 | b[hl + 3];
		hl += 4;
		if (left - hl < 4 * xl) {
			h.err_pos = (uint16_t)hl;
			return h;
		}
		hl += 4 * xl;
	}
	h.hdr_len = hl;
	return h;
}

/* sgpu_desc() (srtpgpu.h) on the device */
__device__ __forceinline__ uint64_t d_desc(uint64_t ix, uint32_t flags)
{
	return (ix & 0xffffull) | ((uint64_t)(uint32_t)(ix >> 16) << 16) |
	       ((uint64_t)flags << 48);
}

/* srtp_get_index (misc.c:22-41), including the int wrap of roc +- 1 */
__device__ __forceinline__ int32_t plan_v(uint32_t roc, uint32_t s_l,
					  uint32_t seq)
{
	if (s_l < 32768)
		return ((int)seq - (int)s_l > 32768) ? (int32_t)(roc - 1)
						     : (int32_t)roc;
	return ((int)s_l - 32768 > (int)seq) ? (int32_t)(roc + 1)
					     : (int32_t)roc;
}

/* ROC rollover seen by a packet (srtp.c:208-213, 318-321) */
__device__ __forceinline__ bool plan_wrap(uint32_t seq, uint32_t sb)
{
	return (int)seq - (int)sb <= -32768;
}

