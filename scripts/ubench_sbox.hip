// ubench_sbox.hip -- AES rounds on the VALU (bitsliced S-box) against the
// T-table rounds the kernels run (LDS lookups).  VERDICT r4 item 3: GCM is
// LDS-bound (k_gcmu LDS floor 0.79-0.83 of the launch, VALU 0.55-0.59,
// profiles/r05_pmc.json), so moving part of its AES onto the VALU pays if
// a VALU round costs less issue than the LDS time it removes.
//
// Two forms of one AES middle round, both on two blocks per lane:
//  * ttab: the kernels' form -- four 256-entry tables, 32 lane replicas
//    (128 KiB, lane l reads replica l & 31: conflict-free ds_read_b32),
//    16 lookups per block-round, round key from SGPRs;
//  * bs: bitsliced -- the two blocks' 32 bytes as 8 bit planes of 32 bits
//    (bit 8c + 2r + k = row r, column c of block k), SubBytes by the
//    Boyar-Peralta circuit (113 XOR/AND/XNOR gates on planes), ShiftRows
//    as byte rotations merged by row masks, MixColumns as
//    x2(a ^ rot1 a) ^ rot1 a ^ rot2(a ^ rot1 a) with 2-bit row rotations
//    inside each byte, AddRoundKey on planes; and bs_nosr: the same
//    without ShiftRows (what a fixsliced schedule would save at best).
// Host: every form checked to give FIPS-197 C.3 (AES-256) on a block,
// then each kernel timed over 256 CUs x 4 SIMDs at 4 waves/SIMD (and 8
// for the LDS-free forms).  Printed: ns per block-round per SIMD, and the
// static VALU / LDS instruction counts of one round (from the ISA,
// scripts/isa_mix.py classes) are what the DESIGN §10 note prices.
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define HD __host__ __device__ __forceinline__
#define ITERS 512

/* ---------------- byte-wise reference (host) ---------------- */
static uint8_t g_sbox[256];

static uint8_t gmul(uint8_t a, uint8_t b)
{
	uint8_t p = 0;
	while (b) {
		if (b & 1)
			p ^= a;
		a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
		b >>= 1;
	}
	return p;
}

static void make_sbox(void)
{
	for (int x = 0; x < 256; x++) {
		uint8_t inv = 0;
		for (int y = 1; y < 256 && x; y++)
			if (gmul((uint8_t)x, (uint8_t)y) == 1)
				inv = (uint8_t)y;
		uint8_t s = inv, r = inv;
		for (int i = 0; i < 4; i++) {
			r = (uint8_t)((r << 1) | (r >> 7));
			s ^= r;
		}
		g_sbox[x] = s ^ 0x63;
	}
}

/* AES-256 key expansion: 60 words, big-endian words of the key bytes */
static void expand256(const uint8_t key[32], uint8_t rk[240])
{
	memcpy(rk, key, 32);
	uint8_t rcon = 1;
	for (int i = 8; i < 60; i++) {
		uint8_t t[4];
		memcpy(t, rk + 4 * (i - 1), 4);
		if (i % 8 == 0) {
			uint8_t u = t[0];
			t[0] = g_sbox[t[1]] ^ rcon;
			t[1] = g_sbox[t[2]];
			t[2] = g_sbox[t[3]];
			t[3] = g_sbox[u];
			rcon = gmul(rcon, 2);
		} else if (i % 8 == 4) {
			for (int j = 0; j < 4; j++)
				t[j] = g_sbox[t[j]];
		}
		for (int j = 0; j < 4; j++)
			rk[4 * i + j] = rk[4 * (i - 8) + j] ^ t[j];
	}
}

/* ---------------- T-table form ---------------- */
/* T_t[x] as a little-endian word of the state column: T0[x] bytes
 * (2s, s, s, 3s) for rows 0..3; T_t = T0 rotated left by 8t bits */
static uint32_t g_t0[256];

static void make_t0(void)
{
	for (int x = 0; x < 256; x++) {
		uint8_t s = g_sbox[x];
		g_t0[x] = (uint32_t)gmul(s, 2) | (uint32_t)s << 8 |
			  (uint32_t)s << 16 | (uint32_t)gmul(s, 3) << 24;
	}
}

HD uint32_t rotl32c(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* one middle round of one block: s = 4 LE column words, T the image
 * (entry (t, x) at word ((t * 256 + x) * 32 + rep)) */
HD void ttab_round(const uint32_t *T, uint32_t rep, uint32_t s[4],
		   const uint32_t k[4])
{
#define L(t, x) T[(((t) * 256u + (x)) << 5) + rep]
	uint32_t o[4];
	for (int c = 0; c < 4; c++)
		o[c] = L(0, s[c] & 255u) ^ L(1, (s[(c + 1) & 3] >> 8) & 255u) ^
		       L(2, (s[(c + 2) & 3] >> 16) & 255u) ^
		       L(3, s[(c + 3) & 3] >> 24) ^ k[c];
#undef L
	s[0] = o[0]; s[1] = o[1]; s[2] = o[2]; s[3] = o[3];
}

/* ---------------- bitsliced form ---------------- */
/* q[b] = bit b of every byte (b = 0 the least significant) */
HD void bs_sbox(uint32_t q[8])
{
	uint32_t x0 = q[7], x1 = q[6], x2 = q[5], x3 = q[4], x4 = q[3],
		 x5 = q[2], x6 = q[1], x7 = q[0];
	uint32_t y1, y2, y3, y4, y5, y6, y7, y8, y9, y10, y11, y12, y13, y14,
		 y15, y16, y17, y18, y19, y20, y21;
	uint32_t t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13,
		 t14, t15, t16, t17, t18, t19, t20, t21, t22, t23, t24, t25,
		 t26, t27, t28, t29, t30, t31, t32, t33, t34, t35, t36, t37,
		 t38, t39, t40, t41, t42, t43, t44, t45, t46, t47, t48, t49,
		 t50, t51, t52, t53, t54, t55, t56, t57, t58, t59, t60, t61,
		 t62, t63, t64, t65, t66, t67;
	uint32_t z0, z1, z2, z3, z4, z5, z6, z7, z8, z9, z10, z11, z12, z13,
		 z14, z15, z16, z17;
	uint32_t s0, s1, s2, s3, s4, s5, s6, s7;
	/* top linear layer */
	y14 = x3 ^ x5; y13 = x0 ^ x6; y9 = x0 ^ x3; y8 = x0 ^ x5;
	t0 = x1 ^ x2; y1 = t0 ^ x7; y4 = y1 ^ x3; y12 = y13 ^ y14;
	y2 = y1 ^ x0; y5 = y1 ^ x6; y3 = y5 ^ y8; t1 = x4 ^ y12;
	y15 = t1 ^ x5; y20 = t1 ^ x1; y6 = y15 ^ x7; y10 = y15 ^ t0;
	y11 = y20 ^ y9; y7 = x7 ^ y11; y17 = y10 ^ y11; y19 = y10 ^ y8;
	y16 = t0 ^ y11; y21 = y13 ^ y16; y18 = x0 ^ y16;
	/* non-linear middle */
	t2 = y12 & y15; t3 = y3 & y6; t4 = t3 ^ t2; t5 = y4 & x7;
	t6 = t5 ^ t2; t7 = y13 & y16; t8 = y5 & y1; t9 = t8 ^ t7;
	t10 = y2 & y7; t11 = t10 ^ t7; t12 = y9 & y11; t13 = y14 & y17;
	t14 = t13 ^ t12; t15 = y8 & y10; t16 = t15 ^ t12; t17 = t4 ^ t14;
	t18 = t6 ^ t16; t19 = t9 ^ t14; t20 = t11 ^ t16; t21 = t17 ^ y20;
	t22 = t18 ^ y19; t23 = t19 ^ y21; t24 = t20 ^ y18;
	t25 = t21 ^ t22; t26 = t21 & t23; t27 = t24 ^ t26; t28 = t25 & t27;
	t29 = t28 ^ t22; t30 = t23 ^ t24; t31 = t22 ^ t26; t32 = t31 & t30;
	t33 = t32 ^ t24; t34 = t23 ^ t33; t35 = t27 ^ t33; t36 = t24 & t35;
	t37 = t36 ^ t34; t38 = t27 ^ t36; t39 = t29 & t38; t40 = t25 ^ t39;
	t41 = t40 ^ t37; t42 = t29 ^ t33; t43 = t29 ^ t40; t44 = t33 ^ t37;
	t45 = t42 ^ t41;
	z0 = t44 & y15; z1 = t37 & y6; z2 = t33 & x7; z3 = t43 & y16;
	z4 = t40 & y1; z5 = t29 & y7; z6 = t42 & y11; z7 = t45 & y17;
	z8 = t41 & y10; z9 = t44 & y12; z10 = t37 & y3; z11 = t33 & y4;
	z12 = t43 & y13; z13 = t40 & y5; z14 = t29 & y2; z15 = t42 & y9;
	z16 = t45 & y14; z17 = t41 & y8;
	/* bottom linear layer */
	t46 = z15 ^ z16; t47 = z10 ^ z11; t48 = z5 ^ z13; t49 = z9 ^ z10;
	t50 = z2 ^ z12; t51 = z2 ^ z5; t52 = z7 ^ z8; t53 = z0 ^ z3;
	t54 = z6 ^ z7; t55 = z16 ^ z17; t56 = z12 ^ t48; t57 = t50 ^ t53;
	t58 = z4 ^ t46; t59 = z3 ^ t54; t60 = t46 ^ t57; t61 = z14 ^ t57;
	t62 = t52 ^ t58; t63 = t49 ^ t58; t64 = z4 ^ t59; t65 = t61 ^ t62;
	t66 = z1 ^ t63; s0 = t59 ^ t63; s6 = t56 ^ ~t62; s7 = t48 ^ ~t60;
	t67 = t64 ^ t65; s3 = t53 ^ t66; s4 = t51 ^ t66; s5 = t47 ^ t65;
	s1 = t64 ^ ~s3; s2 = t55 ^ ~t67;
	q[7] = s0; q[6] = s1; q[5] = s2; q[4] = s3;
	q[3] = s4; q[2] = s5; q[1] = s6; q[0] = s7;
}

HD uint32_t rotr32c(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
HD uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

/* ShiftRows: row r of column c takes column c + r's: the word rotated
 * right by 8r bits, merged by the row masks */
HD uint32_t bs_sr1(uint32_t x)
{
	uint32_t y = bfi(0x0C0C0C0Cu, rotr32c(x, 8), x);
	y = bfi(0x30303030u, rotr32c(x, 16), y);
	return bfi(0xC0C0C0C0u, rotr32c(x, 24), y);
}

/* row rotations inside a column (byte): rot1(x) row r <- row r + 1 */
HD uint32_t bs_rot1(uint32_t x)
{
	return ((x >> 2) & 0x3F3F3F3Fu) | ((x << 6) & 0xC0C0C0C0u);
}

HD uint32_t bs_rot2(uint32_t x)
{
	return ((x >> 4) & 0x0F0F0F0Fu) | ((x << 4) & 0xF0F0F0F0u);
}

HD void bs_mix(uint32_t q[8])
{
	uint32_t r1[8], t[8];
	for (int b = 0; b < 8; b++) {
		r1[b] = bs_rot1(q[b]);
		t[b] = q[b] ^ r1[b];
	}
	/* x2(t): bit b <- bit b - 1, bit 0 <- bit 7, bits 1, 3, 4 ^= bit 7 */
	const uint32_t h = t[7];
	uint32_t x2[8] = {h, t[0] ^ h, t[1], t[2] ^ h, t[3] ^ h, t[4], t[5],
			  t[6]};
	for (int b = 0; b < 8; b++)
		q[b] = x2[b] ^ r1[b] ^ bs_rot2(t[b]);
}

template <bool SR>
HD void bs_round(uint32_t q[8], const uint32_t k[8])
{
	bs_sbox(q);
	if (SR)
		for (int b = 0; b < 8; b++)
			q[b] = bs_sr1(q[b]);
	bs_mix(q);
	for (int b = 0; b < 8; b++)
		q[b] ^= k[b];
}

/* host: two blocks (16 bytes each, AES byte order) <-> planes */
static void to_planes(const uint8_t blk[2][16], uint32_t q[8])
{
	memset(q, 0, 32);
	for (int k = 0; k < 2; k++)
		for (int i = 0; i < 16; i++) {
			const int c = i / 4, r = i % 4, p = 8 * c + 2 * r + k;
			for (int b = 0; b < 8; b++)
				q[b] |= (uint32_t)((blk[k][i] >> b) & 1) << p;
		}
}

static void from_planes(const uint32_t q[8], uint8_t blk[2][16])
{
	for (int k = 0; k < 2; k++)
		for (int i = 0; i < 16; i++) {
			const int c = i / 4, r = i % 4, p = 8 * c + 2 * r + k;
			uint8_t v = 0;
			for (int b = 0; b < 8; b++)
				v |= (uint8_t)(((q[b] >> p) & 1) << b);
			blk[k][i] = v;
		}
}

/* ---------------- kernels: ITERS middle rounds ---------------- */
__global__ void __launch_bounds__(1024)
k_ttab(const uint32_t *t0, const uint32_t *rkw, uint32_t *out)
{
	extern __shared__ uint32_t T[];         /* 4 x 256 x 32 words */
	for (uint32_t i = threadIdx.x; i < 4u * 256u * 32u; i += blockDim.x) {
		const uint32_t t = i >> 13, x = (i >> 5) & 255u;
		T[i] = rotl32c(t0[x], 8 * (int)t);
	}
	__syncthreads();
	const uint32_t rep = threadIdx.x & 31u;
	const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t a[4] = {g, g * 3u, g ^ 0x55u, ~g}, b[4] = {g + 1, g * 5u, 7u, g};
#pragma unroll 1
	for (int it = 0; it < ITERS; it++) {
		const uint32_t *k = rkw + 4 * (it & 7);
		uint32_t ks[4];
		for (int c = 0; c < 4; c++)
			ks[c] = (uint32_t)__builtin_amdgcn_readfirstlane(k[c]);
		ttab_round(T, rep, a, ks);
		ttab_round(T, rep, b, ks);
	}
	out[g] = a[0] ^ a[1] ^ a[2] ^ a[3] ^ b[0] ^ b[1] ^ b[2] ^ b[3];
}

template <bool SR>
__global__ void __launch_bounds__(1024)
k_bs(const uint32_t *rkq, uint32_t *out)
{
	const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t q[8];
	for (int b = 0; b < 8; b++)
		q[b] = g * (2654435761u + b) ^ (b * 0x9e3779b9u);
#pragma unroll 1
	for (int it = 0; it < ITERS; it++) {
		const uint32_t *k = rkq + 8 * (it & 7);
		uint32_t ks[8];
		for (int b = 0; b < 8; b++)
			ks[b] = (uint32_t)__builtin_amdgcn_readfirstlane(k[b]);
		bs_round<SR>(q, ks);
	}
	uint32_t r = 0;
	for (int b = 0; b < 8; b++)
		r ^= q[b];
	out[g] = r;
}

/* ---------------- host ---------------- */
static int check_forms(void)
{
	/* FIPS-197 C.3 */
	uint8_t key[32], pt[16], rk[240];
	static const uint8_t ct_ref[16] = {0x8e, 0xa2, 0xb7, 0xca, 0x51, 0x67,
		0x45, 0xbf, 0xea, 0xfc, 0x49, 0x90, 0x4b, 0x49, 0x60, 0x89};
	for (int i = 0; i < 32; i++)
		key[i] = (uint8_t)i;
	for (int i = 0; i < 16; i++)
		pt[i] = (uint8_t)(0x11 * i);
	expand256(key, rk);
	/* T-table form, one replica */
	static uint32_t T[4 * 256 * 32];
	for (int i = 0; i < 4 * 256 * 32; i++)
		T[i] = rotl32c(g_t0[(i >> 5) & 255], 8 * (i >> 13));
	uint32_t s[4];
	for (int c = 0; c < 4; c++) {
		uint32_t w = 0, kw = 0;
		for (int r = 0; r < 4; r++) {
			w |= (uint32_t)pt[4 * c + r] << 8 * r;
			kw |= (uint32_t)rk[4 * c + r] << 8 * r;
		}
		s[c] = w ^ kw;
	}
	for (int rd = 1; rd < 14; rd++) {
		uint32_t k[4];
		for (int c = 0; c < 4; c++) {
			k[c] = 0;
			for (int r = 0; r < 4; r++)
				k[c] |= (uint32_t)rk[16 * rd + 4 * c + r] << 8 * r;
		}
		ttab_round(T, 0, s, k);
	}
	uint8_t ct_t[16];
	for (int c = 0; c < 4; c++)      /* final round: S-box + ShiftRows */
		for (int r = 0; r < 4; r++)
			ct_t[4 * c + r] = g_sbox[(s[(c + r) & 3] >> 8 * r) & 255] ^
					  rk[224 + 4 * c + r];
	/* bitsliced form: block 0 = pt, block 1 = pt (both must match) */
	uint8_t blk[2][16], kb[2][16];
	uint32_t q[8], kq[8];
	for (int k = 0; k < 2; k++)
		for (int i = 0; i < 16; i++)
			blk[k][i] = pt[i] ^ rk[i];
	to_planes(blk, q);
	for (int rd = 1; rd < 14; rd++) {
		for (int k = 0; k < 2; k++)
			memcpy(kb[k], rk + 16 * rd, 16);
		to_planes(kb, kq);
		bs_round<true>(q, kq);
	}
	bs_sbox(q);
	for (int b = 0; b < 8; b++)
		q[b] = bs_sr1(q[b]);
	for (int k = 0; k < 2; k++)
		memcpy(kb[k], rk + 224, 16);
	to_planes(kb, kq);
	for (int b = 0; b < 8; b++)
		q[b] ^= kq[b];
	uint8_t out[2][16];
	from_planes(q, out);
	/* S-box circuit over all bytes */
	int sbox_bad = 0;
	for (int x = 0; x < 256; x += 32) {
		uint8_t v[2][16];
		for (int i = 0; i < 32; i++)
			v[i / 16][i % 16] = (uint8_t)(x + i);
		to_planes(v, q);
		bs_sbox(q);
		from_planes(q, v);
		for (int i = 0; i < 32; i++)
			sbox_bad += v[i / 16][i % 16] != g_sbox[x + i];
	}
	const int ok_t = !memcmp(ct_t, ct_ref, 16);
	const int ok_b = !memcmp(out[0], ct_ref, 16) &&
			 !memcmp(out[1], ct_ref, 16);
	printf("check: sbox circuit %s, ttab AES-256 %s, bitsliced AES-256 %s\n",
	       sbox_bad ? "WRONG" : "ok", ok_t ? "ok" : "WRONG",
	       ok_b ? "ok" : "WRONG");
	return !sbox_bad && ok_t && ok_b;
}

int main(void)
{
	make_sbox();
	make_t0();
	if (!check_forms())
		return 1;
	int ncu = 0;
	hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
	uint32_t *t0_d, *rk_d, *out_d;
	uint32_t rk_h[64];
	for (int i = 0; i < 64; i++)
		rk_h[i] = 0x9e3779b9u * (i + 1);
	hipMalloc(&t0_d, 1024);
	hipMalloc(&rk_d, sizeof(rk_h));
	const int maxg = ncu * 2;
	hipMalloc(&out_d, (size_t)maxg * 1024 * 4);
	hipMemcpy(t0_d, g_t0, 1024, hipMemcpyHostToDevice);
	hipMemcpy(rk_d, rk_h, sizeof(rk_h), hipMemcpyHostToDevice);
	hipFuncSetAttribute((const void *)k_ttab,
			    hipFuncAttributeMaxDynamicSharedMemorySize,
			    4 * 256 * 32 * 4);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	/* grid: 1 workgroup of 1024 per CU = 4 waves/SIMD, or 2 (bs only) */
	struct { const char *name; int form; int wps; } runs[] = {
		{"ttab (LDS T-tables, 2 blocks/lane)", 0, 4},
		{"bs (bitsliced, ShiftRows, 2 blocks/lane)", 1, 4},
		{"bs (bitsliced, ShiftRows, 2 blocks/lane)", 1, 8},
		{"bs_nosr (bitsliced, no ShiftRows)", 2, 4},
		{"bs_nosr (bitsliced, no ShiftRows)", 2, 8},
	};
	for (auto &r : runs) {
		const int grid = ncu * r.wps / 4;
		float best = 1e30f;
		for (int rep = 0; rep < 5; rep++) {
			hipEventRecord(e0, 0);
			if (r.form == 0)
				hipLaunchKernelGGL(k_ttab, dim3(grid), dim3(1024),
						   4 * 256 * 32 * 4, 0, t0_d, rk_d,
						   out_d);
			else if (r.form == 1)
				hipLaunchKernelGGL(k_bs<true>, dim3(grid),
						   dim3(1024), 0, 0, rk_d, out_d);
			else
				hipLaunchKernelGGL(k_bs<false>, dim3(grid),
						   dim3(1024), 0, 0, rk_d, out_d);
			hipEventRecord(e1, 0);
			hipEventSynchronize(e1);
			float ms;
			hipEventElapsedTime(&ms, e0, e1);
			if (rep && ms < best)
				best = ms;
		}
		/* block-rounds: 2 per lane per iteration */
		const double br = (double)grid * 1024 * ITERS * 2;
		printf("%-44s %d waves/SIMD: %.3f ms, %.3f ns per block-round per "
		       "CU, %.1f G block-rounds/s\n", r.name, r.wps, best,
		       best * 1e6 / (br / ncu), br / best / 1e6);
	}
	return 0;
}
