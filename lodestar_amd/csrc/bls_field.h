// BLS12-381 field tower for gfx950 (CDNA4): Fp, Fp2, Fp6, Fp12.
//
// Fp elements are 12 x 32-bit limbs (little-endian limb order) in Montgomery
// form, R = 2^384, always fully reduced to [0, p).  One lane owns one field
// element: no cross-lane traffic, integer VALU only (no MFMA -- nothing here is
// a dense contraction).  The 381-bit Montgomery product is CIOS with the
// "no final carry" shortcut (p's top limb < 2^31 - 1), lowered by hipcc to
// 288 v_mad_u64_u32 per product (the roofline unit).
//
// fp_mul / fp_sqr are deliberately __noinline__: every higher-level routine
// (Fp2 ... Miller loop, final exponentiation) calls the same ~10 KB body, which
// keeps the hot kernels inside the instruction cache.
//
// Tower: Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(u+1)), Fp12 = Fp6[w]/(w^2-v),
// the same tower blst uses (the arithmetic behind the reference's
// bls.Signature.verifyMultipleSignatures, packages/beacon-node/src/chain/bls/maybeBatch.ts:19).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_constants.h"

#define LB_DEV __device__ __forceinline__
#define LB_NOINL __device__ __noinline__
// Tower-level routines (Fp6/Fp12 products, G2 group law, Miller loop, final
// exponentiation) are inlined into the kernels by default: kernels then run at
// one wave per SIMD with 256 VGPRs + 256 AGPRs and almost no scratch, instead
// of spilling every call level's live state through the AMDGPU call ABI
// (profiles/pmc_traffic.json: ~106 GB of spill traffic per Miller launch with
// out-of-line tower routines).  Only fp_mul / fp_sqr stay out of line.
#ifndef LB_TOWER_NOINLINE
#define LB_TOWER LB_DEV
#else
#define LB_TOWER LB_NOINL
#endif

namespace lb {

struct fp {
  uint32_t l[12];
};
struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

static constexpr uint32_t P_[12] = LB_P_LIMBS;

// ----------------------------------------------------------------------------
// Fp basics
// ----------------------------------------------------------------------------
LB_DEV void fp_set(fp& r, const uint32_t* c) {
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = c[j];
}
LB_DEV void fp_zero(fp& r) {
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = 0;
}
LB_DEV void fp_one(fp& r) { fp_set(r, LB_ONE); }

LB_DEV bool fp_is_zero(const fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) acc |= a.l[j];
  return acc == 0;
}
LB_DEV bool fp_eq(const fp& a, const fp& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) acc |= a.l[j] ^ b.l[j];
  return acc == 0;
}
LB_DEV void fp_cmov(fp& r, const fp& a, bool c) {
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = c ? a.l[j] : r.l[j];
}

LB_DEV void fp_add(fp& r, const fp& a, const fp& b) {
  uint32_t t[12], s[12];
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = __builtin_addc(a.l[j], b.l[j], c, &c);
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = __builtin_subc(t[j], P_[j], br, &br);
  // a + b < 2p < 2^382: no carry out of limb 11; keep t iff t < p
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = br ? t[j] : s[j];
}

LB_DEV void fp_sub(fp& r, const fp& a, const fp& b) {
  uint32_t t[12];
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = __builtin_subc(a.l[j], b.l[j], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = __builtin_addc(t[j], P_[j] & mask, c, &c);
}

LB_DEV void fp_dbl(fp& r, const fp& a) { fp_add(r, a, a); }

LB_DEV void fp_neg(fp& r, const fp& a) {
  fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}

// Montgomery CIOS, no-final-carry variant (p[11] < 2^31 - 1), a, b < p -> r < p.
LB_DEV void fp_mul_body(fp& r, const fp& a, const fp& b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = b.l[i];
    uint64_t A = (uint64_t)a.l[0] * bi + t[0];
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * LB_P_INV32;
    uint64_t C = (uint64_t)m * P_[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; j++) {
      A = (uint64_t)a.l[j] * bi + (uint64_t)t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * P_[j] + (uint64_t)t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[11] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  uint32_t s[12];
  uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = __builtin_subc(t[j], P_[j], br, &br);
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = br ? t[j] : s[j];
}

// Montgomery squaring: 66 cross products (doubled) + 12 squares + one
// 12x12 reduction = 222 v_mad_u64_u32 instead of 288.
LB_DEV void fp_sqr_body(fp& r, const fp& a) {
  uint32_t t[24];
#pragma unroll
  for (int j = 0; j < 24; j++) t[j] = 0;
  // cross products a_i a_j, i < j
#pragma unroll
  for (int i = 0; i < 11; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 12; j++) {
      c = (uint64_t)a.l[i] * a.l[j] + (uint64_t)t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 12] = (uint32_t)(c >> 32);
  }
  // double
  t[23] = t[22] >> 31;
#pragma unroll
  for (int j = 22; j > 0; j--) t[j] = (t[j] << 1) | (t[j - 1] >> 31);
  t[0] <<= 1;
  // + squares
  {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint64_t sq = (uint64_t)a.l[i] * a.l[i];
      c = (uint64_t)t[2 * i] + (uint32_t)sq + (c >> 32);
      t[2 * i] = (uint32_t)c;
      c = (uint64_t)t[2 * i + 1] + (uint32_t)(sq >> 32) + (c >> 32);
      t[2 * i + 1] = (uint32_t)c;
    }
  }
  // Montgomery reduction of the 768-bit t (t < p^2 < 2^762)
  uint32_t carry_hi = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t m = t[i] * LB_P_INV32;
    uint64_t c = (uint64_t)m * P_[0] + t[i];
#pragma unroll
    for (int j = 1; j < 12; j++) {
      c = (uint64_t)m * P_[j] + (uint64_t)t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    c = (uint64_t)t[i + 12] + (c >> 32) + carry_hi;
    t[i + 12] = (uint32_t)c;
    carry_hi = (uint32_t)(c >> 32);
  }
  uint32_t s[12];
  uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = __builtin_subc(t[12 + j], P_[j], br, &br);
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = br ? t[12 + j] : s[j];
}

#ifdef LB_COUNT_OPS
__device__ unsigned long long g_lb_fpmul_count;
#define LB_COUNT_MUL() atomicAdd(&g_lb_fpmul_count, 1ull)
#else
#define LB_COUNT_MUL() ((void)0)
#endif

// Register calling convention: 24 scalar arguments in, a struct of 12 scalars
// out.  (A byval/by-reference fp argument would be passed through scratch
// memory by the AMDGPU ABI and expose its latency on every call.)
struct fp_ret {
  uint32_t v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11;
};
#define LB_FP_PARAMS(x)                                                                                   \
  uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, uint32_t x##6, \
      uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11
#define LB_FP_PACK(x) {{x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11}}
#define LB_FP_ARGS(f) \
  f.l[0], f.l[1], f.l[2], f.l[3], f.l[4], f.l[5], f.l[6], f.l[7], f.l[8], f.l[9], f.l[10], f.l[11]

LB_NOINL fp_ret fp_mul_r(LB_FP_PARAMS(a), LB_FP_PARAMS(b)) {
  LB_COUNT_MUL();
  const fp A = LB_FP_PACK(a), B = LB_FP_PACK(b);
  fp r;
  fp_mul_body(r, A, B);
  return fp_ret{r.l[0], r.l[1], r.l[2], r.l[3], r.l[4], r.l[5], r.l[6], r.l[7], r.l[8], r.l[9], r.l[10], r.l[11]};
}
LB_NOINL fp_ret fp_sqr_r(LB_FP_PARAMS(a)) {
  LB_COUNT_MUL();
  const fp A = LB_FP_PACK(a);
  fp r;
  fp_sqr_body(r, A);
  return fp_ret{r.l[0], r.l[1], r.l[2], r.l[3], r.l[4], r.l[5], r.l[6], r.l[7], r.l[8], r.l[9], r.l[10], r.l[11]};
}
LB_DEV void fp_unret(fp& r, const fp_ret& v) {
  r.l[0] = v.v0;
  r.l[1] = v.v1;
  r.l[2] = v.v2;
  r.l[3] = v.v3;
  r.l[4] = v.v4;
  r.l[5] = v.v5;
  r.l[6] = v.v6;
  r.l[7] = v.v7;
  r.l[8] = v.v8;
  r.l[9] = v.v9;
  r.l[10] = v.v10;
  r.l[11] = v.v11;
}
LB_DEV void fp_mul(fp& r, const fp& a, const fp& b) { fp_unret(r, fp_mul_r(LB_FP_ARGS(a), LB_FP_ARGS(b))); }
LB_DEV void fp_sqr(fp& r, const fp& a) { fp_unret(r, fp_sqr_r(LB_FP_ARGS(a))); }

LB_DEV void fp_mul_const(fp& r, const fp& a, const uint32_t* c) {
  fp k;
  fp_set(k, c);
  fp_mul(r, a, k);
}

// raw (non-Montgomery, < p) -> Montgomery
LB_DEV void fp_to_mont(fp& r, const fp& a) { fp_mul_const(r, a, LB_R2); }
// Montgomery -> raw
LB_DEV void fp_from_mont(fp& r, const fp& a) {
  fp one_raw;
  fp_zero(one_raw);
  one_raw.l[0] = 1;
  fp_mul(r, a, one_raw);
}

// small constant multiples via additions
LB_DEV void fp_mul3(fp& r, const fp& a) {
  fp t;
  fp_add(t, a, a);
  fp_add(r, t, a);
}

// a^((p-3)/4): the single fixed exponent behind inversion, sqrt and Legendre.
// 4-bit fixed window; the 16-entry table lives in private memory (scratch).
LB_NOINL void fp_pow_p34(fp& r, const fp& a) {
  fp tab[16];
  fp_one(tab[0]);
  tab[1] = a;
  for (int i = 2; i < 16; i++) fp_mul(tab[i], tab[i - 1], a);
  fp acc = tab[LB_EXP_P34[0]];
  for (int k = 1; k < LB_EXP_P34_NIBBLES; k++) {
    fp_sqr(acc, acc);
    fp_sqr(acc, acc);
    fp_sqr(acc, acc);
    fp_sqr(acc, acc);
    const int nib = LB_EXP_P34[k];
    if (nib) fp_mul(acc, acc, tab[nib]);
  }
  r = acc;
}

// a^-1 = a^(p-2) = a * (a^((p-3)/4))^4   (a != 0; inv(0) returns 0)
LB_DEV void fp_inv(fp& r, const fp& a) {
  fp t;
  fp_pow_p34(t, a);
  fp_sqr(t, t);
  fp_sqr(t, t);
  fp_mul(r, t, a);
}

// Legendre-based square test: a^((p-1)/2) = a * (a^((p-3)/4))^2 in {0, 1, -1}
LB_DEV bool fp_is_square(const fp& a) {
  fp t, one;
  fp_pow_p34(t, a);
  fp_sqr(t, t);
  fp_mul(t, t, a);
  fp_one(one);
  return fp_is_zero(a) || fp_eq(t, one);
}

// s = a^((p+1)/4); returns true iff s^2 == a
LB_DEV bool fp_sqrt(fp& r, const fp& a) {
  fp t, s2;
  fp_pow_p34(t, a);
  fp_mul(t, t, a);
  fp_sqr(s2, t);
  r = t;
  return fp_eq(s2, a);
}

// ---- byte conversions (big-endian, 48 bytes) --------------------------------
// raw limbs from 48 big-endian bytes; returns true iff value < p
LB_DEV bool fp_from_be48_raw(fp& r, const uint8_t* b) {
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const uint8_t* q = b + 44 - 4 * j;
    r.l[j] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  uint32_t br = 0, s;
#pragma unroll
  for (int j = 0; j < 12; j++) s = __builtin_subc(r.l[j], P_[j], br, &br);
  (void)s;
  return br != 0;  // borrow => r < p
}
LB_DEV void fp_to_be48_raw(uint8_t* b, const fp& a) {
#pragma unroll
  for (int j = 0; j < 12; j++) {
    uint8_t* q = b + 44 - 4 * j;
    const uint32_t v = a.l[j];
    q[0] = (uint8_t)(v >> 24);
    q[1] = (uint8_t)(v >> 16);
    q[2] = (uint8_t)(v >> 8);
    q[3] = (uint8_t)v;
  }
}
// canonical value comparisons (Montgomery input)
// ZCash sign: canonical(a) > (p-1)/2
LB_DEV bool fp_lex_largest(const fp& a) {
  fp c;
  fp_from_mont(c, a);
  // compare c > (p-1)/2  <=>  (p-1)/2 - c borrows
  static constexpr uint32_t H[12] = LB_HALF_P_RAW_LIMBS;
  uint32_t br = 0, s;
#pragma unroll
  for (int j = 0; j < 12; j++) s = __builtin_subc(H[j], c.l[j], br, &br);
  (void)s;
  return br != 0;
}
LB_DEV uint32_t fp_parity(const fp& a) {
  fp c;
  fp_from_mont(c, a);
  return c.l[0] & 1u;
}

// ----------------------------------------------------------------------------
// Fp2
// ----------------------------------------------------------------------------
LB_DEV void fp2_set(fp2& r, const uint32_t* c) {
  fp_set(r.c0, c);
  fp_set(r.c1, c + 12);
}
LB_DEV void fp2_zero(fp2& r) {
  fp_zero(r.c0);
  fp_zero(r.c1);
}
LB_DEV void fp2_one(fp2& r) {
  fp_one(r.c0);
  fp_zero(r.c1);
}
LB_DEV bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
LB_DEV bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
LB_DEV void fp2_cmov(fp2& r, const fp2& a, bool c) {
  fp_cmov(r.c0, a.c0, c);
  fp_cmov(r.c1, a.c1, c);
}
LB_DEV void fp2_add(fp2& r, const fp2& a, const fp2& b) {
  fp_add(r.c0, a.c0, b.c0);
  fp_add(r.c1, a.c1, b.c1);
}
LB_DEV void fp2_sub(fp2& r, const fp2& a, const fp2& b) {
  fp_sub(r.c0, a.c0, b.c0);
  fp_sub(r.c1, a.c1, b.c1);
}
LB_DEV void fp2_dbl(fp2& r, const fp2& a) {
  fp_add(r.c0, a.c0, a.c0);
  fp_add(r.c1, a.c1, a.c1);
}
LB_DEV void fp2_neg(fp2& r, const fp2& a) {
  fp_neg(r.c0, a.c0);
  fp_neg(r.c1, a.c1);
}
LB_DEV void fp2_conj(fp2& r, const fp2& a) {
  r.c0 = a.c0;
  fp_neg(r.c1, a.c1);
}
// Karatsuba: 3 Fp products
LB_DEV void fp2_mul(fp2& r, const fp2& a, const fp2& b) {
  fp t0, t1, s0, s1;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add(s0, a.c0, a.c1);
  fp_add(s1, b.c0, b.c1);
  fp_mul(s0, s0, s1);
  fp_sub(r.c0, t0, t1);
  fp_sub(s0, s0, t0);
  fp_sub(r.c1, s0, t1);
}
// (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u : 2 Fp products
LB_DEV void fp2_sqr(fp2& r, const fp2& a) {
  fp s, d, m;
  fp_add(s, a.c0, a.c1);
  fp_sub(d, a.c0, a.c1);
  fp_mul(m, a.c0, a.c1);
  fp_mul(r.c0, s, d);
  fp_add(r.c1, m, m);
}
LB_DEV void fp2_mul_fp(fp2& r, const fp2& a, const fp& k) {
  fp_mul(r.c0, a.c0, k);
  fp_mul(r.c1, a.c1, k);
}
LB_DEV void fp2_mul_const(fp2& r, const fp2& a, const uint32_t* c) {
  fp2 k;
  fp2_set(k, c);
  fp2_mul(r, a, k);
}
// multiply by xi = 1 + u
LB_DEV void fp2_mul_xi(fp2& r, const fp2& a) {
  fp t0, t1;
  fp_sub(t0, a.c0, a.c1);
  fp_add(t1, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}
LB_DEV void fp2_mul3(fp2& r, const fp2& a) {
  fp_mul3(r.c0, a.c0);
  fp_mul3(r.c1, a.c1);
}
LB_DEV void fp2_inv(fp2& r, const fp2& a) {
  fp n, t;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  fp_inv(n, n);
  fp_mul(r.c0, a.c0, n);
  fp_mul(t, a.c1, n);
  fp_neg(r.c1, t);
}
// RFC 9380 sgn0 for Fp2
LB_DEV uint32_t fp2_sgn0(const fp2& a) {
  const uint32_t s0 = fp_parity(a.c0);
  const uint32_t z0 = fp_is_zero(a.c0) ? 1u : 0u;
  const uint32_t s1 = fp_parity(a.c1);
  return s0 | (z0 & s1);
}
// ZCash sign flag for Fp2: c1 decides unless zero
LB_DEV bool fp2_lex_largest(const fp2& a) {
  return fp_is_zero(a.c1) ? fp_lex_largest(a.c0) : fp_lex_largest(a.c1);
}

// Square root in Fp2 via the norm (p = 3 mod 4, u^2 = -1).  Two Fp
// exponentiations by (p-3)/4; returns false iff a is not a square.  Which of
// the two roots is produced does not matter: every caller normalises the sign.
//   n = a0^2 + a1^2, s = n^((p+1)/4)     (a square iff s^2 == n)
//   t = (a0 + s)/2, c = t^((p-3)/4)
//   t c^2 == 1  -> x = (t c, a1 c / 2)
//   t c^2 == -1 -> x = (-a1 c / 2, t c)
LB_DEV bool fp2_sqrt(fp2& r, const fp2& a) {
  fp half, c, x0, t, n, s;
  fp_set(half, LB_HALF);
  if (fp_is_zero(a.c1)) {
    // a in Fp: sqrt(a0) or u * sqrt(-a0)
    fp_pow_p34(c, a.c0);
    fp_mul(x0, a.c0, c);  // a0^((p+1)/4)
    fp_mul(t, x0, c);     // a0^((p-1)/2)
    fp one;
    fp_one(one);
    const bool is_qr = fp_eq(t, one) || fp_is_zero(a.c0);
    if (is_qr) {
      r.c0 = x0;
      fp_zero(r.c1);
    } else {
      fp_zero(r.c0);
      r.c1 = x0;  // (a0 c)^2 = -a0
    }
    return true;
  }
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  if (!fp_sqrt(s, n)) return false;
  fp_add(t, a.c0, s);
  fp_mul(t, t, half);
  fp_pow_p34(c, t);
  fp_mul(x0, t, c);  // t^((p+1)/4)
  fp chk;
  fp_sqr(chk, x0);
  fp a1c;
  fp_mul(a1c, a.c1, c);
  fp_mul(a1c, a1c, half);
  if (fp_eq(chk, t)) {
    r.c0 = x0;
    r.c1 = a1c;
  } else {
    fp_neg(r.c0, a1c);
    r.c1 = x0;
  }
  return true;
}

// ----------------------------------------------------------------------------
// Fp6
// ----------------------------------------------------------------------------
LB_DEV void fp6_zero(fp6& r) {
  fp2_zero(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
LB_DEV void fp6_one(fp6& r) {
  fp2_one(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
LB_DEV void fp6_add(fp6& r, const fp6& a, const fp6& b) {
  fp2_add(r.c0, a.c0, b.c0);
  fp2_add(r.c1, a.c1, b.c1);
  fp2_add(r.c2, a.c2, b.c2);
}
LB_DEV void fp6_sub(fp6& r, const fp6& a, const fp6& b) {
  fp2_sub(r.c0, a.c0, b.c0);
  fp2_sub(r.c1, a.c1, b.c1);
  fp2_sub(r.c2, a.c2, b.c2);
}
LB_DEV void fp6_neg(fp6& r, const fp6& a) {
  fp2_neg(r.c0, a.c0);
  fp2_neg(r.c1, a.c1);
  fp2_neg(r.c2, a.c2);
}
// multiply by v: (a0, a1, a2) -> (xi a2, a0, a1)
LB_DEV void fp6_mul_v(fp6& r, const fp6& a) {
  fp2 t;
  fp2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}
// Karatsuba (Devegili et al.): 6 Fp2 products
LB_TOWER void fp6_mul(fp6& r, const fp6& a, const fp6& b) {
  fp2 t0, t1, t2, s, u;
  fp2_mul(t0, a.c0, b.c0);
  fp2_mul(t1, a.c1, b.c1);
  fp2_mul(t2, a.c2, b.c2);
  fp6 o;
  // c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2)
  fp2_add(s, a.c1, a.c2);
  fp2_add(u, b.c1, b.c2);
  fp2_mul(s, s, u);
  fp2_sub(s, s, t1);
  fp2_sub(s, s, t2);
  fp2_mul_xi(s, s);
  fp2_add(o.c0, t0, s);
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  fp2_add(s, a.c0, a.c1);
  fp2_add(u, b.c0, b.c1);
  fp2_mul(s, s, u);
  fp2_sub(s, s, t0);
  fp2_sub(s, s, t1);
  fp2_mul_xi(u, t2);
  fp2_add(o.c1, s, u);
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  fp2_add(s, a.c0, a.c2);
  fp2_add(u, b.c0, b.c2);
  fp2_mul(s, s, u);
  fp2_sub(s, s, t0);
  fp2_sub(s, s, t2);
  fp2_add(o.c2, s, t1);
  r = o;
}
// a * (b0 + b1 v): 5 Fp2 products
LB_DEV void fp6_mul_01(fp6& r, const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0, t1, s, u;
  fp2_mul(t0, a.c0, b0);
  fp2_mul(t1, a.c1, b1);
  fp6 o;
  // c0 = t0 + xi (a2 b1)
  fp2_mul(s, a.c2, b1);
  fp2_mul_xi(s, s);
  fp2_add(o.c0, t0, s);
  // c1 = (a0+a1)(b0+b1) - t0 - t1
  fp2_add(s, a.c0, a.c1);
  fp2_add(u, b0, b1);
  fp2_mul(s, s, u);
  fp2_sub(s, s, t0);
  fp2_sub(o.c1, s, t1);
  // c2 = t1 + a2 b0
  fp2_mul(s, a.c2, b0);
  fp2_add(o.c2, t1, s);
  r = o;
}
// a * (b1 v): 3 Fp2 products
LB_DEV void fp6_mul_1(fp6& r, const fp6& a, const fp2& b1) {
  fp2 t0, t1, t2;
  fp2_mul(t0, a.c2, b1);
  fp2_mul_xi(t0, t0);
  fp2_mul(t1, a.c0, b1);
  fp2_mul(t2, a.c1, b1);
  r.c0 = t0;
  r.c1 = t1;
  r.c2 = t2;
}
LB_DEV void fp6_inv(fp6& r, const fp6& a) {
  fp2 c0, c1, c2, t, s;
  fp2_sqr(c0, a.c0);
  fp2_mul(t, a.c1, a.c2);
  fp2_mul_xi(t, t);
  fp2_sub(c0, c0, t);
  fp2_sqr(c1, a.c2);
  fp2_mul_xi(c1, c1);
  fp2_mul(t, a.c0, a.c1);
  fp2_sub(c1, c1, t);
  fp2_sqr(c2, a.c1);
  fp2_mul(t, a.c0, a.c2);
  fp2_sub(c2, c2, t);
  fp2_mul(t, a.c2, c1);
  fp2_mul(s, a.c1, c2);
  fp2_add(t, t, s);
  fp2_mul_xi(t, t);
  fp2_mul(s, a.c0, c0);
  fp2_add(t, t, s);
  fp2_inv(t, t);
  fp2_mul(r.c0, c0, t);
  fp2_mul(r.c1, c1, t);
  fp2_mul(r.c2, c2, t);
}

// ----------------------------------------------------------------------------
// Fp12
// ----------------------------------------------------------------------------
LB_DEV void fp12_one(fp12& r) {
  fp6_one(r.c0);
  fp6_zero(r.c1);
}
LB_DEV bool fp12_is_one(const fp12& a) {
  fp2 one;
  fp2_one(one);
  return fp2_eq(a.c0.c0, one) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}
LB_DEV void fp12_conj(fp12& r, const fp12& a) {
  r.c0 = a.c0;
  fp6_neg(r.c1, a.c1);
}
// Karatsuba over Fp6: 3 Fp6 products = 18 Fp2 products
LB_TOWER void fp12_mul(fp12& r, const fp12& a, const fp12& b) {
  fp6 t0, t1, s, u;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s, a.c0, a.c1);
  fp6_add(u, b.c0, b.c1);
  fp6_mul(s, s, u);
  fp6_sub(s, s, t0);
  fp6_sub(r.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
// complex squaring: 2 Fp6 products
LB_TOWER void fp12_sqr(fp12& r, const fp12& a) {
  fp6 t, s, u;
  fp6_mul(t, a.c0, a.c1);
  fp6_add(s, a.c0, a.c1);
  fp6_mul_v(u, a.c1);
  fp6_add(u, a.c0, u);
  fp6_mul(s, s, u);
  fp6_sub(s, s, t);
  fp6_mul_v(u, t);
  fp6_sub(r.c0, s, u);
  fp6_add(r.c1, t, t);
}
// Granger-Scott squaring for f in the cyclotomic subgroup (after the easy part
// of the final exponentiation).  View Fp12 = Fp4[w]/(w^3 - s), Fp4 = Fp2[s]/(s^2 - xi):
//   f = A + B w + C w^2,  A = (c0.c0, c1.c1), B = (c1.c0, c0.c2), C = (c0.c1, c1.c2)
//   f^2 = (3A^2 - 2conj(A)) + (3 s C^2 + 2conj(B)) w + (3B^2 - 2conj(C)) w^2
// 9 Fp2 squarings = 18 Fp products instead of 36.
LB_DEV void fp4_sqr(fp2& rx, fp2& ry, const fp2& x, const fp2& y) {
  fp2 t0, t1, t2;
  fp2_sqr(t0, x);
  fp2_sqr(t1, y);
  fp2_add(t2, x, y);
  fp2_sqr(t2, t2);
  fp2_sub(t2, t2, t0);
  fp2_sub(ry, t2, t1);
  fp2_mul_xi(t1, t1);
  fp2_add(rx, t0, t1);
}
// r = 3 a - 2 b   /   r = 3 a + 2 b
LB_DEV void fp2_3a_m2b(fp2& r, const fp2& a, const fp2& b) {
  fp2 t;
  fp2_sub(t, a, b);
  fp2_dbl(t, t);
  fp2_add(r, t, a);
}
LB_DEV void fp2_3a_p2b(fp2& r, const fp2& a, const fp2& b) {
  fp2 t;
  fp2_add(t, a, b);
  fp2_dbl(t, t);
  fp2_add(r, t, a);
}
LB_TOWER void fp12_cyc_sqr(fp12& r, const fp12& f) {
  fp2 Ax, Ay, Bx, By, Cx, Cy;
  fp4_sqr(Ax, Ay, f.c0.c0, f.c1.c1);
  fp4_sqr(Bx, By, f.c1.c0, f.c0.c2);
  fp4_sqr(Cx, Cy, f.c0.c1, f.c1.c2);
  fp12 o;
  fp2_3a_m2b(o.c0.c0, Ax, f.c0.c0);
  fp2_3a_p2b(o.c1.c1, Ay, f.c1.c1);
  fp2 sCx;
  fp2_mul_xi(sCx, Cy);  // s C^2 = xi Cy + Cx s
  fp2_3a_p2b(o.c1.c0, sCx, f.c1.c0);
  fp2_3a_m2b(o.c0.c2, Cx, f.c0.c2);
  fp2_3a_m2b(o.c0.c1, Bx, f.c0.c1);
  fp2_3a_p2b(o.c1.c2, By, f.c1.c2);
  r = o;
}

// f * l, l = (l0 + l1 v) + (l4 v) w  (the Miller-loop line shape): 13 Fp2 products
LB_TOWER void fp12_mul_line(fp12& r, const fp12& f, const fp2& l0, const fp2& l1, const fp2& l4) {
  fp6 t0, t1, s;
  fp6_mul_01(t0, f.c0, l0, l1);
  fp6_mul_1(t1, f.c1, l4);
  fp6_add(s, f.c0, f.c1);
  fp2 m;
  fp2_add(m, l1, l4);
  fp6_mul_01(s, s, l0, m);
  fp6_sub(s, s, t0);
  fp6_sub(r.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
LB_DEV void fp12_inv(fp12& r, const fp12& a) {
  fp6 t, s;
  fp6_mul(t, a.c0, a.c0);
  fp6_mul(s, a.c1, a.c1);
  fp6_mul_v(s, s);
  fp6_sub(t, t, s);
  fp6_inv(t, t);
  fp6_mul(r.c0, a.c0, t);
  fp6_mul(s, a.c1, t);
  fp6_neg(r.c1, s);
}

// Frobenius f -> f^(p^k), k = 1, 2, 3.  Coefficient of w^e (e = 2j + i for
// c_i.c_j) picks up gamma_{k,e} = xi^(e (p^k - 1)/6); odd k conjugates.
LB_DEV void fp12_frob_coeffs(fp12& r, const fp12& a, bool conj, const uint32_t* g1, const uint32_t* g2,
                              const uint32_t* g3, const uint32_t* g4, const uint32_t* g5) {
  fp2 x;
  // e=0: c0.c0
  if (conj) fp2_conj(r.c0.c0, a.c0.c0); else r.c0.c0 = a.c0.c0;
  // e=2: c0.c1 ; e=4: c0.c2 ; e=1: c1.c0 ; e=3: c1.c1 ; e=5: c1.c2
  if (conj) fp2_conj(x, a.c0.c1); else x = a.c0.c1;
  fp2_mul_const(r.c0.c1, x, g2);
  if (conj) fp2_conj(x, a.c0.c2); else x = a.c0.c2;
  fp2_mul_const(r.c0.c2, x, g4);
  if (conj) fp2_conj(x, a.c1.c0); else x = a.c1.c0;
  fp2_mul_const(r.c1.c0, x, g1);
  if (conj) fp2_conj(x, a.c1.c1); else x = a.c1.c1;
  fp2_mul_const(r.c1.c1, x, g3);
  if (conj) fp2_conj(x, a.c1.c2); else x = a.c1.c2;
  fp2_mul_const(r.c1.c2, x, g5);
}
LB_DEV void fp12_frob1(fp12& r, const fp12& a) {
  fp12_frob_coeffs(r, a, true, LB_FROB1_1, LB_FROB1_2, LB_FROB1_3, LB_FROB1_4, LB_FROB1_5);
}
LB_DEV void fp12_frob2(fp12& r, const fp12& a) {
  fp12_frob_coeffs(r, a, false, LB_FROB2_1, LB_FROB2_2, LB_FROB2_3, LB_FROB2_4, LB_FROB2_5);
}
LB_DEV void fp12_frob3(fp12& r, const fp12& a) {
  fp12_frob_coeffs(r, a, true, LB_FROB3_1, LB_FROB3_2, LB_FROB3_3, LB_FROB3_4, LB_FROB3_5);
}

}  // namespace lb
