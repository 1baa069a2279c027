// Carry-free column products for Fp (DESIGN.md §4 "Field core").
//
// The product-scanning asm (bls_fp_ps.h) accumulates a column of 32 x 32-bit limb products
// in 96 bits: every v_mad_u64_u32 is followed by a v_addc_co_u32 for its carry.  Here the
// operands are split into 13 digits of 30 bits: a digit product is < 2^60, so a whole column
// of up to 13 products (13 x 2^60 < 2^64) accumulates in one 64-bit register with the mad
// alone.  A column array is normalised to 30-bit digits (a shift, a mask and a 64-bit add per
// column) before the Montgomery reduction adds its 13 m_i p terms to the same columns.  The
// reduction takes 12 digits of 30 bits and a last one of 24 (30 x 12 + 24 = 384), so the
// Montgomery radix stays R = 2^384 and these bodies were drop-in replacements of the asm ones
// (same arguments and results; operands up to 2^384 give a result < 2^384, canonical when the
// contract's bounds hold, as the asm bodies do).  Measured (tools/microbench/fp2_bench.hip,
// DESIGN.md §4 "Field core"): the squaring 16 % fewer cycles than the asm one; the product and
// the lazy Fp2 product's halves (mulw, redc) no faster once the digit conversions are paid --
// and the gfx950 build of these converting bodies disagreed with this header's host build on
// the device self-test (round 6, unresolved), so the library keeps the asm bodies; this header
// stays as the measured experiment (host-tested: tests/test_fp_cols.py).
// LB_HD: device code in the library; plain inline C++ for the host tests
// (tests/native/fp_cols_host.cpp, tests/test_fp_cols.py).
#pragma once
#include <stdint.h>

#ifndef LB_HD
#define LB_HD __device__ __forceinline__
#endif

namespace lb {
namespace cols {

constexpr uint32_t M30 = (1u << 30) - 1;
constexpr uint32_t M24 = (1u << 24) - 1;

struct Digits13 {
  uint32_t d[13];
};
// p (LB_P_LIMBS) as 13 digits of 30 bits
constexpr Digits13 p_digits() {
  constexpr uint32_t P32[12] = LB_P_LIMBS;
  Digits13 r{};
  for (int i = 0; i < 13; i++) {
    const int o = 30 * i, w = o / 32, s = o % 32;
    uint64_t v = (uint64_t)(w < 12 ? P32[w] : 0u) | ((uint64_t)(w + 1 < 12 ? P32[w + 1] : 0u) << 32);
    r.d[i] = (uint32_t)(v >> s) & M30;
  }
  return r;
}
// -p^-1 mod 2^30 (Newton: each step doubles the correct low bits)
constexpr uint32_t p_inv30() {
  constexpr Digits13 P = p_digits();
  uint32_t inv = 1;
  for (int k = 0; k < 6; k++) inv *= 2u - P.d[0] * inv;
  return (0u - inv) & M30;
}
constexpr Digits13 PD = p_digits();
constexpr uint32_t PINV30 = p_inv30();
static_assert(((PD.d[0] * PINV30) & M30) == M30, "-p^-1 mod 2^30");

// 12 limbs -> 13 digits (bits 0 .. 389; the value is < 2^384)
LB_HD void to_d13(const uint32_t* a, uint32_t* d) {
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int o = 30 * i, w = o / 32, s = o % 32;
    const uint32_t lo = w < 12 ? a[w] >> s : 0u;
    const uint32_t hi = (s > 2 && w + 1 < 12) ? a[w + 1] << (32 - s) : 0u;
    d[i] = (lo | hi) & M30;
  }
}
// 24 limbs -> 26 digits
LB_HD void to_d26(const uint32_t* a, uint32_t* d) {
#pragma unroll
  for (int i = 0; i < 26; i++) {
    const int o = 30 * i, w = o / 32, s = o % 32;
    const uint32_t lo = w < 24 ? a[w] >> s : 0u;
    const uint32_t hi = (s > 2 && w + 1 < 24) ? a[w + 1] << (32 - s) : 0u;
    d[i] = (lo | hi) & M30;
  }
}

// c[0 .. 24] = column sums of x y (c[25] = 0)
LB_HD void mul_cols(const uint32_t* x, const uint32_t* y, uint64_t* c) {
#pragma unroll
  for (int k = 0; k < 26; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 13; i++)
#pragma unroll
    for (int j = 0; j < 13; j++) c[i + j] += (uint64_t)x[i] * y[j];
}
// the same for x^2: cross products once with a doubled factor (2 x_i < 2^31; a column holds
// at most 6 of them and one square: < 2^64)
LB_HD void sqr_cols(const uint32_t* x, uint64_t* c) {
#pragma unroll
  for (int k = 0; k < 26; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint32_t x2 = x[i] << 1;
#pragma unroll
    for (int j = i + 1; j < 13; j++) c[i + j] += (uint64_t)x2 * x[j];
    c[2 * i] += (uint64_t)x[i] * x[i];
  }
}
// columns [from, to] -> 30-bit digits, the carries moved up (column to + 1 takes the last)
LB_HD void normalize(uint64_t* c, int from, int to) {
#pragma unroll
  for (int k = from; k <= to; k++) {
    c[k + 1] += c[k] >> 30;
    c[k] &= M30;
  }
}
// Montgomery reduction by 2^384 of the normalised columns: m_i for digits 0 .. 11 (30 bits)
// and digit 12 (its low 24 bits), each adding m_i p to columns i .. i + 12 (at most 13 terms
// of < 2^60 on a < 2^31 digit: < 2^64); then columns 12 .. 24 normalised.
LB_HD void reduce384(uint64_t* c) {
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint32_t m = ((uint32_t)c[i] * PINV30) & (i < 12 ? M30 : M24);
#pragma unroll
    for (int j = 0; j < 13; j++) c[i + j] += (uint64_t)m * PD.d[j];
    if (i < 12) c[i + 1] += c[i] >> 30;  // (digit i is now 0 mod 2^30)
  }
  normalize(c, 12, 24);
}
// bits 384 .. 799 of the normalised columns 12 .. 26 -> 12 limbs + a 13th word, then one
// conditional subtraction of p.  The value is < 2p for operands < 2p (and w < p R), as the
// contract states; callers also pass operands up to 2^384, where it is < 2^384 + p: the 13th
// word keeps such a value whole and the subtraction brings it below 2^384 (the asm bodies do
// the same with their carry-out limb), so the result is always < 2^384 and < p whenever the
// value was < 2p.
LB_HD void out384(uint64_t* c, uint32_t* r) {
  c[26] += c[25] >> 30;  // (columns 25 and 26 normalised too: bits 750 .. 809)
  c[25] &= M30;
  uint32_t t[13];
#pragma unroll
  for (int j = 0; j < 13; j++) {
    const int o = 384 + 32 * j, k = o / 30, s = o % 30;
    uint32_t v = (uint32_t)c[k] >> s;
    if (k + 1 < 27) v |= (uint32_t)c[k + 1] << (30 - s);
    if (60 - s < 32 && k + 2 < 27) v |= (uint32_t)c[k + 2] << (60 - s);
    t[j] = v;
  }
  uint32_t s[13];
  uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 13; j++) {
    constexpr uint32_t P32[12] = LB_P_LIMBS;
    const uint64_t d = (uint64_t)t[j] - (j < 12 ? P32[j] : 0u) - br;
    s[j] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
#pragma unroll
  for (int j = 0; j < 12; j++) r[j] = br ? t[j] : s[j];
}
// the normalised columns 0 .. 25 -> 24 limbs (a value < 2^768)
LB_HD void out768(const uint64_t* c, uint32_t* w) {
#pragma unroll
  for (int j = 0; j < 24; j++) {
    const int o = 32 * j, k = o / 30, s = o % 30;
    uint32_t v = (uint32_t)c[k] >> s;
    v |= (uint32_t)c[k + 1] << (30 - s);
    if (60 - s < 32) v |= (uint32_t)c[k + 2] << (60 - s);
    w[j] = v;
  }
}

// r = a b R^-1 mod p (a, b < p; r < p)
LB_HD void mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t x[13], y[13];
  uint64_t c[27];
  to_d13(a, x);
  to_d13(b, y);
  mul_cols(x, y, c);
  c[26] = 0;
  normalize(c, 0, 24);
  reduce384(c);
  out384(c, r);
}
// r = a^2 R^-1 mod p (a < p)
LB_HD void sqr(uint32_t* r, const uint32_t* a) {
  uint32_t x[13];
  uint64_t c[27];
  to_d13(a, x);
  sqr_cols(x, c);
  c[26] = 0;
  normalize(c, 0, 24);
  reduce384(c);
  out384(c, r);
}
// w = a b (24 limbs, no reduction; a, b < 2^384)
LB_HD void mulw(uint32_t* w, const uint32_t* a, const uint32_t* b) {
  uint32_t x[13], y[13];
  uint64_t c[27];
  to_d13(a, x);
  to_d13(b, y);
  mul_cols(x, y, c);
  c[26] = 0;
  normalize(c, 0, 24);
  out768(c, w);
}
// r = w R^-1 mod p for w < p R (24 limbs; r < p)
LB_HD void redc(uint32_t* r, const uint32_t* w) {
  uint32_t d[26];
  uint64_t c[27];
  to_d26(w, d);
#pragma unroll
  for (int k = 0; k < 26; k++) c[k] = d[k];
  c[26] = 0;
  reduce384(c);
  out384(c, r);
}

}  // namespace cols
}  // namespace lb
