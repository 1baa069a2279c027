/*
 * bls_oracle.c -- CPU restatement of the BLS12-381 signature-set verification
 * path, in plain C (6 x 64-bit limbs, Montgomery form, unsigned __int128).
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/ (checked against the pinned Python
 * oracle oracle/bls12_381.py on the golden vectors), by bench.py's
 * cpu_baseline leg (multithreaded, kind "port") and by nothing else; the
 * product path (lodestar_amd/) never loads it.
 *
 * What it restates (the reference's arithmetic is the un-vendored
 * @chainsafe/blst@0.2.10, yarn.lock:304-310; verdict rules are the
 * reference's own TypeScript):
 *   lbo_verify_requests  <- verifySignatureSetsMaybeBatch per request
 *                           (packages/beacon-node/src/chain/bls/maybeBatch.ts:16-46)
 *                           with the main-thread pubkey aggregation
 *                           (chain/bls/utils.ts:6-21) and the empty-aggregate
 *                           rejection (chain/bls/multithread/index.ts:403-409);
 *                           the same request/set semantics as lb_verify_requests
 *                           (include/lodestar_bls.h) and oracle/batch.py.
 *   batch randomness     <- blst mul_n_aggregate with 64-bit scalars; here the
 *                           deterministic DRBG of oracle/batch.py: w = LE64(
 *                           SHA-256(seed || LE32(i))[0..8]) (0 -> 1),
 *                           r = (w mod 2^32) + (w >> 32) lambda, lambda = -x^2,
 *                           applied with the GLV endomorphisms.
 *   hash_to_G2           <- RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_, DST
 *                           BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_
 *   (de)serialisation    <- ZCash encoding as in oracle/bls12_381.py g1/g2_from_bytes
 *   pairing              <- optimal ate, f^(3 (p^12-1)/r) (same value the device's
 *                           lb_pairing returns)
 *
 * Constants come from oracle/gen_c_consts.py (generated from the Python oracle).
 * Build: oracle/build_c.py (gcc -O3 -shared -fPIC -pthread).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct {
  uint64_t l[6];
} fp;
typedef struct {
  fp c0, c1;
} fp2;
typedef struct {
  fp2 c0, c1, c2;
} fp6;
typedef struct {
  fp6 c0, c1;
} fp12;

#include "bls_oracle_consts.h"

/* ---------------------------------------------------------------- Fp ---- */
static inline int fp_geq_p(const uint64_t* t) {
  for (int i = 5; i >= 0; i--) {
    if (t[i] > C_P_RAW[i]) return 1;
    if (t[i] < C_P_RAW[i]) return 0;
  }
  return 1;
}
static inline void sub_p(uint64_t* t) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)t[i] - C_P_RAW[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}
/* CIOS Montgomery product, fully unrolled on scalar locals */
#define MAC(t, x, y, c)                       \
  do {                                        \
    u128 s_ = (u128)(x) * (y) + (t) + (c);    \
    (t) = (uint64_t)s_;                       \
    (c) = (uint64_t)(s_ >> 64);               \
  } while (0)
#define RED(tlo, thi, x, y, c)                \
  do {                                        \
    u128 s_ = (u128)(x) * (y) + (thi) + (c);  \
    (tlo) = (uint64_t)s_;                     \
    (c) = (uint64_t)(s_ >> 64);               \
  } while (0)
#define ROUND(bi)                                                                    \
  do {                                                                               \
    uint64_t c = 0, m;                                                               \
    MAC(t0, a0, bi, c);                                                              \
    MAC(t1, a1, bi, c);                                                              \
    MAC(t2, a2, bi, c);                                                              \
    MAC(t3, a3, bi, c);                                                              \
    MAC(t4, a4, bi, c);                                                              \
    MAC(t5, a5, bi, c);                                                              \
    t6 += c;                                                                         \
    m = t0 * C_P_INV;                                                                \
    c = (uint64_t)(((u128)m * C_P_RAW[0] + t0) >> 64);                               \
    RED(t0, t1, m, C_P_RAW[1], c);                                                   \
    RED(t1, t2, m, C_P_RAW[2], c);                                                   \
    RED(t2, t3, m, C_P_RAW[3], c);                                                   \
    RED(t3, t4, m, C_P_RAW[4], c);                                                   \
    RED(t4, t5, m, C_P_RAW[5], c);                                                   \
    {                                                                                \
      u128 s_ = (u128)t6 + c;                                                        \
      t5 = (uint64_t)s_;                                                             \
      t6 = (uint64_t)(s_ >> 64);                                                     \
    }                                                                                \
  } while (0)
static void fp_mul(fp* r, const fp* A, const fp* B) {
  const uint64_t a0 = A->l[0], a1 = A->l[1], a2 = A->l[2], a3 = A->l[3], a4 = A->l[4], a5 = A->l[5];
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0, t6 = 0;
  ROUND(B->l[0]);
  ROUND(B->l[1]);
  ROUND(B->l[2]);
  ROUND(B->l[3]);
  ROUND(B->l[4]);
  ROUND(B->l[5]);
  uint64_t t[6] = {t0, t1, t2, t3, t4, t5};
  if (t6 || fp_geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}
static inline void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_add(fp* r, const fp* a, const fp* b) {
  uint64_t t[6], c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    t[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || fp_geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}
static void fp_sub(fp* r, const fp* a, const fp* b) {
  uint64_t t[6], br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)t[i] + C_P_RAW[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r->l, t, 48);
}
static inline int fp_is_zero(const fp* a) {
  uint64_t acc = 0;
  for (int i = 0; i < 6; i++) acc |= a->l[i];
  return acc == 0;
}
static inline int fp_eq(const fp* a, const fp* b) { return memcmp(a->l, b->l, 48) == 0; }
static inline void fp_zero(fp* r) { memset(r, 0, sizeof(*r)); }
static inline void fp_neg(fp* r, const fp* a) {
  fp z;
  fp_zero(&z);
  fp_sub(r, &z, a);
}
static void fp_pow(fp* r, const fp* a, const uint64_t* e, int nl) {
  fp acc = C_ONE;
  for (int i = nl * 64 - 1; i >= 0; i--) {
    fp_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fp_mul(&acc, &acc, a);
  }
  *r = acc;
}
static void fp_from_raw(fp* r, const uint64_t* raw) {
  fp t, r2;
  memcpy(t.l, raw, 48);
  memcpy(r2.l, C_R2_RAW, 48);
  fp_mul(r, &t, &r2);
}
static void fp_to_raw(uint64_t* raw, const fp* a) {
  fp one_raw, t;
  fp_zero(&one_raw);
  one_raw.l[0] = 1;
  fp_mul(&t, a, &one_raw);
  memcpy(raw, t.l, 48);
}
/* a^((p-3)/4) */
static void fp_pow_p34(fp* r, const fp* a) { fp_pow(r, a, C_EXP_P34, 6); }
static void fp_inv(fp* r, const fp* a) {
  fp t;
  fp_pow_p34(&t, a); /* a^((p-3)/4) */
  fp_sqr(&t, &t);
  fp_sqr(&t, &t); /* a^(p-3) */
  fp_mul(r, &t, a);
}
/* returns 1 and r = sqrt(a) iff a is a square */
static int fp_sqrt(fp* r, const fp* a) {
  fp t, s2;
  fp_pow_p34(&t, a);
  fp_mul(&t, &t, a); /* a^((p+1)/4) */
  fp_sqr(&s2, &t);
  *r = t;
  return fp_eq(&s2, a);
}
/* big-endian 48 bytes -> Montgomery; returns 0 if value >= p */
static int fp_from_be48(fp* r, const uint8_t* b) {
  uint64_t raw[6];
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | b[(5 - i) * 8 + k];
    raw[i] = v;
  }
  if (fp_geq_p(raw)) return 0;
  fp_from_raw(r, raw);
  return 1;
}
static void fp_to_be48(uint8_t* b, const fp* a) {
  uint64_t raw[6];
  fp_to_raw(raw, a);
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[(5 - i) * 8 + k] = (uint8_t)(raw[i] >> (56 - 8 * k));
}
static int fp_lex_largest(const fp* a) {
  uint64_t raw[6];
  fp_to_raw(raw, a);
  for (int i = 5; i >= 0; i--) {
    if (raw[i] > C_HALF_P_RAW[i]) return 1;
    if (raw[i] < C_HALF_P_RAW[i]) return 0;
  }
  return 0;
}
static int fp_parity(const fp* a) {
  uint64_t raw[6];
  fp_to_raw(raw, a);
  return (int)(raw[0] & 1);
}

/* --------------------------------------------------------------- Fp2 ---- */
static inline void fp2_add(fp2* r, const fp2* a, const fp2* b) {
  fp_add(&r->c0, &a->c0, &b->c0);
  fp_add(&r->c1, &a->c1, &b->c1);
}
static inline void fp2_sub(fp2* r, const fp2* a, const fp2* b) {
  fp_sub(&r->c0, &a->c0, &b->c0);
  fp_sub(&r->c1, &a->c1, &b->c1);
}
static inline void fp2_neg(fp2* r, const fp2* a) {
  fp_neg(&r->c0, &a->c0);
  fp_neg(&r->c1, &a->c1);
}
static inline void fp2_conj(fp2* r, const fp2* a) {
  r->c0 = a->c0;
  fp_neg(&r->c1, &a->c1);
}
static inline void fp2_dbl(fp2* r, const fp2* a) { fp2_add(r, a, a); }
static void fp2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, s0, s1;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&s0, &s0, &s1);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&s0, &s0, &t0);
  fp_sub(&r->c1, &s0, &t1);
}
static void fp2_sqr(fp2* r, const fp2* a) {
  fp s, d, m;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&m, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_add(&r->c1, &m, &m);
}
static void fp2_mul_fp(fp2* r, const fp2* a, const fp* k) {
  fp_mul(&r->c0, &a->c0, k);
  fp_mul(&r->c1, &a->c1, k);
}
static void fp2_mul_xi(fp2* r, const fp2* a) {
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static inline int fp2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static inline int fp2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static inline void fp2_zero(fp2* r) { memset(r, 0, sizeof(*r)); }
static inline void fp2_one(fp2* r) {
  r->c0 = C_ONE;
  fp_zero(&r->c1);
}
static void fp2_inv(fp2* r, const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&n, &n);
  fp_mul(&r->c0, &a->c0, &n);
  fp_mul(&t, &a->c1, &n);
  fp_neg(&r->c1, &t);
}
static void fp2_mul3(fp2* r, const fp2* a) {
  fp2 t;
  fp2_add(&t, a, a);
  fp2_add(r, &t, a);
}
/* square root in Fp2 via the norm (p = 3 mod 4, u^2 = -1); 0 if none */
static int fp2_sqrt(fp2* r, const fp2* a) {
  if (fp_is_zero(&a->c1)) {
    fp s, na;
    if (fp_sqrt(&s, &a->c0)) {
      r->c0 = s;
      fp_zero(&r->c1);
      return 1;
    }
    fp_neg(&na, &a->c0);
    if (!fp_sqrt(&s, &na)) return 0;
    fp_zero(&r->c0);
    r->c1 = s;
    return 1;
  }
  fp n, t, s, x0, c, chk, a1c;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  if (!fp_sqrt(&s, &n)) return 0;
  fp_add(&t, &a->c0, &s);
  fp_mul(&t, &t, &C_HALF);
  fp_pow_p34(&c, &t);
  fp_mul(&x0, &t, &c);
  fp_sqr(&chk, &x0);
  fp_mul(&a1c, &a->c1, &c);
  fp_mul(&a1c, &a1c, &C_HALF);
  if (fp_eq(&chk, &t)) {
    r->c0 = x0;
    r->c1 = a1c;
  } else {
    fp_neg(&r->c0, &a1c);
    r->c1 = x0;
  }
  fp2 sq;
  fp2_sqr(&sq, r);
  return fp2_eq(&sq, a);
}
static int fp2_sgn0(const fp2* a) {
  int s0 = fp_parity(&a->c0), z0 = fp_is_zero(&a->c0), s1 = fp_parity(&a->c1);
  return s0 | (z0 & s1);
}
static int fp2_lex_largest(const fp2* a) {
  return fp_is_zero(&a->c1) ? fp_lex_largest(&a->c0) : fp_lex_largest(&a->c1);
}

/* ------------------------------------------------------- Fp6 / Fp12 ---- */
static void fp6_add(fp6* r, const fp6* a, const fp6* b) {
  fp2_add(&r->c0, &a->c0, &b->c0);
  fp2_add(&r->c1, &a->c1, &b->c1);
  fp2_add(&r->c2, &a->c2, &b->c2);
}
static void fp6_sub(fp6* r, const fp6* a, const fp6* b) {
  fp2_sub(&r->c0, &a->c0, &b->c0);
  fp2_sub(&r->c1, &a->c1, &b->c1);
  fp2_sub(&r->c2, &a->c2, &b->c2);
}
static void fp6_neg(fp6* r, const fp6* a) {
  fp2_neg(&r->c0, &a->c0);
  fp2_neg(&r->c1, &a->c1);
  fp2_neg(&r->c2, &a->c2);
}
static void fp6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  fp2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void fp6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 t0, t1, t2, s, u;
  fp6 o;
  fp2_mul(&t0, &a->c0, &b->c0);
  fp2_mul(&t1, &a->c1, &b->c1);
  fp2_mul(&t2, &a->c2, &b->c2);
  fp2_add(&s, &a->c1, &a->c2);
  fp2_add(&u, &b->c1, &b->c2);
  fp2_mul(&s, &s, &u);
  fp2_sub(&s, &s, &t1);
  fp2_sub(&s, &s, &t2);
  fp2_mul_xi(&s, &s);
  fp2_add(&o.c0, &t0, &s);
  fp2_add(&s, &a->c0, &a->c1);
  fp2_add(&u, &b->c0, &b->c1);
  fp2_mul(&s, &s, &u);
  fp2_sub(&s, &s, &t0);
  fp2_sub(&s, &s, &t1);
  fp2_mul_xi(&u, &t2);
  fp2_add(&o.c1, &s, &u);
  fp2_add(&s, &a->c0, &a->c2);
  fp2_add(&u, &b->c0, &b->c2);
  fp2_mul(&s, &s, &u);
  fp2_sub(&s, &s, &t0);
  fp2_sub(&s, &s, &t2);
  fp2_add(&o.c2, &s, &t1);
  *r = o;
}
static void fp6_inv(fp6* r, const fp6* a) {
  fp2 c0, c1, c2, t, s;
  fp2_sqr(&c0, &a->c0);
  fp2_mul(&t, &a->c1, &a->c2);
  fp2_mul_xi(&t, &t);
  fp2_sub(&c0, &c0, &t);
  fp2_sqr(&c1, &a->c2);
  fp2_mul_xi(&c1, &c1);
  fp2_mul(&t, &a->c0, &a->c1);
  fp2_sub(&c1, &c1, &t);
  fp2_sqr(&c2, &a->c1);
  fp2_mul(&t, &a->c0, &a->c2);
  fp2_sub(&c2, &c2, &t);
  fp2_mul(&t, &a->c2, &c1);
  fp2_mul(&s, &a->c1, &c2);
  fp2_add(&t, &t, &s);
  fp2_mul_xi(&t, &t);
  fp2_mul(&s, &a->c0, &c0);
  fp2_add(&t, &t, &s);
  fp2_inv(&t, &t);
  fp2_mul(&r->c0, &c0, &t);
  fp2_mul(&r->c1, &c1, &t);
  fp2_mul(&r->c2, &c2, &t);
}
static void fp12_one(fp12* r) {
  memset(r, 0, sizeof(*r));
  r->c0.c0.c0 = C_ONE;
}
static int fp12_is_one(const fp12* a) {
  fp12 one;
  fp12_one(&one);
  return memcmp(a, &one, sizeof(one)) == 0;
}
static void fp12_conj(fp12* r, const fp12* a) {
  r->c0 = a->c0;
  fp6_neg(&r->c1, &a->c1);
}
static void fp12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s, u;
  fp6_mul(&t0, &a->c0, &b->c0);
  fp6_mul(&t1, &a->c1, &b->c1);
  fp6_add(&s, &a->c0, &a->c1);
  fp6_add(&u, &b->c0, &b->c1);
  fp6_mul(&s, &s, &u);
  fp6_sub(&s, &s, &t0);
  fp6_sub(&r->c1, &s, &t1);
  fp6_mul_v(&t1, &t1);
  fp6_add(&r->c0, &t0, &t1);
}
static void fp12_sqr(fp12* r, const fp12* a) {
  fp6 t, s, u;
  fp6_mul(&t, &a->c0, &a->c1);
  fp6_add(&s, &a->c0, &a->c1);
  fp6_mul_v(&u, &a->c1);
  fp6_add(&u, &a->c0, &u);
  fp6_mul(&s, &s, &u);
  fp6_sub(&s, &s, &t);
  fp6_mul_v(&u, &t);
  fp6_sub(&r->c0, &s, &u);
  fp6_add(&r->c1, &t, &t);
}
static void fp12_inv(fp12* r, const fp12* a) {
  fp6 t, s;
  fp6_mul(&t, &a->c0, &a->c0);
  fp6_mul(&s, &a->c1, &a->c1);
  fp6_mul_v(&s, &s);
  fp6_sub(&t, &t, &s);
  fp6_inv(&t, &t);
  fp6_mul(&r->c0, &a->c0, &t);
  fp6_mul(&s, &a->c1, &t);
  fp6_neg(&r->c1, &s);
}
/* f^(p^k), k = 1, 2, 3: coefficient of w^e (c_i.c_j, e = 2j + i) times xi^(e (p^k-1)/6) */
static void fp12_frob(fp12* r, const fp12* a, int k) {
  const fp2* g = k == 1 ? C_FROB1 : k == 2 ? C_FROB2 : C_FROB3;
  const fp2* src[6] = {&a->c0.c0, &a->c1.c0, &a->c0.c1, &a->c1.c1, &a->c0.c2, &a->c1.c2}; /* by e */
  fp2* dst[6] = {&r->c0.c0, &r->c1.c0, &r->c0.c1, &r->c1.c1, &r->c0.c2, &r->c1.c2};
  fp2 x[6];
  for (int e = 0; e < 6; e++) {
    if (k & 1)
      fp2_conj(&x[e], src[e]);
    else
      x[e] = *src[e];
  }
  for (int e = 0; e < 6; e++) {
    if (e == 0)
      *dst[e] = x[e];
    else
      fp2_mul(dst[e], &x[e], &g[e]);
  }
}
/* Granger-Scott squaring in the cyclotomic subgroup */
static void fp4_sqr(fp2* rx, fp2* ry, const fp2* x, const fp2* y) {
  fp2 t0, t1, t2;
  fp2_sqr(&t0, x);
  fp2_sqr(&t1, y);
  fp2_add(&t2, x, y);
  fp2_sqr(&t2, &t2);
  fp2_sub(&t2, &t2, &t0);
  fp2_sub(ry, &t2, &t1);
  fp2_mul_xi(&t1, &t1);
  fp2_add(rx, &t0, &t1);
}
static void f2_3a_m2b(fp2* r, const fp2* a, const fp2* b) {
  fp2 t;
  fp2_sub(&t, a, b);
  fp2_dbl(&t, &t);
  fp2_add(r, &t, a);
}
static void f2_3a_p2b(fp2* r, const fp2* a, const fp2* b) {
  fp2 t;
  fp2_add(&t, a, b);
  fp2_dbl(&t, &t);
  fp2_add(r, &t, a);
}
static void fp12_cyc_sqr(fp12* r, const fp12* f) {
  fp2 Ax, Ay, Bx, By, Cx, Cy, sCx;
  fp12 o;
  fp4_sqr(&Ax, &Ay, &f->c0.c0, &f->c1.c1);
  fp4_sqr(&Bx, &By, &f->c1.c0, &f->c0.c2);
  fp4_sqr(&Cx, &Cy, &f->c0.c1, &f->c1.c2);
  f2_3a_m2b(&o.c0.c0, &Ax, &f->c0.c0);
  f2_3a_p2b(&o.c1.c1, &Ay, &f->c1.c1);
  fp2_mul_xi(&sCx, &Cy);
  f2_3a_p2b(&o.c1.c0, &sCx, &f->c1.c0);
  f2_3a_m2b(&o.c0.c2, &Cx, &f->c0.c2);
  f2_3a_m2b(&o.c0.c1, &Bx, &f->c0.c1);
  f2_3a_p2b(&o.c1.c2, &By, &f->c1.c2);
  *r = o;
}
/* a^x (x < 0), a cyclotomic */
static void fp12_exp_x(fp12* r, const fp12* a) {
  fp12 acc = *a;
  for (int i = 62; i >= 0; i--) {
    fp12_cyc_sqr(&acc, &acc);
    if ((C_X_ABS >> i) & 1) fp12_mul(&acc, &acc, a);
  }
  fp12_conj(r, &acc);
}
/* f^(3 (p^12 - 1)/r): easy part, then 3(p^4-p^2+1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3 */
static void final_exp(fp12* r, const fp12* f) {
  fp12 t0, t1, f2, a, b, c;
  fp12_conj(&t0, f);
  fp12_inv(&t1, f);
  fp12_mul(&t0, &t0, &t1);
  fp12_frob(&t1, &t0, 2);
  fp12_mul(&f2, &t1, &t0);
  fp12_exp_x(&t0, &f2);
  fp12_conj(&t1, &f2);
  fp12_mul(&a, &t0, &t1);
  fp12_exp_x(&t0, &a);
  fp12_conj(&t1, &a);
  fp12_mul(&a, &t0, &t1);
  fp12_exp_x(&t0, &a);
  fp12_frob(&t1, &a, 1);
  fp12_mul(&b, &t0, &t1);
  fp12_exp_x(&t0, &b);
  fp12_exp_x(&t0, &t0);
  fp12_frob(&t1, &b, 2);
  fp12_mul(&c, &t0, &t1);
  fp12_conj(&t1, &b);
  fp12_mul(&c, &c, &t1);
  fp12_cyc_sqr(&t0, &f2);
  fp12_mul(&t0, &t0, &f2);
  fp12_mul(r, &c, &t0);
}

/* ----------------------------------------------------- curve points ---- */
/* Jacobian (X/Z^2, Y/Z^3), Z == 0 <=> infinity; a = 0 on both curves.
 * The group law is written once per field through this macro. */
#define DEFINE_JAC(G, F)                                                                         \
  typedef struct {                                                                               \
    F X, Y, Z;                                                                                   \
  } G##j;                                                                                        \
  typedef struct {                                                                               \
    F x, y;                                                                                      \
    int inf;                                                                                     \
  } G##a;                                                                                        \
  static inline int G##_is_inf(const G##j* p) { return F##_is_zero(&p->Z); }                    \
  static inline void G##_set_inf(G##j* p) {                                                      \
    memset(p, 0, sizeof(*p));                                                                    \
  }                                                                                              \
  static void G##_from_aff(G##j* r, const G##a* a) {                                             \
    if (a->inf) {                                                                                \
      G##_set_inf(r);                                                                            \
      return;                                                                                    \
    }                                                                                            \
    r->X = a->x;                                                                                 \
    r->Y = a->y;                                                                                 \
    F##_one(&r->Z);                                                                              \
  }                                                                                              \
  static void G##_dbl(G##j* r, const G##j* p) {                                                  \
    if (G##_is_inf(p)) {                                                                         \
      *r = *p;                                                                                   \
      return;                                                                                    \
    }                                                                                            \
    F A, B, C, D, E, Fq, t;                                                                      \
    G##j o;                                                                                      \
    F##_sqr(&A, &p->X);                                                                          \
    F##_sqr(&B, &p->Y);                                                                          \
    F##_sqr(&C, &B);                                                                             \
    F##_add(&t, &p->X, &B);                                                                      \
    F##_sqr(&t, &t);                                                                             \
    F##_sub(&t, &t, &A);                                                                         \
    F##_sub(&t, &t, &C);                                                                         \
    F##_add(&D, &t, &t);                                                                         \
    F##_add(&E, &A, &A);                                                                         \
    F##_add(&E, &E, &A);                                                                         \
    F##_sqr(&Fq, &E);                                                                            \
    F##_add(&t, &D, &D);                                                                         \
    F##_sub(&o.X, &Fq, &t);                                                                      \
    F##_sub(&t, &D, &o.X);                                                                       \
    F##_mul(&o.Y, &E, &t);                                                                       \
    F##_add(&C, &C, &C);                                                                         \
    F##_add(&C, &C, &C);                                                                         \
    F##_add(&C, &C, &C);                                                                         \
    F##_sub(&o.Y, &o.Y, &C);                                                                     \
    F##_mul(&o.Z, &p->Y, &p->Z);                                                                 \
    F##_add(&o.Z, &o.Z, &o.Z);                                                                   \
    *r = o;                                                                                      \
  }                                                                                              \
  static void G##_add(G##j* r, const G##j* p, const G##j* q) {                                   \
    if (G##_is_inf(p)) {                                                                         \
      *r = *q;                                                                                   \
      return;                                                                                    \
    }                                                                                            \
    if (G##_is_inf(q)) {                                                                         \
      *r = *p;                                                                                   \
      return;                                                                                    \
    }                                                                                            \
    F Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, Rr, V, t;                                             \
    G##j o;                                                                                      \
    F##_sqr(&Z1Z1, &p->Z);                                                                       \
    F##_sqr(&Z2Z2, &q->Z);                                                                       \
    F##_mul(&U1, &p->X, &Z2Z2);                                                                  \
    F##_mul(&U2, &q->X, &Z1Z1);                                                                  \
    F##_mul(&S1, &p->Y, &q->Z);                                                                  \
    F##_mul(&S1, &S1, &Z2Z2);                                                                    \
    F##_mul(&S2, &q->Y, &p->Z);                                                                  \
    F##_mul(&S2, &S2, &Z1Z1);                                                                    \
    F##_sub(&H, &U2, &U1);                                                                       \
    F##_sub(&Rr, &S2, &S1);                                                                      \
    if (F##_is_zero(&H)) {                                                                       \
      if (F##_is_zero(&Rr))                                                                      \
        G##_dbl(r, p);                                                                           \
      else                                                                                       \
        G##_set_inf(r);                                                                          \
      return;                                                                                    \
    }                                                                                            \
    F##_add(&I, &H, &H);                                                                         \
    F##_sqr(&I, &I);                                                                             \
    F##_mul(&J, &H, &I);                                                                         \
    F##_add(&Rr, &Rr, &Rr);                                                                      \
    F##_mul(&V, &U1, &I);                                                                        \
    F##_sqr(&o.X, &Rr);                                                                          \
    F##_sub(&o.X, &o.X, &J);                                                                     \
    F##_add(&t, &V, &V);                                                                         \
    F##_sub(&o.X, &o.X, &t);                                                                     \
    F##_sub(&t, &V, &o.X);                                                                       \
    F##_mul(&o.Y, &Rr, &t);                                                                      \
    F##_mul(&t, &S1, &J);                                                                        \
    F##_add(&t, &t, &t);                                                                         \
    F##_sub(&o.Y, &o.Y, &t);                                                                     \
    F##_add(&t, &p->Z, &q->Z);                                                                   \
    F##_sqr(&t, &t);                                                                             \
    F##_sub(&t, &t, &Z1Z1);                                                                      \
    F##_sub(&t, &t, &Z2Z2);                                                                      \
    F##_mul(&o.Z, &t, &H);                                                                       \
    *r = o;                                                                                      \
  }                                                                                              \
  static void G##_neg(G##j* r, const G##j* p) {                                                  \
    *r = *p;                                                                                     \
    F##_neg(&r->Y, &p->Y);                                                                       \
  }                                                                                              \
  static void G##_to_aff(G##a* r, const G##j* p) {                                               \
    if (G##_is_inf(p)) {                                                                         \
      memset(r, 0, sizeof(*r));                                                                  \
      r->inf = 1;                                                                                \
      return;                                                                                    \
    }                                                                                            \
    F zi, zi2, zi3;                                                                              \
    F##_inv(&zi, &p->Z);                                                                         \
    F##_sqr(&zi2, &zi);                                                                          \
    F##_mul(&zi3, &zi2, &zi);                                                                    \
    F##_mul(&r->x, &p->X, &zi2);                                                                 \
    F##_mul(&r->y, &p->Y, &zi3);                                                                 \
    r->inf = 0;                                                                                  \
  }                                                                                              \
  static int G##_eq(const G##j* p, const G##j* q) {                                              \
    int pi = G##_is_inf(p), qi = G##_is_inf(q);                                                  \
    if (pi || qi) return pi && qi;                                                               \
    F z1, z2, a, b;                                                                              \
    F##_sqr(&z1, &p->Z);                                                                         \
    F##_sqr(&z2, &q->Z);                                                                         \
    F##_mul(&a, &p->X, &z2);                                                                     \
    F##_mul(&b, &q->X, &z1);                                                                     \
    if (!F##_eq(&a, &b)) return 0;                                                               \
    F##_mul(&z1, &z1, &p->Z);                                                                    \
    F##_mul(&z2, &z2, &q->Z);                                                                    \
    F##_mul(&a, &p->Y, &z2);                                                                     \
    F##_mul(&b, &q->Y, &z1);                                                                     \
    return F##_eq(&a, &b);                                                                       \
  }                                                                                              \
  /* [|x|]P */                                                                                   \
  static void G##_mul_xabs(G##j* r, const G##j* p) {                                             \
    G##j acc = *p;                                                                               \
    for (int i = 62; i >= 0; i--) {                                                              \
      G##_dbl(&acc, &acc);                                                                       \
      if ((C_X_ABS >> i) & 1) G##_add(&acc, &acc, p);                                            \
    }                                                                                            \
    *r = acc;                                                                                    \
  }                                                                                              \
  /* [a + b lambda]P given E = [lambda]P (Straus-Shamir over 32-bit halves) */                   \
  static void G##_mul_glv(G##j* r, const G##j* p, const G##j* e, uint64_t w) {                   \
    const uint32_t a = (uint32_t)w, b = (uint32_t)(w >> 32);                                     \
    G##j tab[4], acc;                                                                            \
    G##_set_inf(&tab[0]);                                                                        \
    tab[1] = *p;                                                                                 \
    tab[2] = *e;                                                                                 \
    G##_add(&tab[3], p, e);                                                                      \
    G##_set_inf(&acc);                                                                           \
    for (int i = 31; i >= 0; i--) {                                                              \
      G##_dbl(&acc, &acc);                                                                       \
      const uint32_t sel = ((a >> i) & 1u) | (((b >> i) & 1u) << 1);                             \
      if (sel) G##_add(&acc, &acc, &tab[sel]);                                                   \
    }                                                                                            \
    *r = acc;                                                                                    \
  }                                                                                              \
  /* [k]P for a big-endian 32-byte scalar */                                                     \
  static void G##_mul_be32(G##j* r, const G##j* p, const uint8_t* k) {                           \
    G##j acc;                                                                                    \
    G##_set_inf(&acc);                                                                           \
    for (int i = 0; i < 256; i++) {                                                              \
      G##_dbl(&acc, &acc);                                                                       \
      if ((k[i >> 3] >> (7 - (i & 7))) & 1) G##_add(&acc, &acc, p);                              \
    }                                                                                            \
    *r = acc;                                                                                    \
  }

static inline void fp_one(fp* r) { *r = C_ONE; }
DEFINE_JAC(g1, fp)
DEFINE_JAC(g2, fp2)

static int g1_on_curve(const g1a* a) {
  if (a->inf) return 1;
  fp l, r;
  fp_sqr(&l, &a->y);
  fp_sqr(&r, &a->x);
  fp_mul(&r, &r, &a->x);
  fp_add(&r, &r, &C_B1);
  return fp_eq(&l, &r);
}
static int g2_on_curve(const g2a* a) {
  if (a->inf) return 1;
  fp2 l, r;
  fp2_sqr(&l, &a->y);
  fp2_sqr(&r, &a->x);
  fp2_mul(&r, &r, &a->x);
  fp2_add(&r, &r, &C_B2);
  return fp2_eq(&l, &r);
}
static void g2_psi(g2j* r, const g2j* p) {
  fp2 t;
  fp2_conj(&t, &p->X);
  fp2_mul(&r->X, &t, &C_PSI_CX);
  fp2_conj(&t, &p->Y);
  fp2_mul(&r->Y, &t, &C_PSI_CY);
  fp2_conj(&r->Z, &p->Z);
}
/* psi(P) == [x]P  (blst POINTonE2_in_G2) */
static int g2_in_subgroup(const g2j* p) {
  if (g2_is_inf(p)) return 1;
  g2j xp, ps;
  g2_mul_xabs(&xp, p);
  g2_neg(&xp, &xp);
  g2_psi(&ps, p);
  return g2_eq(&ps, &xp);
}
/* phi(P) == [-x^2]P */
static int g1_in_subgroup(const g1j* p) {
  if (g1_is_inf(p)) return 1;
  g1j t, ph = *p;
  g1_mul_xabs(&t, p);
  g1_mul_xabs(&t, &t);
  g1_neg(&t, &t);
  fp_mul(&ph.X, &p->X, &C_G1_BETA);
  return g1_eq(&ph, &t);
}
static void g1_glv_endo(g1j* r, const g1j* p) {
  *r = *p;
  fp_mul(&r->X, &p->X, &C_G1_BETA);
}
static void g2_glv_endo(g2j* r, const g2j* p) {
  g2j t;
  g2_psi(&t, p);
  g2_psi(&t, &t);
  g2_neg(r, &t);
}

/* ----------------------------------------------- (de)serialisation ---- */
enum { ST_OK = 0, ST_BAD_ENCODING = 1, ST_NOT_ON_CURVE = 2, ST_NOT_IN_GROUP = 3, ST_PK_INFINITY = 4,
       ST_EMPTY_AGGREGATE = 5, ST_ZERO_SIGNATURE = 6 };

static int bytes_zero(const uint8_t* b, int n) {
  uint8_t acc = 0;
  for (int i = 0; i < n; i++) acc |= b[i];
  return acc == 0;
}
/* PublicKey.fromBytes(96 bytes, uncompressed), no subgroup check */
static int g1_deserialize96(g1a* out, const uint8_t* b) {
  memset(out, 0, sizeof(*out));
  const uint8_t flags = b[0];
  if (flags & 0x80) return ST_BAD_ENCODING; /* 96 bytes <=> compressed bit clear */
  if (flags & 0xE0) {
    if ((flags & 0x40) && (flags & 0x3F) == 0 && bytes_zero(b + 1, 95)) {
      out->inf = 1;
      return ST_OK;
    }
    return ST_BAD_ENCODING;
  }
  if (!fp_from_be48(&out->x, b) || !fp_from_be48(&out->y, b + 48)) return ST_BAD_ENCODING;
  if (!g1_on_curve(out)) return ST_NOT_ON_CURVE;
  if (fp_is_zero(&out->x) && fp_is_zero(&out->y)) return ST_NOT_IN_GROUP;
  return ST_OK;
}
/* Signature.fromBytes without the subgroup check: 96 (compressed) / 192 bytes */
static int g2_deserialize(g2a* out, const uint8_t* b, uint32_t len) {
  memset(out, 0, sizeof(*out));
  if (len == 0) return ST_BAD_ENCODING;
  const uint8_t flags = b[0];
  const int c = (flags & 0x80) != 0;
  if (len != (c ? 96u : 192u)) return ST_BAD_ENCODING;
  if (c) {
    if (flags & 0x40) {
      if ((flags & 0x3F) == 0 && bytes_zero(b + 1, 95)) {
        out->inf = 1;
        return ST_OK;
      }
      return ST_BAD_ENCODING;
    }
    uint8_t t[48];
    memcpy(t, b, 48);
    t[0] &= 0x1F;
    if (!fp_from_be48(&out->x.c1, t) || !fp_from_be48(&out->x.c0, b + 48)) return ST_BAD_ENCODING;
    fp2 rhs, y;
    fp2_sqr(&rhs, &out->x);
    fp2_mul(&rhs, &rhs, &out->x);
    fp2_add(&rhs, &rhs, &C_B2);
    if (!fp2_sqrt(&y, &rhs)) return ST_NOT_ON_CURVE;
    if (fp2_lex_largest(&y) != ((flags & 0x20) != 0)) fp2_neg(&y, &y);
    out->y = y;
    return ST_OK;
  }
  if (flags & 0xE0) {
    if ((flags & 0x40) && (flags & 0x3F) == 0 && bytes_zero(b + 1, 191)) {
      out->inf = 1;
      return ST_OK;
    }
    return ST_BAD_ENCODING;
  }
  if (!fp_from_be48(&out->x.c1, b) || !fp_from_be48(&out->x.c0, b + 48) || !fp_from_be48(&out->y.c1, b + 96) ||
      !fp_from_be48(&out->y.c0, b + 144))
    return ST_BAD_ENCODING;
  if (!g2_on_curve(out)) return ST_NOT_ON_CURVE;
  if (fp2_is_zero(&out->x) && fp2_is_zero(&out->y)) return ST_NOT_IN_GROUP;
  return ST_OK;
}
static void g1_serialize96(uint8_t* o, const g1a* a) {
  if (a->inf) {
    memset(o, 0, 96);
    o[0] = 0x40;
    return;
  }
  fp_to_be48(o, &a->x);
  fp_to_be48(o + 48, &a->y);
}
static void g2_serialize192(uint8_t* o, const g2a* a) {
  if (a->inf) {
    memset(o, 0, 192);
    o[0] = 0x40;
    return;
  }
  fp_to_be48(o, &a->x.c1);
  fp_to_be48(o + 48, &a->x.c0);
  fp_to_be48(o + 96, &a->y.c1);
  fp_to_be48(o + 144, &a->y.c0);
}

/* ------------------------------------------------------------ SHA-256 ---- */
static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static void sha256_block(uint32_t st[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) |
           blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA_K[i] + w[i];
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}
static void sha256(uint8_t out[32], const uint8_t* msg, size_t len) {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t off = 0;
  while (len - off >= 64) {
    sha256_block(st, msg + off);
    off += 64;
  }
  uint8_t blk[128];
  size_t rem = len - off;
  memset(blk, 0, sizeof(blk));
  memcpy(blk, msg + off, rem);
  blk[rem] = 0x80;
  size_t nb = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) blk[nb - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha256_block(st, blk);
  if (nb == 128) sha256_block(st, blk + 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

/* ------------------------------------------------------- hash_to_G2 ---- */
static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
#define DST_LEN 43
/* expand_message_xmd(msg[32], DST, 256) */
static void expand_xmd_256(uint8_t out[256], const uint8_t msg[32]) {
  uint8_t buf[64 + 32 + 2 + 1 + DST_LEN + 1];
  size_t n = 0;
  memset(buf, 0, 64);
  n = 64;
  memcpy(buf + n, msg, 32);
  n += 32;
  buf[n++] = 1; /* 256 = 0x0100 */
  buf[n++] = 0;
  buf[n++] = 0;
  memcpy(buf + n, DST, DST_LEN);
  n += DST_LEN;
  buf[n++] = DST_LEN;
  uint8_t b0[32], bi[32];
  sha256(b0, buf, n);
  uint8_t tail[32 + 1 + DST_LEN + 1];
  for (int i = 1; i <= 8; i++) {
    size_t m = 0;
    for (int k = 0; k < 32; k++) tail[m++] = (i == 1) ? b0[k] : (uint8_t)(b0[k] ^ bi[k]);
    tail[m++] = (uint8_t)i;
    memcpy(tail + m, DST, DST_LEN);
    m += DST_LEN;
    tail[m++] = DST_LEN;
    sha256(bi, tail, m);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}
/* 64 big-endian bytes mod p */
static void fp_from_be64(fp* r, const uint8_t* b) {
  uint64_t hi[6] = {0}, lo[6] = {0};
  for (int i = 0; i < 4; i++) {
    uint64_t vh = 0, vl = 0;
    for (int k = 0; k < 8; k++) {
      vh = (vh << 8) | b[(3 - i) * 8 + k];
      vl = (vl << 8) | b[32 + (3 - i) * 8 + k];
    }
    hi[i] = vh;
    lo[i] = vl;
  }
  fp h, l;
  fp_from_raw(&h, hi);
  fp_from_raw(&l, lo);
  fp_mul(&h, &h, &C_2P256);
  fp_add(r, &h, &l);
}
static void map_to_curve_sswu(g2a* out, const fp2* u) {
  fp2 tv1, tv2, x1, gx1, x, y, t;
  fp2_sqr(&tv1, u);
  fp2_mul(&tv1, &C_SSWU_Z, &tv1);
  fp2_sqr(&tv2, &tv1);
  fp2_add(&tv2, &tv2, &tv1);
  if (fp2_is_zero(&tv2)) {
    x1 = C_SSWU_BZA;
  } else {
    fp2_inv(&t, &tv2);
    fp_add(&t.c0, &t.c0, &C_ONE);
    fp2_mul(&x1, &t, &C_SSWU_MBA);
  }
  fp2_sqr(&gx1, &x1);
  fp2_add(&gx1, &gx1, &C_SSWU_A);
  fp2_mul(&gx1, &gx1, &x1);
  fp2_add(&gx1, &gx1, &C_SSWU_B);
  if (fp2_sqrt(&y, &gx1)) {
    x = x1;
  } else {
    fp2 gx2;
    fp2_mul(&x, &tv1, &x1);
    fp2_sqr(&gx2, &x);
    fp2_add(&gx2, &gx2, &C_SSWU_A);
    fp2_mul(&gx2, &gx2, &x);
    fp2_add(&gx2, &gx2, &C_SSWU_B);
    fp2_sqrt(&y, &gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(&y)) fp2_neg(&y, &y);
  out->x = x;
  out->y = y;
  out->inf = 0;
}
static void poly_eval(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc;
  fp2_zero(&acc);
  for (int i = n - 1; i >= 0; i--) {
    fp2_mul(&acc, &acc, x);
    fp2_add(&acc, &acc, &c[i]);
  }
  *r = acc;
}
static void iso_map(g2j* r, const g2a* p) {
  fp2 xn, xd, yn, yd, t;
  poly_eval(&xn, C_ISO_XNUM, 4, &p->x);
  poly_eval(&xd, C_ISO_XDEN, 3, &p->x);
  poly_eval(&yn, C_ISO_YNUM, 4, &p->x);
  poly_eval(&yd, C_ISO_YDEN, 4, &p->x);
  if (fp2_is_zero(&xd) || fp2_is_zero(&yd)) {
    g2_set_inf(r);
    return;
  }
  /* Z = xd yd, X = xn xd yd^2, Y = y yn xd^3 yd^2 */
  fp2 yd2, xd3;
  fp2_mul(&r->Z, &xd, &yd);
  fp2_sqr(&yd2, &yd);
  fp2_mul(&t, &xn, &xd);
  fp2_mul(&r->X, &t, &yd2);
  fp2_sqr(&xd3, &xd);
  fp2_mul(&xd3, &xd3, &xd);
  fp2_mul(&t, &p->y, &yn);
  fp2_mul(&t, &t, &xd3);
  fp2_mul(&r->Y, &t, &yd2);
}
static void clear_cofactor(g2j* r, const g2j* p) {
  g2j t1, t2, t3, n;
  g2_mul_xabs(&t1, p);
  g2_neg(&t1, &t1);
  g2_psi(&t2, p);
  g2_dbl(&t3, p);
  g2_psi(&t3, &t3);
  g2_psi(&t3, &t3);
  g2_neg(&n, &t2);
  g2_add(&t3, &t3, &n);
  g2_add(&t2, &t1, &t2);
  g2_mul_xabs(&t2, &t2);
  g2_neg(&t2, &t2);
  g2_add(&t3, &t3, &t2);
  g2_neg(&n, &t1);
  g2_add(&t3, &t3, &n);
  g2_neg(&n, p);
  g2_add(r, &t3, &n);
}
static void hash_to_g2(g2j* r, const uint8_t msg[32]) {
  uint8_t ub[256];
  expand_xmd_256(ub, msg);
  fp2 u0, u1;
  fp_from_be64(&u0.c0, ub);
  fp_from_be64(&u0.c1, ub + 64);
  fp_from_be64(&u1.c0, ub + 128);
  fp_from_be64(&u1.c1, ub + 192);
  g2a q0, q1;
  map_to_curve_sswu(&q0, &u0);
  map_to_curve_sswu(&q1, &u1);
  g2j j0, j1;
  iso_map(&j0, &q0);
  iso_map(&j1, &q1);
  g2_add(&j0, &j0, &j1);
  clear_cofactor(r, &j0);
}

/* ------------------------------------------------------------ pairing ---- */
typedef struct {
  fp2 X, Y, Z;
} g2proj;
static void miller_dbl(g2proj* T, fp2* l0, fp2* l1, fp2* l4, const fp* xp, const fp* yp) {
  fp2 XX, B, C, E, F, A, G, H, t, E2;
  fp2_sqr(&XX, &T->X);
  fp2_sqr(&B, &T->Y);
  fp2_sqr(&C, &T->Z);
  fp2_mul(&E, &C, &C_B2X3);
  fp2_mul3(&F, &E);
  fp2_mul(&A, &T->X, &T->Y);
  fp2_mul_fp(&A, &A, &C_HALF);
  fp2_add(&G, &B, &F);
  fp2_mul_fp(&G, &G, &C_HALF);
  fp2_add(&H, &T->Y, &T->Z);
  fp2_sqr(&H, &H);
  fp2_sub(&H, &H, &B);
  fp2_sub(&H, &H, &C);
  fp2_sub(l0, &B, &E);
  fp2_mul3(&t, &XX);
  fp2_mul_fp(&t, &t, xp);
  fp2_neg(l1, &t);
  fp2_mul_fp(l4, &H, yp);
  fp2_sub(&t, &B, &F);
  fp2_mul(&T->X, &A, &t);
  fp2_sqr(&E2, &E);
  fp2_mul3(&E2, &E2);
  fp2_sqr(&T->Y, &G);
  fp2_sub(&T->Y, &T->Y, &E2);
  fp2_mul(&T->Z, &B, &H);
}
static void miller_add(g2proj* T, const fp2* xq, const fp2* yq, fp2* l0, fp2* l1, fp2* l4, const fp* xp,
                       const fp* yp) {
  fp2 th, la, C, D, E, F, G, H, t, ye;
  fp2_mul(&t, yq, &T->Z);
  fp2_sub(&th, &T->Y, &t);
  fp2_mul(&t, xq, &T->Z);
  fp2_sub(&la, &T->X, &t);
  fp2_mul(l0, &th, xq);
  fp2_mul(&t, &la, yq);
  fp2_sub(l0, l0, &t);
  fp2_mul_fp(&t, &th, xp);
  fp2_neg(l1, &t);
  fp2_mul_fp(l4, &la, yp);
  fp2_sqr(&C, &th);
  fp2_sqr(&D, &la);
  fp2_mul(&E, &la, &D);
  fp2_mul(&F, &T->Z, &C);
  fp2_mul(&G, &T->X, &D);
  fp2_add(&H, &E, &F);
  fp2_sub(&H, &H, &G);
  fp2_sub(&H, &H, &G);
  fp2_mul(&T->X, &la, &H);
  fp2_sub(&t, &G, &H);
  fp2_mul(&t, &th, &t);
  fp2_mul(&ye, &T->Y, &E);
  fp2_sub(&T->Y, &t, &ye);
  fp2_mul(&T->Z, &T->Z, &E);
}
/* a * (b0 + b1 v): 5 Fp2 products */
static void fp6_mul_01(fp6* r, const fp6* a, const fp2* b0, const fp2* b1) {
  fp2 t0, t1, s, u;
  fp6 o;
  fp2_mul(&t0, &a->c0, b0);
  fp2_mul(&t1, &a->c1, b1);
  fp2_mul(&s, &a->c2, b1);
  fp2_mul_xi(&s, &s);
  fp2_add(&o.c0, &t0, &s);
  fp2_add(&s, &a->c0, &a->c1);
  fp2_add(&u, b0, b1);
  fp2_mul(&s, &s, &u);
  fp2_sub(&s, &s, &t0);
  fp2_sub(&o.c1, &s, &t1);
  fp2_mul(&s, &a->c2, b0);
  fp2_add(&o.c2, &t1, &s);
  *r = o;
}
/* a * (b1 v): 3 Fp2 products */
static void fp6_mul_1(fp6* r, const fp6* a, const fp2* b1) {
  fp2 t0, t1, t2;
  fp2_mul(&t0, &a->c2, b1);
  fp2_mul_xi(&t0, &t0);
  fp2_mul(&t1, &a->c0, b1);
  fp2_mul(&t2, &a->c1, b1);
  r->c0 = t0;
  r->c1 = t1;
  r->c2 = t2;
}
/* f * (l0 + l1 v + l4 v w): 13 Fp2 products */
static void fp12_mul_line(fp12* f, const fp2* l0, const fp2* l1, const fp2* l4) {
  fp6 t0, t1, s;
  fp2 m;
  fp6_mul_01(&t0, &f->c0, l0, l1);
  fp6_mul_1(&t1, &f->c1, l4);
  fp6_add(&s, &f->c0, &f->c1);
  fp2_add(&m, l1, l4);
  fp6_mul_01(&s, &s, l0, &m);
  fp6_sub(&s, &s, &t0);
  fp6_sub(&f->c1, &s, &t1);
  fp6_mul_v(&t1, &t1);
  fp6_add(&f->c0, &t0, &t1);
}
/* f_{|x|,Q}(P) conjugated (x < 0); P, Q affine finite */
static void miller_loop(fp12* f, const g1a* P, const g2a* Q) {
  g2proj T;
  fp2 l0, l1, l4;
  T.X = Q->x;
  T.Y = Q->y;
  fp2_one(&T.Z);
  fp12_one(f);
  for (int i = 62; i >= 0; i--) {
    if (i < 62) fp12_sqr(f, f);
    miller_dbl(&T, &l0, &l1, &l4, &P->x, &P->y);
    fp12_mul_line(f, &l0, &l1, &l4);
    if ((C_X_ABS >> i) & 1) {
      miller_add(&T, &Q->x, &Q->y, &l0, &l1, &l4, &P->x, &P->y);
      fp12_mul_line(f, &l0, &l1, &l4);
    }
  }
  fp12_conj(f, f);
}

/* ------------------------------------------------------- verification ---- */
static uint64_t batch_scalar_raw(const uint8_t seed[32], uint32_t i) {
  uint8_t buf[36], d[32];
  memcpy(buf, seed, 32);
  buf[32] = (uint8_t)i;
  buf[33] = (uint8_t)(i >> 8);
  buf[34] = (uint8_t)(i >> 16);
  buf[35] = (uint8_t)(i >> 24);
  sha256(d, buf, 36);
  uint64_t w = 0;
  for (int k = 7; k >= 0; k--) w = (w << 8) | d[k];
  return w ? w : 1;
}

typedef struct {
  uint32_t n_req;
  const uint32_t* req_off;
  const uint8_t* pks;
  const uint32_t* pk_off;
  const uint8_t* msgs;
  const uint8_t* sigs;
  const uint32_t* sig_off;
  const uint8_t* seed;
  uint8_t* valid;
  uint8_t* err;
  volatile uint32_t next;
} job_t;

/* one request: verifySignatureSetsMaybeBatch verdict (+ rejection codes) */
static void verify_request(const job_t* J, uint32_t k) {
  const uint32_t a = J->req_off[k], b = J->req_off[k + 1];
  int bad = (a == b), err_empty = 0, err_pk = 0;
  const int single = (b - a == 1);
  fp12 f;
  fp12_one(&f);
  g2j S;
  g2_set_inf(&S);
  for (uint32_t i = a; i < b && !err_empty; i++) {
    /* pubkey(s) -> aggregated Jacobian */
    const uint32_t pa = J->pk_off ? J->pk_off[i] : i, pb = J->pk_off ? J->pk_off[i + 1] : i + 1;
    g1j pk;
    g1_set_inf(&pk);
    if (pb == pa) {
      err_empty = 1;
      break;
    }
    int pk_bad = 0;
    for (uint32_t t = pa; t < pb; t++) {
      g1a p;
      if (g1_deserialize96(&p, J->pks + (size_t)t * 96) != ST_OK) {
        pk_bad = 1;
        continue;
      }
      g1j pj;
      g1_from_aff(&pj, &p);
      g1_add(&pk, &pk, &pj);
    }
    if (pk_bad) {
      err_pk = 1;
      continue;
    }
    if (bad) continue;
    if (g1_is_inf(&pk)) { /* BLST_PK_IS_INFINITY -> false */
      bad = 1;
      continue;
    }
    if (single && !g1_in_subgroup(&pk)) {
      bad = 1;
      continue;
    }
    g2a sa;
    const uint32_t sa0 = J->sig_off[i], sa1 = J->sig_off[i + 1];
    if (g2_deserialize(&sa, J->sigs + sa0, sa1 - sa0) != ST_OK) {
      bad = 1;
      continue;
    }
    g2j sj;
    g2_from_aff(&sj, &sa);
    if (!g2_in_subgroup(&sj) || (single && sa.inf)) {
      bad = 1;
      continue;
    }
    /* r_i pk_i, r_i sig_i, Miller(r_i pk_i, H(m_i)) */
    const uint64_t w = batch_scalar_raw(J->seed, i);
    g1j e1, rp;
    g1_glv_endo(&e1, &pk);
    g1_mul_glv(&rp, &pk, &e1, w);
    g2j e2, rs;
    g2_glv_endo(&e2, &sj);
    g2_mul_glv(&rs, &sj, &e2, w);
    g2_add(&S, &S, &rs);
    g2j h;
    hash_to_g2(&h, J->msgs + (size_t)i * 32);
    g1a rpa;
    g2a ha;
    g1_to_aff(&rpa, &rp);
    g2_to_aff(&ha, &h);
    if (!rpa.inf && !ha.inf) {
      fp12 fi;
      miller_loop(&fi, &rpa, &ha);
      fp12_mul(&f, &f, &fi);
    }
  }
  J->err[k] = err_empty ? 1 : err_pk ? 2 : 0;
  if (bad || err_empty || err_pk) {
    J->valid[k] = 0;
    return;
  }
  g2a Sa;
  g2_to_aff(&Sa, &S);
  if (!Sa.inf) {
    g1a ng;
    ng.x = C_G1_X;
    ng.y = C_G1_NEG_Y;
    ng.inf = 0;
    fp12 fs;
    miller_loop(&fs, &ng, &Sa);
    fp12_mul(&f, &f, &fs);
  }
  fp12 r;
  final_exp(&r, &f);
  J->valid[k] = (uint8_t)fp12_is_one(&r);
}

static void* worker(void* arg) {
  job_t* J = (job_t*)arg;
  for (;;) {
    const uint32_t k = __atomic_fetch_add(&J->next, 1u, __ATOMIC_RELAXED);
    if (k >= J->n_req) break;
    verify_request(J, k);
  }
  return NULL;
}

/* Same inputs / outputs as lb_verify_requests (include/lodestar_bls.h):
 * out_valid[k] in {0,1}, out_err[k] in {0 ok, 1 empty aggregate, 2 bad pubkey}.
 * Requests are spread over n_threads POSIX threads. */
int lbo_verify_requests(uint32_t n_req, const uint32_t* req_off, const uint8_t* pks, const uint32_t* pk_off,
                        const uint8_t* msgs, const uint8_t* sigs, const uint32_t* sig_off, const uint8_t* seed,
                        uint8_t* out_valid, uint8_t* out_err, int n_threads) {
  if (!req_off || !out_valid || !out_err || !seed) return -1;
  job_t J = {n_req, req_off, pks, pk_off, msgs, sigs, sig_off, seed, out_valid, out_err, 0};
  if (n_threads <= 1) {
    worker(&J);
    return 0;
  }
  pthread_t th[256];
  if (n_threads > 256) n_threads = 256;
  int started = 0;
  for (int t = 0; t < n_threads; t++)
    if (pthread_create(&th[t], NULL, worker, &J) == 0) started++;
  if (!started) worker(&J);
  for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
  return 0;
}

/* hash_to_G2(msg) -> 192-byte uncompressed affine */
int lbo_hash_to_g2(uint32_t n, const uint8_t* msgs, uint8_t* out192) {
  for (uint32_t i = 0; i < n; i++) {
    g2j h;
    g2a a;
    hash_to_g2(&h, msgs + (size_t)i * 32);
    g2_to_aff(&a, &h);
    g2_serialize192(out192 + (size_t)i * 192, &a);
  }
  return 0;
}

/* Signature.fromBytes(validate=true): status (LB_SET_*) + 192-byte re-encoding */
int lbo_decode_signatures(uint32_t n, const uint8_t* sigs, const uint32_t* sig_off, uint8_t* out_status,
                          uint8_t* out192) {
  for (uint32_t i = 0; i < n; i++) {
    g2a a;
    uint8_t st = (uint8_t)g2_deserialize(&a, sigs + sig_off[i], sig_off[i + 1] - sig_off[i]);
    if (st == ST_OK) {
      g2j j;
      g2_from_aff(&j, &a);
      if (!g2_in_subgroup(&j)) st = ST_NOT_IN_GROUP;
    }
    out_status[i] = st;
    if (out192) {
      if (st == ST_OK)
        g2_serialize192(out192 + (size_t)i * 192, &a);
      else
        memset(out192 + (size_t)i * 192, 0, 192);
    }
  }
  return 0;
}

/* e(P, Q) = final_exp(Miller(P, Q)) with the device's exponent 3 (p^12-1)/r,
 * 12 big-endian Fp coefficients (c0.c0.c0, c0.c0.c1, ..., c1.c2.c1) */
int lbo_pairing(uint32_t n, const uint8_t* g1_96, const uint8_t* g2_192, uint8_t* out576) {
  for (uint32_t i = 0; i < n; i++) {
    g1a p;
    g2a q;
    fp12 f, r;
    fp12_one(&f);
    if (g1_deserialize96(&p, g1_96 + (size_t)i * 96) == ST_OK && g2_deserialize(&q, g2_192 + (size_t)i * 192, 192) == ST_OK &&
        !p.inf && !q.inf)
      miller_loop(&f, &p, &q);
    final_exp(&r, &f);
    const fp2* c[6] = {&r.c0.c0, &r.c0.c1, &r.c0.c2, &r.c1.c0, &r.c1.c1, &r.c1.c2};
    uint8_t* o = out576 + (size_t)i * 576;
    for (int k = 0; k < 6; k++) {
      fp_to_be48(o + 96 * k, &c[k]->c0);
      fp_to_be48(o + 96 * k + 48, &c[k]->c1);
    }
  }
  return 0;
}

/* SecretKey.toPublicKey / sign (big-endian 32-byte secret keys), for tests */
int lbo_sk_to_pk(uint32_t n, const uint8_t* sk32, uint8_t* out96) {
  g1a g;
  g.x = C_G1_X;
  g.y = C_G1_Y;
  g.inf = 0;
  g1j gj;
  g1_from_aff(&gj, &g);
  for (uint32_t i = 0; i < n; i++) {
    g1j r;
    g1a a;
    g1_mul_be32(&r, &gj, sk32 + (size_t)i * 32);
    g1_to_aff(&a, &r);
    g1_serialize96(out96 + (size_t)i * 96, &a);
  }
  return 0;
}
int lbo_sign(uint32_t n, const uint8_t* sk32, const uint8_t* msgs, uint8_t* out96) {
  for (uint32_t i = 0; i < n; i++) {
    g2j h, r;
    g2a a;
    hash_to_g2(&h, msgs + (size_t)i * 32);
    g2_mul_be32(&r, &h, sk32 + (size_t)i * 32);
    g2_to_aff(&a, &r);
    uint8_t* o = out96 + (size_t)i * 96;
    if (a.inf) {
      memset(o, 0, 96);
      o[0] = 0xC0;
      continue;
    }
    fp_to_be48(o, &a.x.c1);
    fp_to_be48(o + 48, &a.x.c0);
    o[0] |= (uint8_t)(0x80 | (fp2_lex_largest(&a.y) ? 0x20 : 0));
  }
  return 0;
}
