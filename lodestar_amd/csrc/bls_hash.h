// hash_to_G2 for BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380 §8.8.2) with the
// Ethereum proof-of-possession DST, plus the SHA-256 DRBG for batch scalars.
//
// Reference: every blst verification path hashes the 32-byte signing root with
// this suite (blst Hash_to_G2 inside Pairing.mul_n_aggregate / core_verify,
// reached from packages/beacon-node/src/chain/bls/maybeBatch.ts:19,38).
#pragma once
#include "bls_curve.h"

namespace lb {

// ----------------------------------------------------------------------------
// SHA-256 (FIPS 180-4), one lane per message
// ----------------------------------------------------------------------------
__device__ __constant__ const uint32_t SHA_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

LB_DEV uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

LB_DEV void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u;
  st[1] = 0xbb67ae85u;
  st[2] = 0x3c6ef372u;
  st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu;
  st[5] = 0x9b05688cu;
  st[6] = 0x1f83d9abu;
  st[7] = 0x5be0cd19u;
}

// w: 16 big-endian message words of one block
LB_NOINL void sha256_compress(uint32_t st[8], const uint32_t win[16]) {
  uint32_t w[16];
  for (int i = 0; i < 16; i++) w[i] = win[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + SHA_K[i] + wi;
    const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
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

// Byte-addressed block builder (big-endian words)
struct sha_block {
  uint32_t w[16];
  LB_DEV void clear() {
    for (int i = 0; i < 16; i++) w[i] = 0;
  }
  LB_DEV void put(int pos, uint8_t v) { w[pos >> 2] |= (uint32_t)v << (24 - 8 * (pos & 3)); }
};

// DST = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" (43 bytes) || I2OSP(43, 1)
__device__ __constant__ const uint8_t DST_PRIME[44] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1', 'G', '2', '_', 'X', 'M', 'D', ':',
    'S', 'H', 'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_', 43};

// expand_message_xmd(msg[32], DST, 256) -> 8 digests (64 words)
LB_DEV void expand_message_xmd_32(uint32_t out[64], const uint8_t msg[32]) {
  // b0 = H(Z_pad(64) || msg(32) || I2OSP(256,2) || 0x00 || DST_prime(44)) : 143 bytes, 3 blocks
  uint32_t st[8];
  sha256_init(st);
  sha_block blk;
  blk.clear();
  sha256_compress(st, blk.w);  // the all-zero Z_pad block
  // block 2: msg(32) || 0x01 0x00 || 0x00 || DST_prime[0..28]
  blk.clear();
  for (int i = 0; i < 32; i++) blk.put(i, msg[i]);
  blk.put(32, 0x01);
  blk.put(33, 0x00);
  blk.put(34, 0x00);
  for (int i = 0; i < 29; i++) blk.put(35 + i, DST_PRIME[i]);
  sha256_compress(st, blk.w);
  // block 3: DST_prime[29..43] (15 bytes) || 0x80 || zeros || bitlen(143*8)
  blk.clear();
  for (int i = 0; i < 15; i++) blk.put(i, DST_PRIME[29 + i]);
  blk.put(15, 0x80);
  blk.w[15] = 143u * 8u;
  sha256_compress(st, blk.w);
  uint32_t b0[8];
  for (int i = 0; i < 8; i++) b0[i] = st[i];
  // b_i = H((b0 ^ b_{i-1}) || I2OSP(i,1) || DST_prime) : 77 bytes, 2 blocks
  uint32_t prev[8];
  for (int i = 0; i < 8; i++) prev[i] = 0;
  for (int i = 1; i <= 8; i++) {
    sha256_init(st);
    blk.clear();
    for (int k = 0; k < 8; k++) blk.w[k] = b0[k] ^ prev[k];
    blk.put(32, (uint8_t)i);
    for (int k = 0; k < 31; k++) blk.put(33 + k, DST_PRIME[k]);
    sha256_compress(st, blk.w);
    blk.clear();
    for (int k = 0; k < 13; k++) blk.put(k, DST_PRIME[31 + k]);
    blk.put(13, 0x80);
    blk.w[15] = 77u * 8u;
    sha256_compress(st, blk.w);
    for (int k = 0; k < 8; k++) {
      prev[k] = st[k];
      out[(i - 1) * 8 + k] = st[k];
    }
  }
}

// OS2IP(64 bytes as 16 BE words) mod p, into Montgomery form:
//   x = A * 2^256 + B (A, B < 2^256 < p) -> mont(x) = mm(A, 2^256 R^2) + mm(B, R^2)
LB_DEV void fp_from_64be_words(fp& r, const uint32_t* w) {
  fp A, B;
  for (int j = 0; j < 12; j++) {
    A.l[j] = 0;
    B.l[j] = 0;
  }
  for (int j = 0; j < 8; j++) {
    A.l[j] = w[7 - j];
    B.l[j] = w[15 - j];
  }
  fp a, b;
  fp_mul_const(a, A, LB_C256);
  fp_mul_const(b, B, LB_R2);
  fp_add(r, a, b);
}

LB_DEV void hash_to_field_fp2_2(fp2 u[2], const uint8_t msg[32]) {
  uint32_t ub[64];
  expand_message_xmd_32(ub, msg);
  fp_from_64be_words(u[0].c0, ub + 0);
  fp_from_64be_words(u[0].c1, ub + 16);
  fp_from_64be_words(u[1].c0, ub + 32);
  fp_from_64be_words(u[1].c1, ub + 48);
}

// Square root in Fp2 when a square root s of the norm N(a) = a0^2 + a1^2 is
// already known: one Fp exponentiation (fp2_sqrt's second half).  a must be a
// square; which of the two roots comes out does not matter (callers fix the sign).
LB_DEV void fp2_sqrt_with_norm_root(fp2& r, const fp2& a, const fp& s) {
  if (fp_is_zero(a.c1)) {  // a in Fp (probability ~2^-381 on hashed input)
    fp2 t;
    fp2_sqrt(t, a);
    r = t;
    return;
  }
  fp half, t, c, x0, chk, a1c;
  fp_set(half, LB_HALF);
  fp_add(t, a.c0, s);
  fp_mul(t, t, half);
  fp_pow_p34(c, t);
  fp_mul(x0, t, c);  // t^((p+1)/4)
  fp_sqr(chk, x0);
  fp_mul(a1c, a.c1, c);
  fp_mul(a1c, a1c, half);
  const bool direct = fp_eq(chk, t);
  fp na1c;
  fp_neg(na1c, a1c);
  r.c0 = x0;
  r.c1 = a1c;
  fp_cmov(r.c0, na1c, !direct);
  fp_cmov(r.c1, x0, !direct);
}

// Simplified SWU onto E2': y^2 = x^3 + A'x + B'  (RFC 9380 §6.6.2), branch-free.
// With x2 = Z u^2 x1, g(x2) = Z^3 u^6 g(x1), so N(g(x2)) = N(Z)^3 N(u)^6 N(g(x1))
// and N(Z)^3 is a non-square: ONE exponentiation t = N(g(x1))^((p-3)/4) gives
// the square test of g(x1) and a square root of whichever norm is a square
//   sqrt N(g(x1)) = N(g(x1)) t,   sqrt N(g(x2)) = N(u)^3 N(Z)^(3(p+1)/4) N(g(x1)) t,
// and a second one (fp2_sqrt_with_norm_root) finishes the Fp2 root.  Every lane
// of a wave runs the same instructions (the gx1 / gx2 choice is a select).
LB_DEV void map_to_curve_sswu(g2a& out, const fp2& u) {
  fp2 A, B, Z, tv1, tv2, x1, x2, gx1, gx2, x, gx, y, t;
  fp2_set(A, LB_SSWU_A);
  fp2_set(B, LB_SSWU_B);
  fp2_set(Z, LB_SSWU_Z);
  fp2_sqr(tv1, u);
  fp2_mul(tv1, Z, tv1);  // Z u^2
  fp2_sqr(tv2, tv1);
  fp2_add(tv2, tv2, tv1);  // Z^2 u^4 + Z u^2
  const bool exceptional = fp2_is_zero(tv2);
  fp2_inv(t, tv2);  // inv(0) = 0
  fp one;
  fp_one(one);
  fp_add(t.c0, t.c0, one);
  fp2_mul_const(x1, t, LB_SSWU_MINUS_B_OVER_A);
  fp2 bza;
  fp2_set(bza, LB_SSWU_B_OVER_ZA);
  fp2_cmov(x1, bza, exceptional);
  // gx1 = x1^3 + A x1 + B, x2 = Z u^2 x1, gx2 = x2^3 + A x2 + B
  fp2_sqr(gx1, x1);
  fp2_add(gx1, gx1, A);
  fp2_mul(gx1, gx1, x1);
  fp2_add(gx1, gx1, B);
  fp2_mul(x2, tv1, x1);
  fp2_sqr(gx2, x2);
  fp2_add(gx2, gx2, A);
  fp2_mul(gx2, gx2, x2);
  fp2_add(gx2, gx2, B);
  // norms and the shared exponentiation
  fp n1, e, chk, s1, s2, nu, nu3, c1;
  fp_sqr(n1, gx1.c0);
  fp_sqr(e, gx1.c1);
  fp_add(n1, n1, e);
  fp_pow_p34(e, n1);
  fp_sqr(chk, e);
  fp_mul(chk, chk, n1);
  const bool sq1 = fp_eq(chk, one) || fp_is_zero(n1);
  fp_mul(s1, n1, e);
  fp_sqr(nu, u.c0);
  fp_sqr(e, u.c1);
  fp_add(nu, nu, e);
  fp_sqr(nu3, nu);
  fp_mul(nu3, nu3, nu);
  fp_set(c1, LB_SSWU_NZ3_SQRT);
  fp_mul(s2, nu3, c1);
  fp_mul(s2, s2, s1);
  x = x1;
  gx = gx1;
  fp_cmov(s2, s1, sq1);
  fp2_cmov(x, x2, !sq1);
  fp2_cmov(gx, gx2, !sq1);
  fp2_sqrt_with_norm_root(y, gx, s2);
  fp2 ny;
  fp2_neg(ny, y);
  fp2_cmov(y, ny, fp2_sgn0(u) != fp2_sgn0(y));
  out.x = x;
  out.y = y;
  out.inf = false;
}

// 3-isogeny E2' -> E2, output Jacobian (no inversion):
//   x = xn/xd, y = y' yn/yd ;  Z = xd yd, X = xn xd yd^2, Y = y' yn xd^3 yd^2
LB_DEV void iso_map_g2(g2j& r, const g2a& p) {
  fp2 xn, xd, yn, yd, t;
  fp2_set(xn, LB_ISO_XNUM3);
  fp2_mul(xn, xn, p.x);
  fp2_set(t, LB_ISO_XNUM2);
  fp2_add(xn, xn, t);
  fp2_mul(xn, xn, p.x);
  fp2_set(t, LB_ISO_XNUM1);
  fp2_add(xn, xn, t);
  fp2_mul(xn, xn, p.x);
  fp2_set(t, LB_ISO_XNUM0);
  fp2_add(xn, xn, t);

  fp2_set(t, LB_ISO_XDEN1);
  fp2_add(xd, p.x, t);  // monic
  fp2_mul(xd, xd, p.x);
  fp2_set(t, LB_ISO_XDEN0);
  fp2_add(xd, xd, t);

  fp2_set(yn, LB_ISO_YNUM3);
  fp2_mul(yn, yn, p.x);
  fp2_set(t, LB_ISO_YNUM2);
  fp2_add(yn, yn, t);
  fp2_mul(yn, yn, p.x);
  fp2_set(t, LB_ISO_YNUM1);
  fp2_add(yn, yn, t);
  fp2_mul(yn, yn, p.x);
  fp2_set(t, LB_ISO_YNUM0);
  fp2_add(yn, yn, t);

  fp2_set(t, LB_ISO_YDEN2);
  fp2_add(yd, p.x, t);  // monic
  fp2_mul(yd, yd, p.x);
  fp2_set(t, LB_ISO_YDEN1);
  fp2_add(yd, yd, t);
  fp2_mul(yd, yd, p.x);
  fp2_set(t, LB_ISO_YDEN0);
  fp2_add(yd, yd, t);

  if (fp2_is_zero(xd) || fp2_is_zero(yd)) {  // kernel point -> infinity
    jac_set_inf(r);
    return;
  }
  fp2 yd2, xd2;
  fp2_mul(r.Z, xd, yd);
  fp2_sqr(yd2, yd);
  fp2_mul(t, xn, xd);
  fp2_mul(r.X, t, yd2);
  fp2_sqr(xd2, xd);
  fp2_mul(xd2, xd2, xd);  // xd^3
  fp2_mul(t, p.y, yn);
  fp2_mul(t, t, xd2);
  fp2_mul(r.Y, t, yd2);
}

// clear_cofactor (RFC 9380 G.3): (x^2 - x - 1)P + (x - 1)psi(P) + psi^2(2P), x < 0.
// With z = |x|, A = [z]P, B = psi(P) - A, C = [z]B:
//   h = D - C,  D = psi^2(2P) - P - B,
// ordered so that at most two points are live around each ladder; D is parked
// in `stash` (the output slot, when the caller has one) across the second
// ladder instead of occupying 72 VGPRs there.
LB_DEV void clear_cofactor_g2(g2j& r, const g2j& p, g2j* stash = nullptr) {
  g2j A, B, D, t;
  jac_mul_xabs(A, p);
  g2_psi(B, p);
  jac_neg(A, A);
  jac_add(B, B, A);  // B = psi(P) - A
  jac_dbl(t, p);
  g2_psi(t, t);
  g2_psi(t, t);      // psi^2(2P)
  jac_neg(D, p);
  jac_add(t, t, D);  // psi^2(2P) - P
  jac_neg(D, B);
  jac_add(D, t, D);  // D
  if (stash) {
    *stash = D;
    __asm__ volatile("" ::: "memory");  // reload D after the ladder, not kept live
  }
  jac_mul_xabs(t, B);  // C
  jac_neg(t, t);
  if (stash) D = *stash;
  jac_add(r, D, t);
}

// One half of hash_to_curve: u_j = hash_to_field(msg)[j] -> SSWU -> iso (Jacobian).
// Two lanes per message run j = 0, 1 concurrently (the halves are independent).
LB_DEV void hash_to_g2_half(g2j& r, const uint8_t msg[32], int j) {
  uint32_t ub[64];
  expand_message_xmd_32(ub, msg);
  fp2 u;
  fp_from_64be_words(u.c0, ub + 32 * j);
  fp_from_64be_words(u.c1, ub + 32 * j + 16);
  g2a q;
  map_to_curve_sswu(q, u);
  iso_map_g2(r, q);
}
// Q0 + Q1 -> clear_cofactor
LB_DEV void hash_to_g2_finish(g2j& r, const g2j& q0, const g2j& q1, g2j* stash = nullptr) {
  g2j s;
  jac_add(s, q0, q1);
  clear_cofactor_g2(r, s, stash);
}

// hash_to_curve(msg) -> Jacobian point of G2
LB_DEV void hash_to_g2(g2j& r, const uint8_t msg[32]) {
  fp2 u[2];
  hash_to_field_fp2_2(u, msg);
  g2a q0, q1;
  map_to_curve_sswu(q0, u[0]);
  map_to_curve_sswu(q1, u[1]);
  g2j j0, j1;
  iso_map_g2(j0, q0);
  iso_map_g2(j1, q1);
  jac_add(j0, j0, j1);
  clear_cofactor_g2(r, j0);
}

// Deterministic batch randomness (SURVEY.md §8c "Batch
// randomness"): w_i = LE64(SHA-256(seed[32] || LE32(i))[0..8]), 0 -> 1.
// The batch scalar is r_i = (w_i mod 2^32) + (w_i >> 32) lambda (mod r),
// lambda = -x^2: 2^64 distinct values like blst's 64-bit scalars, but applied
// as a 2 x 32-bit GLV multiplication (jac_mul_glv).
LB_DEV uint64_t batch_scalar(const uint8_t seed[32], uint32_t idx) {
  uint32_t st[8];
  sha256_init(st);
  sha_block blk;
  blk.clear();
  for (int i = 0; i < 32; i++) blk.put(i, seed[i]);
  blk.put(32, (uint8_t)idx);
  blk.put(33, (uint8_t)(idx >> 8));
  blk.put(34, (uint8_t)(idx >> 16));
  blk.put(35, (uint8_t)(idx >> 24));
  blk.put(36, 0x80);
  blk.w[15] = 36u * 8u;
  sha256_compress(st, blk.w);
  // digest bytes 0..7 as little-endian u64
  uint64_t r = 0;
  for (int i = 0; i < 8; i++) {
    const uint8_t byte = (uint8_t)(st[i >> 2] >> (24 - 8 * (i & 3)));
    r |= (uint64_t)byte << (8 * i);
  }
  return r == 0 ? 1 : r;
}

}  // namespace lb
