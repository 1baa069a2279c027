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
  // fully unrolled: the schedule's ring w[] then lives in registers (a rolled loop
  // indexes it dynamically, i.e. in scratch memory -- a memory round trip per round,
  // which a lone set's k_lp_prep waits out 19 times 64)
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = win[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
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
  // the state after the all-zero Z_pad block is a constant: SHA-256's compression of one zero
  // block from the initial state (checked against hashlib in tests/test_oracle_kats.py)
  uint32_t st[8] = {0xda5698beu, 0x17b9b469u, 0x62335799u, 0x779fbecau,
                    0x8ce5d491u, 0xc0d26243u, 0xbafef9eau, 0x1837a9d8u};
  sha_block blk;
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

// sqrt(W / m) in Fp2 (W / m a square; m in Fp), given s with s^2 = N(W), with no
// inversion: with t = (W0 + s) / 2 and c = (t m)^((p-3)/4), z = t c satisfies
// z^2 = (t / m) chi(t m) and 1 / z = c m (chi = 1), so
//   chi(t m) = 1  -> y = (z, W1 c / 2)
//   chi(t m) = -1 -> y = (-W1 c / 2, z)     ((W0 - s) / 2 is the square then)
// W1 = 0 (W / m in Fp, probability ~2^-381 on hashed input): sqrt(u / v) =
// u (u v)^((p-3)/4), or i sqrt(-u / v).  Which root comes out does not matter
// (the caller fixes the sign).  Step for step in tests/test_sswu_fraction.py.
LB_DEV void fp2_sqrt_ratio_frac(fp2& y, const fp2& W, const fp& m, const fp& s) {
  fp half, t, c, z, chk, a1c, na1c;
  fp_set(half, LB_HALF);
  if (fp_is_zero(W.c1)) {
    fp u = W.c0;
    fp_mul(t, u, m);
    fp_pow_p34(c, t);
    fp_mul(z, u, c);
    fp_sqr(chk, z);
    fp_mul(chk, chk, m);
    if (fp_eq(chk, u)) {
      y.c0 = z;
      fp_zero(y.c1);
    } else {
      fp_neg(u, u);
      fp_mul(t, u, m);
      fp_pow_p34(c, t);
      fp_zero(y.c0);
      fp_mul(y.c1, u, c);
    }
    return;
  }
  fp_add(t, W.c0, s);
  fp_mul(t, t, half);
  fp_mul(c, t, m);
  fp_pow_p34(c, c);
  fp_mul(z, t, c);
  fp_sqr(chk, z);
  fp_mul(chk, chk, m);
  fp_mul(a1c, W.c1, c);
  fp_mul(a1c, a1c, half);
  const bool direct = fp_eq(chk, t);
  fp_neg(na1c, a1c);
  y.c0 = z;
  y.c1 = a1c;
  fp_cmov(y.c0, na1c, !direct);
  fp_cmov(y.c1, z, !direct);
}

// Simplified SWU onto E2': y^2 = x^3 + A'x + B' (RFC 9380 §6.6.2) followed by the
// 3-isogeny to E2, with no inversion anywhere (no binary GCD
// in k_hash_half).  x1 = n / d is kept as a fraction,
//   n = -B (tv2 + 1), d = A tv2   (tv2 = Z^2 u^4 + Z u^2; tv2 = 0: n = B, d = Z A),
// g(x1) = U / V with U = n^3 + A n d^2 + B d^3, V = d^3, and U / V = W / m with
// W = U conj(V), m = N(V) in Fp.  ONE exponentiation e = N(W)^((p-3)/4) gives the
// square test of g(x1) and sqrt N(W) = N(W) e; for x2 = Z u^2 x1 (g(x2) = Z^3 u^6
// g(x1), W2 = (Z u^2)^3 W) the norm root is N(u)^3 sqrt(-N(Z)^3) N(W) e, as before.
// fp2_sqrt_ratio_frac finishes the affine y (its sign fixed against u).  The
// isogeny is homogenised in (x_n, d): XN = xn(x) d^3, XD = xd(x) d^2, YN = yn(x) d^3,
// YD = yd(x) d^3, so x_E = XN / (XD d), y_E = y YN / YD and the Jacobian output is
//   Z = XD d YD,  X = XN XD d YD^2,  Y = y YN (XD d)^3 YD^2.
LB_DEV void map_to_g2_sswu_iso(g2j& r, const fp2& u) {
  fp2 A, B, Zc, tv1, tv2, n, d, d2, d3, U, W, t;
  fp2_set(A, LB_SSWU_A);
  fp2_set(B, LB_SSWU_B);
  fp2_set(Zc, LB_SSWU_Z);
  fp2_sqr(tv1, u);
  fp2_mul(tv1, Zc, tv1);  // Z u^2
  fp2_sqr(tv2, tv1);
  fp2_add(tv2, tv2, tv1);  // Z^2 u^4 + Z u^2
  const bool exceptional = fp2_is_zero(tv2);
  fp2 one;
  fp2_one(one);
  fp2_add(t, tv2, one);
  fp2_mul(n, B, t);
  fp2_neg(n, n);
  fp2_mul(d, A, tv2);
  fp2 za;
  fp2_mul(za, Zc, A);
  fp2_cmov(n, B, exceptional);
  fp2_cmov(d, za, exceptional);
  fp2_sqr(d2, d);
  fp2_mul(d3, d2, d);
  // U = n (n^2 + A d^2) + B d^3
  fp2_mul(t, A, d2);
  fp2_sqr(U, n);
  fp2_add(U, U, t);
  fp2_mul(U, U, n);
  fp2_mul(t, B, d3);
  fp2_add(U, U, t);
  fp2 vc;
  fp2_conj(vc, d3);
  fp2_mul(W, U, vc);
  fp m, nW, e, chk, s1, s2, nu, c1;
  fp_sqr(m, d3.c0);
  fp_sqr(e, d3.c1);
  fp_add(m, m, e);  // N(V)
  fp_sqr(nW, W.c0);
  fp_sqr(e, W.c1);
  fp_add(nW, nW, e);
  fp_pow_p34(e, nW);
  fp_sqr(chk, e);
  fp_mul(chk, chk, nW);
  fp onep;
  fp_one(onep);
  const bool sq1 = fp_eq(chk, onep) || fp_is_zero(nW);
  fp_mul(s1, nW, e);
  fp_sqr(nu, u.c0);
  fp_sqr(e, u.c1);
  fp_add(nu, nu, e);
  fp_sqr(s2, nu);
  fp_mul(s2, s2, nu);
  fp_set(c1, LB_SSWU_NZ3_SQRT);
  fp_mul(s2, s2, c1);
  fp_mul(s2, s2, s1);
  fp_cmov(s2, s1, sq1);
  // x2 branch: x_n = tv1 n, W2 = tv1^3 W
  fp2 xn_, W2;
  fp2_mul(xn_, tv1, n);
  fp2_sqr(t, tv1);
  fp2_mul(t, t, tv1);
  fp2_mul(W2, t, W);
  fp2_cmov(xn_, n, sq1);
  fp2_cmov(W2, W, sq1);
  fp2 y;
  fp2_sqrt_ratio_frac(y, W2, m, s2);
  fp2 ny;
  fp2_neg(ny, y);
  fp2_cmov(y, ny, fp2_sgn0(u) != fp2_sgn0(y));
  // isogeny, Horner in x_n with the d powers (d, d2, d3 live)
  fp2 XN, XD, YN, YD;
  fp2_set(XN, LB_ISO_XNUM3);
  fp2_mul(XN, XN, xn_);
  fp2_mul_const(t, d, LB_ISO_XNUM2);
  fp2_add(XN, XN, t);
  fp2_mul(XN, XN, xn_);
  fp2_mul_const(t, d2, LB_ISO_XNUM1);
  fp2_add(XN, XN, t);
  fp2_mul(XN, XN, xn_);
  fp2_mul_const(t, d3, LB_ISO_XNUM0);
  fp2_add(XN, XN, t);

  fp2_mul_const(t, d, LB_ISO_XDEN1);
  fp2_add(XD, xn_, t);  // monic
  fp2_mul(XD, XD, xn_);
  fp2_mul_const(t, d2, LB_ISO_XDEN0);
  fp2_add(XD, XD, t);

  fp2_set(YN, LB_ISO_YNUM3);
  fp2_mul(YN, YN, xn_);
  fp2_mul_const(t, d, LB_ISO_YNUM2);
  fp2_add(YN, YN, t);
  fp2_mul(YN, YN, xn_);
  fp2_mul_const(t, d2, LB_ISO_YNUM1);
  fp2_add(YN, YN, t);
  fp2_mul(YN, YN, xn_);
  fp2_mul_const(t, d3, LB_ISO_YNUM0);
  fp2_add(YN, YN, t);

  fp2_mul_const(t, d, LB_ISO_YDEN2);
  fp2_add(YD, xn_, t);  // monic
  fp2_mul(YD, YD, xn_);
  fp2_mul_const(t, d2, LB_ISO_YDEN1);
  fp2_add(YD, YD, t);
  fp2_mul(YD, YD, xn_);
  fp2_mul_const(t, d3, LB_ISO_YDEN0);
  fp2_add(YD, YD, t);

  if (fp2_is_zero(XD) || fp2_is_zero(YD)) {  // kernel point -> infinity
    jac_set_inf(r);
    return;
  }
  fp2 XDd, YD2;
  fp2_mul(XDd, XD, d);
  fp2_mul(r.Z, XDd, YD);
  fp2_sqr(YD2, YD);
  fp2_mul(t, XN, XDd);
  fp2_mul(r.X, t, YD2);
  fp2_sqr(t, XDd);
  fp2_mul(t, t, XDd);  // (XD d)^3
  fp2_mul(YN, YN, y);
  fp2_mul(YN, YN, t);
  fp2_mul(r.Y, YN, YD2);
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

// Register-lean form of clear_cofactor_g2 for the throughput kernel (k_hash_finish):
// every point that is not being worked on waits in global memory (two per-lane slots),
// so across each |x|-ladder only its accumulator and the doubling's temporaries are
// live -- the base is re-read at the ladder's 5 additions and for the final Z product.
// The same operations in the same order as clear_cofactor_g2 (bit-identical output for
// a finite P; an infinite one gives an infinity of another X, Y).
// A compiler barrier before each re-read keeps it a load (no value held across the loop).
LB_DEV void g2_load_barrier(g2j& r, const g2j* m) {
  __asm__ volatile("" ::: "memory");
  r = *m;
}
LB_DEV void g2_mul_xabs_mem(g2j& r, const g2j* pm) {
  // (no branch on infinity: P = (X:Y:0) ends with Z = Z_acc * 0, infinity again)
  g2j acc;
  g2_load_barrier(acc, pm);
  fp2_one(acc.Z);
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((LB_X_ABS >> i) & 1ull) {
      __asm__ volatile("" ::: "memory");
      g2a q;
      q.x = pm->X;
      q.y = pm->Y;
      q.inf = false;
      jac_add_aff(acc, acc, q);
    }
  }
  __asm__ volatile("" ::: "memory");
  const fp2 z = pm->Z;
  fmul(acc.Z, acc.Z, z);
  r = acc;
}
// g2_in_subgroup (psi(P) == [x]P) with P (not infinity) in memory: across the ladder
// only its accumulator is live (k_decode_sigs parks the decoded point in its output slot).
LB_DEV bool g2_in_subgroup_mem(const g2j* pm) {
  g2j xp, ps;
  g2_mul_xabs_mem(xp, pm);
  jac_neg(xp, xp);
  g2_load_barrier(ps, pm);
  g2_psi(ps, ps);
  return jac_eq(ps, xp);
}

// On entry sP holds P; sB is a second slot.  r = h_eff P.
LB_DEV void clear_cofactor_g2_mem(g2j& r, g2j* sP, g2j* sB) {
  g2j A, B, t, D;
  g2_mul_xabs_mem(A, sP);  // A = [z]P
  g2_load_barrier(t, sP);
  g2_psi(B, t);
  jac_neg(A, A);
  jac_add(B, B, A);  // B = psi(P) - A
  *sB = B;
  g2_load_barrier(t, sP);
  jac_neg(D, t);
  jac_dbl(t, t);
  g2_psi(t, t);
  g2_psi(t, t);      // psi^2(2P)
  jac_add(t, t, D);  // psi^2(2P) - P
  g2_load_barrier(B, sB);
  jac_neg(D, B);
  jac_add(D, t, D);  // D
  *sP = D;           // (P is no longer needed)
  g2_mul_xabs_mem(t, sB);  // C
  jac_neg(t, t);
  g2_load_barrier(D, sP);
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
  map_to_g2_sswu_iso(r, u);
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
  g2j j0, j1;
  map_to_g2_sswu_iso(j0, u[0]);
  map_to_g2_sswu_iso(j1, u[1]);
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
