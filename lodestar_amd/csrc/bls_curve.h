// G1 (over Fp) and G2 (over Fp2) group law, endomorphisms, subgroup checks and
// ZCash point (de)serialisation for gfx950.  One lane per point.
//
// Reference semantics restated here (blst via @chainsafe/bls, not vendored):
//  * PublicKey.fromBytes / toBytes(uncompressed)  -- multithread/worker.ts:110-116,
//    multithread/jobItem.ts:59,80 (96-byte uncompressed affine G1, 0x40 = infinity)
//  * Signature.fromBytes(bytes, affine, validate=true) -- maybeBatch.ts:24,37,
//    jobItem.ts:73: 96-byte compressed or 192-byte uncompressed G2, then the
//    G2 subgroup check (psi(P) == [x]P, equivalent to [r]P == O on BLS12-381).
//  * PublicKey.aggregate / Signature.aggregate -- chain/bls/utils.ts:13,
//    jobItem.ts:80-81 (Jacobian sums).
#pragma once
#include "bls_field.h"

namespace lb {

// ---- overloads so the group law is written once for both fields ------------
LB_DEV void fadd(fp& r, const fp& a, const fp& b) { fp_add(r, a, b); }
LB_DEV void fadd(fp2& r, const fp2& a, const fp2& b) { fp2_add(r, a, b); }
LB_DEV void fsub(fp& r, const fp& a, const fp& b) { fp_sub(r, a, b); }
LB_DEV void fsub(fp2& r, const fp2& a, const fp2& b) { fp2_sub(r, a, b); }
LB_DEV void fdbl(fp& r, const fp& a) { fp_dbl(r, a); }
LB_DEV void fdbl(fp2& r, const fp2& a) { fp2_dbl(r, a); }
LB_DEV void fneg(fp& r, const fp& a) { fp_neg(r, a); }
LB_DEV void fneg(fp2& r, const fp2& a) { fp2_neg(r, a); }
LB_DEV void fmul(fp& r, const fp& a, const fp& b) { fp_mul(r, a, b); }
LB_DEV void fmul(fp2& r, const fp2& a, const fp2& b) { fp2_mul(r, a, b); }
LB_DEV void fsqr(fp& r, const fp& a) { fp_sqr(r, a); }
LB_DEV void fsqr(fp2& r, const fp2& a) { fp2_sqr(r, a); }
LB_DEV void finv(fp& r, const fp& a) { fp_inv(r, a); }
LB_DEV void finv(fp2& r, const fp2& a) { fp2_inv(r, a); }
LB_DEV bool fis_zero(const fp& a) { return fp_is_zero(a); }
LB_DEV bool fis_zero(const fp2& a) { return fp2_is_zero(a); }
LB_DEV bool feq(const fp& a, const fp& b) { return fp_eq(a, b); }
LB_DEV bool feq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
LB_DEV void fzero(fp& r) { fp_zero(r); }
LB_DEV void fzero(fp2& r) { fp2_zero(r); }
LB_DEV void fone(fp& r) { fp_one(r); }
LB_DEV void fone(fp2& r) { fp2_one(r); }

template <class F>
struct jac {
  F X, Y, Z;  // x = X/Z^2, y = Y/Z^3; Z == 0 <=> infinity
};
template <class F>
struct aff {
  F x, y;
  bool inf;
};
typedef jac<fp> g1j;
typedef jac<fp2> g2j;
typedef aff<fp> g1a;
typedef aff<fp2> g2a;

template <class F>
LB_DEV void jac_set_inf(jac<F>& r) {
  fone(r.X);
  fone(r.Y);
  fzero(r.Z);
}
template <class F>
LB_DEV bool jac_is_inf(const jac<F>& p) {
  return fis_zero(p.Z);
}
template <class F>
LB_DEV void jac_from_aff(jac<F>& r, const aff<F>& a) {
  if (a.inf) {
    jac_set_inf(r);
  } else {
    r.X = a.x;
    r.Y = a.y;
    fone(r.Z);
  }
}
template <class F>
LB_DEV void jac_neg(jac<F>& r, const jac<F>& p) {
  r.X = p.X;
  fneg(r.Y, p.Y);
  r.Z = p.Z;
}

// The group law below is written register-lean: each formula computes Z3 as
// soon as its inputs allow, so the input Z (and Z^2) die early; a G2 point is
// 72 VGPRs and every out-of-line Fp product clobbers v0-v50, so the order in
// which intermediates die decides whether a 2-waves/SIMD kernel spills.

// dbl-2009-l (a = 0): 2M + 5S.  Z3 = 2YZ, so 2-torsion and infinity map to Z3 = 0.
template <class F>
LB_DEV void jac_dbl_impl(jac<F>& r, const jac<F>& p) {
  F A, B, C, D, E, t;
  F Z3;
  fmul(Z3, p.Y, p.Z);  // first: p.Z dies here
  fdbl(Z3, Z3);
  fsqr(B, p.Y);
  fsqr(A, p.X);
  fadd(t, p.X, B);
  fsqr(C, B);
  fsqr(t, t);
  fsub(t, t, A);
  fsub(t, t, C);
  fdbl(D, t);
  fdbl(E, A);
  fadd(E, E, A);
  fsqr(t, E);  // F = E^2
  F X3;
  fsub(X3, t, D);
  fsub(X3, X3, D);
  fsub(t, D, X3);
  F Y3;
  fmul(Y3, E, t);
  fdbl(C, C);
  fdbl(C, C);
  fdbl(C, C);
  fsub(Y3, Y3, C);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// add-2007-bl with the exceptional cases resolved (P == Q -> dbl, P == -Q -> O);
// W = 2 Z1 Z2 = (Z1 + Z2)^2 - Z1Z1 - Z2Z2 first, so Z1, Z2 die early.
template <class F>
LB_DEV void jac_add_impl(jac<F>& r, const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) {
    r = q;
    return;
  }
  if (jac_is_inf(q)) {
    r = p;
    return;
  }
  F Z1Z1, Z2Z2, W, U1, U2, S1, S2, H, Rr, t;
  fsqr(Z1Z1, p.Z);
  fsqr(Z2Z2, q.Z);
  fadd(W, p.Z, q.Z);
  fsqr(W, W);
  fsub(W, W, Z1Z1);
  fsub(W, W, Z2Z2);
  fmul(t, q.Z, Z2Z2);
  fmul(S1, p.Y, t);
  fmul(t, p.Z, Z1Z1);
  fmul(S2, q.Y, t);
  fmul(U1, p.X, Z2Z2);
  fmul(U2, q.X, Z1Z1);
  fsub(H, U2, U1);
  fsub(Rr, S2, S1);
  if (fis_zero(H)) {
    if (fis_zero(Rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  jac<F> o;
  fmul(o.Z, W, H);
  F I, J, V;
  fdbl(I, H);
  fsqr(I, I);
  fmul(J, H, I);
  fmul(V, U1, I);
  fdbl(Rr, Rr);
  fsqr(o.X, Rr);
  fsub(o.X, o.X, J);
  fsub(o.X, o.X, V);
  fsub(o.X, o.X, V);
  fsub(t, V, o.X);
  fmul(o.Y, Rr, t);
  fmul(t, S1, J);
  fdbl(t, t);
  fsub(o.Y, o.Y, t);
  r = o;
}

// madd-2007-bl: p Jacobian + q affine; Z3 = (Z1 + H)^2 - Z1Z1 - HH as soon as H is known.
template <class F>
LB_DEV void jac_add_aff_impl(jac<F>& r, const jac<F>& p, const aff<F>& q) {
  if (q.inf) {
    r = p;
    return;
  }
  if (jac_is_inf(p)) {
    jac_from_aff(r, q);
    return;
  }
  F Z1Z1, U2, S2, H, HH, Rr, t;
  fsqr(Z1Z1, p.Z);
  fmul(t, p.Z, Z1Z1);
  fmul(S2, q.y, t);
  fmul(U2, q.x, Z1Z1);
  fsub(H, U2, p.X);
  fsub(Rr, S2, p.Y);
  if (fis_zero(H)) {
    if (fis_zero(Rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  jac<F> o;
  fsqr(HH, H);
  fadd(t, p.Z, H);
  fsqr(t, t);
  fsub(t, t, Z1Z1);
  fsub(o.Z, t, HH);
  F I, J, V;
  fdbl(I, HH);
  fdbl(I, I);
  fmul(J, H, I);
  fmul(V, p.X, I);
  fdbl(Rr, Rr);
  fsqr(o.X, Rr);
  fsub(o.X, o.X, J);
  fsub(o.X, o.X, V);
  fsub(o.X, o.X, V);
  fsub(t, V, o.X);
  fmul(o.Y, Rr, t);
  fmul(t, p.Y, J);
  fdbl(t, t);
  fsub(o.Y, o.Y, t);
  r = o;
}

// G1 point ops always inline; G2 point ops follow LB_TOWER (see bls_field.h).
LB_DEV void jac_dbl(g1j& r, const g1j& p) { jac_dbl_impl(r, p); }
LB_DEV void jac_add(g1j& r, const g1j& p, const g1j& q) { jac_add_impl(r, p, q); }
LB_DEV void jac_add_aff(g1j& r, const g1j& p, const g1a& q) { jac_add_aff_impl(r, p, q); }
LB_TOWER void jac_dbl(g2j& r, const g2j& p) { jac_dbl_impl(r, p); }
LB_TOWER void jac_add(g2j& r, const g2j& p, const g2j& q) { jac_add_impl(r, p, q); }
LB_TOWER void jac_add_aff(g2j& r, const g2j& p, const g2a& q) { jac_add_aff_impl(r, p, q); }

template <class F>
LB_DEV void jac_to_aff(aff<F>& r, const jac<F>& p) {
  if (jac_is_inf(p)) {
    fzero(r.x);
    fzero(r.y);
    r.inf = true;
    return;
  }
  F zi, zi2, zi3;
  finv(zi, p.Z);
  fsqr(zi2, zi);
  fmul(zi3, zi2, zi);
  fmul(r.x, p.X, zi2);
  fmul(r.y, p.Y, zi3);
  r.inf = false;
}

// Affine forms of a G1 and a G2 point with ONE shared Fp inversion
// (Montgomery's trick over the pair): with t = Z1 N(Z2),
//   1/Z1 = N(Z2)/t,  1/Z2 = conj(Z2) Z1/t.
// Saves one of the two ~460-product exponentiations per verified set (the
// pipeline needs r_i pk_i and H(m_i) affine for the Miller loop).
LB_DEV void jac_pair_to_aff(g1a& pa, g2a& qa, const g1j& p, const g2j& q) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  fp one, z1, n2, e, t, ti, z1i, n2i, zi2, zi3;
  fp_one(one);
  z1 = p.Z;
  fp_cmov(z1, one, pi);
  fp_sqr(n2, q.Z.c0);
  fp_sqr(e, q.Z.c1);
  fp_add(n2, n2, e);
  fp_cmov(n2, one, qi);
  fp_mul(t, z1, n2);
  fp_inv(ti, t);
  fp_mul(z1i, ti, n2);
  fp_mul(n2i, ti, z1);
  // G1
  fp_sqr(zi2, z1i);
  fp_mul(zi3, zi2, z1i);
  fp_mul(pa.x, p.X, zi2);
  fp_mul(pa.y, p.Y, zi3);
  pa.inf = pi;
  // G2: 1/Z2 = conj(Z2) / N(Z2)
  fp2 z2i, w2, w3;
  fp2_conj(z2i, q.Z);
  fp2_mul_fp(z2i, z2i, n2i);
  fp2_sqr(w2, z2i);
  fp2_mul(w3, w2, z2i);
  fp2_mul(qa.x, q.X, w2);
  fp2_mul(qa.y, q.Y, w3);
  qa.inf = qi;
}

template <class F>
LB_DEV bool jac_eq(const jac<F>& p, const jac<F>& q) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1, z2z2, a, b;
  fsqr(z1z1, p.Z);
  fsqr(z2z2, q.Z);
  fmul(a, p.X, z2z2);
  fmul(b, q.X, z1z1);
  if (!feq(a, b)) return false;
  fmul(z1z1, z1z1, p.Z);
  fmul(z2z2, z2z2, q.Z);
  fmul(a, p.Y, z2z2);
  fmul(b, q.Y, z1z1);
  return feq(a, b);
}

// [k]P, k a 64-bit scalar (batch-verification randomness), left to right.
template <class F>
LB_DEV void jac_mul_u64(jac<F>& r, const jac<F>& p, uint64_t k) {
  jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int i = 63; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((k >> i) & 1ull) jac_add(acc, acc, p);
  }
  r = acc;
}

// Field element times an Fp scalar (an Fp2 scales coefficient-wise).
LB_DEV void fmul_fp(fp& r, const fp& a, const fp& k) { fp_mul(r, a, k); }
LB_DEV void fmul_fp(fp2& r, const fp2& a, const fp& k) { fp2_mul_fp(r, a, k); }

// Shared-Z ladders.  A Jacobian point P = (X, Y, Z) is the affine point (X, Y)
// of the isomorphic curve y^2 = x^3 + b Z^6, and so is every point (c X, +-Y, Z)
// of the same Z; dbl-2009-l and madd-2007-bl do not involve b, so a ladder over
// such points runs on that curve with mixed additions (7M + 4S instead of the
// 11M + 5S of a Jacobian addition), and its result (X', Y', Z') there is
// (X', Y', Z' Z) here.

// [a + b lambda]P for the batch-randomness scalar r = a + b lambda (mod r),
// a, b = the 32-bit halves of the 64-bit DRBG output, lambda = -x^2.  lambda is
// a primitive cube root of unity mod r (lambda^2 + lambda + 1 = x^4 - x^2 + 1 =
// r), so with [lambda]P = (w X, Y, Z) (phi on G1: w = beta; -psi^2 on G2: w in
// Fp, LB_G2_OMEGA) the joint table is free: P + [lambda]P = -[lambda^2]P =
// (w^2 X, -Y, Z).  Straus-Shamir over 32 bit pairs: 32 doublings + 32 mixed
// additions per wave (a wave adds as soon as ONE lane's bit pair is non-zero),
// the table selected with conditional moves (no private-memory table).
// The ladder runs on the shared-Z curve; the caller multiplies the result's Z
// by P's Z (jac_mul_glv), or knows it is 1.  LB_GLV_TABLE_REGS keeps w X and
// w^2 X in registers; by default they are recomputed per step (2 Fp products)
// to keep the live state at acc + (X, Y).
template <class F>
LB_DEV void jac_mul_glv_xy(jac<F>& r, const F& X, const F& Y, const uint32_t* w_c, const uint32_t* w2_c,
                           uint64_t raw) {
  const uint32_t a = (uint32_t)raw, b = (uint32_t)(raw >> 32);
#ifdef LB_GLV_TABLE_REGS
  F xw, xw2;
  {
    fp w;
    fp_set(w, w_c);
    fmul_fp(xw, X, w);
    fp_set(w, w2_c);
    fmul_fp(xw2, X, w);
  }
#endif
  jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int i = 31; i >= 0; i--) {
    jac_dbl(acc, acc);
    const uint32_t sel = ((a >> i) & 1u) | (((b >> i) & 1u) << 1);
    if (sel) {
      aff<F> q;
      q.inf = false;
#ifdef LB_GLV_TABLE_REGS
      q.x = sel == 1 ? X : sel == 2 ? xw : xw2;
#else
      if (sel == 1) {
        q.x = X;
      } else {
        fp w;
        fp_set(w, sel == 2 ? w_c : w2_c);
        fmul_fp(q.x, X, w);
      }
#endif
      q.y = Y;
      if (sel == 3) fneg(q.y, Y);
      jac_add_aff(acc, acc, q);
    }
  }
  r = acc;
}
template <class F>
LB_DEV void jac_mul_glv(jac<F>& r, const jac<F>& p, const uint32_t* w_c, const uint32_t* w2_c, uint64_t raw) {
  if (jac_is_inf(p)) {
    jac_set_inf(r);
    return;
  }
  jac_mul_glv_xy(r, p.X, p.Y, w_c, w2_c, raw);
  fmul(r.Z, r.Z, p.Z);
}

// [k]P for a 32-byte big-endian scalar (secret keys: SecretKey.fromBytes is BE)
template <class F>
LB_DEV void jac_mul_be32(jac<F>& r, const jac<F>& p, const uint8_t k[32]) {
  jac<F> acc;
  jac_set_inf(acc);
  for (int i = 0; i < 256; i++) {
    jac_dbl(acc, acc);
    if ((k[i >> 3] >> (7 - (i & 7))) & 1) jac_add(acc, acc, p);
  }
  r = acc;
}

// [|x|]P for the BLS parameter |x| = 0xd201000000010000 (fixed bit pattern:
// 63 doublings, 5 additions; the branch is wave-uniform).
// Shared-Z ladder (above): the 5 additions are mixed additions of (X, Y).
template <class F>
LB_DEV void jac_mul_xabs(jac<F>& r, const jac<F>& p) {
  if (jac_is_inf(p)) {
    r = p;
    return;
  }
  aff<F> q;
  q.x = p.X;
  q.y = p.Y;
  q.inf = false;
  jac<F> acc;
  jac_from_aff(acc, q);
  // rolled: unrolled, the 63 inlined doublings made k_hash_finish (two ladders) 514 KB of
  // straight-line code against a 64 KB instruction cache (the bit test is wave-uniform)
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((LB_X_ABS >> i) & 1ull) jac_add_aff(acc, acc, q);
  }
  fmul(acc.Z, acc.Z, p.Z);
  r = acc;
}

// ---- curve equations --------------------------------------------------------
LB_DEV bool g1_aff_on_curve(const g1a& a) {
  if (a.inf) return true;
  fp l, rr, b;
  fp_sqr(l, a.y);
  fp_sqr(rr, a.x);
  fp_mul(rr, rr, a.x);
  fp_set(b, LB_B1);
  fp_add(rr, rr, b);
  return fp_eq(l, rr);
}
LB_DEV bool g2_aff_on_curve(const g2a& a) {
  if (a.inf) return true;
  fp2 l, rr, b;
  fp2_sqr(l, a.y);
  fp2_sqr(rr, a.x);
  fp2_mul(rr, rr, a.x);
  fp2_set(b, LB_B2);
  fp2_add(rr, rr, b);
  return fp2_eq(l, rr);
}

// psi(x, y) = (conj(x) cx, conj(y) cy) on Jacobian coordinates
LB_DEV void g2_psi(g2j& r, const g2j& p) {
  fp2 t;
  fp2_conj(t, p.X);
  fp2_mul_const(r.X, t, LB_PSI_CX);
  fp2_conj(t, p.Y);
  fp2_mul_const(r.Y, t, LB_PSI_CY);
  fp2_conj(r.Z, p.Z);
}

// GLV endomorphisms with eigenvalue lambda = -x^2 (mod r) on G1 and G2:
//   G1: phi(x, y) = (beta x, y)      (the map g1_in_subgroup checks)
//   G2: -psi^2, since psi = [x] on G2 (the map g2_in_subgroup checks)
LB_DEV void g1_glv_endo(g1j& r, const g1j& p) {
  r = p;
  fp_mul_const(r.X, p.X, LB_G1_BETA);
}
LB_DEV void g2_glv_endo(g2j& r, const g2j& p) {
  g2j t;
  g2_psi(t, p);
  g2_psi(t, t);
  jac_neg(r, t);
}

// G2 membership: psi(P) == [x]P = -[|x|]P  (Scott 2021; blst POINTonE2_in_G2).
LB_DEV bool g2_in_subgroup(const g2j& p) {
  if (jac_is_inf(p)) return true;
  g2j xp, ps;
  jac_mul_xabs(xp, p);
  jac_neg(xp, xp);
  g2_psi(ps, p);
  return jac_eq(ps, xp);
}

// G1 membership: phi(P) == [-x^2]P with phi(x, y) = (beta x, y).
LB_DEV bool g1_in_subgroup(const g1j& p) {
  if (jac_is_inf(p)) return true;
  g1j t;
  jac_mul_xabs(t, p);
  jac_mul_xabs(t, t);  // [x^2]P
  jac_neg(t, t);
  g1j ph = p;
  fp_mul_const(ph.X, p.X, LB_G1_BETA);
  return jac_eq(ph, t);
}

// ---- ZCash serialisation ---------------------------------------------------
enum : uint8_t {
  LB_ST_OK = 0,
  LB_ST_BAD_ENCODING = 1,
  LB_ST_NOT_ON_CURVE = 2,
  LB_ST_NOT_IN_GROUP = 3,
  LB_ST_PK_INFINITY = 4,
  LB_ST_EMPTY_AGGREGATE = 5,
};

LB_DEV bool bytes_zero(const uint8_t* b, int n) {
  uint32_t acc = 0;
  for (int i = 0; i < n; i++) acc |= b[i];
  return acc == 0;
}

// 48 big-endian bytes (with the 3 flag bits masked) -> Montgomery fp; false if >= p
LB_DEV bool fp_read_masked(fp& r, const uint8_t* b, bool mask_flags) {
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  if (mask_flags) tmp[0] &= 0x1f;
  fp raw;
  if (!fp_from_be48_raw(raw, tmp)) return false;
  fp_to_mont(r, raw);
  return true;
}

// POINTonE1_Deserialize_Z + the binding's length rule (48 iff compressed).
LB_DEV uint8_t g1_deserialize(g1a& out, const uint8_t* b, uint32_t len) {
  out.inf = false;
  if (len == 0) return LB_ST_BAD_ENCODING;
  const uint8_t f = b[0];
  const bool comp = (f & 0x80) != 0;
  if (len != (comp ? 48u : 96u)) return LB_ST_BAD_ENCODING;
  if (comp) {
    if (f & 0x40) {
      if ((f & 0x3f) == 0 && bytes_zero(b + 1, 47)) {
        out.inf = true;
        fp_zero(out.x);
        fp_zero(out.y);
        return LB_ST_OK;
      }
      return LB_ST_BAD_ENCODING;
    }
    if (!fp_read_masked(out.x, b, true)) return LB_ST_BAD_ENCODING;
    fp rhs, bb;
    fp_sqr(rhs, out.x);
    fp_mul(rhs, rhs, out.x);
    fp_set(bb, LB_B1);
    fp_add(rhs, rhs, bb);
    if (!fp_sqrt(out.y, rhs)) return LB_ST_NOT_ON_CURVE;
    if (fp_lex_largest(out.y) != ((f & 0x20) != 0)) fp_neg(out.y, out.y);
    return LB_ST_OK;
  }
  if (f & 0xe0) {
    if ((f & 0x40) && (f & 0x3f) == 0 && bytes_zero(b + 1, 95)) {
      out.inf = true;
      fp_zero(out.x);
      fp_zero(out.y);
      return LB_ST_OK;
    }
    return LB_ST_BAD_ENCODING;
  }
  if (!fp_read_masked(out.x, b, false)) return LB_ST_BAD_ENCODING;
  if (!fp_read_masked(out.y, b + 48, false)) return LB_ST_BAD_ENCODING;
  if (!g1_aff_on_curve(out)) return LB_ST_NOT_ON_CURVE;
  if (fp_is_zero(out.x) && fp_is_zero(out.y)) return LB_ST_NOT_IN_GROUP;
  return LB_ST_OK;
}

// POINTonE2_Deserialize_Z + length rule (96 iff compressed); x = (c1 || c0).
LB_DEV uint8_t g2_deserialize(g2a& out, const uint8_t* b, uint32_t len) {
  out.inf = false;
  if (len == 0) return LB_ST_BAD_ENCODING;
  const uint8_t f = b[0];
  const bool comp = (f & 0x80) != 0;
  if (len != (comp ? 96u : 192u)) return LB_ST_BAD_ENCODING;
  if (comp) {
    if (f & 0x40) {
      if ((f & 0x3f) == 0 && bytes_zero(b + 1, 95)) {
        out.inf = true;
        fp2_zero(out.x);
        fp2_zero(out.y);
        return LB_ST_OK;
      }
      return LB_ST_BAD_ENCODING;
    }
    if (!fp_read_masked(out.x.c1, b, true)) return LB_ST_BAD_ENCODING;
    if (!fp_read_masked(out.x.c0, b + 48, false)) return LB_ST_BAD_ENCODING;
    fp2 rhs, bb;
    fp2_sqr(rhs, out.x);
    fp2_mul(rhs, rhs, out.x);
    fp2_set(bb, LB_B2);
    fp2_add(rhs, rhs, bb);
    if (!fp2_sqrt(out.y, rhs)) return LB_ST_NOT_ON_CURVE;
    if (fp2_lex_largest(out.y) != ((f & 0x20) != 0)) fp2_neg(out.y, out.y);
    return LB_ST_OK;
  }
  if (f & 0xe0) {
    if ((f & 0x40) && (f & 0x3f) == 0 && bytes_zero(b + 1, 191)) {
      out.inf = true;
      fp2_zero(out.x);
      fp2_zero(out.y);
      return LB_ST_OK;
    }
    return LB_ST_BAD_ENCODING;
  }
  if (!fp_read_masked(out.x.c1, b, false)) return LB_ST_BAD_ENCODING;
  if (!fp_read_masked(out.x.c0, b + 48, false)) return LB_ST_BAD_ENCODING;
  if (!fp_read_masked(out.y.c1, b + 96, false)) return LB_ST_BAD_ENCODING;
  if (!fp_read_masked(out.y.c0, b + 144, false)) return LB_ST_BAD_ENCODING;
  if (!g2_aff_on_curve(out)) return LB_ST_NOT_ON_CURVE;
  if (fp2_is_zero(out.x) && fp2_is_zero(out.y)) return LB_ST_NOT_IN_GROUP;
  return LB_ST_OK;
}

LB_DEV void fp_write_be(uint8_t* out, const fp& a) {
  fp raw;
  fp_from_mont(raw, a);
  fp_to_be48_raw(out, raw);
}

// blst_p1_affine_serialize / POINTonE1_Serialize (uncompressed, 96 bytes)
LB_DEV void g1_serialize(uint8_t* out, const g1a& a) {
  if (a.inf) {
    for (int i = 0; i < 96; i++) out[i] = 0;
    out[0] = 0x40;
    return;
  }
  fp_write_be(out, a.x);
  fp_write_be(out + 48, a.y);
}
LB_DEV void g1_compress(uint8_t* out, const g1a& a) {
  if (a.inf) {
    for (int i = 0; i < 48; i++) out[i] = 0;
    out[0] = 0xc0;
    return;
  }
  fp_write_be(out, a.x);
  out[0] |= 0x80 | (fp_lex_largest(a.y) ? 0x20 : 0);
}
LB_DEV void g2_serialize(uint8_t* out, const g2a& a) {
  if (a.inf) {
    for (int i = 0; i < 192; i++) out[i] = 0;
    out[0] = 0x40;
    return;
  }
  fp_write_be(out, a.x.c1);
  fp_write_be(out + 48, a.x.c0);
  fp_write_be(out + 96, a.y.c1);
  fp_write_be(out + 144, a.y.c0);
}
LB_DEV void g2_compress(uint8_t* out, const g2a& a) {
  if (a.inf) {
    for (int i = 0; i < 96; i++) out[i] = 0;
    out[0] = 0xc0;
    return;
  }
  fp_write_be(out, a.x.c1);
  fp_write_be(out + 48, a.x.c0);
  out[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
}

}  // namespace lb
