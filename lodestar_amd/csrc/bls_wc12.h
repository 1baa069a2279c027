// Wave-cooperative Fp12 arithmetic for the per-request tails on gfx950.
//
// The tails of a verification -- the Miller loop of (-g1, S_k) and the final
// exponentiation -- are single Fp12 dependency chains (~10k Fp products).  One
// lane per request runs them in 15-20 ms regardless of batch size.  Here one
// wave per request runs each Fp12 operation as ONE round of parallel Fp
// products (lane k computes product k, K = 18 ... 54 per op) followed by the
// linear combinations that form the 12 output coefficients (lanes 0..11),
// with the operands in LDS.  The programs (which linear forms to multiply,
// how to combine) are generated from the same tower formulas as bls_field.h by
// gen_wc12.py and pinned against the oracle by tests/test_wc12_programs.py.
#pragma once
#include "bls_pairing.h"
#include "bls_wc12_tables.h"

namespace lb {

// LDS slots of one wave (each an Fp12 as 12 Fp coefficients in tower order)
enum : int {
  WC_F = 0,   // input / scratch
  WC_T0,
  WC_T1,
  WC_F2,
  WC_A,
  WC_B,
  WC_C,
  WC_ACC,
  WC_FS,      // Miller value of (-g1, S)
  WC_LINE,    // current line (B[0..5])
  WC_G1,      // Frobenius constants gamma_{k,e} at B[2e], B[2e+1]
  WC_G2,
  WC_G3,
  WC_NSLOTS
};
struct wc_smem {
  fp slot[WC_NSLOTS][12];
  fp prod[64];
  fp part[64];
  // the op programs, copied from constant memory once per kernel: every lane
  // walks its own term list, and lane-divergent constant/global loads on that
  // path would put a memory round trip under every term
  wc_desc ops[LB_WC_NOPS];
  uint16_t term[LB_WC_NTERMS];  // coef << 8 | code
};

LB_DEV void wc_init_tables(wc_smem& S) {
  for (int t = threadIdx.x; t < LB_WC_NTERMS; t += blockDim.x)
    S.term[t] = (uint16_t)((uint8_t)LB_WC_COEF[t] << 8 | LB_WC_CODE[t]);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(LB_WC_OPS);
  uint32_t* dst = reinterpret_cast<uint32_t*>(S.ops);
  for (int t = threadIdx.x; t < (int)(sizeof(S.ops) / 4); t += blockDim.x) dst[t] = src[t];
  __syncthreads();
}

// ---- lazy accumulation: a lane sums up to 8 (|coef|-weighted) canonical terms
// (the signed sum plus the negative weight times p stays in [0, 8p), 8p < 2^384),
// then reduces once with conditional subtractions of 4p, 2p, p.
static constexpr uint32_t WC_P2[12] = LB_P2_LIMBS;
static constexpr uint32_t WC_P4[12] = LB_P4_LIMBS;

struct lz {
  uint32_t l[12];
};
// a -= m if a >= m
LB_DEV void lz_csub(lz& a, const uint32_t* m) {
  uint32_t s[12], br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = __builtin_subc(a.l[j], m[j], br, &br);
#pragma unroll
  for (int j = 0; j < 12; j++) a.l[j] = br ? a.l[j] : s[j];
}
// sum of the terms [t0, t1) (values val(code)) into r, reduced to < 2p
// (operands of fp_mul: x y < 4p^2 < p R) or to < p (canonical outputs).
// Limb-wise 64-bit accumulation: positive terms into P, negative ones into N,
// no carry chain per term (a 12-limb carry chain pads every step with s_nop on
// gfx950); one signed carry pass at the end forms P - N + kneg p, kneg = the
// negative weight, which is >= 0 and < w p <= 8p < 2^384.
template <class Val>
LB_DEV void lz_sum(fp& r, const uint16_t* term, int t0, int t1, Val val, bool canonical) {
  uint64_t P[12], N[12];
#pragma unroll
  for (int j = 0; j < 12; j++) P[j] = N[j] = 0;
  int w = 0;
  uint32_t kneg = 0;
  for (int t = t0; t < t1; t++) {
    const uint16_t tm = term[t];
    const int c = (int8_t)(tm >> 8);
    const fp& v = val(tm & 255);
    if (c > 0) {
      for (int q = 0; q < c; q++) {
#pragma unroll
        for (int j = 0; j < 12; j++) P[j] += v.l[j];
      }
      w += c;
    } else {
      for (int q = 0; q < -c; q++) {
#pragma unroll
        for (int j = 0; j < 12; j++) N[j] += v.l[j];
      }
      w -= c;
      kneg += (uint32_t)(-c);
    }
  }
  lz a;
  int64_t carry = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const int64_t t = (int64_t)P[j] - (int64_t)N[j] + (int64_t)((uint64_t)P_[j] * kneg) + carry;
    a.l[j] = (uint32_t)t;
    carry = t >> 32;  // arithmetic: a limb's partial result may be negative
  }
  if (w > 4) lz_csub(a, WC_P4);
  if (w > 2) lz_csub(a, WC_P2);
  if (canonical && w > 1) lz_csub(a, P_);
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = a.l[j];
}

// dst = op(a, b).  Every lane of the workgroup (TPB = 64) must call it.
//   1. lane k < K: x_k, y_k = lazy sums of operand coefficients; P_k = x_k y_k
//   2. lane c < NC: partial sum of one output chunk (products and operands)
//   3. lane o < 12: output o = sum of its chunks (canonical)
// In-place (dst == a or b) is safe: phase 3 reads only the partial sums.
// Out of line: ~500 call sites per final exponentiation would otherwise
// inline into a kernel far larger than the instruction cache.
LB_NOINL void wc_apply(wc_smem& S, int op, int dst, int a, int b) {
  const wc_desc& d = S.ops[op];
  const int lane = threadIdx.x;
  const fp* A = S.slot[a];
  const fp* B = d.square ? S.slot[a] : S.slot[b];
  if (lane < d.K) {
    fp x, y;
    const int x0 = d.xoff[lane], y0 = d.yoff[lane], y1 = lane + 1 < d.K ? d.xoff[lane + 1] : d.yoff[d.K];
    lz_sum(x, S.term, x0, y0, [&](int code) -> const fp& { return A[code & 63]; }, false);
    lz_sum(y, S.term, y0, y1, [&](int code) -> const fp& { return B[code & 63]; }, false);
    fp p;
    fp_mul(p, x, y);
    S.prod[lane] = p;
  }
  __syncthreads();
  if (lane < d.NC) {
    const fp* Bo = S.slot[b];
    fp part;
    lz_sum(part, S.term, d.coff[lane], d.coff[lane + 1],
           [&](int code) -> const fp& {
             const int idx = code & 63, kind = code >> 6;
             return kind == 0 ? A[idx] : kind == 1 ? Bo[idx] : S.prod[idx];
           },
           true);
    S.part[lane] = part;
  }
  __syncthreads();
  if (lane < 12) {
    const int c0 = d.cs[lane], c1 = d.cs[lane + 1];
    fp o = S.part[c0];
    for (int c = c0 + 1; c < c1; c++) fp_add(o, o, S.part[c]);
    S.slot[dst][lane] = o;
  }
  __syncthreads();
}

LB_DEV void wc_copy(wc_smem& S, int dst, int src) {
  if (threadIdx.x < 12) S.slot[dst][threadIdx.x] = S.slot[src][threadIdx.x];
  __syncthreads();
}
LB_DEV void wc_set_one(wc_smem& S, int dst) {
  if (threadIdx.x < 12) {
    fp v;
    if (threadIdx.x == 0)
      fp_one(v);
    else
      fp_zero(v);
    S.slot[dst][threadIdx.x] = v;
  }
  __syncthreads();
}
LB_DEV void wc_store(fp12& r, const wc_smem& S, int src) {
  fp* o = &r.c0.c0.c0;
  for (int i = 0; i < 12; i++) o[i] = S.slot[src][i];
}
LB_DEV void wc_load12(wc_smem& S, int dst, const fp12& v) {
  if (threadIdx.x < 12) S.slot[dst][threadIdx.x] = (&v.c0.c0.c0)[threadIdx.x];
  __syncthreads();
}
// Frobenius constants into the gamma slots (once per kernel)
LB_DEV void wc_init_gammas(wc_smem& S) {
  const int c = threadIdx.x;
  if (c < 12) {
    const int e = c >> 1, part = c & 1;
    const uint32_t* g1[6] = {LB_ONE, LB_FROB1_1, LB_FROB1_2, LB_FROB1_3, LB_FROB1_4, LB_FROB1_5};
    const uint32_t* g2[6] = {LB_ONE, LB_FROB2_1, LB_FROB2_2, LB_FROB2_3, LB_FROB2_4, LB_FROB2_5};
    const uint32_t* g3[6] = {LB_ONE, LB_FROB3_1, LB_FROB3_2, LB_FROB3_3, LB_FROB3_4, LB_FROB3_5};
    fp v;
    if (e == 0) {  // unused (the e = 0 coefficient is passed through)
      fp_zero(v);
      S.slot[WC_G1][c] = v;
      S.slot[WC_G2][c] = v;
      S.slot[WC_G3][c] = v;
    } else {
      fp_set(v, g1[e] + 12 * part);
      S.slot[WC_G1][c] = v;
      fp_set(v, g2[e] + 12 * part);
      S.slot[WC_G2][c] = v;
      fp_set(v, g3[e] + 12 * part);
      S.slot[WC_G3][c] = v;
    }
  }
  __syncthreads();
}

// dst = src^x (x < 0, src cyclotomic); uses WC_ACC
LB_DEV void wc_exp_x(wc_smem& S, int dst, int src) {
  wc_copy(S, WC_ACC, src);
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    wc_apply(S, LB_WC_CYC, WC_ACC, WC_ACC, WC_ACC);
    if ((LB_X_ABS >> i) & 1ull) wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, src);
  }
  wc_apply(S, LB_WC_CONJ, dst, WC_ACC, WC_ACC);
}

// out = in^-1 for 12 Fp coefficients in LDS; out of line so its register
// pressure (one lane, once per final exponentiation) stays out of the kernel
LB_NOINL void wc_fp12_inv_lane(fp* out, const fp* in) {
  fp12 f, fi;
  fp* pf = &f.c0.c0.c0;
  for (int i = 0; i < 12; i++) pf[i] = in[i];
  fp12_inv(fi, f);
  const fp* o = &fi.c0.c0.c0;
  for (int i = 0; i < 12; i++) out[i] = o[i];
}

// slot dst = f^(3 (p^12 - 1)/r) for f in slot src (== final_exp in bls_pairing.h)
LB_DEV void wc_final_exp(wc_smem& S, int dst, int src) {
  // easy part: f^(p^6 - 1) = conj(f) / f: the Fp12 inversion runs in lane 0
  wc_apply(S, LB_WC_CONJ, WC_T0, src, src);
  if (threadIdx.x == 0) wc_fp12_inv_lane(S.slot[WC_T1], S.slot[src]);
  __syncthreads();
  wc_apply(S, LB_WC_MUL, WC_T0, WC_T0, WC_T1);
  wc_apply(S, LB_WC_FROB2, WC_T1, WC_T0, WC_G2);
  wc_apply(S, LB_WC_MUL, WC_F2, WC_T1, WC_T0);
  // hard part: (x-1)^2 (x+p) (x^2+p^2-1) + 3
  wc_exp_x(S, WC_T0, WC_F2);
  wc_apply(S, LB_WC_CONJ, WC_T1, WC_F2, WC_F2);
  wc_apply(S, LB_WC_MUL, WC_A, WC_T0, WC_T1);
  wc_exp_x(S, WC_T0, WC_A);
  wc_apply(S, LB_WC_CONJ, WC_T1, WC_A, WC_A);
  wc_apply(S, LB_WC_MUL, WC_A, WC_T0, WC_T1);
  wc_exp_x(S, WC_T0, WC_A);
  wc_apply(S, LB_WC_FROB1, WC_T1, WC_A, WC_G1);
  wc_apply(S, LB_WC_MUL, WC_B, WC_T0, WC_T1);
  wc_exp_x(S, WC_T0, WC_B);
  wc_exp_x(S, WC_T0, WC_T0);
  wc_apply(S, LB_WC_FROB2, WC_T1, WC_B, WC_G2);
  wc_apply(S, LB_WC_MUL, WC_C, WC_T0, WC_T1);
  wc_apply(S, LB_WC_CONJ, WC_T1, WC_B, WC_B);
  wc_apply(S, LB_WC_MUL, WC_C, WC_C, WC_T1);
  wc_apply(S, LB_WC_CYC, WC_T0, WC_F2, WC_F2);
  wc_apply(S, LB_WC_MUL, WC_T0, WC_T0, WC_F2);
  wc_apply(S, LB_WC_MUL, dst, WC_C, WC_T0);
}

// slot dst = Miller value of pair q from the stored lines (bls_pairing.h layout)
LB_DEV void wc_miller_from_lines(wc_smem& S, int dst, const uint32_t* __restrict__ lines, size_t n_pairs, size_t q) {
  wc_set_one(S, dst);
  int j = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i < 62) wc_apply(S, LB_WC_SQR, dst, dst, dst);
    for (int rep = 0; rep < 2; rep++) {
      if (rep == 1 && !((LB_X_ABS >> i) & 1ull)) break;
      if (threadIdx.x < 6) {
        const uint32_t* p = lines + ((size_t)j * 72 + 12 * threadIdx.x) * n_pairs + q;
        fp v;
        for (int w = 0; w < 12; w++) v.l[w] = p[(size_t)w * n_pairs];
        S.slot[WC_LINE][threadIdx.x] = v;
      }
      __syncthreads();
      wc_apply(S, LB_WC_LINE, dst, dst, WC_LINE);
      j++;
    }
  }
  wc_apply(S, LB_WC_CONJ, dst, dst, dst);  // x < 0
}

LB_DEV bool wc_is_one(const wc_smem& S, int src) {
  fp one;
  fp_one(one);
  bool ok = fp_eq(S.slot[src][0], one);
  for (int i = 1; i < 12; i++) ok = ok && fp_is_zero(S.slot[src][i]);
  return ok;
}

}  // namespace lb
