// Miller loops: per set f_i = Miller(r_i pk_i, H(m_i)); per request Miller(-g1, S_k).
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

// f_S[k] = Miller(-g1, S_k)
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_miller_S(uint32_t n_req, const g2a* __restrict__ S, fp12* __restrict__ fS) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req) return;
  fp12 r;
  fp12_one(r);
  g2a q = S[k];
  if (!q.inf) {
    g1a g;
    fp_set(g.x, LB_G1_X);
    fp_set(g.y, LB_G1_NEG_Y);
    g.inf = false;
    miller_loop(r, g, q);
  }
  fS[k] = r;
}

// f_i = Miller(r_i pk_i, H(m_i))
__global__ void __launch_bounds__(TPB, LB_HEAVY_WAVES) k_miller_sets(uint32_t n, const g1j* __restrict__ rpk, const g2j* __restrict__ h,
                                                     fp12* __restrict__ f) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp12 r;
  fp12_one(r);
  g1a p;
  g2a q;
  jac_pair_to_aff(p, q, rpk[i], h[i]);
  if (!p.inf && !q.inf) miller_loop(r, p, q);
  f[i] = r;
}

// Lines of pairs [base, base + n) of the verification's pair list (n_pairs
// total): pair base + i is (P[i], Q[i]) (Jacobian in, one shared inversion).
template <int WAVES>
__global__ void __launch_bounds__(TPB, WAVES) k_lines(uint32_t n, uint32_t n_pairs, uint32_t base,
                                                               const g1j* __restrict__ P, const g2j* __restrict__ Q,
                                                               uint32_t* __restrict__ lines) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a p;
  g2a q;
  jac_pair_to_aff(p, q, P[i], Q[i]);
  miller_lines(p, q, lines, n_pairs, base + i);
}

// f *= line j of the pairs a + lane, a + lane + LPR, ... < b: two pairs at a time
// through the sparse x sparse product (23 Fp2 products per two lines instead of 26)
template <int LPR>
LB_DEV void acc_lines(fp12& f, const uint32_t* __restrict__ lines, uint32_t n_pairs, uint32_t a, uint32_t b,
                      uint32_t lane, int j) {
  fp2 l0, l1, l4;
  uint32_t i = a + lane;
#ifndef LB_NO_LINE_PAIRS
#pragma unroll 1
  for (; i + LPR < b; i += 2 * LPR) {
    fp2 m0, m1, m4, y1, y2;
    fp6 x;
    line_get(lines, n_pairs, i, j, l0, l1, l4);
    line_get(lines, n_pairs, i + LPR, j, m0, m1, m4);
    line_mul_line(x, y1, y2, l0, l1, l4, m0, m1, m4);
    fp12_mul_by_sparse2(f, f, x, y1, y2);
  }
#endif
#pragma unroll 1
  for (; i < b; i += LPR) {
    line_get(lines, n_pairs, i, j, l0, l1, l4);
    fp12_mul_line(f, f, l0, l1, l4);
  }
}

// Miller(-g1, S) with its lines computed on the fly (one lane); out of line so
// the accumulation loop of k_miller_acc keeps its own register allocation
__device__ __noinline__ void miller_neg_g1(fp12* __restrict__ out, const g2a* __restrict__ S) {
  fp12 r;
  fp12_one(r);
  const g2a q = *S;
  if (!q.inf) {
    g1a g;
    fp_set(g.x, LB_G1_X);
    fp_set(g.y, LB_G1_NEG_Y);
    g.inf = false;
    miller_loop(r, g, q);
  }
  *out = r;
}

// Per request k: F_k = f_S[k] * prod_{i in request} Miller(r_i pk_i, H_i), from
// the stored lines.  LB_ACC_LPR lanes per request (64 / LB_ACC_LPR requests per
// wave); lane l accumulates the set pairs a + l, a + l + LPR, ... into ONE f,
// so the Fp12 squaring of each loop step is shared by ~128 / LPR pairs; the
// lane values are then multiplied in an LDS tree.  Also reduces the request's
// set statuses (verdict / rejection flags) as k_prod_tree did.
// halves != 0: the "requests" are the halves of the call's requests (a lone call
// on an idle GPU runs twice as many waves, k_split_requests / k_join_halves); an
// empty half is then not a false verdict.
// Sx != nullptr: one extra (last) workgroup computes Fx = Miller(-g1, Sx) for
// the merged check, alongside the per-request waves (its sum S_all came from
// the bucket MSM before this launch), so neither the lines of that pair nor
// their wave-cooperative Miller value sit on the call's serial tail.
template <int LPR>
__global__ void __launch_bounds__(TPB, LB_W_ACC) k_miller_acc(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                                    uint32_t n_pairs, const uint32_t* __restrict__ lines,
                                                                    const fp12* __restrict__ fS,
                                                                    const uint8_t* __restrict__ sig_status,
                                                                    const uint8_t* __restrict__ pk_status,
                                                                    fp12* __restrict__ F, uint8_t* __restrict__ req_bad,
                                                                    uint8_t* __restrict__ req_err, uint32_t halves,
                                                                    const g2a* __restrict__ Sx, fp12* __restrict__ Fx) {
  constexpr uint32_t RPW = TPB / LPR;  // requests per workgroup
  if (Sx && blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x == 0) miller_neg_g1(Fx, Sx);
    return;
  }
  __shared__ LdsRec<fp12> sh[TPB];
  __shared__ uint32_t bad[RPW], err_empty[RPW], err_pk[RPW];
  const uint32_t sub = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  const uint32_t k = blockIdx.x * RPW + sub;
  const bool live = k < n_req;
  const uint32_t a = live ? req_off[k] : 0, b = live ? req_off[k + 1] : 0;
  if (lane == 0) {
    bad[sub] = (a == b && !halves) ? 1u : 0u;
    err_empty[sub] = 0;
    err_pk[sub] = 0;
  }
  __syncthreads();
  for (uint32_t i = a + lane; i < b; i += LPR) {
    const uint8_t ss = sig_status[i], ps = pk_status[i];
    if (ss != LB_ST_OK || ps != LB_ST_OK) atomicOr(&bad[sub], 1u);
    if (ps == LB_ST_EMPTY_AGGREGATE) atomicOr(&err_empty[sub], 1u);
    if (ps == LB_ST_BAD_ENCODING) atomicOr(&err_pk[sub], 1u);
  }
  fp12 f;
  fp12_one(f);
  int j = 0;
#pragma unroll 1
  for (int bit = 62; bit >= 0; bit--) {
    // the doubling line, then the addition line when bit is set: one loop body,
    // so the (large) line accumulation is instantiated once
    const int reps = 1 + (int)((LB_X_ABS >> bit) & 1ull);
#pragma unroll 1
    for (int rep = 0; rep < reps; rep++) {
      if (rep == 0 && bit < 62) fp12_sqr(f, f);
      acc_lines<LPR>(f, lines, n_pairs, a, b, lane, j);
      j++;
    }
  }
  fp12_conj(f, f);  // x < 0
  sh[threadIdx.x].v = f;
  __syncthreads();
  for (uint32_t s = (uint32_t)LPR / 2; s > 0; s >>= 1) {
    if (lane < s) {
      fp12 m = sh[threadIdx.x].v, o = sh[threadIdx.x + s].v;
      fp12_mul(m, m, o);
      sh[threadIdx.x].v = m;
    }
    __syncthreads();
  }
  if (live && lane == 0) {
    fp12 tot = sh[threadIdx.x].v;
    if (fS) {  // null: the tail kernel multiplies Miller(-g1, S_k) in (k_tail)
      fp12 s = fS[k];
      fp12_mul(tot, tot, s);
    }
    F[k] = tot;
    req_bad[k] = bad[sub] ? 1 : 0;
    req_err[k] = err_empty[sub] ? LB_REQ_EMPTY_AGGREGATE : err_pk[sub] ? LB_REQ_BAD_PUBKEY : LB_REQ_OK;
  }
}

// Request halves for a lone call: off2[2k] = off[k], off2[2k+1] = off[k] + ceil(n_k / 2).
__global__ void __launch_bounds__(TPB) k_split_requests(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                        uint32_t* __restrict__ off2) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n_req) return;
  const uint32_t a = req_off[k];
  off2[2 * k] = a;
  if (k < n_req) off2[2 * k + 1] = a + (req_off[k + 1] - a + 1) / 2;
}

// Join the halves: F_k = F2[2k] F2[2k+1] (x Miller(-g1, S_k) when fS is given),
// verdict / rejection flags OR-ed; an empty request is false (maybeBatch.ts:31-33).
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_join_halves(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                               const fp12* __restrict__ F2, const uint8_t* __restrict__ bad2,
                                                               const uint8_t* __restrict__ err2,
                                                               const fp12* __restrict__ fS, fp12* __restrict__ F,
                                                               uint8_t* __restrict__ req_bad, uint8_t* __restrict__ req_err) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req) return;
  fp12 x = F2[2 * k], y = F2[2 * k + 1];
  fp12_mul(x, x, y);
  if (fS) {
    fp12 s = fS[k];
    fp12_mul(x, x, s);
  }
  F[k] = x;
  req_bad[k] = (bad2[2 * k] | bad2[2 * k + 1] | (req_off[k + 1] == req_off[k] ? 1 : 0)) ? 1 : 0;
  const uint8_t e0 = err2[2 * k], e1 = err2[2 * k + 1];
  req_err[k] = (e0 == LB_REQ_EMPTY_AGGREGATE || e1 == LB_REQ_EMPTY_AGGREGATE) ? LB_REQ_EMPTY_AGGREGATE
               : (e0 == LB_REQ_BAD_PUBKEY || e1 == LB_REQ_BAD_PUBKEY)     ? LB_REQ_BAD_PUBKEY
                                                                            : LB_REQ_OK;
}

// tuning variants selected at run time (LB_LINES_WAVES, LB_ACC_LPR)
#define LB_INST_LINES(W)                                                                                       \
  template __global__ void k_lines<W>(uint32_t, uint32_t, uint32_t, const g1j* __restrict__, const g2j* __restrict__, \
                                      uint32_t* __restrict__);
LB_INST_LINES(1)
LB_INST_LINES(2)
#define LB_INST_ACC(L)                                                                                           \
  template __global__ void k_miller_acc<L>(uint32_t, const uint32_t* __restrict__, uint32_t,                    \
                                           const uint32_t* __restrict__, const fp12* __restrict__,              \
                                           const uint8_t* __restrict__, const uint8_t* __restrict__,            \
                                           fp12* __restrict__, uint8_t* __restrict__, uint8_t* __restrict__, uint32_t, \
                                           const g2a* __restrict__, fp12* __restrict__);
LB_INST_ACC(64)
LB_INST_ACC(32)
LB_INST_ACC(16)

}  // namespace lb
