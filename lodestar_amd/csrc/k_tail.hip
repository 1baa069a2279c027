// Per-request tails, one wave per request (wave-cooperative Fp12, bls_wc12.h):
// lines of (-g1, S_k), Miller value from those lines, F_k * f_S, final
// exponentiation, verdict.  Replaces the one-lane-per-request k_miller_S +
// k_final chain (15-20 ms of latency each) for the default pipeline.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"
#include "bls_wc12.h"

namespace lb {

// lines of the pairs (-g1, S_k), k < n_req, stored as pairs base + k
// (skip: optional flag; nonzero -> nothing to do, the merged check passed)
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_lines_S(uint32_t n_req, uint32_t n_pairs, uint32_t base,
                                                          const g2a* __restrict__ S, uint32_t* __restrict__ lines,
                                                          const uint8_t* __restrict__ skip) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req || (skip && *skip)) return;
  g1a p;
  fp_set(p.x, LB_G1_X);
  fp_set(p.y, LB_G1_NEG_Y);
  p.inf = false;
  const g2a q = S[k];
  miller_lines(p, q, lines, n_pairs, (size_t)base + k);
}

// one workgroup (one wave) per request: valid[k] = final_exp(F_k * Miller(-g1, S_k)) == 1.
// lines == nullptr: F_k already holds the Miller(-g1, S) factor (the merged
// check folded into k_miller_acc): valid[k] = final_exp(F_k) == 1.
// skip (optional): nonzero when the merged check of the whole call passed ->
// valid[k] = !req_bad[k] without any arithmetic.
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_tail(uint32_t n_req, uint32_t n_pairs, uint32_t base,
                                                       const uint32_t* __restrict__ lines,
                                                       const fp12* __restrict__ F,
                                                       const uint8_t* __restrict__ req_bad,
                                                       uint8_t* __restrict__ valid,
                                                       const uint8_t* __restrict__ skip) {
  __shared__ wc_smem S;
  const uint32_t k = blockIdx.x;
  if (k >= n_req) return;
  if (req_bad[k] || (skip && *skip)) {  // uniform per workgroup
    if (threadIdx.x == 0) valid[k] = req_bad[k] ? 0 : 1;
    return;
  }
  wc_init_tables(S);
  wc_init_gammas(S);
  if (lines) wc_miller_from_lines(S, WC_FS, lines, n_pairs, (size_t)base + k);
  wc_load12(S, WC_F, F[k]);
  if (lines) wc_apply(S, LB_WC_MUL, WC_F, WC_F, WC_FS);
  wc_final_exp(S, WC_F, WC_F);
  if (threadIdx.x == 0) valid[k] = wc_is_one(S, WC_F) ? 1 : 0;
}

// Miller value of each set pair from its stored lines, one wave per pair
// (wave-cooperative; the latency path for small calls, where one lane per pair
// would run a ~6.5k-product chain)
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_pair_wc(uint32_t n, uint32_t n_pairs,
                                                          const uint32_t* __restrict__ lines, fp12* __restrict__ f) {
  __shared__ wc_smem S;
  const uint32_t q = blockIdx.x;
  if (q >= n) return;
  wc_init_tables(S);
  wc_miller_from_lines(S, WC_FS, lines, n_pairs, q);
  if (threadIdx.x < 12) (&f[q].c0.c0.c0)[threadIdx.x] = S.slot[WC_FS][threadIdx.x];
}

// Merged check of a whole call (the worker's merged batch, worker.ts:41-96):
// S_all = sum S_k and F_all = prod F_k over the requests not already false.
// S == nullptr: S_all already came from the bucket MSM (k_msm_final); only F_all.
// Fx != nullptr: Miller(-g1, S_all) computed by k_miller_acc, multiplied in.
// F == nullptr: S_all only (the steps organisation forms F_all by levels, k_steps.hip).
// One wave; the tail kernel then verifies (F_all, S_all) once, and the
// per-request tails only run if that merged check fails.
// The worker's bookkeeping of its merged batch (worker.ts:66-85): batchRetries
// (1 when the merged check failed and requests were re-verified alone) and
// batchSigsSuccess (sets verified inside a passing merged check).
__global__ void __launch_bounds__(TPB) k_merge_stats(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                     const uint8_t* __restrict__ req_bad,
                                                     const uint8_t* __restrict__ mflag, uint32_t* __restrict__ out) {
  __shared__ uint32_t cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  uint32_t c = 0;
  for (uint32_t k = threadIdx.x; k < n_req; k += TPB)
    if (!req_bad[k]) c += req_off[k + 1] - req_off[k];
  atomicAdd(&cnt, c);
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool passed = mflag[0] != 0;
    out[0] = passed ? 0u : 1u;
    out[1] = passed ? cnt : 0u;
  }
}

// Partial of a call for the multi-GPU combine (north_star): the
// call's merged Miller product P = F_all * Miller(-g1, S_all) BEFORE the final
// exponentiation, as 576 bytes (12 big-endian canonical Fp coefficients,
// c0.c0.c0 ... c1.c2.c1, the lb_pairing order).  The host multiplies the
// partials of all GPUs and checks final_exp(prod) == 1 once (k_gt_check).
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_partial(uint32_t n_pairs, uint32_t base,
                                                          const uint32_t* __restrict__ lines,
                                                          const fp12* __restrict__ F_all, uint8_t* __restrict__ out576) {
  __shared__ wc_smem S;
  wc_init_tables(S);
  if (lines) wc_miller_from_lines(S, WC_FS, lines, n_pairs, base);  // (nullptr: F_all holds the factor)
  wc_load12(S, WC_F, F_all[0]);
  if (lines) wc_apply(S, LB_WC_MUL, WC_F, WC_F, WC_FS);
  if (threadIdx.x < 12) fp_write_be(out576 + 48 * threadIdx.x, S.slot[WC_F][threadIdx.x]);
}

// out[0] = 1 iff final_exp(prod_i partial_i) == 1 for n partials of 576 bytes
// (the host-side combine of the per-GPU partials; one wave).  A coefficient
// that is not < p makes the product invalid (out[0] = 0, out[1] = 1).
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_gt_check(uint32_t n, const uint8_t* __restrict__ in576,
                                                           uint8_t* __restrict__ out) {
  __shared__ wc_smem S;
  __shared__ uint32_t bad;
  if (threadIdx.x == 0) bad = 0;
  wc_init_tables(S);
  wc_init_gammas(S);
  wc_set_one(S, WC_ACC);
  for (uint32_t i = 0; i < n; i++) {
    if (threadIdx.x < 12) {
      fp v;
      if (!fp_read_masked(v, in576 + (size_t)i * 576 + 48 * threadIdx.x, false)) {
        atomicOr(&bad, 1u);
        fp_zero(v);
      }
      S.slot[WC_B][threadIdx.x] = v;
    }
    __syncthreads();
    wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, WC_B);
  }
  wc_copy(S, WC_C, WC_ACC);
  wc_final_exp(S, WC_F, WC_C);
  if (threadIdx.x == 0) {
    out[0] = (!bad && wc_is_one(S, WC_F)) ? 1 : 0;
    out[1] = bad ? 1 : 0;
  }
}

// The product of n partials (as k_gt_check) as 12 records of one-lane limbs for the
// round-program final exponentiation (k_lp_final_lane); out[1] = 1 when a coefficient
// is not < p (the product is then invalid).
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_gt_prod(uint32_t n, const uint8_t* __restrict__ in576,
                                                          uint32_t* __restrict__ out16, uint8_t* __restrict__ out) {
  __shared__ wc_smem S;
  __shared__ uint32_t bad;
  if (threadIdx.x == 0) bad = 0;
  wc_init_tables(S);
  wc_set_one(S, WC_ACC);
  for (uint32_t i = 0; i < n; i++) {
    if (threadIdx.x < 12) {
      fp v;
      if (!fp_read_masked(v, in576 + (size_t)i * 576 + 48 * threadIdx.x, false)) {
        atomicOr(&bad, 1u);
        fp_zero(v);
      }
      S.slot[WC_B][threadIdx.x] = v;
    }
    __syncthreads();
    wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, WC_B);
  }
  if (threadIdx.x < 12) {
    const fp v = S.slot[WC_ACC][threadIdx.x];
#pragma unroll
    for (int j = 0; j < 12; j++) out16[16 * threadIdx.x + j] = v.l[j];
#pragma unroll
    for (int j = 12; j < 16; j++) out16[16 * threadIdx.x + j] = 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[1] = bad ? 1 : 0;
}

__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_merge(uint32_t n_req, const g2a* __restrict__ S,
                                                        const fp12* __restrict__ F,
                                                        const uint8_t* __restrict__ req_bad,
                                                        g2a* __restrict__ S_all, fp12* __restrict__ F_all,
                                                        const fp12* __restrict__ Fx) {
  __shared__ LdsRec<g2j> shs[TPB];
  __shared__ LdsRec<fp12> shf[TPB];
  g2j acc;
  jac_set_inf(acc);
  fp12 f;
  fp12_one(f);
  if (Fx && threadIdx.x == 0) f = Fx[0];
  for (uint32_t k = threadIdx.x; k < n_req; k += TPB) {
    if (req_bad[k]) continue;
    if (S) {
      const g2a s = S[k];
      if (!s.inf) jac_add_aff(acc, acc, s);
    }
    if (F) {
      fp12 t = F[k];
      fp12_mul(f, f, t);
    }
  }
  shs[threadIdx.x].v = acc;
  shf[threadIdx.x].v = f;
  __syncthreads();
  for (int st = TPB / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
      if (S) {
        g2j m = shs[threadIdx.x].v, o = shs[threadIdx.x + st].v;
        jac_add(m, m, o);
        shs[threadIdx.x].v = m;
      }
      if (F) {
        fp12 a = shf[threadIdx.x].v, b = shf[threadIdx.x + st].v;
        fp12_mul(a, a, b);
        shf[threadIdx.x].v = a;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (S) {
      g2j tot = shs[0].v;
      g2a sa;
      jac_to_aff(sa, tot);
      S_all[0] = sa;
    }
    if (F) F_all[0] = shf[0].v;
  }
}

}  // namespace lb
