// Per-request tails, one wave per request (wave-cooperative Fp12, bls_wc12.h):
// lines of (-g1, S_k), Miller value from those lines, F_k * f_S, final
// exponentiation, verdict.  Replaces the one-lane-per-request k_miller_S +
// k_final chain (15-20 ms of latency each) for the default pipeline.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"
#include "bls_wc12.h"

namespace lb {

// lines of the pairs (-g1, S_k), k < n_req, stored as pairs base + k
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_lines_S(uint32_t n_req, uint32_t n_pairs, uint32_t base,
                                                          const g2a* __restrict__ S, uint32_t* __restrict__ lines) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req) return;
  g1a p;
  fp_set(p.x, LB_G1_X);
  fp_set(p.y, LB_G1_NEG_Y);
  p.inf = false;
  const g2a q = S[k];
  miller_lines(p, q, lines, n_pairs, (size_t)base + k);
}

// one workgroup (one wave) per request: valid[k] = final_exp(F_k * Miller(-g1, S_k)) == 1
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_tail(uint32_t n_req, uint32_t n_pairs, uint32_t base,
                                                       const uint32_t* __restrict__ lines,
                                                       const fp12* __restrict__ F,
                                                       const uint8_t* __restrict__ req_bad,
                                                       uint8_t* __restrict__ valid) {
  __shared__ wc_smem S;
  const uint32_t k = blockIdx.x;
  if (k >= n_req) return;
  if (req_bad[k]) {  // uniform per workgroup
    if (threadIdx.x == 0) valid[k] = 0;
    return;
  }
  wc_init_gammas(S);
  wc_miller_from_lines(S, WC_FS, lines, n_pairs, (size_t)base + k);
  wc_load12(S, WC_F, F[k]);
  wc_apply(S, LB_WC_MUL, WC_F, WC_F, WC_FS);
  wc_final_exp(S, WC_F, WC_F);
  if (threadIdx.x == 0) valid[k] = wc_is_one(S, WC_F) ? 1 : 0;
}

}  // namespace lb
