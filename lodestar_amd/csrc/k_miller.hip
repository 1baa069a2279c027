// Miller loops: per set f_i = Miller(r_i pk_i, H(m_i)); per request Miller(-g1, S_k).
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

// f_S[k] = Miller(-g1, S_k)
__global__ void __launch_bounds__(TPB, LB_HEAVY_WAVES) k_miller_S(uint32_t n_req, const g2a* __restrict__ S, fp12* __restrict__ fS) {
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
__global__ void __launch_bounds__(TPB, LB_HEAVY_WAVES) k_miller_sets(uint32_t n, const g1a* __restrict__ rpk, const g2a* __restrict__ h,
                                                     fp12* __restrict__ f) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp12 r;
  fp12_one(r);
  g1a p = rpk[i];
  g2a q = h[i];
  if (!p.inf && !q.inf) miller_loop(r, p, q);
  f[i] = r;
}

}  // namespace lb
