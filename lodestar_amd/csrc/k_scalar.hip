// Random-scalar stages: r_i sig_i, r_i pk_i, per-request sum S_k.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

// r_i sig_i  (r_i = a_i + b_i lambda, jac_mul_glv: shared-Z ladder, free cube-root table)
__global__ void __launch_bounds__(TPB, LB_W_SSIG) k_scalar_sig(uint32_t n, const uint8_t* __restrict__ seed,
                                                    const g2j* __restrict__ sig,
                                                    const uint8_t* __restrict__ sig_status,
                                                    g2j* __restrict__ rsig, const uint8_t* __restrict__ skip) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (skip && *skip)) return;
  g2j rs;
  jac_set_inf(rs);
  if (sig_status[i] == LB_ST_OK) {
    uint8_t sd[32];
    for (int k = 0; k < 32; k++) sd[k] = seed[k];
    const uint64_t r = batch_scalar(sd, i);
    jac_mul_glv_xy(rs, sig[i].X, sig[i].Y, LB_G2_OMEGA, LB_G2_OMEGA2, r);
    fp2 z = sig[i].Z;  // 1 for decoded signatures; reloaded rather than kept live
    fp2_mul(rs.Z, rs.Z, z);
  }
  rsig[i] = rs;
}

// r_i pk_i (Jacobian; made affine together with H(m_i), jac_pair_to_aff);
// core-verify pubkey subgroup check for single-set requests
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_scalar_pk(uint32_t n, const uint8_t* __restrict__ seed,
                                                   const g1j* __restrict__ pk, const uint8_t* __restrict__ single_flag,
                                                   uint8_t* __restrict__ pk_status, g1j* __restrict__ rpk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st = pk_status[i];
  g1j p = pk[i];
  if (st == LB_ST_OK && single_flag[i] && !g1_in_subgroup(p)) st = LB_ST_NOT_IN_GROUP;
  g1j rp;
  jac_set_inf(rp);
  if (st == LB_ST_OK) {
    uint8_t sd[32];
    for (int k = 0; k < 32; k++) sd[k] = seed[k];
    const uint64_t r = batch_scalar(sd, i);
    jac_mul_glv(rp, p, LB_G1_BETA, LB_G1_BETA2, r);
  }
  rpk[i] = rp;
  pk_status[i] = st;
}

// S_k = sum_{i in request k} r_i sig_i : one wave per request, strided + LDS tree
// skip (k_scalar_sig too): optional flag, nonzero -> nothing to do (the merged
// check, whose sum came from the bucket MSM, passed: no per-request tails)
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_sum_tree(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                  const g2j* __restrict__ rsig, g2a* __restrict__ S,
                                                  const uint8_t* __restrict__ skip) {
  __shared__ LdsRec<g2j> sh[TPB];
  const uint32_t k = blockIdx.x;
  if (k >= n_req || (skip && *skip)) return;
  const uint32_t a = req_off[k], b = req_off[k + 1];
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t i = a + threadIdx.x; i < b; i += TPB) {
    g2j t = rsig[i];
    jac_add(acc, acc, t);
  }
  sh[threadIdx.x].v = acc;
  __syncthreads();
  for (int s = TPB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s && a + threadIdx.x + s < b) {
      g2j m = sh[threadIdx.x].v, o = sh[threadIdx.x + s].v;
      jac_add(m, m, o);
      sh[threadIdx.x].v = m;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    g2j tot = sh[0].v;
    g2a sa;
    jac_to_aff(sa, tot);
    S[k] = sa;
  }
}

}  // namespace lb
