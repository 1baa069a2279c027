// Per-request product tree of the Miller values (one wave per request, LDS tree).
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

// F_k = f_S[k] * prod f_i, request status and errors: one wave per request
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_prod_tree(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                   const fp12* __restrict__ f, const fp12* __restrict__ fS,
                                                   const uint8_t* __restrict__ sig_status,
                                                   const uint8_t* __restrict__ pk_status, fp12* __restrict__ F,
                                                   uint8_t* __restrict__ req_bad, uint8_t* __restrict__ req_err) {
  __shared__ LdsRec<fp12> sh[TPB];
  __shared__ uint32_t bad, err_empty, err_pk;
  const uint32_t k = blockIdx.x;
  if (k >= n_req) return;
  const uint32_t a = req_off[k], b = req_off[k + 1];
  if (threadIdx.x == 0) {
    bad = (a == b) ? 1u : 0u;
    err_empty = 0;
    err_pk = 0;
  }
  __syncthreads();
  fp12 acc;
  fp12_one(acc);
  bool first = true;
  for (uint32_t i = a + threadIdx.x; i < b; i += TPB) {
    const uint8_t ss = sig_status[i], ps = pk_status[i];
    if (ss != LB_ST_OK || ps != LB_ST_OK) atomicOr(&bad, 1u);
    if (ps == LB_ST_EMPTY_AGGREGATE) atomicOr(&err_empty, 1u);
    if (ps == LB_ST_BAD_ENCODING) atomicOr(&err_pk, 1u);
    fp12 t = f[i];
    if (first) {
      acc = t;
      first = false;
    } else {
      fp12_mul(acc, acc, t);
    }
  }
  sh[threadIdx.x].v = acc;
  __syncthreads();
  for (int s = TPB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s && a + threadIdx.x + s < b) {
      fp12 m = sh[threadIdx.x].v, o = sh[threadIdx.x + s].v;
      fp12_mul(m, m, o);
      sh[threadIdx.x].v = m;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    fp12 tot = sh[0].v;
    if (fS) {  // null: the tail kernel multiplies Miller(-g1, S_k) in (k_tail)
      fp12 s = fS[k];
      fp12_mul(tot, tot, s);
    }
    F[k] = tot;
    req_bad[k] = bad ? 1 : 0;
    req_err[k] = err_empty ? LB_REQ_EMPTY_AGGREGATE : err_pk ? LB_REQ_BAD_PUBKEY : LB_REQ_OK;
  }
}

}  // namespace lb
