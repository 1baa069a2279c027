// Per-request final exponentiation and the == 1 verdict.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_final(uint32_t n_req, const fp12* __restrict__ F,
                                               const uint8_t* __restrict__ req_bad, uint8_t* __restrict__ valid) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req) return;
  if (req_bad[k]) {
    valid[k] = 0;
    return;
  }
  fp12 acc = F[k], r;
  final_exp(r, acc);
  valid[k] = fp12_is_one(r) ? 1 : 0;
}

}  // namespace lb
