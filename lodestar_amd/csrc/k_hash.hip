// hash_to_G2 stages (two lanes per message, then finish), and the one-lane variant.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

// hash_to_G2, first half: lane 2i+j maps u_j of message i (SSWU + 3-isogeny)
__global__ void __launch_bounds__(TPB, LB_W_MAP) k_hash_half(uint32_t n, const uint8_t* __restrict__ msgs,
                                                   g2j* __restrict__ q) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  uint8_t m[32];
  const uint8_t* src = msgs + (size_t)(t >> 1) * 32;
  for (int k = 0; k < 32; k++) m[k] = src[k];
  g2j r;
  hash_to_g2_half(r, m, (int)(t & 1));
  q[t] = r;
}
// hash_to_G2, second half: Q0 + Q1, clear cofactor (Jacobian out: the
// affine conversion shares its inversion with r_i pk_i, jac_pair_to_aff)
// LB_HASH_FINISH_MEM (default): the register-lean cofactor clearing, the two halves' slots
// of q (consumed here) holding the points that are not being worked on
__global__ void __launch_bounds__(TPB, LB_W_HASH) k_hash_finish(uint32_t n, g2j* __restrict__ q, g2j* __restrict__ out_h) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2j h;
#ifdef LB_HASH_FINISH_REGS
  g2j q0 = q[2 * i], q1 = q[2 * i + 1];
  hash_to_g2_finish(h, q0, q1, out_h + i);  // out_h[i] doubles as the stash
#else
  {
    g2j q0 = q[2 * i], q1 = q[2 * i + 1], s;
    jac_add(s, q0, q1);
    q[2 * i] = s;
  }
  clear_cofactor_g2_mem(h, q + 2 * i, q + 2 * i + 1);
#endif
  out_h[i] = h;
}

// ---- hash_to_G2 in one lane (stage-level API) ------------------------------
__global__ void __launch_bounds__(TPB, LB_HEAVY_WAVES) k_hash(uint32_t n, const uint8_t* __restrict__ msgs, g2a* __restrict__ out_h) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t m[32];
  for (int k = 0; k < 32; k++) m[k] = msgs[(size_t)i * 32 + k];
  g2j h;
  hash_to_g2(h, m);
  g2a ha;
  jac_to_aff(ha, h);
  out_h[i] = ha;
}

}  // namespace lb
