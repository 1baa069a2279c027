// Stage-level parity kernel: full pairing e(P, Q) (Miller loop + final exponentiation).
#include "bls_kernels.h"

namespace lb {

__global__ void k_pairing(uint32_t n, const uint8_t* __restrict__ g1b, const uint8_t* __restrict__ g2b,
                          uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a p;
  g2a q;
  const uint8_t s1 = g1_deserialize(p, g1b + (size_t)i * 96, 96);
  const uint8_t s2 = g2_deserialize(q, g2b + (size_t)i * 192, 192);
  fp12 f, r;
  fp12_one(f);
  if (s1 == LB_ST_OK && s2 == LB_ST_OK && !p.inf && !q.inf) miller_loop(f, p, q);
  final_exp(r, f);
  uint8_t* o = out + (size_t)i * 576;
  const fp2* c[6] = {&r.c0.c0, &r.c0.c1, &r.c0.c2, &r.c1.c0, &r.c1.c1, &r.c1.c2};
  for (int k = 0; k < 6; k++) {
    fp_write_be(o + 96 * k, c[k]->c0);
    fp_write_be(o + 96 * k + 48, c[k]->c1);
  }
}
}  // namespace lb
