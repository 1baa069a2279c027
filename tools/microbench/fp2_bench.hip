// Fp2 / Fp12 product microbenchmark on gfx950 at 1-4 waves per SIMD: the lazy-reduction
// Fp2 product (bls_field.h, default) vs -DLB_NO_LAZY (three Montgomery products).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DLB_NO_LAZY] -o fp2_bench fp2_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../lodestar_amd/csrc/bls_field.h"
// (round 6 measured -DLB_FP_COLS=1/2/12/15 builds against a bls_field.h that took the column
// bodies of fp_cols.h per product kind, commit "Carry-free column field core"; the library has
// since gone back to the asm bodies only, so the flag now only labels the output)
#ifndef LB_FP_COLS
#define LB_FP_COLS 0
#endif
using namespace lb;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ void seed_fp(fp& a, uint32_t s) {
  for (int j = 0; j < 12; j++) a.l[j] = s * 2654435761u + j * 40503u + (s >> 3) + j * s * 77u;
  a.l[11] &= 0x0fffffff;
}
template <int V>
__global__ void __launch_bounds__(64, 1) k_fp2(uint32_t* out, int iters) {
  fp2 a, b, c;
  seed_fp(a.c0, threadIdx.x + 1); seed_fp(a.c1, threadIdx.x + 2); seed_fp(b.c0, blockIdx.x + 7);
  seed_fp(b.c1, blockIdx.x + 9); seed_fp(c.c0, threadIdx.x * 3 + 5); seed_fp(c.c1, threadIdx.x * 5 + 1);
  fp12 f;
  f.c0.c0 = a; f.c0.c1 = b; f.c0.c2 = c; f.c1.c0 = b; f.c1.c1 = a; f.c1.c2 = c;
  for (int k = 0; k < iters; k++) {
    if (V == 0) { fp2_mul(a, a, b); fp2_mul(c, c, b); }
    if (V == 1) { fp12_sqr(f, f); }
    if (V == 2) { fp12_mul_line(f, f, a, b, c); }
    if (V == 3) { fp_mul(a.c0, a.c0, b.c0); fp_mul(c.c1, c.c1, b.c1); }
    if (V == 4) { fp_sqr(a.c0, a.c0); fp_sqr(c.c1, c.c1); }
  }
  uint32_t s = 0;
  for (int j = 0; j < 12; j++) s ^= a.c0.l[j] ^ c.c1.l[j] ^ f.c0.c0.c0.l[j] ^ f.c1.c2.c1.l[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <typename K>
static void run(K kern, uint32_t* buf, int blocks, int iters, double per_lane, const char* name, int lds) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), lds, 0, buf, iters);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), lds, 0, buf, iters);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * 64 * iters * per_lane;
  printf("%-10s blocks=%5d %8.3f ms  %.3e op/s  cyc/wave-op(chip)=%.0f\n", name, blocks, ms, ops / (ms * 1e-3),
         1024 * 2.4e9 / (ops / (ms * 1e-3)) * 64);
}
int main() {
  uint32_t* buf; CHK(hipMalloc(&buf, 64 << 20));
#ifdef LB_NO_LAZY
  printf("variant: LB_NO_LAZY\n");
#else
  printf("variant: lazy, LB_FP_COLS=%d\n", LB_FP_COLS);
#endif
  for (int occ : {1, 2, 4}) {
    const int blocks = 1024 * occ;
    const int lds = 160 * 1024 / 4 / occ - 1024;  // pins occupancy: 4*occ workgroups of 64 per CU
    printf("-- %d waves/SIMD\n", occ);
    run(k_fp2<0>, buf, blocks, 64, 2, "fp2_mul", lds);
    run(k_fp2<1>, buf, blocks, 16, 1, "fp12_sqr", lds);
    run(k_fp2<2>, buf, blocks, 16, 1, "fp12_line", lds);
    run(k_fp2<3>, buf, blocks, 256, 2, "fp_mul", lds);
    run(k_fp2<4>, buf, blocks, 256, 2, "fp_sqr", lds);
  }
  return 0;
}
