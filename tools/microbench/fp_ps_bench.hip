// Field-multiply microbenchmark on gfx950: the product-scanning asm multiply
// (bls_fp_ps.h) against the compiler's CIOS lowering, at 1-8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fp_ps_bench fp_ps_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../lodestar_amd/csrc/bls_field.h"
using namespace lb;

// the compiler-lowered CIOS product the library used before bls_fp_ps.h (baseline)
namespace lb {
// Montgomery CIOS, no-final-carry variant (p[11] < 2^31 - 1), a, b < p -> r < p.
__device__ __forceinline__ void fp_mul_cios_body(fp& r, const fp& a, const fp& b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = b.l[i];
    uint64_t A = (uint64_t)a.l[0] * bi + t[0];
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * LB_P_INV32;
    uint64_t C = (uint64_t)m * P_[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; j++) {
      A = (uint64_t)a.l[j] * bi + (uint64_t)t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * P_[j] + (uint64_t)t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[11] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  uint32_t s[12];
  uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = __builtin_subc(t[j], P_[j], br, &br);
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = br ? t[j] : s[j];
}

}  // namespace lb
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

LB_NOINL fp_ret fp_mul_cios_r(LB_FP_PARAMS(a), LB_FP_PARAMS(b)) {
  const fp A = LB_FP_PACK(a), B = LB_FP_PACK(b);
  fp r;
  fp_mul_cios_body(r, A, B);
  return fp_ret{r.l[0], r.l[1], r.l[2], r.l[3], r.l[4], r.l[5], r.l[6], r.l[7], r.l[8], r.l[9], r.l[10], r.l[11]};
}
LB_DEV void mul_cios(fp& r, const fp& a, const fp& b) { fp_unret(r, fp_mul_cios_r(LB_FP_ARGS(a), LB_FP_ARGS(b))); }
LB_NOINL fp_ret fp_mul_ps_r(LB_FP_PARAMS(a), LB_FP_PARAMS(b)) {
  const fp A = LB_FP_PACK(a), B = LB_FP_PACK(b);
  fp r;
  fp_mul_ps_body(r, A, B);
  return fp_ret{r.l[0], r.l[1], r.l[2], r.l[3], r.l[4], r.l[5], r.l[6], r.l[7], r.l[8], r.l[9], r.l[10], r.l[11]};
}
LB_NOINL fp_ret fp_sqr_ps_r(LB_FP_PARAMS(a)) {
  const fp A = LB_FP_PACK(a);
  fp r;
  fp_sqr_ps_body(r, A);
  return fp_ret{r.l[0], r.l[1], r.l[2], r.l[3], r.l[4], r.l[5], r.l[6], r.l[7], r.l[8], r.l[9], r.l[10], r.l[11]};
}
LB_DEV void mul_ps(fp& r, const fp& a, const fp& b) { fp_unret(r, fp_mul_ps_r(LB_FP_ARGS(a), LB_FP_ARGS(b))); }
LB_DEV void sqr_ps(fp& r, const fp& a) { fp_unret(r, fp_sqr_ps_r(LB_FP_ARGS(a))); }

__device__ void seed_fp(fp& a, uint32_t s) {
  for (int j = 0; j < 12; j++) a.l[j] = s * 2654435761u + j * 40503u + (s >> 3) + j * s * 77u;
  a.l[11] &= 0x0fffffff;
}
template <int V>
__global__ void k_mul(uint32_t* out, int iters) {
  fp a, b, c;
  seed_fp(a, threadIdx.x + 1); seed_fp(b, blockIdx.x + 7); seed_fp(c, threadIdx.x * 3 + 5);
  for (int k = 0; k < iters; k++) {
    if (V == 0) { mul_cios(a, a, b); mul_cios(c, c, b); }
    if (V == 1) { mul_ps(a, a, b); mul_ps(c, c, b); }
    if (V == 2) { fp_sqr(a, a); fp_sqr(c, c); }
    if (V == 3) { sqr_ps(a, a); sqr_ps(c, c); }
  }
  uint32_t s = 0;
  for (int j = 0; j < 12; j++) s ^= a.l[j] ^ c.l[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_check(uint32_t* bad, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp a, b, r1, r2, one;
  seed_fp(a, i * 7 + 3); seed_fp(b, i * 13 + 11);
  fp_one(one);
  fp_mul(a, a, one); fp_mul(b, b, one);
  if (i == 0) { for (int j = 0; j < 12; j++) { a.l[j] = P_[j]; b.l[j] = P_[j]; } a.l[0] -= 1; b.l[0] -= 1; }  // p-1
  for (int k = 0; k < 16; k++) {
    mul_cios(r1, a, b); mul_ps(r2, a, b);
    if (!fp_eq(r1, r2)) atomicAdd(bad, 1u);
    fp_sqr(r1, a); sqr_ps(r2, a);
    if (!fp_eq(r1, r2)) atomicAdd(bad + 1, 1u);
    a = r1; fp_add(b, b, r2);
  }
}
template <typename K>
static void run(K kern, uint32_t* buf, int blocks, int threads, int iters, double per_lane, const char* name) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, iters);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, iters);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * threads * iters * per_lane;
  printf("%-14s blocks=%5d thr=%4d %8.3f ms  %.3e op/s  cyc/wave-op(chip)=%.0f  lane latency %.3f us/op\n", name, blocks, threads, ms,
         ops / (ms * 1e-3), 1024 * 2.4e9 / (ops / (ms * 1e-3)) * 64, ms * 1e3 / (iters * per_lane));
}
int main() {
  uint32_t* buf; CHK(hipMalloc(&buf, 64 << 20));
  uint32_t* bad; CHK(hipMalloc(&bad, 8)); CHK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, bad, 1024 * 256);
  uint32_t hb[2] = {0, 0}; CHK(hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost));
  printf("mismatch mul_ps: %u  sqr_ps: %u\n", hb[0], hb[1]);
  for (int occ : {1, 2, 4, 8}) {
    int blocks = 256 * 4 * occ;
    printf("-- %d waves/SIMD (%d blocks of 64)\n", occ, blocks);
    run(k_mul<0>, buf, blocks, 64, 256, 2, "fp_mul(cios)");
    run(k_mul<1>, buf, blocks, 64, 256, 2, "fp_mul(ps)");
    run(k_mul<2>, buf, blocks, 64, 256, 2, "fp_sqr(lib)");
    run(k_mul<3>, buf, blocks, 64, 256, 2, "fp_sqr(ps)");
  }
  run(k_mul<0>, buf, 1, 64, 2048, 2, "cios_1w");
  run(k_mul<1>, buf, 1, 64, 2048, 2, "ps_1w");
  run(k_mul<3>, buf, 1, 64, 2048, 2, "sqrps_1w");
  return (hb[0] || hb[1]) ? 1 : 0;
}
