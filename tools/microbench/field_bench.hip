// Field-arithmetic microbenchmark on gfx950: throughput (full chip) and
// single-lane latency of the Fp / Fp2 / Fp12 primitives in bls_field.h, plus a
// self-check fp_sqr(a) == fp_mul(a, a).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o field_bench field_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../lodestar_amd/csrc/bls_field.h"

using namespace lb;
#define CHK(x)                                                        \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);         \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__device__ void seed_fp(fp& a, uint32_t s) {
  for (int j = 0; j < 12; j++) a.l[j] = s * 2654435761u + j * 40503u + (s >> 3);
  a.l[11] &= 0x0fffffff;
}

__global__ void k_mul(uint32_t* out, int iters) {
  fp a, b, c;
  seed_fp(a, threadIdx.x + 1);
  seed_fp(b, blockIdx.x + 7);
  seed_fp(c, threadIdx.x * 3 + 5);
  for (int k = 0; k < iters; k++) {
    fp_mul(a, a, b);
    fp_mul(c, c, b);
  }
  uint32_t s = 0;
  for (int j = 0; j < 12; j++) s ^= a.l[j] ^ c.l[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_sqr(uint32_t* out, int iters) {
  fp a, c;
  seed_fp(a, threadIdx.x + 1);
  seed_fp(c, threadIdx.x * 3 + 5);
  for (int k = 0; k < iters; k++) {
    fp_sqr(a, a);
    fp_sqr(c, c);
  }
  uint32_t s = 0;
  for (int j = 0; j < 12; j++) s ^= a.l[j] ^ c.l[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fp2mul(uint32_t* out, int iters) {
  fp2 a, b;
  seed_fp(a.c0, threadIdx.x + 1);
  seed_fp(a.c1, threadIdx.x + 2);
  seed_fp(b.c0, blockIdx.x + 3);
  seed_fp(b.c1, blockIdx.x + 4);
  for (int k = 0; k < iters; k++) fp2_mul(a, a, b);
  uint32_t s = 0;
  for (int j = 0; j < 12; j++) s ^= a.c0.l[j] ^ a.c1.l[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fp12mul(uint32_t* out, int iters) {
  fp12 a, b;
  fp2* pa = &a.c0.c0;
  fp2* pb = &b.c0.c0;
  for (int i = 0; i < 6; i++) {
    seed_fp(pa[i].c0, threadIdx.x + i);
    seed_fp(pa[i].c1, threadIdx.x + 2 * i);
    seed_fp(pb[i].c0, blockIdx.x + i);
    seed_fp(pb[i].c1, blockIdx.x + 3 * i);
  }
  for (int k = 0; k < iters; k++) fp12_mul(a, a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a.c0.c0.c0.l[0];
}
__global__ void k_check(uint32_t* bad, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp a, r1, r2, one;
  seed_fp(a, i * 7 + 3);
  // reduce a below p first
  fp_one(one);
  fp_mul(a, a, one);
  for (int k = 0; k < 8; k++) {
    fp_mul(r1, a, a);
    fp_sqr(r2, a);
    if (!fp_eq(r1, r2)) atomicAdd(bad, 1u);
    a = r1;
  }
}

template <typename K>
static void run(K kern, uint32_t* buf, int blocks, int threads, int iters, double per_lane, const char* name) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, iters);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, iters);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * threads * iters * per_lane;
  printf("%-12s blocks=%5d thr=%4d  %8.3f ms  %.3e op/s   lane latency %.2f us/op\n", name, blocks, threads, ms,
         ops / (ms * 1e-3), ms * 1e3 / (iters * per_lane));
}

int main() {
  uint32_t* buf;
  CHK(hipMalloc(&buf, 64 << 20));
  uint32_t* bad;
  CHK(hipMalloc(&bad, 4));
  CHK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, bad, 1024 * 256);
  uint32_t hb = 0;
  CHK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("sqr==mul self-check mismatches: %u\n", hb);
  run(k_mul, buf, 2048, 256, 256, 2, "fp_mul");
  run(k_sqr, buf, 2048, 256, 256, 2, "fp_sqr");
  run(k_fp2mul, buf, 2048, 256, 128, 1, "fp2_mul");
  run(k_fp12mul, buf, 1024, 256, 16, 1, "fp12_mul");
  run(k_mul, buf, 1, 64, 2048, 2, "fp_mul_1w");
  run(k_sqr, buf, 1, 64, 2048, 2, "fp_sqr_1w");
  run(k_fp12mul, buf, 1, 64, 64, 1, "fp12_mul_1w");
  return hb ? 1 : 0;
}
