// Microbenchmark: integer multiply-add issue rates on gfx950 (MI355X).
// Establishes the roofline peak used by bench.py (v_mad_u64_u32 per second).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// 8 independent 64-bit accumulators: acc = a*b + acc  (one v_mad_u64_u32 each)
__global__ void k_mad64(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) { acc[i] = (uint64_t)(a + i) * b + acc[i]; }
    asm volatile("" : "+v"(a));
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 8 independent 32-bit mul_lo (v_mul_lo_u32)
__global__ void k_mullo(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a = seed ^ threadIdx.x;
  uint32_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x + 1;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = acc[i] * a;
    asm volatile("" : "+v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 8 independent 24-bit mads (v_mad_u32_u24)
__global__ void k_mad24(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a = (seed ^ threadIdx.x) & 0xffffff;
  uint32_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x + 1;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (acc[i] & 0xffffff) * a + acc[i];
    asm volatile("" : "+v"(a));
  }
  out[0] = acc[0];
}

// 8 independent f64 FMAs
__global__ void k_fma64(double* out, double seed, int iters) {
  double a = seed + threadIdx.x, b = 1.0000001;
  double acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = __builtin_fma(acc[i], b, a);
    asm volatile("" : "+v"(a));
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 8 independent 32-bit adds (full-rate reference)
__global__ void k_add32(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a = seed ^ threadIdx.x;
  uint32_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x + 1;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (acc[i] ^ a) + i;
    asm volatile("" : "+v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


struct fp { uint32_t l[12]; };
#define PINV 0xfffcfffdu
static constexpr uint32_t PC[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
__device__ __forceinline__ fp fp_mul_cios(const fp& a, const fp& b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint32_t bi = b.l[i];
    uint64_t A = (uint64_t)a.l[0] * bi + t[0];
    t[0] = (uint32_t)A;
    uint32_t m = t[0] * PINV;
    uint64_t C = (uint64_t)m * PC[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; j++) {
      A = (uint64_t)a.l[j] * bi + (uint64_t)t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * PC[j] + (uint64_t)t[j] + (C >> 32);
      t[j-1] = (uint32_t)C;
    }
    t[11] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  uint32_t s[12]; uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) { s[j] = __builtin_subc(t[j], PC[j], borrow, &borrow); }
  fp r;
#pragma unroll
  for (int j = 0; j < 12; j++) r.l[j] = borrow ? t[j] : s[j];
  return r;
}
__global__ void k_fpmul(uint32_t* out, uint32_t seed, int iters) {
  fp a, b, c;
#pragma unroll
  for (int j = 0; j < 12; j++) { a.l[j] = seed * (j + 3) + threadIdx.x; b.l[j] = seed ^ (j * 977); c.l[j] = j + blockIdx.x; }
  a.l[11] &= 0xffffff; b.l[11] &= 0xffffff; c.l[11] &= 0xffffff;
  for (int k = 0; k < iters; k++) { a = fp_mul_cios(a, b); c = fp_mul_cios(c, b); }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) s ^= a.l[j] ^ c.l[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K, typename T>
static double run(K kern, T* buf, int blocks, int threads, int iters, double ops_per_iter_lane, const char* name) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, (T)7, iters);  // warmup
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, (T)7, iters);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double ops = (double)blocks * threads * iters * ops_per_iter_lane;
  double rate = ops / (ms * 1e-3);
  printf("%-10s blocks=%d threads=%d  %.3f ms  %.3e ops/s  (%.2f ops/clk/CU @2.4GHz)\n", name, blocks, threads, ms, rate,
         rate / 256 / 2.4e9);
  return rate;
}

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  void* buf; CHK(hipMalloc(&buf, 64 << 20));
  int blocks = 256 * 8, threads = 256, iters = 4096;
  run(k_mad64, (uint64_t*)buf, blocks, threads, iters, 8, "mad_u64");
  run(k_mullo, (uint32_t*)buf, blocks, threads, iters, 8, "mul_lo32");
  run(k_fma64, (double*)buf, blocks, threads, iters, 8, "fma_f64");
  run(k_add32, (uint32_t*)buf, blocks, threads, iters, 16, "xor+add32");
  run(k_fpmul, (uint32_t*)buf, blocks, threads, 256, 2, "fp_mul_cios");
  run(k_fpmul, (uint32_t*)buf, 256*4, 64, 256, 2, "fpmul_1w");
  run(k_mad64, (uint64_t*)buf, 256, 64, iters, 8, "mad_u64_1w");
  run(k_mad64, (uint64_t*)buf, 256 * 4, 64, iters, 8, "mad_u64_4w");
  return 0;
}
