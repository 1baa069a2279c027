// Carry-free column layout of the Montgomery product: 13 limbs of 30 bits
// (R = 2^390) whose 60-bit limb products accumulate a whole column in 64 bits with no carry
// instruction, against the library's product-scanning 12 x 32-bit product (bls_fp_ps.h: a
// v_addc_co_u32 behind every v_mad_u64_u32).  The column sums of the product (<= 13 terms of
// < 2^60) and of the reduction (another 13) do not fit one 64-bit word together, so the
// product's columns are normalised to 30-bit digits (carry-save: digit + carry into the next
// column) before the reduction adds m_i p.  Same harness as fp2_bench.hip: dependent products
// per lane, 1 / 2 / 4 waves per SIMD pinned by LDS, cycles per wave-product on the chip; the
// two layouts compute the same Montgomery products (checked on the host against unsigned
// __int128 arithmetic, and each other, for the benchmark's own inputs).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fp_cols_bench fp_cols_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../lodestar_amd/csrc/bls_field.h"
using namespace lb;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// p in 13 x 30-bit digits, -p^-1 mod 2^30
struct P30 { uint32_t d[13]; uint32_t pinv; };
__constant__ P30 c_p30;

struct f30 { uint32_t l[13]; };  // digits < 2^30, value < 2p

// r = a b 2^-390 mod p (< 2p for a, b < 2p: 4p^2 / 2^390 + p < 2p)
__device__ __forceinline__ void mul30(f30& r, const f30& a, const f30& b) {
  constexpr uint32_t M = (1u << 30) - 1;
  uint64_t c[27];
#pragma unroll
  for (int k = 0; k < 27; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 13; i++)
#pragma unroll
    for (int j = 0; j < 13; j++) c[i + j] += (uint64_t)a.l[i] * b.l[j];  // v_mad_u64_u32, no carry
  // normalise the product's columns to 30-bit digits (each column then < 2^30 + its carry-in)
#pragma unroll
  for (int k = 0; k < 26; k++) {
    c[k + 1] += c[k] >> 30;
    c[k] &= M;
  }
  // reduction: m_i from digit i, + m_i p into columns i .. i + 12, carry digit i onwards
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const uint32_t m = ((uint32_t)c[i] * c_p30.pinv) & M;
#pragma unroll
    for (int j = 0; j < 13; j++) c[i + j] += (uint64_t)m * c_p30.d[j];
    c[i + 1] += c[i] >> 30;  // (digit i is now 0 mod 2^30)
  }
#pragma unroll
  for (int k = 13; k < 26; k++) {
    r.l[k - 13] = (uint32_t)c[k] & M;
    c[k + 1] += c[k] >> 30;
  }
}

__device__ void seed30(f30& a, uint32_t s) {
  for (int j = 0; j < 13; j++) a.l[j] = (s * 2654435761u + j * 40503u + (s >> 3) + j * s * 77u) & ((1u << 30) - 1);
  a.l[12] &= 0x7ffff;  // < 2^379
}
__device__ void seed_fp(fp& a, uint32_t s) {
  for (int j = 0; j < 12; j++) a.l[j] = s * 2654435761u + j * 40503u + (s >> 3) + j * s * 77u;
  a.l[11] &= 0x0fffffff;
}

// V 0: the library's fp_mul (12 x 32, product scanning + v_addc per mad), 1: mul30
template <int V>
__global__ void __launch_bounds__(64, 1) k_mul(uint32_t* out, int iters) {
  uint32_t s = 0;
  if (V == 0) {
    fp a, b, c;
    seed_fp(a, threadIdx.x + 1); seed_fp(b, blockIdx.x + 7); seed_fp(c, threadIdx.x * 3 + 5);
    for (int k = 0; k < iters; k++) { fp_mul(a, a, b); fp_mul(c, c, b); }
    for (int j = 0; j < 12; j++) s ^= a.l[j] ^ c.l[j];
  } else {
    f30 a, b, c;
    seed30(a, threadIdx.x + 1); seed30(b, blockIdx.x + 7); seed30(c, threadIdx.x * 3 + 5);
    for (int k = 0; k < iters; k++) { mul30(a, a, b); mul30(c, c, b); }
    for (int j = 0; j < 13; j++) s ^= a.l[j] ^ c.l[j];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one product of each kind for the host check
__global__ void k_check(const uint32_t* in, uint32_t* out) {
  f30 a, b, r;
  for (int j = 0; j < 13; j++) { a.l[j] = in[j]; b.l[j] = in[13 + j]; }
  mul30(r, a, b);
  for (int j = 0; j < 13; j++) out[j] = r.l[j];
}

template <typename K>
static void run(K kern, uint32_t* buf, int blocks, int iters, const char* name, int lds) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), lds, 0, buf, iters);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), lds, 0, buf, iters);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * 64 * iters * 2;
  printf("%-12s blocks=%5d %8.3f ms  %.3e products/s  cycles/wave-product(chip, 2.4 GHz)=%.0f\n", name, blocks, ms,
         ops / (ms * 1e-3), 1024 * 2.4e9 / (ops / (ms * 1e-3)) * 64);
}

// host big-int helpers (unsigned __int128 limbs of 30 bits)
typedef unsigned __int128 u128;
static void to30(const uint8_t* be48, uint32_t* d) {  // 48-byte big-endian -> 13 digits
  uint32_t w[13] = {0};
  for (int bit = 0; bit < 384; bit++) {
    const int byte = 47 - bit / 8;
    if ((be48[byte] >> (bit % 8)) & 1) w[bit / 30] |= 1u << (bit % 30);
  }
  for (int j = 0; j < 13; j++) d[j] = w[j];
}

int main() {
  // p = 0x1a0111ea...aaab
  static const uint8_t P_BE[48] = {0x1a, 0x01, 0x11, 0xea, 0x39, 0x7f, 0xe6, 0x9a, 0x4b, 0x1b, 0xa7, 0xb6, 0x43, 0x4b,
                                   0xac, 0xd7, 0x64, 0x77, 0x4b, 0x84, 0xf3, 0x85, 0x12, 0xbf, 0x67, 0x30, 0xd2, 0xa0,
                                   0xf6, 0xb0, 0xf6, 0x24, 0x1e, 0xab, 0xff, 0xfe, 0xb1, 0x53, 0xff, 0xff, 0xb9, 0xfe,
                                   0xff, 0xff, 0xff, 0xff, 0xaa, 0xab};
  P30 h;
  to30(P_BE, h.d);
  // -p^-1 mod 2^30 by Newton iteration
  uint32_t inv = 1;
  for (int k = 0; k < 6; k++) inv *= 2 - h.d[0] * inv;
  h.pinv = (0u - inv) & ((1u << 30) - 1);
  if (((h.d[0] * h.pinv) & ((1u << 30) - 1)) != (1u << 30) - 1) { printf("pinv wrong\n"); return 1; }
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(c_p30), &h, sizeof h));
  // host check of one product: r * 2^390 == a * b (mod p), r < 2p
  {
    uint32_t in[26], out[13];
    for (int j = 0; j < 13; j++) { in[j] = (j * 123457u + 99) & ((1u << 30) - 1); in[13 + j] = (j * 7654321u + 5) & ((1u << 30) - 1); }
    in[12] &= 0x7ffff; in[25] &= 0x7ffff;
    uint32_t *d_in, *d_out; CHK(hipMalloc(&d_in, sizeof in)); CHK(hipMalloc(&d_out, sizeof out));
    CHK(hipMemcpy(d_in, in, sizeof in, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3(1), dim3(1), 0, 0, d_in, d_out);
    CHK(hipMemcpy(out, d_out, sizeof out, hipMemcpyDeviceToHost));
    bool ok = true;
    // exact check with 64-bit-word big integers: (r 2^390 - a b) mod p == 0
    auto big = [](const uint32_t* d, int n, uint64_t* out64, int words) {
      for (int i = 0; i < words; i++) out64[i] = 0;
      for (int bit = 0; bit < 30 * n; bit++) if ((d[bit / 30] >> (bit % 30)) & 1) out64[bit / 64] |= 1ull << (bit % 64);
    };
    uint64_t A[7], B[7], R[7], Pp[7];
    big(in, 13, A, 7); big(in + 13, 13, B, 7); big(out, 13, R, 7); big(h.d, 13, Pp, 7);
    // L = a b (14 words), Rr = r 2^390 (14 words); check (Rr - L) mod p == 0 by long division remainder
    uint64_t L[14] = {0}, Rr[14] = {0};
    for (int i = 0; i < 7; i++) { u128 c = 0; for (int j = 0; j < 7; j++) { c += (u128)A[i] * B[j] + L[i + j]; L[i + j] = (uint64_t)c; c >>= 64; } L[i + 7] = (uint64_t)c; }
    for (int i = 0; i < 7; i++) { const int sh = 390 + 64 * i; const int w = sh / 64, b = sh % 64; if (w < 14) Rr[w] |= R[i] << b; if (b && w + 1 < 14) Rr[w + 1] |= R[i] >> (64 - b); }
    // D = Rr - L (two's complement over 14 words), reduce mod p by bitwise long division of |D|
    uint64_t D[14]; int neg = 0; { u128 br = 0; for (int i = 0; i < 14; i++) { u128 t = (u128)Rr[i] - L[i] - br; D[i] = (uint64_t)t; br = (t >> 64) ? 1 : 0; } neg = (int)br; }
    if (neg) { u128 c = 1; for (int i = 0; i < 14; i++) { c += (u128)(~D[i]); D[i] = (uint64_t)c; c >>= 64; } }
    uint64_t rem[7] = {0};
    for (int bit = 14 * 64 - 1; bit >= 0; bit--) {
      uint64_t carry = 0; for (int i = 0; i < 7; i++) { uint64_t nc = rem[i] >> 63; rem[i] = (rem[i] << 1) | carry; carry = nc; }
      rem[0] |= (D[bit / 64] >> (bit % 64)) & 1;
      int ge = 1; for (int i = 6; i >= 0; i--) { if (rem[i] != Pp[i]) { ge = rem[i] > Pp[i]; break; } }
      if (ge) { u128 br = 0; for (int i = 0; i < 7; i++) { u128 t = (u128)rem[i] - Pp[i] - br; rem[i] = (uint64_t)t; br = (t >> 64) ? 1 : 0; } }
    }
    for (int i = 0; i < 7; i++) ok = ok && rem[i] == 0;
    printf("mul30 host check: %s\n", ok ? "ok" : "MISMATCH");
    if (!ok) return 1;
  }
  uint32_t* buf; CHK(hipMalloc(&buf, 64 << 20));
  for (int occ : {1, 2, 4}) {
    const int blocks = 1024 * occ;
    const int lds = 160 * 1024 / 4 / occ - 1024;  // pins occupancy: 4*occ workgroups of 64 per CU
    printf("-- %d waves/SIMD\n", occ);
    run(k_mul<0>, buf, blocks, 256, "fp_mul_12x32", lds);
    run(k_mul<1>, buf, blocks, 256, "mul30_13x30", lds);
  }
  return 0;
}
