// Test-only HIP library for the row-cooperative Fp layer (bls_coop.h): one
// element per 16-lane row, 16 words per element in memory (limbs 0..11, the
// rest zero).  tests/test_gpu_coop.py checks every output against Python big
// integers; op 1 also times a dependent chain of products (s_memtime ticks).
// Never linked into the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_coop.h"

namespace {
using namespace lb::co;

// op 0: out = mont_mul(a, b)
// op 1: x = a; k times x = mont_mul(x, b); out = x; cyc[item] = ticks of the chain
// op 2: T = c0 a + c1 b + c2 c + c3 d + K p (coefs/K from aux[item*8 ..]):
//       out = norm(T) (13 limbs), out2 = reduce(T)
// op 3: out = canon(a); aux_out[item*4 + 0..2] = is_zero, gt_half(canon(from_mont... raw)), bit0
// op 4: out = a - b (borrow lookahead), aux_out[item*4] = a >= b
// op 5: out = a^-1 mod p (row_inv_raw; raw a < p); cyc[item] = ticks of the wave's inversions
__global__ void k_coop(int op, uint32_t n, uint32_t k, const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                       const uint32_t* __restrict__ c, const uint32_t* __restrict__ d, const int32_t* __restrict__ aux,
                       uint32_t* __restrict__ out, uint32_t* __restrict__ out2, uint32_t* __restrict__ aux_out,
                       unsigned long long* __restrict__ cyc) {
  const uint32_t item = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const uint32_t j = lane16();
  if (item >= n) return;  // whole rows exit together
  const size_t o = (size_t)item * 16 + j;
  const uint32_t pj = p_limb();
  const uint32_t va = a[o];
  if (op == 0) {
    out[o] = mont_mul(va, b[o], pj);
  } else if (op == 1) {
    uint32_t x = va;
    const uint32_t y = b[o];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (uint32_t i = 0; i < k; i++) x = mont_mul(x, y, pj);
    out[o] = x;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (j == 0) cyc[item] = t1 - t0;
  } else if (op == 2) {
    const int32_t* q = aux + (size_t)item * 8;
    const uint32_t v[4] = {va, b[o], c[o], d[o]};
    uint64_t P = 0, N = 0;
#pragma unroll 1
    for (int t = 0; t < 4; t++) {
      const int32_t cf = q[t];
      if (cf >= 0)
        P += (uint64_t)(uint32_t)cf * v[t];
      else
        N += (uint64_t)(uint32_t)(-cf) * v[t];
    }
    P += (uint64_t)(uint32_t)q[4] * pj;
    const uint32_t T = norm<true>((int64_t)(P - N));
    out[o] = T;
    out2[o] = reduce(T, pj);
  } else if (op == 3) {
    const uint32_t cv = canon(va, pj);
    out[o] = cv;
    const bool z = row_is_zero(cv), g = row_gt_half(cv);
    const uint32_t b0 = row_bit0(cv);
    if (j == 0) {
      aux_out[item * 4 + 0] = z;
      aux_out[item * 4 + 1] = g;
      aux_out[item * 4 + 2] = b0;
    }
  } else if (op == 4) {
    bool ge;
    out[o] = sub_cmp(va, b[o], ge);
    if (j == 0) aux_out[item * 4] = ge;
  } else if (op == 5) {
    // out = a^-1 mod p (raw a < p, 0 -> 0): every row of the wave, one after the other
    uint32_t r = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint64_t m = ballot(j == 0); m; m &= m - 1) {
      const uint32_t base = (uint32_t)__builtin_ctzll(m);
      const bool mine = (lane64() & ~15u) == base;
      const uint32_t ri = row_inv_raw(va, mine, base, pj);
      if (mine) r = ri;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[o] = r;
    if (j == 0) cyc[item] = t1 - t0;
  }
}

}  // namespace

extern "C" int lbt_coop_op(int op, uint32_t n, uint32_t k, const uint32_t* a, const uint32_t* b, const uint32_t* c,
                           const uint32_t* d, const int32_t* aux, uint32_t* out, uint32_t* out2, uint32_t* aux_out,
                           unsigned long long* cyc, uint32_t waves_per_block, float* ms) {
  const size_t ew = (size_t)n * 16 * 4;
  uint32_t *da = nullptr, *db = nullptr, *dc = nullptr, *dd = nullptr, *dout = nullptr, *dout2 = nullptr, *daux_out = nullptr;
  int32_t* daux = nullptr;
  unsigned long long* dcyc = nullptr;
  if (hipMalloc(&da, ew) || hipMalloc(&db, ew) || hipMalloc(&dc, ew) || hipMalloc(&dd, ew) || hipMalloc(&dout, ew) ||
      hipMalloc(&dout2, ew) || hipMalloc(&daux, (size_t)n * 32 + 32) || hipMalloc(&daux_out, (size_t)n * 16 + 16) ||
      hipMalloc(&dcyc, (size_t)n * 8 + 8))
    return -2;
  hipMemcpy(da, a, ew, hipMemcpyHostToDevice);
  hipMemcpy(db, b ? b : a, ew, hipMemcpyHostToDevice);
  hipMemcpy(dc, c ? c : a, ew, hipMemcpyHostToDevice);
  hipMemcpy(dd, d ? d : a, ew, hipMemcpyHostToDevice);
  if (aux) hipMemcpy(daux, aux, (size_t)n * 32, hipMemcpyHostToDevice);
  hipMemset(dout, 0, ew);
  hipMemset(dout2, 0, ew);
  const uint32_t tpb = 64 * (waves_per_block ? waves_per_block : 1);
  const uint32_t rows_per_block = tpb / 16;
  const uint32_t grid = (n + rows_per_block - 1) / rows_per_block;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_coop, dim3(grid), dim3(tpb), 0, 0, op, n, k, da, db, dc, dd, daux, dout, dout2, daux_out, dcyc);
  hipEventRecord(e1, 0);
  int rc = hipDeviceSynchronize() == hipSuccess ? 0 : -3;
  if (ms) hipEventElapsedTime(ms, e0, e1);
  hipMemcpy(out, dout, ew, hipMemcpyDeviceToHost);
  if (out2) hipMemcpy(out2, dout2, ew, hipMemcpyDeviceToHost);
  if (aux_out) hipMemcpy(aux_out, daux_out, (size_t)n * 16, hipMemcpyDeviceToHost);
  if (cyc) hipMemcpy(cyc, dcyc, (size_t)n * 8, hipMemcpyDeviceToHost);
  hipFree(da);
  hipFree(db);
  hipFree(dc);
  hipFree(dd);
  hipFree(dout);
  hipFree(dout2);
  hipFree(daux);
  hipFree(daux_out);
  hipFree(dcyc);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return rc;
}
