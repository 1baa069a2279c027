// Test-only HIP library: the field primitives behind the lazy-reduction Fp2
// product and the register-window exponentiation, one element per lane, raw
// little-endian 32-bit limbs in Montgomery form.  tests/test_gpu_field.py feeds
// edge cases (0, 1, p - 1, limbs of all ones, 2p - 1 where the bound allows)
// and checks every output against Python big integers.  Never linked into the
// product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_field.h"

namespace {
using namespace lb;

LB_DEV void load(fp& a, const uint32_t* p) {
#pragma unroll
  for (int j = 0; j < 12; j++) a.l[j] = p[j];
}
LB_DEV void store(uint32_t* p, const fp& a) {
#pragma unroll
  for (int j = 0; j < 12; j++) p[j] = a.l[j];
}

// op 0: fp2_mul (a, b: 24 limbs each) -> 24 limbs
// op 1: fp_mulw (a, b: 12 limbs)      -> 24 limbs (double width)
// op 2: fp_redc (a: 24 limbs)         -> 12 limbs
// op 3: fp_pow_p34 (a: 12 limbs)      -> 12 limbs
// op 4: fp_mul (a, b: 12 limbs)       -> 12 limbs
// op 5: fp_sqr (a: 12 limbs)          -> 12 limbs
__global__ void k_selftest(int op, uint32_t n, const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                           uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (op == 0) {
    fp2 x, y, r;
    load(x.c0, a + 24 * i);
    load(x.c1, a + 24 * i + 12);
    load(y.c0, b + 24 * i);
    load(y.c1, b + 24 * i + 12);
    fp2_mul(r, x, y);
    store(out + 24 * i, r.c0);
    store(out + 24 * i + 12, r.c1);
  } else if (op == 1) {
    fp x, y;
    load(x, a + 12 * i);
    load(y, b + 12 * i);
    uint32_t w[24];
    fp_mulw(w, x, y);
    for (int j = 0; j < 24; j++) out[24 * i + j] = w[j];
  } else if (op == 2) {
    uint32_t w[24];
    for (int j = 0; j < 24; j++) w[j] = a[24 * i + j];
    fp r;
    fp_redc(r, w);
    store(out + 12 * i, r);
  } else if (op == 3) {
    fp x, r;
    load(x, a + 12 * i);
    fp_pow_p34(r, x);
    store(out + 12 * i, r);
  } else if (op == 4) {
    fp x, y, r;
    load(x, a + 12 * i);
    load(y, b + 12 * i);
    fp_mul(r, x, y);
    store(out + 12 * i, r);
  } else {
    fp x, r;
    load(x, a + 12 * i);
    fp_sqr(r, x);
    store(out + 12 * i, r);
  }
}
}  // namespace

// Host-buffer entry: copies in, runs op over n elements, copies out.  0 = ok.
extern "C" int lbt_field_op(int op, uint32_t n, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  const size_t wa = (op == 0 || op == 2) ? 24 : 12, wb = op == 0 ? 24 : 12;
  const size_t wo = (op == 0 || op == 1) ? 24 : 12;
  uint32_t *da = nullptr, *db = nullptr, *dout = nullptr;
  if (hipMalloc(&da, n * wa * 4) != hipSuccess || hipMalloc(&db, n * wb * 4) != hipSuccess ||
      hipMalloc(&dout, n * wo * 4) != hipSuccess)
    return 1;
  int rc = 0;
  if (hipMemcpy(da, a, n * wa * 4, hipMemcpyHostToDevice) != hipSuccess) rc = 2;
  if (!rc && b && hipMemcpy(db, b, n * wb * 4, hipMemcpyHostToDevice) != hipSuccess) rc = 2;
  if (!rc) {
    hipLaunchKernelGGL(k_selftest, dim3((n + 63) / 64), dim3(64), 0, 0, op, n, da, db, dout);
    if (hipDeviceSynchronize() != hipSuccess) rc = 3;
  }
  if (!rc && hipMemcpy(out, dout, n * wo * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = 4;
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return rc;
}
