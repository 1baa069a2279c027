// Latency of the wave-cooperative Fp12 ops (bls_wc12.h) on gfx950: one
// workgroup runs N ops of one kind back to back; reports us per op.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o wc_bench wc_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../lodestar_amd/csrc/bls_kernels.h"
#include "../../lodestar_amd/csrc/bls_wc12.h"

using namespace lb;
#define CHK(x)                                                \
  do {                                                        \
    hipError_t e = (x);                                       \
    if (e != hipSuccess) {                                    \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                \
    }                                                         \
  } while (0)

__global__ void __launch_bounds__(64, 1) k_bench(int op, int n, uint32_t* out, long long* cyc) {
  __shared__ wc_smem S;
  wc_init_tables(S);
  wc_init_gammas(S);
  if (threadIdx.x < 12) {
    fp v;
    for (int j = 0; j < 12; j++) v.l[j] = (threadIdx.x + 1) * 2654435761u + j;
    v.l[11] &= 0x0fffffff;
    S.slot[WC_F][threadIdx.x] = v;
    S.slot[WC_T0][threadIdx.x] = v;
    S.slot[WC_LINE][threadIdx.x] = v;
  }
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < n; i++) {
    if (op == 100) {
      __syncthreads();  // barrier-only baseline
    } else if (op == 101) {
      if (threadIdx.x < 12) {  // one fp_mul per lane, no LDS program
        fp a = S.slot[WC_F][threadIdx.x], b = S.slot[WC_T0][threadIdx.x];
        fp_mul(a, a, b);
        S.slot[WC_F][threadIdx.x] = a;
      }
      __syncthreads();
    } else {
      wc_apply(S, op, WC_F, WC_F, op == LB_WC_LINE ? WC_LINE : WC_T0);
    }
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    out[0] = S.slot[WC_F][0].l[0];
  }
}

int main() {
  uint32_t* out;
  long long* cyc;
  CHK(hipMalloc(&out, 64));
  CHK(hipMalloc(&cyc, 64));
  const int n = 200;
  const char* names[] = {"MUL", "SQR", "CYC", "LINE", "FROB1", "FROB2", "FROB3", "CONJ"};
  int ops[] = {100, 101, LB_WC_MUL, LB_WC_SQR, LB_WC_CYC, LB_WC_LINE, LB_WC_FROB1, LB_WC_CONJ};
  for (int k = 0; k < 8; k++) {
    const int op = ops[k];
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, op, n, out, cyc);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, op, n, out, cyc);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    long long c = 0;
    CHK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    printf("%-10s %8.2f us/op  %9.0f clk64/op\n", op == 100 ? "barrier" : op == 101 ? "fp_mul x12" : names[op],
           ms * 1e3 / n, (double)c / n);
  }
  return 0;
}
