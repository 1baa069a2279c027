// Helper kernels: point sums, serialization, stage-level parity kernels, synthetic signer.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

// ---- generic point sums (one workgroup, LDS tree) ------------------------
template <class F>
__global__ void __launch_bounds__(256) k_jac_sum(uint32_t n, const jac<F>* __restrict__ in, jac<F>* __restrict__ out) {
  __shared__ LdsRec<jac<F>> sh[256];
  jac<F> acc;
  jac_set_inf(acc);
  for (uint32_t i = threadIdx.x; i < n; i += 256) {
    jac<F> t = in[i];
    jac_add(acc, acc, t);
  }
  sh[threadIdx.x].v = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      jac<F> m = sh[threadIdx.x].v, o = sh[threadIdx.x + s].v;
      jac_add(m, m, o);
      sh[threadIdx.x].v = m;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = sh[0].v;
}

// A priority call's host <-> device copies as a kernel: the GPU reads / writes the pinned
// host buffer over PCIe.  hipMemcpyAsync goes to an SDMA engine, where a priority call's
// few KB waited behind the throughput calls' megabytes of staging (40-80 ms under load,
// profiles/r05/node_q/).  Grid-stride, 16 bytes per thread where both ends are aligned.
__global__ void __launch_bounds__(256) k_copy_bytes(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                    uint32_t n) {
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t done = 0;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
    const uint32_t n16 = n >> 4;
    for (uint32_t k = i; k < n16; k += stride)
      reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
    done = n16 << 4;
  }
  for (uint32_t k = done + i; k < n; k += stride) dst[k] = src[k];
}

__global__ void k_g1_serialize(uint32_t n, const g1j* __restrict__ in, uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1j p = in[i];
  g1a a;
  jac_to_aff(a, p);
  g1_serialize(out96 + (size_t)i * 96, a);
}
__global__ void k_g2_serialize(uint32_t n, const g2j* __restrict__ in, uint8_t* __restrict__ out192) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2j p = in[i];
  g2a a;
  jac_to_aff(a, p);
  g2_serialize(out192 + (size_t)i * 192, a);
}
// ---- device-resident pubkey table (index2pubkey mirror) ----------------------
// syncPubkeys (state-transition/src/cache/pubkeyCache.ts:56-77) pushes
// PublicKey.fromBytes(pubkey) per new validator: decode only (48-byte
// compressed as the state holds it, or 96-byte uncompressed), no group check.
__global__ void __launch_bounds__(TPB) k_table_decode(uint32_t n, const uint8_t* __restrict__ in, uint32_t len,
                                                      g1a* __restrict__ out, uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a p;
  status[i] = g1_deserialize(p, in + (size_t)i * len, len);
  out[i] = p;
}
// PublicKey.fromBytes(bytes, affine, validate=true) (blst key_validate: a valid
// encoding, not infinity, in G1), re-encoded uncompressed; the BLS-to-execution
// change pubkeys of a capella+ block (signatureSets/blsToExecutionChange.ts:30)
__global__ void __launch_bounds__(TPB) k_pubkey_validate(uint32_t n, const uint8_t* __restrict__ in, uint32_t len,
                                                         uint8_t* __restrict__ out96, uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a p;
  uint8_t st = g1_deserialize(p, in + (size_t)i * len, len);
  if (st == LB_ST_OK && p.inf) st = LB_ST_PK_INFINITY;
  if (st == LB_ST_OK) {
    g1j j;
    jac_from_aff(j, p);
    if (!g1_in_subgroup(j)) st = LB_ST_NOT_IN_GROUP;
  }
  if (st != LB_ST_OK) p.inf = true;
  g1_serialize(out96 + (size_t)i * 96, p);
  status[i] = st;
}

__global__ void k_g1a_serialize(uint32_t n, const g1a* __restrict__ in, uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a a = in[i];
  g1_serialize(out96 + (size_t)i * 96, a);
}

__global__ void k_g2a_serialize(uint32_t n, const g2a* __restrict__ in, uint8_t* __restrict__ out192) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a = in[i];
  g2_serialize(out192 + (size_t)i * 192, a);
}

// ---- stage-level kernels for parity tests ---------------------------------
__global__ void k_scalars(const uint8_t* __restrict__ seed, uint32_t first, uint32_t n, uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t sd[32];
  for (int k = 0; k < 32; k++) sd[k] = seed[k];
  out[i] = batch_scalar(sd, first + i);
}
__global__ void k_g1_mul(uint32_t n, const uint8_t* __restrict__ in, const uint64_t* __restrict__ k,
                         uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a a;
  g1_deserialize(a, in + (size_t)i * 96, 96);
  g1j p, r;
  jac_from_aff(p, a);
  jac_mul_u64(r, p, k[i]);
  jac_to_aff(a, r);
  g1_serialize(out + (size_t)i * 96, a);
}
__global__ void k_g2_mul(uint32_t n, const uint8_t* __restrict__ in, const uint64_t* __restrict__ k,
                         uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  g2_deserialize(a, in + (size_t)i * 192, 192);
  g2j p, r;
  jac_from_aff(p, a);
  jac_mul_u64(r, p, k[i]);
  jac_to_aff(a, r);
  g2_serialize(out + (size_t)i * 192, a);
}

// ---- synthetic data generation (bench / tests): SecretKey.toPublicKey, sign --
__global__ void __launch_bounds__(TPB) k_sk_to_pk(uint32_t n, const uint8_t* __restrict__ sk32,
                                                  uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t k[32];
  for (int b = 0; b < 32; b++) k[b] = sk32[(size_t)i * 32 + b];
  g1j g, r;
  fp_set(g.X, LB_G1_X);
  fp_set(g.Y, LB_G1_Y);
  fp_one(g.Z);
  jac_mul_be32(r, g, k);
  g1a a;
  jac_to_aff(a, r);
  g1_serialize(out96 + (size_t)i * 96, a);
}
__global__ void __launch_bounds__(TPB) k_sign(uint32_t n, const uint8_t* __restrict__ sk32,
                                              const uint8_t* __restrict__ msgs, uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t k[32], m[32];
  for (int b = 0; b < 32; b++) {
    k[b] = sk32[(size_t)i * 32 + b];
    m[b] = msgs[(size_t)i * 32 + b];
  }
  g2j h, r;
  hash_to_g2(h, m);
  jac_mul_be32(r, h, k);
  g2a a;
  jac_to_aff(a, r);
  g2_compress(out96 + (size_t)i * 96, a);
}

template __global__ void k_jac_sum<fp>(uint32_t, const jac<fp>* __restrict__, jac<fp>* __restrict__);
template __global__ void k_jac_sum<fp2>(uint32_t, const jac<fp2>* __restrict__, jac<fp2>* __restrict__);

}  // namespace lb
