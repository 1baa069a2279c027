// Per-set input stages: request flags, signature decode + G2 subgroup check, pubkey decode/aggregation.
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

__global__ void __launch_bounds__(TPB) k_req_flags(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                   uint8_t* __restrict__ single_flag) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req) return;
  const uint32_t a = req_off[k], b = req_off[k + 1];
  for (uint32_t i = a; i < b; i++) single_flag[i] = (b - a == 1) ? 1 : 0;
}

// Signature.fromBytes(validate=true); for single-set requests also the
// ZeroSignatureError of @chainsafe/bls Signature.verify.
__global__ void __launch_bounds__(TPB, LB_W_DECODE) k_decode_sigs(uint32_t n, const uint8_t* __restrict__ sigs,
                                                     const uint32_t* __restrict__ sig_off,
                                                     const uint8_t* __restrict__ single_flag,
                                                     g2j* __restrict__ out_sig, uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t a = sig_off[i], b = sig_off[i + 1];
  g2a s;
  uint8_t st = g2_deserialize(s, sigs + a, b - a);
  g2j sj;
  jac_set_inf(sj);
  if (st == LB_ST_OK) jac_from_aff(sj, s);
#ifdef LB_DECODE_REGS
  out_sig[i] = sj;
  if (st == LB_ST_OK) {
    const bool in_group = g2_in_subgroup(sj);
    if (!in_group) st = LB_ST_NOT_IN_GROUP;
    else if (single_flag && single_flag[i] && s.inf) st = LB_ST_ZERO_SIGNATURE;
  }
  status[i] = st;
#else
  // the decoded point waits in its output slot across the subgroup check's ladder;
  // the status is final before it (only a failed check rewrites it), so nothing but
  // the ladder's own state lives across it
  if (st == LB_ST_OK && s.inf && single_flag && single_flag[i]) st = LB_ST_ZERO_SIGNATURE;
  const bool ladder = st == LB_ST_OK && !s.inf;  // (infinity is in the group)
  out_sig[i] = sj;
  status[i] = st;
  if (ladder && !g2_in_subgroup_mem(out_sig + i)) status[i] = LB_ST_NOT_IN_GROUP;
#endif
}

// Sets with exactly one pubkey (the common case): one lane per set.
__global__ void __launch_bounds__(TPB) k_pubkeys_single(uint32_t n_sets, PkSource pks,
                                                        const uint32_t* __restrict__ pk_off, g1j* __restrict__ out_pk,
                                                        uint8_t* __restrict__ pk_status) {
  const uint32_t set = blockIdx.x * blockDim.x + threadIdx.x;
  if (set >= n_sets) return;
  const uint32_t a = pk_off ? pk_off[set] : set, b = pk_off ? pk_off[set + 1] : set + 1;
  if (b - a > 1) return;  // aggregate: k_pubkeys_agg
  g1j acc;
  jac_set_inf(acc);
  uint8_t st = LB_ST_EMPTY_AGGREGATE;
  if (b == a + 1) {
    g1a p;
    st = pk_load(p, pks, a);
    if (st == LB_ST_OK) {
      jac_from_aff(acc, p);
      if (p.inf) st = LB_ST_PK_INFINITY;
    } else {
      st = LB_ST_BAD_ENCODING;
    }
  }
  out_pk[set] = acc;
  pk_status[set] = st;
}

// Sets with >= 2 pubkeys (PublicKey.aggregate, chain/bls/utils.ts:13): one
// wave per set, grid-stride over sets; lanes decode strided, LDS tree sum.
__global__ void __launch_bounds__(TPB) k_pubkeys_agg(uint32_t n_sets, PkSource pks,
                                                     const uint32_t* __restrict__ pk_off, g1j* __restrict__ out_pk,
                                                     uint8_t* __restrict__ pk_status) {
  __shared__ LdsRec<g1j> sh[TPB];
  __shared__ uint32_t bad;
  if (!pk_off) return;
  for (uint32_t set = blockIdx.x; set < n_sets; set += gridDim.x) {
    const uint32_t a = pk_off[set], b = pk_off[set + 1];
    if (b - a <= 1) continue;  // uniform across the block
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    g1j acc;
    jac_set_inf(acc);
    for (uint32_t k = a + threadIdx.x; k < b; k += TPB) {
      g1a p;
      const uint8_t st = pk_load(p, pks, k);
      if (st != LB_ST_OK) {
        atomicOr(&bad, 1u);
      } else {
        jac_add_aff(acc, acc, p);
      }
    }
    sh[threadIdx.x].v = acc;
    __syncthreads();
    for (int s = TPB / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s && a + threadIdx.x + s < b) {
        g1j o = sh[threadIdx.x + s].v;
        g1j m = sh[threadIdx.x].v;
        jac_add(m, m, o);
        sh[threadIdx.x].v = m;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      out_pk[set] = sh[0].v;
      pk_status[set] = bad ? LB_ST_BAD_ENCODING : jac_is_inf(sh[0].v) ? LB_ST_PK_INFINITY : LB_ST_OK;
    }
    __syncthreads();
  }
}

// Same-message jobs (jobItemWorkReq sameMessage, chain/bls/multithread/jobItem.ts:64-86):
// one wave per job j sums the job's validated signatures (decoded ONCE by
// k_decode_sigs) and writes the aggregate's 192-byte uncompressed encoding
// (Signature.aggregate(sigs).toBytes(uncompressed)) and the aggregated pubkey's
// 96-byte encoding as the inputs of a 1-set request.  A job with any signature
// that failed Signature.fromBytes(validate=true) would have thrown on the main
// thread (-> per-set retry, index.ts:411-414): its aggregate is written as an
// invalid encoding (all zero bytes: compression flag clear, infinity flag clear
// -> BAD_ENCODING), so its request is false, and job_bad[j] = 1.
__global__ void __launch_bounds__(TPB) k_same_message_agg(uint32_t n_jobs, const uint32_t* __restrict__ job_off,
                                                          const g2j* __restrict__ sig,
                                                          const uint8_t* __restrict__ sig_status,
                                                          const g1j* __restrict__ job_pk, uint8_t* __restrict__ out_pk96,
                                                          uint8_t* __restrict__ out_sig192,
                                                          uint8_t* __restrict__ job_bad) {
  __shared__ LdsRec<g2j> sh[TPB];
  __shared__ uint32_t bad;
  for (uint32_t j = blockIdx.x; j < n_jobs; j += gridDim.x) {
    const uint32_t a = job_off[j], b = job_off[j + 1];
    if (threadIdx.x == 0) bad = (a == b) ? 1u : 0u;
    __syncthreads();
    g2j acc;
    jac_set_inf(acc);
    for (uint32_t i = a + threadIdx.x; i < b; i += TPB) {
      if (sig_status[i] != LB_ST_OK) {
        atomicOr(&bad, 1u);
      } else {
        g2j t = sig[i];
        jac_add(acc, acc, t);
      }
    }
    sh[threadIdx.x].v = acc;
    __syncthreads();
    for (int s = TPB / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s && a + threadIdx.x + s < b) {
        g2j o = sh[threadIdx.x + s].v;
        g2j m = sh[threadIdx.x].v;
        jac_add(m, m, o);
        sh[threadIdx.x].v = m;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      uint8_t* os = out_sig192 + (size_t)j * 192;
      if (bad) {
        for (int k = 0; k < 192; k++) os[k] = 0;
      } else {
        g2j tot = sh[0].v;
        g2a s;
        jac_to_aff(s, tot);
        g2_serialize(os, s);
      }
      g1j p = job_pk[j];
      g1a pa;
      jac_to_aff(pa, p);
      g1_serialize(out_pk96 + (size_t)j * 96, pa);
      job_bad[j] = bad ? 1 : 0;
    }
    __syncthreads();
  }
}

}  // namespace lb
