// Random-scalar multi-scalar multiplication of the merged check:
//   S_all = sum over the sets i of the call's good requests of r_i sig_i,
// r_i = a_i + b_i lambda (the 2 x 32-bit GLV form of the batch scalar, see
// batch_scalar), as ONE bucket (Pippenger) MSM over the 2N half-points
//   P_2i = sig_i (scalar a_i),  P_2i+1 = [lambda] sig_i = (omega X_i, Y_i) (scalar b_i)
// instead of one 32-step GLV ladder per set (k_scalar_sig) and a sum per
// request (k_sum_tree).  This is the sum blst's mul_n_aggregate / finalverify
// accumulate for verifyMultipleSignatures (BN/chain/bls/maybeBatch.ts:19-26,
// SURVEY.md §8a row a14); the per-request sums S_k are only needed when the
// merged check fails (worker.ts:74-85 retry), and are then computed by the
// per-set ladders (run_tails in bls_host.hip).
//
// Geometry: signed digits of c = 11 bits, W = 3 windows (bits 0-10, 11-21,
// 22-31; the top window's raw 10 bits plus the carry stay <= 1024, so no
// fourth window), 1024 buckets per window (|digit| 1..1024), 3072 in all.
//   k_msm_scalars  one wave per request: request status, DRBG scalar, the six
//                  digits of a set's two half-points, bucket histogram
//   k_msm_scan     one workgroup: bucket offsets and chunk offsets (prefix sums)
//   k_msm_scatter  one lane per (point, window): counting-sort placement
//   k_msm_chunks   one lane per chunk of <= T entries of ONE bucket: mixed
//                  (Jacobian + affine) additions, the bulk of the work
//   k_msm_buckets  four lanes per bucket: sum of its chunk partials
//   k_msm_bits     256 threads per bit position p = 11 w + k: G_p = sum of the
//                  buckets d of window w with bit k of d set (two per thread,
//                  then an LDS tree)
//   k_msm_final    one wave: lane p doubles G_p p times, LDS tree, affine
// so sum_w 2^(11w) sum_d d B_(w,d) = sum_p 2^p G_p with no serial running sum
// over the 1024 buckets (critical path: T madds + ~8 adds + 13 adds + 32 dbl).
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
#include "bls_kernels.h"

namespace lb {

static_assert(32 - LB_MSM_C * (LB_MSM_W - 1) <= LB_MSM_C - 1, "top window must not carry");
static_assert((1u << (LB_MSM_C - 1)) == LB_MSM_NB, "bucket count = 2^(c-1)");
static_assert(LB_MSM_POS == LB_MSM_C * (LB_MSM_W - 1) + 11, "bit positions");

// keys of the W windows of one 32-bit scalar s: bucket (w NB + |d| - 1) with the
// digit's sign in bit 31, or LB_MSM_NONE for a zero digit
LB_DEV void msm_keys(uint32_t s, uint32_t* __restrict__ out) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < LB_MSM_W; w++) {
    const uint32_t raw = ((s >> (LB_MSM_C * w)) & ((1u << LB_MSM_C) - 1u)) + carry;
    int32_t d;
    if (raw > LB_MSM_NB) {  // never in the top window (static_assert above)
      d = (int32_t)raw - (int32_t)(1u << LB_MSM_C);
      carry = 1;
    } else {
      d = (int32_t)raw;
      carry = 0;
    }
    const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
    out[w] = d == 0 ? LB_MSM_NONE : ((uint32_t)w * LB_MSM_NB + mag - 1u) | (d < 0 ? 0x80000000u : 0u);
  }
}

// Request k is good when every set has a valid signature and pubkey (the
// request flags of k_miller_acc / k_prod_tree; bad requests are excluded from
// the merged check, k_merge).  For each set of a good request with a finite
// signature: its scalar (the caller's raw values, or the DRBG of the seed),
// the keys of its two half-points, and the bucket histogram.  Everything else
// gets LB_MSM_NONE keys.
__global__ void __launch_bounds__(TPB) k_msm_scalars(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                     const uint8_t* __restrict__ seed, const uint64_t* __restrict__ raw,
                                                     const g2j* __restrict__ sig, const uint8_t* __restrict__ sig_status,
                                                     const uint8_t* __restrict__ pk_status, uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ hist) {
  __shared__ uint32_t bad;
  const uint32_t k = blockIdx.x;
  if (k >= n_req) return;
  const uint32_t a = req_off[k], b = req_off[k + 1];
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (uint32_t i = a + threadIdx.x; i < b; i += TPB)
    if (sig_status[i] != LB_ST_OK || (pk_status && pk_status[i] != LB_ST_OK)) atomicOr(&bad, 1u);
  __syncthreads();
  const bool good = bad == 0;
  uint8_t sd[32];
  if (!raw)
    for (int j = 0; j < 32; j++) sd[j] = seed[j];
  for (uint32_t i = a + threadIdx.x; i < b; i += TPB) {
    uint32_t kk[2 * LB_MSM_W];
#pragma unroll
    for (int j = 0; j < 2 * LB_MSM_W; j++) kk[j] = LB_MSM_NONE;
    if (good && !jac_is_inf(sig[i])) {
      const uint64_t r = raw ? raw[i] : batch_scalar(sd, i);
      msm_keys((uint32_t)r, kk);
      msm_keys((uint32_t)(r >> 32), kk + LB_MSM_W);
#pragma unroll
      for (int j = 0; j < 2 * LB_MSM_W; j++)
        if (kk[j] != LB_MSM_NONE) atomicAdd(&hist[kk[j] & 0x7fffffffu], 1u);
    }
#pragma unroll
    for (int j = 0; j < 2 * LB_MSM_W; j++) keys[(size_t)i * 2 * LB_MSM_W + j] = kk[j];
  }
}

// Exclusive prefix sums over the 3072 buckets (one workgroup of 1024 lanes, 3
// buckets per lane): off = entries, coff = chunks of <= T entries; off/coff
// [LB_MSM_BUCKETS] are the totals.  Zeroes the scatter cursors.
// (T: the chunk size -- LB_MSM_T, or LB_MSM_T_LONE for a lone mid-size call's shorter chains)
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t* __restrict__ hist, uint32_t* __restrict__ off,
                                                   uint32_t* __restrict__ coff, uint32_t* __restrict__ cursor,
                                                   uint32_t T) {
  constexpr uint32_t PER = LB_MSM_BUCKETS / 1024;
  static_assert(PER * 1024 == LB_MSM_BUCKETS, "3 buckets per lane");
  __shared__ uint32_t se[1024], sc[1024];
  const uint32_t t = threadIdx.x;
  uint32_t e = 0, c = 0, h[PER];
#pragma unroll
  for (uint32_t j = 0; j < PER; j++) {
    h[j] = hist[t * PER + j];
    e += h[j];
    c += (h[j] + T - 1) / T;
    cursor[t * PER + j] = 0;
  }
  se[t] = e;
  sc[t] = c;
  __syncthreads();
  // Hillis-Steele inclusive scan of the lane totals
  for (uint32_t s = 1; s < 1024; s <<= 1) {
    const uint32_t ve = t >= s ? se[t - s] : 0u, vc = t >= s ? sc[t - s] : 0u;
    __syncthreads();
    se[t] += ve;
    sc[t] += vc;
    __syncthreads();
  }
  uint32_t re = se[t] - e, rc = sc[t] - c;
#pragma unroll
  for (uint32_t j = 0; j < PER; j++) {
    off[t * PER + j] = re;
    coff[t * PER + j] = rc;
    re += h[j];
    rc += (h[j] + T - 1) / T;
  }
  if (t == 1023) {
    off[LB_MSM_BUCKETS] = re;
    coff[LB_MSM_BUCKETS] = rc;
  }
}

// Counting-sort placement: sorted[pos] = point index | sign, grouped by bucket.
// (The order inside a bucket follows the atomics; the bucket's sum is the same
// group element either way.)
__global__ void __launch_bounds__(256) k_msm_scatter(uint32_t n_ent, const uint32_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ off, uint32_t* __restrict__ cursor,
                                                     uint32_t* __restrict__ sorted) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_ent) return;
  const uint32_t key = keys[e];
  if (key == LB_MSM_NONE) return;
  const uint32_t bk = key & 0x7fffffffu;
  const uint32_t pos = off[bk] + atomicAdd(&cursor[bk], 1u);
  // entry e = (set, half, window): point index = 2 set + half = e / W
  sorted[pos] = (e / LB_MSM_W) | (key & 0x80000000u);
}

// half-point of a sorted entry: sig_i or [lambda] sig_i = (omega X, Y), negated by the sign bit
LB_DEV void msm_point(g2a& q, const g2j* __restrict__ sig, uint32_t v) {
  const uint32_t j = v & 0x7fffffffu;
  const g2j& s = sig[j >> 1];
  q.x = s.X;
  if (j & 1u) {
    fp w;
    fp_set(w, LB_G2_OMEGA);
    fp2_mul_fp(q.x, q.x, w);
  }
  q.y = s.Y;
  if (v >> 31) fp2_neg(q.y, q.y);
  q.inf = false;
}

// bucket of chunk c: the last b with coff[b] <= c (empty buckets share their
// successor's offset, so the last one is the non-empty bucket holding c)
LB_DEV uint32_t msm_chunk_bucket(const uint32_t* __restrict__ coff, uint32_t c) {
  uint32_t lo = 0, hi = LB_MSM_BUCKETS;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (coff[mid] <= c)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// One lane per chunk: the sum of <= T affine half-points of one bucket
// (decoded signatures are affine: Z = 1), by mixed additions.
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_msm_chunks(uint32_t max_chunks, const uint32_t* __restrict__ off,
                                                                 const uint32_t* __restrict__ coff,
                                                                 const uint32_t* __restrict__ sorted,
                                                                 const g2j* __restrict__ sig, g2j* __restrict__ csum,
                                                                 uint32_t T) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= max_chunks || c >= coff[LB_MSM_BUCKETS]) return;
  const uint32_t bk = msm_chunk_bucket(coff, c);
  const uint32_t e0 = off[bk] + (c - coff[bk]) * T;
  const uint32_t e1 = min(e0 + T, off[bk + 1]);
  g2a q;
  msm_point(q, sig, sorted[e0]);
  g2j acc;
  jac_from_aff(acc, q);
#pragma unroll 1
  for (uint32_t e = e0 + 1; e < e1; e++) {
    msm_point(q, sig, sorted[e]);
    jac_add_aff(acc, acc, q);
  }
  csum[c] = acc;
}

// B_b = sum of bucket b's chunk partials (infinity when empty): LB_MSM_BLANES lanes per bucket
// (round 6: a C2 bucket holds ~8 chunks, which one lane added in 7 dependent Jacobian additions
// of ~75 us each; 4 lanes take two chunks each and a 2-level LDS tree joins them: 3)
// (lanes: LB_MSM_BLANES, or 1 -- one lane per bucket, round 5 -- with LB_MSM_LANES=0)
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_msm_buckets(const uint32_t* __restrict__ coff,
                                                                  const g2j* __restrict__ csum, g2j* __restrict__ bsum,
                                                                  uint32_t lanes) {
  __shared__ LdsRec<g2j> sh[TPB];
  static_assert(TPB % LB_MSM_BLANES == 0, "a bucket's lanes in one workgroup");
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t bk = t / lanes, sub = t % lanes;
  g2j acc;
  jac_set_inf(acc);
  if (bk < LB_MSM_BUCKETS) {
    const uint32_t c0 = coff[bk], c1 = coff[bk + 1];
    bool have = false;
#pragma unroll 1
    for (uint32_t c = c0 + sub; c < c1; c += lanes) {
      g2j v = csum[c];
      if (have) {
        jac_add(acc, acc, v);
      } else {
        acc = v;
        have = true;
      }
    }
  }
  sh[threadIdx.x].v = acc;
  __syncthreads();
#pragma unroll 1
  for (uint32_t s = lanes / 2; s > 0; s >>= 1) {
    if (sub < s) {
      g2j m = sh[threadIdx.x].v, o = sh[threadIdx.x + s].v;
      jac_add(m, m, o);
      sh[threadIdx.x].v = m;
    }
    __syncthreads();
  }
  if (sub == 0 && bk < LB_MSM_BUCKETS) bsum[bk] = sh[threadIdx.x].v;
}

// One workgroup of LB_MSM_BITS_TPB threads per bit position p = 11 w + k: G_p = sum of the
// buckets d of window w whose bit k is set (512 of them for k < 10, only d = 1024 for k = 10):
// two buckets per thread, then an LDS tree (round 6: 256 threads, 9 dependent additions
// instead of one wave's 8 + 6)
template <int T>
__global__ void __launch_bounds__(T, T == TPB ? LB_W_SCALAR : 1) k_msm_bits(const g2j* __restrict__ bsum,
                                                                           g2j* __restrict__ G) {
  __shared__ LdsRec<g2j> sh[T];  // (T = TPB: the narrow form's 19 KB, not the wide one's 78 KB)
  const uint32_t p = blockIdx.x;
  if (p >= LB_MSM_POS) return;
  const uint32_t w = p / LB_MSM_C, k = p % LB_MSM_C;
  const uint32_t n = k < LB_MSM_C - 1 ? LB_MSM_NB / 2 : 1u;
  g2j acc;
  jac_set_inf(acc);
  bool have = false;
#pragma unroll 1
  for (uint32_t m = threadIdx.x; m < n; m += T) {
    const uint32_t low = m & ((1u << k) - 1u), high = m >> k;
    const uint32_t d = (high << (k + 1)) | (1u << k) | low;  // 1 <= d <= 1024, bit k set
    g2j t = bsum[w * LB_MSM_NB + d - 1];
    if (have) {
      jac_add(acc, acc, t);
    } else {
      acc = t;
      have = true;
    }
  }
  sh[threadIdx.x].v = acc;
  __syncthreads();
#pragma unroll 1
  for (uint32_t s = T / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      g2j m = sh[threadIdx.x].v, o = sh[threadIdx.x + s].v;
      jac_add(m, m, o);
      sh[threadIdx.x].v = m;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) G[p] = sh[0].v;
}

// One wave: S = sum_p 2^p G_p (lane p doubles p times, then an LDS tree), affine.
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_msm_final(const g2j* __restrict__ G, g2a* __restrict__ S) {
  __shared__ LdsRec<g2j> sh[TPB];
  const uint32_t p = threadIdx.x;
  g2j acc;
  jac_set_inf(acc);
  if (p < LB_MSM_POS) {
    acc = G[p];
#pragma unroll 1
    for (uint32_t t = 0; t < p; t++) jac_dbl(acc, acc);
  }
  sh[p].v = acc;
  __syncthreads();
  for (uint32_t s = TPB / 2; s > 0; s >>= 1) {
    if (p < s) {
      g2j m = sh[p].v, o = sh[p + s].v;
      jac_add(m, m, o);
      sh[p].v = m;
    }
    __syncthreads();
  }
  if (p == 0) {
    g2j tot = sh[0].v;
    g2a sa;
    jac_to_aff(sa, tot);
    S[0] = sa;
  }
}

// lb_g2_msm (tests): 192-byte uncompressed affine points -> Jacobian (Z = 1),
// status OK iff the encoding decodes to a point on the curve
__global__ void __launch_bounds__(TPB) k_msm_load(uint32_t n, const uint8_t* __restrict__ in192, g2j* __restrict__ out,
                                                  uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  const uint8_t st = g2_deserialize(a, in192 + (size_t)i * 192, 192);
  g2j p;
  jac_set_inf(p);
  if (st == LB_ST_OK) jac_from_aff(p, a);
  out[i] = p;
  status[i] = st;
}

template __global__ void k_msm_bits<TPB>(const g2j* __restrict__, g2j* __restrict__);
template __global__ void k_msm_bits<LB_MSM_BITS_TPB>(const g2j* __restrict__, g2j* __restrict__);

}  // namespace lb
