// Shared declarations of the verification kernels (defined in k_*.hip, one
// translation unit per stage group so the build compiles them in parallel;
// bls_all.hip is the single-TU build used for the op-counting variant).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/lodestar_bls.h"
#include "bls_pairing.h"


#define LB_ST_ZERO_SIGNATURE 6

// ============================================================================
// Kernels
// ============================================================================
static constexpr int TPB = 64;  // one wave per workgroup: flexible residency at high VGPR counts
// min waves per SIMD for the heavy per-lane kernels: 1 = 512-register budget
// (256 VGPR + 256 AGPR), which keeps the inlined tower arithmetic spill-free
#ifndef LB_HEAVY_WAVES
#define LB_HEAVY_WAVES 1
#endif
// Per-stage occupancy (min waves per SIMD, i.e. a 512 / W register budget),
// measured on MI355X (profiles/occupancy_r01.log): the per-set stages run
// faster at 2 waves/SIMD despite some spilling (a lone wave issues
// v_mad_u64_u32 at ~60% of the SIMD's rate); the per-request tails (one lane
// per request, a long serial chain) and the Miller accumulation keep the
// spill-free 1-wave budget.
// Re-measured in round 5 (profiles/r05/occupancy/): hash_finish / decode at 1 wave cost
// the pipeline 6-7 % (co-residency with other calls' kernels), at 3 waves 0.3-2.5 %.
#ifndef LB_W_HASH
#define LB_W_HASH 2
#endif
// k_hash_half (SHA-256 + SSWU + isogeny): 2, not 4 -- the binary-GCD inversion
// in its call graph takes 228 VGPRs, so 4 waves/SIMD is out of reach, and a
// 128-register target for the kernel body only adds spills (1,328 vs 704 B/lane)
#ifndef LB_W_MAP
#define LB_W_MAP 2
#endif
#ifndef LB_W_DECODE
#define LB_W_DECODE 2
#endif
#ifndef LB_W_SCALAR
#define LB_W_SCALAR 2
#endif
#ifndef LB_W_SSIG  // k_scalar_sig (r sigma: two live G2 points)
#define LB_W_SSIG LB_W_SCALAR
#endif
#ifndef LB_W_ACC
#define LB_W_ACC 1
#endif
#ifndef LB_W_TAIL
#define LB_W_TAIL 1
#endif


// Bucket MSM of the merged check (k_msm.hip): signed digits of LB_MSM_C bits in
// LB_MSM_W windows of the 32-bit GLV half-scalars, LB_MSM_NB buckets per window,
// chunks of <= LB_MSM_T entries, bit positions 0 .. LB_MSM_POS - 1.
#define LB_MSM_C 11
#define LB_MSM_W 3
#define LB_MSM_NB 1024u
#define LB_MSM_BUCKETS (LB_MSM_W * LB_MSM_NB)
#define LB_MSM_T 16u
#define LB_MSM_T_LONE 4u  // (a lone call of at most LB_LP_DEC_MAX sets: shorter chunk chains, more chunks)
#define LB_MSM_POS 33u
#define LB_MSM_NONE 0xffffffffu

namespace lb {
// One lane's tower value in an LDS tree, padded so the record stride is an odd number of
// 16-byte units: a wave's ds_read_b128 / ds_write_b128 of lane-strided records then hits
// every bank once per lane group (MI355X_MICROARCH.md, LDS table).  An fp12 at its bare
// 144-dword stride maps 16 lanes onto 4 bank groups (SQ_LDS_BANK_CONFLICT / IDX_ACTIVE 0.36
// in k_miller_acc's epilogue); a Jacobian G2 point at 72 dwords onto 8.
template <class T, bool PAD = ((sizeof(T) / 16) % 2 == 0)>
struct alignas(16) LdsRec {
  T v;
  uint32_t pad[4];
};
template <class T>
struct alignas(16) LdsRec<T, false> {
  T v;
};

// Where a set's pubkeys come from: the call's 96-byte uncompressed encodings
// (the worker wire format, chain/bls/multithread/worker.ts:110-116) or the
// device-resident pubkey table addressed by validator index (the index2pubkey
// mirror, state-transition/src/cache/pubkeyCache.ts:56-77; lb_pubkey_table_*).
struct PkSource {
  const uint8_t* bytes;   // pk_offsets[n_sets] x 96 B (when index == nullptr)
  const uint32_t* index;  // pk_offsets[n_sets] validator indices, or nullptr
  const g1a* table;       // decoded affine table entries
  uint32_t table_n;
};
// Pubkey k of the call; an index outside the table is a bad pubkey (LB_REQ_BAD_PUBKEY).
// In a mixed package (index AND bytes given) an index with bit 31 set is row
// (j & LB_PK_ROW_MASK) of the call's 96-byte pubkey rows (the host checked the rows
// exist); bit 30 marks a row holding a 48-byte compressed encoding.
LB_DEV uint8_t pk_load(g1a& p, const PkSource& s, uint32_t k) {
  if (s.index) {
    const uint32_t j = s.index[k];
    if ((j & LB_PK_ROW_FLAG) && s.bytes)
      return g1_deserialize(p, s.bytes + (size_t)(j & LB_PK_ROW_MASK) * 96, (j & LB_PK_ROW48_FLAG) ? 48u : 96u);
    if (j >= s.table_n) {
      p.inf = true;
      return LB_ST_BAD_ENCODING;
    }
    p = s.table[j];
    return LB_ST_OK;
  }
  return g1_deserialize(p, s.bytes + (size_t)k * 96, 96);
}

// Row layout of the steps organisation (k_steps.hip): requests in size-descending
// order, pair (k, i) of request k at slot rowoff[i] + pos[k]; meta[0] = rows.
struct Rows {
  const uint32_t* rowoff;
  const uint32_t* inv;
  const uint32_t* pos;
  const uint32_t* meta;
  // lanes per set of the step-major accumulation (1, 2 or 4: 68 / split lines per lane; a lone
  // mid-size call's k_step_acc is the one-lane latency of its lanes' lines, k_steps.hip)
  uint32_t split = 1;
};

__global__ void __launch_bounds__(TPB) k_req_flags(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                   uint8_t* __restrict__ single_flag);
__global__ void __launch_bounds__(TPB, LB_W_DECODE) k_decode_sigs(uint32_t n, const uint8_t* __restrict__ sigs,
                                                     const uint32_t* __restrict__ sig_off,
                                                     const uint8_t* __restrict__ single_flag,
                                                     g2j* __restrict__ out_sig, uint8_t* __restrict__ status);
__global__ void __launch_bounds__(TPB) k_pubkeys_single(uint32_t n_sets, PkSource pks,
                                                        const uint32_t* __restrict__ pk_off, g1j* __restrict__ out_pk,
                                                        uint8_t* __restrict__ pk_status);
__global__ void __launch_bounds__(TPB) k_pubkeys_agg(uint32_t n_sets, PkSource pks,
                                                     const uint32_t* __restrict__ pk_off, g1j* __restrict__ out_pk,
                                                     uint8_t* __restrict__ pk_status);
__global__ void __launch_bounds__(TPB) k_table_decode(uint32_t n, const uint8_t* __restrict__ in, uint32_t len,
                                                      g1a* __restrict__ out, uint8_t* __restrict__ status);
__global__ void k_g1a_serialize(uint32_t n, const g1a* __restrict__ in, uint8_t* __restrict__ out96);
__global__ void __launch_bounds__(TPB) k_pubkey_validate(uint32_t n, const uint8_t* __restrict__ in, uint32_t len,
                                                         uint8_t* __restrict__ out96, uint8_t* __restrict__ status);
__global__ void __launch_bounds__(TPB, LB_W_MAP) k_hash_half(uint32_t n, const uint8_t* __restrict__ msgs,
                                                   g2j* __restrict__ q);
__global__ void __launch_bounds__(TPB, LB_W_HASH) k_hash_finish(uint32_t n, g2j* __restrict__ q, g2j* __restrict__ out_h);
__global__ void __launch_bounds__(TPB, LB_W_SSIG) k_scalar_sig(uint32_t n, const uint8_t* __restrict__ seed,
                                                    const g2j* __restrict__ sig,
                                                    const uint8_t* __restrict__ sig_status,
                                                    g2j* __restrict__ rsig, const uint8_t* __restrict__ skip);
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_scalar_pk(uint32_t n, const uint8_t* __restrict__ seed,
                                                   const g1j* __restrict__ pk, const uint8_t* __restrict__ single_flag,
                                                   uint8_t* __restrict__ pk_status, g1j* __restrict__ rpk);
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_sum_tree(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                  const g2j* __restrict__ rsig, g2a* __restrict__ S,
                                                  const uint8_t* __restrict__ skip);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_miller_S(uint32_t n_req, const g2a* __restrict__ S, fp12* __restrict__ fS);
__global__ void __launch_bounds__(TPB, LB_HEAVY_WAVES) k_miller_sets(uint32_t n, const g1j* __restrict__ rpk, const g2j* __restrict__ h,
                                                     fp12* __restrict__ f);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_prod_tree(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                   const fp12* __restrict__ f, const fp12* __restrict__ fS,
                                                   const uint8_t* __restrict__ sig_status,
                                                   const uint8_t* __restrict__ pk_status, fp12* __restrict__ F,
                                                   uint8_t* __restrict__ req_bad, uint8_t* __restrict__ req_err);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_final(uint32_t n_req, const fp12* __restrict__ F,
                                               const uint8_t* __restrict__ req_bad, uint8_t* __restrict__ valid);
__global__ void __launch_bounds__(TPB, LB_HEAVY_WAVES) k_hash(uint32_t n, const uint8_t* __restrict__ msgs, g2a* __restrict__ out_h);
template <class F>
__global__ void __launch_bounds__(256) k_jac_sum(uint32_t n, const jac<F>* __restrict__ in, jac<F>* __restrict__ out);
__global__ void __launch_bounds__(256) k_copy_bytes(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                    uint32_t n);
__global__ void k_g1_serialize(uint32_t n, const g1j* __restrict__ in, uint8_t* __restrict__ out96);
__global__ void k_g2_serialize(uint32_t n, const g2j* __restrict__ in, uint8_t* __restrict__ out192);
__global__ void k_g2a_serialize(uint32_t n, const g2a* __restrict__ in, uint8_t* __restrict__ out192);
__global__ void k_pairing(uint32_t n, const uint8_t* __restrict__ g1b, const uint8_t* __restrict__ g2b,
                          uint8_t* __restrict__ out);
__global__ void k_scalars(const uint8_t* __restrict__ seed, uint32_t first, uint32_t n, uint64_t* __restrict__ out);
__global__ void k_g1_mul(uint32_t n, const uint8_t* __restrict__ in, const uint64_t* __restrict__ k,
                         uint8_t* __restrict__ out);
__global__ void k_g2_mul(uint32_t n, const uint8_t* __restrict__ in, const uint64_t* __restrict__ k,
                         uint8_t* __restrict__ out);
__global__ void __launch_bounds__(TPB) k_sk_to_pk(uint32_t n, const uint8_t* __restrict__ sk32,
                                                  uint8_t* __restrict__ out96);
__global__ void __launch_bounds__(TPB) k_sign(uint32_t n, const uint8_t* __restrict__ sk32,
                                              const uint8_t* __restrict__ msgs, uint8_t* __restrict__ out96);
template <int WAVES>
__global__ void __launch_bounds__(TPB, WAVES) k_lines(uint32_t n, uint32_t n_pairs, uint32_t base,
                                                               const g1j* __restrict__ P, const g2j* __restrict__ Q,
                                                               uint32_t* __restrict__ lines);
template <int LPR>
__global__ void __launch_bounds__(TPB, LB_W_ACC) k_miller_acc(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                                    uint32_t n_pairs, const uint32_t* __restrict__ lines,
                                                                    const fp12* __restrict__ fS,
                                                                    const uint8_t* __restrict__ sig_status,
                                                                    const uint8_t* __restrict__ pk_status,
                                                                    fp12* __restrict__ F, uint8_t* __restrict__ req_bad,
                                                                    uint8_t* __restrict__ req_err, uint32_t halves,
                                                                    const g2a* __restrict__ Sx, fp12* __restrict__ Fx);
__global__ void __launch_bounds__(TPB) k_split_requests(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                        uint32_t* __restrict__ off2);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_join_halves(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                               const fp12* __restrict__ F2, const uint8_t* __restrict__ bad2,
                                                               const uint8_t* __restrict__ err2,
                                                               const fp12* __restrict__ fS, fp12* __restrict__ F,
                                                               uint8_t* __restrict__ req_bad, uint8_t* __restrict__ req_err);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_lines_S(uint32_t n_req, uint32_t n_pairs, uint32_t base,
                                                          const g2a* __restrict__ S, uint32_t* __restrict__ lines,
                                                          const uint8_t* __restrict__ skip);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_tail(uint32_t n_req, uint32_t n_pairs, uint32_t base,
                                                       const uint32_t* __restrict__ lines,
                                                       const fp12* __restrict__ F,
                                                       const uint8_t* __restrict__ req_bad,
                                                       uint8_t* __restrict__ valid,
                                                       const uint8_t* __restrict__ skip);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_pair_wc(uint32_t n, uint32_t n_pairs,
                                                          const uint32_t* __restrict__ lines, fp12* __restrict__ f);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_merge(uint32_t n_req, const g2a* __restrict__ S,
                                                        const fp12* __restrict__ F,
                                                        const uint8_t* __restrict__ req_bad,
                                                        g2a* __restrict__ S_all, fp12* __restrict__ F_all,
                                                        const fp12* __restrict__ Fx);
__global__ void __launch_bounds__(TPB) k_merge_stats(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                     const uint8_t* __restrict__ req_bad,
                                                     const uint8_t* __restrict__ mflag, uint32_t* __restrict__ out);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_partial(uint32_t n_pairs, uint32_t base,
                                                          const uint32_t* __restrict__ lines,
                                                          const fp12* __restrict__ F_all, uint8_t* __restrict__ out576);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_gt_check(uint32_t n, const uint8_t* __restrict__ in576,
                                                           uint8_t* __restrict__ out);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_gt_prod(uint32_t n, const uint8_t* __restrict__ in576,
                                                          uint32_t* __restrict__ out16, uint8_t* __restrict__ out);
__global__ void __launch_bounds__(TPB) k_same_message_agg(uint32_t n_jobs, const uint32_t* __restrict__ job_off,
                                                          const g2j* __restrict__ sig,
                                                          const uint8_t* __restrict__ sig_status,
                                                          const g1j* __restrict__ job_pk, uint8_t* __restrict__ out_pk96,
                                                          uint8_t* __restrict__ out_sig192,
                                                          uint8_t* __restrict__ job_bad);
__global__ void __launch_bounds__(TPB) k_signing_root_att(uint32_t n, const uint8_t* __restrict__ data,
                                                          const uint8_t* __restrict__ domains, uint32_t dstride,
                                                          uint8_t* __restrict__ out);
__global__ void __launch_bounds__(TPB) k_signing_root_chunks(uint32_t n, uint32_t m, const uint8_t* __restrict__ chunks,
                                                             const uint8_t* __restrict__ domains, uint32_t dstride,
                                                             uint8_t* __restrict__ out);
__global__ void __launch_bounds__(TPB) k_msm_scalars(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                     const uint8_t* __restrict__ seed, const uint64_t* __restrict__ raw,
                                                     const g2j* __restrict__ sig, const uint8_t* __restrict__ sig_status,
                                                     const uint8_t* __restrict__ pk_status, uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ hist);
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t* __restrict__ hist, uint32_t* __restrict__ off,
                                                   uint32_t* __restrict__ coff, uint32_t* __restrict__ cursor,
                                                   uint32_t T);
__global__ void __launch_bounds__(256) k_msm_scatter(uint32_t n_ent, const uint32_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ off, uint32_t* __restrict__ cursor,
                                                     uint32_t* __restrict__ sorted);
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_msm_chunks(uint32_t max_chunks, const uint32_t* __restrict__ off,
                                                                 const uint32_t* __restrict__ coff,
                                                                 const uint32_t* __restrict__ sorted,
                                                                 const g2j* __restrict__ sig, g2j* __restrict__ csum,
                                                                 uint32_t T);
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_msm_buckets(const uint32_t* __restrict__ coff,
                                                                  const g2j* __restrict__ csum, g2j* __restrict__ bsum,
                                                                  uint32_t lanes);
static constexpr uint32_t LB_MSM_BLANES = 4;      // k_msm_buckets: lanes per bucket
static constexpr uint32_t LB_MSM_BITS_TPB = 256;  // k_msm_bits: threads per bit position
template <int T>  // (T threads per bit position: TPB, or LB_MSM_BITS_TPB for a lone call)
__global__ void __launch_bounds__(T, T == TPB ? LB_W_SCALAR : 1) k_msm_bits(const g2j* __restrict__ bsum,
                                                                           g2j* __restrict__ G);
__global__ void __launch_bounds__(TPB, LB_W_SCALAR) k_msm_final(const g2j* __restrict__ G, g2a* __restrict__ S);
__global__ void __launch_bounds__(256) k_rows_hist(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                   uint32_t* __restrict__ hist);
__global__ void __launch_bounds__(1024) k_rows_scan(uint32_t n_sets, const uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ gt, uint32_t* __restrict__ rowoff,
                                                    uint32_t* __restrict__ meta);
__global__ void __launch_bounds__(256) k_rows_pos(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                  const uint32_t* __restrict__ gt, uint32_t* __restrict__ cursor,
                                                  uint32_t* __restrict__ pos, uint32_t* __restrict__ inv);
template <int WAVES>
__global__ void __launch_bounds__(TPB, WAVES) k_lines_rows(uint32_t n_sets, uint32_t n_pairs, Rows R,
                                                           const uint32_t* __restrict__ req_off,
                                                           const g1j* __restrict__ P, g2j* __restrict__ Q,
                                                           uint32_t* __restrict__ lines);
__global__ void __launch_bounds__(TPB) k_req_status(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                    const uint8_t* __restrict__ sig_status,
                                                    const uint8_t* __restrict__ pk_status,
                                                    uint8_t* __restrict__ req_bad, uint8_t* __restrict__ req_err);
template <int MODE, int WAVES>
__global__ void __launch_bounds__(TPB, WAVES) k_step_acc(uint32_t n_sets, uint32_t n_pairs, Rows R,
                                                            const uint32_t* __restrict__ req_off,
                                                            const uint32_t* __restrict__ lines,
                                                            uint32_t* __restrict__ G);
__global__ void __launch_bounds__(256, 1) k_level_prod(uint32_t n_req, uint32_t n_sets, uint32_t n_pairs,
                                                       uint32_t s_pair, Rows R, const uint32_t* __restrict__ req_off,
                                                       const uint32_t* __restrict__ G,
                                                       const uint8_t* __restrict__ req_bad,
                                                       const uint32_t* __restrict__ lines, fp12* __restrict__ Pl);
// the level products in two stages (round 6): lane products of each level's share, then
// wave-cooperative products of groups of LB_LVL_GROUP partials (k_steps.hip)
static constexpr uint32_t LB_LVL_GROUP = 8;
__global__ void __launch_bounds__(256, 1) k_level_part(uint32_t n_req, uint32_t n_sets, Rows R,
                                                       const uint32_t* __restrict__ req_off,
                                                       const uint32_t* __restrict__ G,
                                                       const uint8_t* __restrict__ req_bad, uint32_t per,
                                                       fp12* __restrict__ part, uint8_t* __restrict__ has);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_level_wc(uint32_t per_in, const fp12* __restrict__ in,
                                                             const uint8_t* __restrict__ in_has, uint32_t per_out,
                                                             fp12* __restrict__ out, uint8_t* __restrict__ out_has,
                                                             uint32_t n_pairs, uint32_t s_pair,
                                                             const uint32_t* __restrict__ lines, fp12* __restrict__ Pl);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_horner_all(const fp12* __restrict__ Pl, fp12* __restrict__ F_all);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_req_horner(uint32_t n_req, uint32_t n_sets, Rows R,
                                                             const uint32_t* __restrict__ req_off,
                                                             const uint32_t* __restrict__ G,
                                                             const uint8_t* __restrict__ req_bad,
                                                             fp12* __restrict__ F, const uint8_t* __restrict__ skip);
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_req_join(uint32_t n_req, uint32_t split,
                                                           const fp12* __restrict__ parts,
                                                           const uint8_t* __restrict__ req_bad,
                                                           fp12* __restrict__ F, const uint8_t* __restrict__ skip);
__global__ void __launch_bounds__(TPB) k_msm_load(uint32_t n, const uint8_t* __restrict__ in192, g2j* __restrict__ out,
                                                  uint8_t* __restrict__ status);
}  // namespace lb
