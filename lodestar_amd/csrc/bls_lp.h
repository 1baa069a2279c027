// Latency path (round-program interpreter, k_lp.hip): sizes and opcodes shared
// with the generator (lodestar_amd/lpgen/compile.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_kernels.h"

#ifndef LB_LP_ROWS
#define LB_LP_ROWS 32                     // units per round = 16-lane rows per workgroup
#endif
#define LB_LP_TPB (LB_LP_ROWS * 16)       // 8 waves: 2 per SIMD (256 VGPRs for the one-lane inversion)
// k_lp_verify's waves per SIMD target: 4 = two workgroups per CU (128 VGPRs, 12 spilled;
// LDS 2 x 68 KB): 512-set calls 6.9 -> 4.6 ms, 1024-set 12.4 -> 8.5 ms, 1 and 128 sets
// unchanged (profiles/r05/lp_direct/lp_v*); 2 = one per CU (152 VGPRs)
#ifndef LB_LP_VERIFY_WPE
#define LB_LP_VERIFY_WPE 4
#endif
#define LB_LP_MAX_REGS 1024               // LDS registers (64 B each)
// the merged-check programs (k_lp_mtail, one workgroup per call) hold the call's 63 level
// products as inputs (k_horner_all folded in): a larger register file, 96 KB of LDS
#define LB_LP_MTAIL_REGS 1536
#define LB_LP_MAX_FLAGS 512
#define LB_LP_STAMPS (6 + 6 * LB_LP_TPB / 64)  // diagnostic s_memtime points per round (k_lp_program stamps): 6 of
                                              // the workgroup, run_unit start / end of every wave, 4 inside its unit
#define LB_LP_BLOCK_CAP 1536              // words of one round's encoded block
#define LB_LP_RING 16384                  // LDS ring of the program stream (words, power of 2)
#define LB_LP_CHUNK 2048                  // stream words fetched per round (4 per thread; rounds average
                                          // ~0.9k words, the final program ~1.04k)
#define LB_LP_HDR 10                      // header words of an encoded program
#define LB_LP_TREE_LEVELS 20              // product-tree levels (requests up to 2^20 sets)

#define LB_LP_OP_MUL 0
#define LB_LP_OP_LIN 1
#define LB_LP_OP_SEL 2
#define LB_LP_OP_INV 3
#define LB_LP_OP_CANON 4
#define LB_LP_OP_ISZERO 5
#define LB_LP_OP_BIT0 6
#define LB_LP_OP_GTHALF 7
#define LB_LP_OP_FOP 8
#define LB_LP_OP_LIN2 9  // a linear form over both term lists of the record (x + y)

// programs in the embedded blob (gen_lp.py -> lp_programs.bin, bls_lp_progs.h)
#define LB_LP_PROG_SET_SINGLE 0
#define LB_LP_PROG_SET_BATCH 1
#define LB_LP_PROG_MUL 2
#define LB_LP_PROG_FINAL 3
#define LB_LP_PROG_MTAIL_CHECK 4    // the throughput pipeline's merged check (lpgen/bls.py mtail_program)
#define LB_LP_PROG_MTAIL_PARTIAL 5  // ... its two-phase form: the shard's partial
#define LB_LP_PROG_FINAL_LANE 6     // final exponentiation == 1 of a one-lane Fp12 (lb_gt_check)
#define LB_LP_PROG_RTAIL 7          // one request's tail after a failed merged check (k_lp_rtail)
#define LB_LP_PROG_MTAIL_CHECK_WIDE 8    // the merged-check programs compiled for LB_LP_MTAIL_ROWS rows
#define LB_LP_PROG_MTAIL_PARTIAL_WIDE 9  // (a lone call's k_lp_mtail: 1,024 threads)
#define LB_LP_PROG_MSM_BITS0 10  // a lone call's MSM bit sums: 8 one-lane Jacobian points -> their sum
#define LB_LP_PROG_MSM_BITS1 11  // ... 8 partial sums -> one
#define LB_LP_PROG_MSM_BITS2 12  // ... 8 partial sums -> G_p, one-lane Jacobian (k_lp_msm_bits)
#define LB_LP_PROG_SIG_DECODE 13  // a small same-message package's signature decode (k_lp_dec, 8 rows)
#define LB_LP_PROG_HASH_FINISH 14  // a lone mid-size call's clear_cofactor(Q0 + Q1) (k_lp_hf, 16 rows)
#define LB_LP_PROG_LINES 15  // a lone mid-size call's Miller lines of one pair (k_lp_lines, 16 rows)
#define LB_LP_PROG_HASH_FINISH_NARROW 16  // the hash finish compiled for LB_LP_NARROW_ROWS rows
#define LB_LP_PROG_HASH_FULL 17  // a lone mid-size call's whole hash_to_G2 curve part (k_lp_hash, 8 rows)
#define LB_LP_NPROGS 18
#define LB_LP_HASH_REGS 384  // gen_lp.py MAX_REGS_HASH
#define LB_LP_NARROW_ROWS 8  // gen_lp.py DEC_ROWS
#define LB_LP_LINES_MAX 5120  // lone steps calls of at most this many sets store their lines via k_lp_lines (6,144: -0.5 ms)
#define LB_LP_LINES_NOUT (68 * 6)
#define LB_LP_HF_ROWS 16           // gen_lp.py HF_ROWS
#define LB_LP_HF_MAX 3072          // lone calls of at most this many sets finish their hash on k_lp_hf
#define LB_LP_DEC_ROWS 8          // gen_lp.py DEC_ROWS
#define LB_LP_DEC_REGS 128        // gen_lp.py MAX_REGS_DEC
#define LB_SM_DEC_MAX 512         // packages of at most this many signatures decode on k_lp_dec
#define LB_LP_DEC_MAX 5120        // ... and lone pipeline calls of at most this many sets
#define LB_MSM_BITS_GROUP 8      // lpgen/bls.py MSM_BITS_GROUP
#define LB_MSM_BITS_INST (LB_MSM_POS * (LB_MSM_NB / 2 / LB_MSM_BITS_GROUP))  // level-0 instances: 33 x 64
#define LB_RTAIL_NIN 16                 // rtail inputs: F_k (12 Fp), S_k affine (4 Fp); inflag S_inf
#define LB_LP_RTAIL_REGS 512            // (its program holds ~240 registers: 32 KB of LDS)
#define LB_MTAIL_LEVELS 63                  // the step-major accumulation's Horner levels (k_steps.hip)
#define LB_MTAIL_NIN (12 * LB_MTAIL_LEVELS + 6 * LB_MSM_POS)  // mtail inputs: the 63 level products, the MSM's
                                                              // 33 bit sums

namespace lb {
// k_lp.hip: instance b (one workgroup of LB_LP_TPB threads) runs the round program at
// prog on in[b * in_stride ...]; stamps (diagnostic, usually nullptr): s_memtime after
// every round of instance 0
__global__ void __launch_bounds__(LB_LP_TPB) k_lp_program(const uint32_t* __restrict__ prog, uint32_t n,
                                                          const uint32_t* __restrict__ in, uint32_t in_stride,
                                                          const uint32_t* __restrict__ in_flags, uint32_t flag_stride,
                                                          uint32_t* __restrict__ out, uint32_t out_stride,
                                                          uint32_t* __restrict__ out_flags, uint32_t oflag_stride,
                                                          unsigned long long* __restrict__ stamps);

// the small-call pipeline (k_lp.hip): one call's device state
struct LpCall {
  const uint32_t* prog_single;
  const uint32_t* prog_batch;
  const uint32_t* prog_mul;
  const uint32_t* prog_final;
  const uint32_t* req_off;
  const uint32_t* set_req;
  const uint32_t* in16;
  const uint32_t* flags;
  uint8_t* sig_st;    // prep status in, the signature's final status out (LB_SET_*)
  uint8_t* pk_st;     // k_pubkeys_* status in, + the G1 check of 1-set requests
  uint32_t* F;        // n_sets x 12 x 16 words: Miller values, then the tree's nodes
  uint32_t* cnt;      // LB_LP_TREE_LEVELS x n_sets arrival counters (zeroed)
  uint8_t* valid;     // n_req (zeroed)
  uint8_t* req_err;   // n_req (zeroed)
  uint32_t n_sets;
  // diagnostics: [0] s_memrealtime (100 MHz) and [1] s_memtime (shader
  // clock) when set 0's workgroup starts, [2] / [3] the same when request 0's verdict is
  // written (zeroed; [2] and [3] by the workgroup that writes it)
  unsigned long long* clk;
};
static constexpr uint32_t LB_LP_NIN = 11, LB_LP_NFL = 67;  // set program inputs / input flags
__global__ void __launch_bounds__(TPB) k_lp_prep(uint32_t n, const uint32_t* __restrict__ req_off, uint32_t n_req,
                                                 const uint8_t* __restrict__ msgs, const uint8_t* __restrict__ sigs,
                                                 const uint32_t* __restrict__ sig_off, const g1j* __restrict__ pk,
                                                 const uint8_t* __restrict__ seed, uint32_t* __restrict__ in16,
                                                 uint32_t* __restrict__ flags, uint8_t* __restrict__ sig_st,
                                                 uint32_t* __restrict__ set_req,
                                                 uint8_t* __restrict__ valid, uint8_t* __restrict__ req_err,
                                                 uint32_t* __restrict__ cnt, uint32_t n_cnt, unsigned long long* __restrict__ clk);
__global__ void __launch_bounds__(LB_LP_TPB, LB_LP_VERIFY_WPE) k_lp_verify(LpCall c);
// The throughput pipeline's merged check as a round program (one workgroup): in16 =
// LB_MTAIL_NIN records (k_mtail_prep); mflag (check program): [0] = final_exp == 1;
// out16 (partial program): the shard's partial, 12 records in the one-lane form.
#ifndef LB_LP_MTAIL_ROWS
#define LB_LP_MTAIL_ROWS 64  // (bls_lp_progs.h: the rows gen_lp.py compiled the wide merged-check programs for)
#endif
__global__ void __launch_bounds__(LB_LP_MTAIL_ROWS * 16) k_lp_mtail(const uint32_t* __restrict__ prog,
                                                        const uint32_t* __restrict__ in16, uint8_t* __restrict__ mflag,
                                                        uint32_t* __restrict__ out16);
// A lone call's MSM bit sums as three levels of round programs (bls_host.hip): the bucket sums
// gathered into level-0 records (8 per instance, 64 instances per bit position; infinity where a
// position has fewer buckets), then instance b of a level runs `prog` on in16 + b * n_in * 16 and
// writes out16 + b * n_out * 16 (level 2: the 33 G_p straight into the merged-check program's
// input records)
__global__ void __launch_bounds__(256) k_msm_bits_prep(const g2j* __restrict__ bsum, uint32_t* __restrict__ in16);
__global__ void __launch_bounds__(LB_LP_TPB, LB_LP_VERIFY_WPE) k_lp_msm_bits(const uint32_t* __restrict__ prog,
                                                                             uint32_t n, uint32_t n_in,
                                                                             uint32_t n_out,
                                                                             const uint32_t* __restrict__ in16,
                                                                             uint32_t* __restrict__ out16);
// A small same-message package's signature decode (bls_host.hip sm path): k_sm_dec_prep parses
// every signature's bytes (g2_deserialize's encoding rules) into the program's records, flags and
// a pre-status; k_lp_dec runs the sig_decode program per signature (one 8-row workgroup);
// k_sm_dec_finish forms k_decode_sigs' outputs (point, status) from them.
__global__ void __launch_bounds__(256) k_sm_dec_prep(uint32_t n, const uint8_t* __restrict__ sigs,
                                                     const uint32_t* __restrict__ sig_off, uint32_t* __restrict__ in16,
                                                     uint32_t* __restrict__ fl, uint8_t* __restrict__ pre);
__global__ void __launch_bounds__(LB_LP_DEC_ROWS * 16) k_lp_dec(const uint32_t* __restrict__ prog, uint32_t n,
                                                                const uint32_t* __restrict__ in16,
                                                                const uint32_t* __restrict__ fl,
                                                                uint32_t* __restrict__ out16,
                                                                uint32_t* __restrict__ ofl);
__global__ void __launch_bounds__(256) k_sm_dec_finish(uint32_t n, const uint8_t* __restrict__ pre,
                                                       const uint32_t* __restrict__ in16,
                                                       const uint32_t* __restrict__ fl,
                                                       const uint32_t* __restrict__ out16,
                                                       const uint32_t* __restrict__ ofl, g2j* __restrict__ sig,
                                                       uint8_t* __restrict__ status,
                                                       const uint8_t* __restrict__ single_flag);
// A lone mid-size call's hash finish (bls_host.hip): Q0, Q1 of every set into records
// (k_hf_prep), the hash_finish program per set on a 16-row workgroup (k_lp_hf), H back into
// Jacobian points (k_hf_finish)
// LB_LP_HASH_FULL: hash_to_field on one lane per set (k_hu_prep: u0, u1 as 4 records), the
// hash_full program per set (k_lp_hash), H back into Jacobian by k_hf_finish
__global__ void __launch_bounds__(256) k_hu_prep(uint32_t n, const uint8_t* __restrict__ msgs,
                                                 uint32_t* __restrict__ in16);
__global__ void __launch_bounds__(LB_LP_HF_ROWS * 16) k_lp_hash(const uint32_t* __restrict__ prog, uint32_t n,
                                                                const uint32_t* __restrict__ in16,
                                                                uint32_t* __restrict__ out16);
__global__ void __launch_bounds__(256) k_hf_prep(uint32_t n, const g2j* __restrict__ q, uint32_t* __restrict__ in16);
__global__ void __launch_bounds__(LB_LP_HF_ROWS * 16) k_lp_hf(const uint32_t* __restrict__ prog, uint32_t n,
                                                              const uint32_t* __restrict__ in16,
                                                              uint32_t* __restrict__ out16);
__global__ void __launch_bounds__(256) k_hf_finish(uint32_t n, const uint32_t* __restrict__ out16,
                                                   g2j* __restrict__ h);
// A lone mid-size steps call's lines (bls_host.hip): slot q's pair (r pk, H) into records
// (k_lines_prep, the row layout of k_lines_rows), the lines program per slot on a 16-row
// workgroup (k_lp_lines), its 68 lines into the SoA line store at slot q (k_lines_store)
__global__ void __launch_bounds__(256) k_lines_prep(uint32_t n_sets, Rows R, const uint32_t* __restrict__ req_off,
                                                    const g1j* __restrict__ P, const g2j* __restrict__ Q,
                                                    uint32_t* __restrict__ in16);
__global__ void __launch_bounds__(LB_LP_HF_ROWS * 16) k_lp_lines(const uint32_t* __restrict__ prog, uint32_t n,
                                                                 const uint32_t* __restrict__ in16,
                                                                 uint32_t* __restrict__ out16);
__global__ void __launch_bounds__(256) k_lines_store(uint32_t n_sets, uint32_t n_pairs, const uint32_t* __restrict__ out16,
                                                     uint32_t* __restrict__ lines);
// final_exp(F) == 1 of 12 one-lane records (lb_gt_check's combined product): out[0]
__global__ void __launch_bounds__(LB_LP_TPB) k_lp_final_lane(const uint32_t* __restrict__ prog,
                                                             const uint32_t* __restrict__ in16,
                                                             uint8_t* __restrict__ out);
// in16 of the merged check: the 63 level products P_l (one-lane fp12) and the MSM's bit sums G
__global__ void __launch_bounds__(256) k_mtail_prep(const fp12* __restrict__ Pl, const g2j* __restrict__ G,
                                                    uint32_t* __restrict__ in16);
// k_lp_rtail's inputs: LB_RTAIL_NIN 16-word records and one input flag per request
__global__ void __launch_bounds__(256) k_rtail_prep(uint32_t n_req, const fp12* __restrict__ F,
                                                    const g2a* __restrict__ S, uint32_t* __restrict__ in16,
                                                    uint32_t* __restrict__ inflag);
// the per-request tails of a failed merged check as round programs, one workgroup per request:
// valid[k] = final_exp(F_k * Miller(-g1, S_k)) == 1; requests already false or a passed merged
// check (skip) are settled without arithmetic, as k_tail does
__global__ void __launch_bounds__(LB_LP_TPB, LB_LP_VERIFY_WPE) k_lp_rtail(const uint32_t* __restrict__ prog,
                                                                          uint32_t n_req,
                                                                          const uint32_t* __restrict__ in16,
                                                                          const uint32_t* __restrict__ inflag,
                                                                          const uint8_t* __restrict__ req_bad,
                                                                          uint8_t* __restrict__ valid,
                                                                          const uint8_t* __restrict__ skip);
// 12 records of one-lane limbs -> fp12
__global__ void __launch_bounds__(64) k_records_to_fp12(const uint32_t* __restrict__ in16, fp12* __restrict__ F);
}  // namespace lb
