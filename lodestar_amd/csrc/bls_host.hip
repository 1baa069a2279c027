// MI355X (gfx950) BLS12-381 signature-set verification pipeline + C ABI.
//
// One lane per signature set for the per-set stages; one workgroup per set
// for pubkey aggregation; one lane per request for the request reductions.
// Integer VALU only (v_mad_u64_u32 chains); see DESIGN.md for the roofline.
//
// Pipeline of lb_verify_requests (reference: BlsMultiThreadWorkerPool job ->
// worker verifyManySignatureSets -> verifySignatureSetsMaybeBatch,
// packages/beacon-node/src/chain/bls/multithread/worker.ts:30-108,
// chain/bls/maybeBatch.ts:16-46):
//   k_req_flags       per request : 1-set requests need core-verify checks
//   k_decode_sigs     per set     : Signature.fromBytes(validate=true)
//   k_pubkeys_*       per set     : PublicKey.fromBytes + PublicKey.aggregate
//   k_hash_half/finish per message: hash_to_G2(signing root), two lanes per message
//   k_scalar_pk       per set     : r_i pk_i (GLV, 2 x 32-bit)
//   k_msm_*           per call    : S_all = sum r_i sig_i over the good requests, one
//                                   bucket MSM (k_msm.hip) for the merged check; or
//   k_scalar_sig + k_sum_tree     : r_i sig_i, S_k per request (small calls, and the
//                                   per-request tails after a failed merged check)
//   k_lines + k_miller_acc        : Miller(r_i pk_i, H_i) from stored lines, several
//     (or k_miller_sets + k_prod_tree) pairs per lane, product per request
//   k_lines_S + k_tail per request: Miller(-g1, S_k), final exponentiation, == 1,
//                                   one wave per request (wave-cooperative Fp12)
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "bls_kernels.h"
#include "bls_lp.h"
#ifdef LB_LP_PROGS_HEADER  // (a variant's programs, tools/lp_rows_variant.py)
#include LB_LP_PROGS_HEADER
#else
#include "bls_lp_progs.h"
#endif

using namespace lb;

// the latency path's round programs (gen_lp.py), embedded by lp_blob.hip
extern "C" const uint32_t lb_lp_blob[];

#ifdef LB_COUNT_OPS
static unsigned long long opcount_read_reset() {
  unsigned long long v = 0, z = 0;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_lb_fpmul_count), sizeof(v));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lb_fpmul_count), &z, sizeof(z));
  return v;
}
#endif

// ============================================================================
// Host side: context, workspace, C ABI
// ============================================================================
// What a call keeps between its front half (everything up to the merged
// product) and its tails (per-request final exponentiations), so a two-phase
// call (lb_verify_requests_partial_async) can stop after the front half, hand
// its Fp12 partial to the host and resume with the host's combined verdict.
struct PipeState {
  uint32_t n_req = 0, n_sets = 0, n_pairs = 0;
  bool merged = false, tail_wave = true;
  // merged check's S_all from the bucket MSM: the per-request S_k (per-set
  // ladders + sums) are computed only when the tails run
  bool msm = false;
  const uint8_t* d_seed = nullptr;
  const g2j* d_sig = nullptr;
  const uint8_t* d_sig_st = nullptr;
  g2j* d_rsig = nullptr;
  const uint32_t* d_req_off = nullptr;
  uint32_t* d_lines = nullptr;
  g2a* d_S = nullptr;
  fp12* d_F = nullptr;
  uint8_t* d_bad = nullptr;
  uint8_t* d_valid = nullptr;
  uint8_t* d_mflag = nullptr;
  uint32_t* d_mstats = nullptr;
  // steps organisation of the Miller accumulation (k_steps.hip): the lanes'
  // level products G (per-request F_k only when the tails need them)
  bool steps = false;
  Rows rows{};
  const uint32_t* d_G = nullptr;
  fp12* d_Fparts = nullptr;  // (a split accumulation: k_req_horner's parts per request, k_req_join)
  // the failed merged check's per-request tails as round programs (k_lp_rtail): staged inputs
  uint32_t* d_rt_in = nullptr;
  uint32_t* d_rt_fl = nullptr;
};

// A same-message package in flight (lb_verify_same_message_batch[_async]):
// what its completion needs after phase 1 (the jobs' aggregated sets) to
// publish verdicts and, for failed jobs, to run phase 2 (every set of those
// jobs alone) on the same slot from the device-resident decoded signatures.
struct SmState {
  bool active = false;
  int phase = 0;                     // 1: phase 1 in flight, 2: phase 2 (retries) in flight
  uint32_t nr = 0, retried_jobs = 0, fast_sets = 0;
  bool by_index = false;
  uint32_t nj = 0, ns = 0;
  uint8_t* out_valid = nullptr;     // caller: n_sets verdicts
  uint8_t* out_job_fast = nullptr;  // caller (optional): n_jobs flags
  const uint32_t* h_joff = nullptr;  // pinned copy of job_offsets
  const uint8_t* h_res = nullptr;    // pinned phase-1 results: valid, err, job_bad, pk status (al(nj) each)
  uint32_t* h_rset = nullptr;        // pinned: phase-2 set indices, then job indices (ns each)
  uint8_t* h_rout = nullptr;         // pinned: phase-2 verdicts, errors (al(ns) each)
  // device-resident phase-1 data
  const uint8_t* d_pks = nullptr;    // 96-byte keys or u32 indices (by_index)
  const uint8_t* d_rows = nullptr;   // by_index: the mixed package's key rows (or nullptr)
  const g2j* d_sig = nullptr;        // decoded signatures (validate=true done once)
  const uint8_t* d_sst = nullptr;
  const uint8_t* d_msgs = nullptr;
  const uint8_t* d_seed = nullptr;
  size_t ws_off = 0;                 // bump offset after phase 1 (phase 2 allocates from here)
  int err = 0;                       // a failed phase-2 launch: reported by this ticket's wait
  std::string err_msg;
};

// One in-flight call: two streams (DAG), own workspace, staging and events.
struct Slot {
  hipStream_t st[2] = {};
  // LB_PRIO_CUS with LB_PRIO_DYN=1: the slot's streams without and with the CU mask;
  // st[] is one pair or the other, chosen when a call is submitted (pick_streams)
  hipStream_t st_full[2] = {}, st_mask[2] = {};
  hipEvent_t dep[8] = {};
  hipEvent_t done = nullptr;
  char* d_ws = nullptr;
  size_t ws_cap = 0;
  char* h_pin = nullptr;
  size_t pin_cap = 0;
  static constexpr int kMaxStages = 32;
  hipEvent_t ev0[kMaxStages] = {}, ev1[kMaxStages] = {};
  const char* stage_name[kMaxStages] = {};
  int n_stages = 0;
  unsigned long long stage_ops[kMaxStages] = {};
  hipEvent_t wall0 = nullptr, wall1 = nullptr;
  bool busy = false;
  uint64_t ticket = 0;
  uint32_t* h_stats = nullptr;  // pinned: [batch_retries, batch_sigs_success] of the call in flight
  PipeState ps;
  // two-phase calls: front half enqueued, tails wait for lb_verify_requests_finish
  bool partial_pending = false;
  hipEvent_t partial_ev = nullptr;
  uint8_t* h_partial = nullptr;  // pinned, 576 B
  // host-buffer calls: device outputs, their pinned copies and the caller's
  // buffers they are copied into when the call retires (finish_slot)
  uint8_t *dv_valid = nullptr, *dv_err = nullptr, *dv_sst = nullptr;
  char* h_out = nullptr;
  uint8_t *out_valid = nullptr, *out_err = nullptr, *out_sst = nullptr;
  uint32_t out_nr = 0, out_ns = 0;
  SmState sm;
  // an async call on an otherwise idle GPU runs as the two-stream DAG with the
  // stream of an idle slot (borrowed); that slot is lent (busy) until the call retires
  Slot* borrowed = nullptr;
  Slot* lent_to = nullptr;
  // a synchronous call's second stream (borrow_second_stream): pick_streams keeps it
  hipStream_t guard_st = nullptr;
  // latency-path calls: the kernel's clock stamps (pinned, LpCall::clk), published to
  // ctx->lp_clk when the call retires
  unsigned long long* h_clk = nullptr;
  bool lp_call = false;
};

// The context's last error message.  lb_gt_check may run on one thread while another
// submits and retires calls (include/lodestar_bls.h), and both can fail: every write
// and read of the message takes a lock.
class ErrorText {
 public:
  ErrorText& operator=(std::string v) {
    std::lock_guard<std::mutex> g(mu_);
    s_ = std::move(v);
    return *this;
  }
  operator std::string() const {
    std::lock_guard<std::mutex> g(mu_);
    return s_;
  }

 private:
  mutable std::mutex mu_;
  std::string s_;
};

// A released two-phase call (LB_TP_RELEASE): what lb_partial_wait, lb_verify_requests_finish
// and lb_wait need once its slot has moved on -- the partial, and the call itself (the
// caller's buffers stay valid until lb_wait returns) for a re-run when the combine fails.
// Until its ticket is waited for, a released call's outputs hold provisional verdicts (every
// request not already false valid), so a record is never overwritten while it can still
// change them: lb_verify_requests_partial_async refuses a call whose ring entry is live
// (tp_reusable).  `failed`: the re-run after a failed combined check could not be submitted;
// lb_wait then returns that error instead of the provisional verdicts.
struct TwoPhaseRec {
  uint64_t ticket = 0;
  bool device = false, finished = false, have_partial = false, failed = false, waited = false;
  uint64_t rerun = 0;  // the one-phase re-run's ticket (failed combine)
  lb_request_batch batch{};
  uint8_t *valid = nullptr, *err = nullptr, *sst = nullptr;
  uint8_t partial[LB_GT_BYTES];
};

// Stats of a retired call, kept per ticket (lb_wait reports the stats of ITS
// ticket even when another call retired the slot first).
struct TicketStats {
  uint64_t ticket = 0;
  uint32_t batch_retries = 0, batch_sigs_success = 0;
  float wall_ms = 0.f;
};

struct lb_ctx {
  int device = -1;
  // One single-stream slot per hardware queue HIP gives this process: GPU_MAX_HW_QUEUES
  // (HIP's default and the box's setting are 4; at most kMaxSlots) -- more streams than
  // queues share a queue and measured -20 %, profiles/ab_r01i.txt.  That many calls are
  // in flight on the async API; a synchronous call runs on slot 0 as the two-stream DAG
  // by borrowing slot 1's stream for its duration.  LB_SLOTS overrides the count.
  // (24 hardware queues failed: HSA_STATUS_ERROR_OUT_OF_RESOURCES at k_miller_acc's dispatch,
  // whose 3.3 KB/lane private segment is reserved per queue; profiles/ab_r03/r03g_q24_fail.txt)
  static constexpr int kMaxSlots = 16;
  int n_slots = 4;
  int streams_per_slot[kMaxSlots + 1] = {2};  // (set for every slot in lb_create)
  // slots[n_slots] is the priority lane: one stream at the device's highest
  // priority, outside the async round robin, for latency-critical calls
  // (lb_verify_requests_priority_async, and lb_verify_requests of at most
  // lp_max_sets sets): they never queue behind the calls in flight
  Slot slots[kMaxSlots + 1];
  Slot& prio() { return slots[n_slots]; }
  bool prio_kcopy = true;  // the priority slot's host copies as kernels (slot_copy, LB_PRIO_KCOPY)
  int prio_cus = 0;  // CUs the throughput slots leave to the priority lane (LB_PRIO_CUS)
  // LB_PRIO_DYN=1 (with LB_PRIO_CUS): the throughput calls take the masked streams only
  // while the priority lane has been used within the last prio_hold_ms (LB_PRIO_HOLD_MS)
  bool prio_dyn = false;
  int prio_dyn_slots = 0;  // slots [0, prio_dyn_slots) own masked streams (LB_PRIO_DYN_SLOTS)
  double prio_hold_ms = 250.0;
  // steady-clock ns of the priority lane's last use (or lb_mark_priority from another
  // thread: an atomic, the one field of a context another thread may write)
  std::atomic<int64_t> last_prio_ns{INT64_MIN / 2};
  int next_slot = 0;
  uint64_t next_ticket = 1;
  // the last tickets issued to two-phase calls: lb_verify_requests_finish accepts a
  // ticket whose call a slot reuse already resumed only if it is one of these
  static constexpr int kTwoPhaseRing = 256;
  uint64_t two_phase[kTwoPhaseRing] = {};
  int two_phase_pos = 0;
  // LB_TP_RELEASE (default 1): a two-phase call completes as if the combined check passed and
  // frees its slot when its partial is out, instead of holding the slot through the host's
  // combine (-5..-7 % at N = 1); a failed combined check re-runs the shard
  // as a one-phase call.  One record per two-phase ticket (ring by ticket).
  bool tp_release = true;  // the mode of the two-phase call being submitted
  // LB_TP_RELEASE as configured; after a failed combined check the next tp_pause_calls two-phase
  // calls take the legacy mode: a re-run repeats the whole shard (one wrong set per C2 call:
  // 1.07 M sets/s released against 1.98 M legacy, bench.py adversarial_two_phase), the legacy
  // mode runs only the per-request tails, so a stream of failing batches (invalid gossip)
  // costs the tails alone while a clean stream keeps the release
  bool tp_release_cfg = true;
  uint32_t tp_pause = 0;
  uint32_t tp_pause_calls = 32;  // (LB_TP_PAUSE; 0: always release)
  bool fault_rerun = false;  // LB_FAULT_RERUN=1 (tests only): a failed combine's re-run fails to submit
  TwoPhaseRec tp[kTwoPhaseRing];
  ErrorText err;
  hipStream_t stream = nullptr;  // slot 0 stream 0 (synchronous helper calls)
  // Miller organisation: stored lines + one wave per pair (k_lines/k_pair_wc,
  // lowest latency) up to wave_max_sets; one pair per lane (k_miller_sets)
  // below lines_min_sets; stored lines + multi-pair accumulation per request
  // (k_lines/k_miller_acc, highest throughput) from there.  LB_MILLER=wave|lane|lines forces one.
  int miller_mode = 0;  // 0 auto, 1 lane, 2 lines, 3 wave
  // 1025: every call the latency path does not take (lp_max_sets) uses the stored lines;
  // 1.5k-6k-set calls 25-29 -> 17-19 ms, C5 27.2 -> 21.0 ms (profiles/r06/orgs_probe_r06f.json)
  uint32_t lines_min_sets = 1025;
  uint32_t wave_max_sets = 1024;
  // LB_LINES_WAVES: 1 or 2 waves/SIMD for k_lines(_rows): 2 spills (3.4 -> 4.7 ms alone) but its
  // waves share SIMDs with other calls' in the pipeline (profiles/ab_r03/ab_r03r, ab_r03s)
  int lines_waves = 2;
  int lines_waves_small = 1;  // k_lines for the calls below the steps organisation
  int acc_lpr = 64;     // LB_ACC_LPR: lanes per request in k_miller_acc (64, 32, 16)
  int acc_split = -1;   // LB_ACC_SPLIT: 1 always / 0 never split requests in halves; -1 = lone calls only
  // Miller accumulation of the stored lines: 1 = step-major lanes + level products +
  // one Horner chain (k_steps.hip, default), 0 = pair-major k_miller_acc (LB_ACC=pairs)
  int acc_steps = 1;
  // LB_DAG=0: a call never borrows a second stream (every kernel of a lone call runs
  // alone on the GPU: bench.py's per-kernel iso timings and their rocprof profile)
  bool dag = true;
  // LB_STEP_MODE: k_step_acc variant (0 registers + paired lines, 1 accumulator in LDS,
  // 2 registers + one line at a time; k_steps.hip)
  // defaults (round 4): the accumulator in LDS at one wave per SIMD -- alone 4.64-4.70 ms per
  // C2 launch against 6.04-6.10 for one line at a time at 2 waves/SIMD (which spilled 1,408
  // B/lane: 18.3 GB of traffic per launch, 13.9x the algorithmic bytes; now 2.6 GB, 2.0x), the
  // pipeline 3.55-3.62 vs 3.54-3.57 M sets/s, three interleaved runs each
  // (profiles/r04/step_ab/).  Round 3 had measured 2/2 ahead of 2/1 (profiles/ab_r03/ab_r03s).
  // Round 5, in the final pipeline (merged-check program, two-phase flow): one line at a time
  // at 2 waves/SIMD (LB_STEP_MODE=2 LB_STEP_WAVES=2) measured ahead -- 3.61-3.67 M (mean 3.650
  // over 5 runs) against the LDS build's 3.53-3.61 M (mean 3.569) -- but alone it takes 5.7 ms
  // against 4.4-4.5 and moves 18.4 GB per launch (13.9x its algorithmic bytes: spills) against
  // 2.6 GB (profiles/r05/knobs/, final/pmc_traffic_r05s3.json); the LDS build stays the default
  // until a 2-wave build without the spills exists (half the accumulator in LDS: 18 KB a
  // workgroup, 8 per CU)
  int step_mode = 1;
  int step_waves = 1;  // LB_STEP_WAVES: occupancy target of k_step_acc (1 or 2)
  // LB_STAGE_EVENTS=0: no per-stage timing events (two HIP calls per kernel of the
  // submission; the N-API addon sets it, lb_last_stage_times is then empty)
  bool stage_events = true;
  // per-request tails: one wave per request (k_lines_S + k_tail, wave-cooperative
  // Fp12) or LB_TAIL=lane: one lane per request (k_miller_S + k_final)
  bool tail_wave = true;
  // merged check of the whole call first (one tail), per-request tails only
  // when it fails; used from merge_min_req requests up (LB_MERGE_MIN, 0 = off)
  uint32_t merge_min_req = 8;
  // merged calls of at least msm_min_sets sets take S_all from the bucket MSM
  // (k_msm.hip) instead of per-set ladders (LB_MSM_MIN, 0 = never)
  uint32_t msm_min_sets = 1025;  // (same probe: from 1025 sets the MSM beats the ladders)
  // merged steps calls: the level products as lane products + wave-cooperative passes
  // (k_level_part / k_level_wc) instead of k_level_prod's one-lane LDS tree (LB_LEVEL=0)
  bool level_wc = true;
  // lone calls: the MSM's bucket sums on LB_MSM_BLANES lanes per bucket and its bit sums on 256
  // threads (LB_MSM_LANES=0: one lane per bucket and one wave per bit, round 5, always), the
  // merged-check program on 64 rows (LB_WIDE_TAIL=0: 32 rows always)
  bool msm_lanes = true;
  bool wide_tail = true;
  bool msm_bits_lp = true;  // (LB_MSM_BITS_LP=0: a lone call's bit sums by k_msm_bits' 256 threads)
  uint32_t step_split = 0;  // LB_STEP_SPLIT: 1, 2 or 4 lanes per set always (0: by size, lone calls only)
  // same-message packages of at most LB_SM_DEC_MAX signatures decode them as round programs
  // (k_lp_dec; LB_SM_LP_DECODE=0: k_decode_sigs always)
  bool sm_lp_decode = true;
  // lone pipeline calls of at most LB_LP_DEC_MAX sets decode their signatures the same way
  // (LB_LP_DECODE=0: k_decode_sigs)
  bool lp_decode = true;
  bool lp_hash_finish = true;  // (LB_LP_HASH_FINISH: the same calls' hash finish as round programs)
  bool msm_short = true;  // (LB_MSM_SHORT: a lone mid-size call's MSM chunks of LB_MSM_T_LONE entries)
  uint32_t msm_short_max = 16384u, msm_t_lone = LB_MSM_T_LONE;  // (LB_MSM_SHORT_MAX / LB_MSM_T_LONE probes)
  // (the lone-call round-program size bounds; env LB_LP_DEC_MAX / LB_LP_HF_MAX / LB_LP_LINES_MAX probe others)
  uint32_t lp_dec_max = LB_LP_DEC_MAX, lp_hf_max = LB_LP_HF_MAX, lp_lines_max = LB_LP_LINES_MAX;
  // (LB_LP_HASH_FULL: lone calls of at most this many sets run hash_to_G2's whole curve part as one
  // program per set, k_lp_hash -- profiles/r06/orgs_probe_r06hf3.json; 0: never)
  uint32_t lp_hash_full = 2048;
  uint32_t lp_narrow = 1;  // (LB_LP_NARROW=1: the hash-finish program on LB_LP_NARROW_ROWS rows, default; 0: 16 rows)
  bool lp_lines = true;  // (LB_LP_LINES: a lone steps call's lines as round programs, up to LB_LP_LINES_MAX sets)
  // device-resident pubkey table (index2pubkey mirror, lb_pubkey_table_*)
  g1a* d_table = nullptr;
  uint32_t table_n = 0, table_cap = 0;
  // timing of the last completed verify call
  int n_stages = 0;
  float stage_ms[Slot::kMaxStages] = {};
  const char* stage_name[Slot::kMaxStages] = {};
  unsigned long long stage_ops[Slot::kMaxStages] = {};
  float wall_ms = 0.f;
  uint32_t batch_retries = 0, batch_sigs_success = 0;
  static constexpr int kTicketRing = 64;
  TicketStats tstats[kTicketRing];
  // lb_gt_check runs on its own stream and buffers, so the host combine of the
  // shards' partials never drains the slots' calls in flight
  hipStream_t aux_stream = nullptr;
  // the merged check's one-wave chain of every slot (highest priority) when
  // LB_TAIL_PRIO=1; nullptr (default): the slot's own stream
  hipStream_t tail_stream = nullptr;
  uint8_t* d_aux = nullptr;
  uint8_t* h_aux = nullptr;
  size_t aux_cap = 0;
  // latency path: the round programs in device memory (uploaded on first use);
  // calls of at most lp_max_sets sets run it instead of the throughput pipeline
  // (LB_LP_MAX, lb_set_latency_path; 0 = never)
  uint32_t* d_lp = nullptr;
  uint32_t lp_max_sets = 1024;
  uint32_t lp_lone_max = 896;  // (LB_LP_LONE_MAX, 0 = off: lone calls above it take the pipeline, run_pipeline)
  bool lp_explicit = false;    // (the bound set by lb_set_latency_path / LB_LP_MAX: no lone rule)
  // the merged check of a steps + MSM call as a round program (k_lp_mtail: S_all from the
  // MSM's bit sums, Miller(-g1, S_all), final exponentiation on one workgroup) instead of
  // msm_final + lines of S_all + the one-wave k_tail (LB_MTAIL=0: the one-wave chain)
  bool mtail_lp = true;
  // LB_RTAIL (default 1): a failed merged check's per-request tails (Miller(-g1, S_k), F_k times
  // it, final exponentiation) as one round program per request (k_lp_rtail) instead of one-lane
  // lines of S_k (k_lines_S) + the one-wave chain (k_tail)
  bool rtail_lp = true;
  bool gt_lp = true;  // lb_gt_check's final exponentiation as a round program (LB_GT_LP=0: one wave)
  int hw_queues = 0;  // hardware queues this context opens (priced by lb_create's guard)
  int q_plain = 0, q_high = 0, q_masked = 0;  // its streams in the process tally (g_q_*)
  bool lane = false;  // lb_create_lane: a latency-lane context (one slot, no CU-masked streams)
  int last_call_streams = 0;  // streams of the last submitted verify call (begin_call)
  unsigned long long lp_clk[4] = {};  // clock stamps of the last retired latency-path call
};

namespace {

#define LB_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ctx->err = std::string(#call) + ": " + hipGetErrorString(e_);                    \
      return LB_ERR_DEVICE;                                                            \
    }                                                                                  \
  } while (0)

#define LB_TRY(x)                 \
  do {                            \
    int rc_ = (x);                \
    if (rc_ != LB_OK) return rc_; \
  } while (0)

inline uint32_t blocks_for(uint32_t n, uint32_t tpb = TPB) { return (n + tpb - 1) / tpb; }

struct Bump {
  char* base;
  size_t off = 0;
  size_t cap;
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* p = reinterpret_cast<T*>(base + off);
    off += sizeof(T) * count;
    return p;
  }
};

int ensure_ws(lb_ctx* ctx, Slot& sl, size_t bytes) {
  if (bytes <= sl.ws_cap) return LB_OK;
  if (sl.d_ws) {
    LB_HIP(hipStreamSynchronize(sl.st[0]));
    LB_HIP(hipStreamSynchronize(sl.st[1]));
    LB_HIP(hipFree(sl.d_ws));
    sl.d_ws = nullptr;
    sl.ws_cap = 0;
  }
  size_t cap = bytes + bytes / 4 + (1 << 20);
  if (hipMalloc(&sl.d_ws, cap) != hipSuccess) {
    ctx->err = "hipMalloc workspace failed";
    return LB_ERR_OUT_OF_MEMORY;
  }
  sl.ws_cap = cap;
  return LB_OK;
}
int ensure_ws(lb_ctx* ctx, size_t bytes) { return ensure_ws(ctx, ctx->slots[0], bytes); }

int ensure_pin(lb_ctx* ctx, Slot& sl, size_t bytes) {
  if (bytes <= sl.pin_cap) return LB_OK;
  if (sl.h_pin) {
    LB_HIP(hipStreamSynchronize(sl.st[0]));
    LB_HIP(hipHostFree(sl.h_pin));
    sl.h_pin = nullptr;
    sl.pin_cap = 0;
  }
  size_t cap = bytes + bytes / 4 + (1 << 20);
  if (hipHostMalloc(&sl.h_pin, cap, hipHostMallocDefault) != hipSuccess) {
    ctx->err = "hipHostMalloc staging failed";
    return LB_ERR_OUT_OF_MEMORY;
  }
  sl.pin_cap = cap;
  return LB_OK;
}

#ifdef LB_COUNT_OPS
#define LB_COUNT_SYNC() LB_HIP(hipDeviceSynchronize())
#define LB_COUNT_TAKE(i) sl.stage_ops[i] = opcount_read_reset()
#else
#define LB_COUNT_SYNC() ((void)0)
#define LB_COUNT_TAKE(i) ((void)0)
#endif

// Launch `kern` on stream `s` of slot `sl`, bracketed by timing events.
#define LB_STAGE_ON(name, strm, kern, grid, block, ...)                                    \
  do {                                                                                     \
    const int si_ = (ctx->stage_events && sl.n_stages < Slot::kMaxStages) ? sl.n_stages++ : -1; \
    hipStream_t strm_ = (strm);                                                            \
    LB_COUNT_SYNC();                                                                       \
    if (si_ >= 0) {                                                                        \
      LB_COUNT_TAKE(si_);                                                                  \
      sl.stage_name[si_] = name;                                                           \
      LB_HIP(hipEventRecord(sl.ev0[si_], strm_));                                          \
    }                                                                                      \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, strm_, __VA_ARGS__);             \
    LB_HIP(hipGetLastError());                                                             \
    if (si_ >= 0) LB_HIP(hipEventRecord(sl.ev1[si_], strm_));                              \
    LB_COUNT_SYNC();                                                                       \
    if (si_ >= 0) {                                                                        \
      LB_COUNT_TAKE(si_);                                                                  \
    }                                                                                      \
  } while (0)
#define LB_STAGE(name, s, kern, grid, block, ...) LB_STAGE_ON(name, sl.st[s], kern, grid, block, __VA_ARGS__)

#define LB_LAUNCH(kern, grid, block, ...)                                                  \
  do {                                                                                     \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, ctx->stream, __VA_ARGS__);       \
    LB_HIP(hipGetLastError());                                                             \
  } while (0)

int lp_ensure(lb_ctx* ctx);
static uint32_t level_blocks(uint32_t n_sets, uint32_t n_req, bool wide);
static uint32_t step_split_for(uint32_t n_sets);
int slot_copy(lb_ctx* ctx, Slot& sl, void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t st);

// The latency path (k_lp.hip) for a small call: pubkeys -> per-set inputs -> one
// workgroup per set (set program, the request's product tree, the root's final
// exponentiation).  No merged check: every request is verified on its own, in
// parallel, which is what the reference's verdicts are per request anyway.
int run_lp(lb_ctx* ctx, Slot& sl, uint32_t n_req, uint32_t n_sets, const uint32_t* d_req_off, const uint8_t* d_pks,
           const uint32_t* d_pk_off, const uint32_t* d_pk_idx, const uint8_t* d_msgs, const uint8_t* d_sigs,
           const uint32_t* d_sig_off, const uint8_t* d_seed, uint8_t* d_valid, uint8_t* d_req_err,
           uint8_t* d_set_status, Bump& ws) {
  LB_TRY(lp_ensure(ctx));
  const uint32_t ns = n_sets ? n_sets : 1;
  g1j* d_pk = ws.take<g1j>(ns);
  uint8_t* d_pk_st = ws.take<uint8_t>(ns);
  uint32_t* d_in16 = ws.take<uint32_t>((size_t)ns * LB_LP_NIN * 16);
  uint32_t* d_fl = ws.take<uint32_t>((size_t)ns * LB_LP_NFL);
  uint8_t* d_sig_st = d_set_status ? d_set_status : ws.take<uint8_t>(ns);
  uint32_t* d_setreq = ws.take<uint32_t>(ns);
  uint32_t* d_F = ws.take<uint32_t>((size_t)ns * 12 * 16);
  uint32_t* d_cnt = ws.take<uint32_t>((size_t)LB_LP_TREE_LEVELS * ns);
  unsigned long long* d_clk = ws.take<unsigned long long>(4);
  if (ws.off > ws.cap) {
    ctx->err = "workspace overflow";
    return LB_ERR_OUT_OF_MEMORY;
  }
  if (!n_sets) {  // every request empty: false (otherwise k_lp_prep zeroes the outputs)
    LB_HIP(hipMemsetAsync(d_valid, 0, n_req, sl.st[0]));
    LB_HIP(hipMemsetAsync(d_req_err, 0, n_req, sl.st[0]));
    return LB_OK;
  }
  const PkSource src{d_pks, d_pk_idx, ctx->d_table, ctx->table_n};
  LB_STAGE("pubkeys", 0, k_pubkeys_single, blocks_for(n_sets), TPB, n_sets, src, d_pk_off, d_pk, d_pk_st);
  if (d_pk_off)
    LB_STAGE("pubkeys_agg", 0, k_pubkeys_agg, n_sets < 16384u ? n_sets : 16384u, TPB, n_sets, src, d_pk_off, d_pk,
             d_pk_st);
  LB_STAGE("lp_prep", 0, k_lp_prep, blocks_for(n_sets), TPB, n_sets, d_req_off, n_req, d_msgs, d_sigs, d_sig_off,
           (const g1j*)d_pk, d_seed, d_in16, d_fl, d_sig_st, d_setreq, d_valid, d_req_err, d_cnt,
           (uint32_t)LB_LP_TREE_LEVELS * ns, d_clk);
  LpCall c;
  c.prog_single = ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_SET_SINGLE].off;
  c.prog_batch = ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_SET_BATCH].off;
  c.prog_mul = ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_MUL].off;
  c.prog_final = ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_FINAL].off;
  c.req_off = d_req_off;
  c.set_req = d_setreq;
  c.in16 = d_in16;
  c.flags = d_fl;
  c.sig_st = d_sig_st;
  c.pk_st = d_pk_st;
  c.F = d_F;
  c.cnt = d_cnt;
  c.valid = d_valid;
  c.req_err = d_req_err;
  c.n_sets = n_sets;
  c.clk = d_clk;
  LB_STAGE("lp_verify", 0, k_lp_verify, n_sets, LB_LP_TPB, c);
  LB_TRY(slot_copy(ctx, sl, sl.h_clk, d_clk, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, sl.st[0]));
  sl.lp_call = true;
  PipeState& ps = sl.ps;
  ps = PipeState{};
  ps.n_req = n_req;
  ps.n_sets = n_sets;
  ps.d_valid = d_valid;
  return LB_OK;
}

// stream `to` of the slot waits for everything enqueued so far on stream `from`
int stream_wait(lb_ctx* ctx, Slot& sl, int from, int to, int ev) {
  LB_HIP(hipEventRecord(sl.dep[ev], sl.st[from]));
  LB_HIP(hipStreamWaitEvent(sl.st[to], sl.dep[ev], 0));
  return LB_OK;
}

// Core pipeline on device-resident inputs (all pointers are device pointers),
// as a two-stream DAG inside the slot:
//   A: flags -> pubkeys -> r_i pk_i -> [evPK] -> decode sigs -> r_i sig_i -> S_k (tree)
//      -> Miller(-g1, S_k) -> [wait B] -> per-request product (tree) -> final exp
//   B: hash_to_G2 (two lanes per message) -> [wait evPK] -> lines of (r_i pk_i, H_i)
// with the Miller values accumulated per request from the stored lines
// (k_miller_acc, several pairs per lane sharing the Fp12 squarings); the
// original one-pair-per-lane Miller (k_miller_sets + k_prod_tree) remains
// selectable with LB_MILLER=lane for comparison.
// Tails of a call (after the per-request products F_k): with a merged check,
// the per-request tails run only when d_mflag[0] == 0 (k_lines_S / k_tail skip
// themselves otherwise); without one, every request runs its tail.
int run_tails(lb_ctx* ctx, Slot& sl) {
  const PipeState& p = sl.ps;
  if (p.merged) {
    if (p.msm) {  // the S_k of the per-request tails (skipped when the merged check passed)
      LB_STAGE("scalar_sig", 0, k_scalar_sig, blocks_for(p.n_sets), TPB, p.n_sets, p.d_seed, p.d_sig, p.d_sig_st,
               p.d_rsig, (const uint8_t*)p.d_mflag);
      LB_STAGE("sum_tree", 0, k_sum_tree, p.n_req, TPB, p.n_req, p.d_req_off, (const g2j*)p.d_rsig, p.d_S,
               (const uint8_t*)p.d_mflag);
    }
    if (!p.d_rt_in)
      LB_STAGE("lines_S", 0, k_lines_S, blocks_for(p.n_req), TPB, p.n_req, p.n_pairs, p.n_sets, (const g2a*)p.d_S,
               p.d_lines, (const uint8_t*)p.d_mflag);
    if (p.steps) {
      const uint32_t sp = p.rows.split;
      LB_STAGE("req_horner", 0, k_req_horner, p.n_req * sp, TPB, p.n_req, p.n_sets, p.rows, p.d_req_off, p.d_G,
               (const uint8_t*)p.d_bad, sp > 1 ? p.d_Fparts : p.d_F, (const uint8_t*)p.d_mflag);
      if (sp > 1)
        LB_STAGE("req_horner", 0, k_req_join, p.n_req, TPB, p.n_req, sp, (const fp12*)p.d_Fparts,
                 (const uint8_t*)p.d_bad, p.d_F, (const uint8_t*)p.d_mflag);
    }
    if (p.d_rt_in) {
      hipLaunchKernelGGL(k_rtail_prep, dim3((p.n_req * LB_RTAIL_NIN + 255) / 256), dim3(256), 0, sl.st[0], p.n_req,
                         (const fp12*)p.d_F, (const g2a*)p.d_S, p.d_rt_in, p.d_rt_fl);
      LB_HIP(hipGetLastError());
      LB_STAGE("rtail", 0, k_lp_rtail, p.n_req, LB_LP_TPB, ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_RTAIL].off, p.n_req,
               (const uint32_t*)p.d_rt_in, (const uint32_t*)p.d_rt_fl, (const uint8_t*)p.d_bad, p.d_valid,
               (const uint8_t*)p.d_mflag);
    } else {
      LB_STAGE("tail", 0, k_tail, p.n_req, TPB, p.n_req, p.n_pairs, p.n_sets, (const uint32_t*)p.d_lines,
               (const fp12*)p.d_F, (const uint8_t*)p.d_bad, p.d_valid, (const uint8_t*)p.d_mflag);
    }
    hipLaunchKernelGGL(k_merge_stats, dim3(1), dim3(TPB), 0, sl.st[0], p.n_req, p.d_req_off, (const uint8_t*)p.d_bad,
                       (const uint8_t*)p.d_mflag, p.d_mstats);
    LB_HIP(hipGetLastError());
    LB_HIP(hipMemcpyAsync(sl.h_stats, p.d_mstats, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, sl.st[0]));
  } else if (p.tail_wave) {
    LB_STAGE("tail", 0, k_tail, p.n_req, TPB, p.n_req, p.n_pairs, p.n_sets, (const uint32_t*)p.d_lines,
             (const fp12*)p.d_F, (const uint8_t*)p.d_bad, p.d_valid, (const uint8_t*)nullptr);
  } else {
    LB_STAGE("final_exp", 0, k_final, blocks_for(p.n_req), TPB, p.n_req, (const fp12*)p.d_F, (const uint8_t*)p.d_bad,
             p.d_valid);
  }
  return LB_OK;
}

// lone calls of lp_lone_max < n_sets <= lp_max_sets leave the latency path for the pipeline
// (run_pipeline's lone_mid; the synchronous entry points then take slot 0's two-stream DAG)
static bool lp_lone_rule(const lb_ctx* ctx, uint32_t n_sets) {
  return !ctx->lp_explicit && ctx->lp_lone_max && n_sets > ctx->lp_lone_max && n_sets <= ctx->lp_max_sets;
}

static bool any_slot_busy(const lb_ctx* ctx) {
  for (int s = 0; s <= ctx->n_slots; s++)
    if (ctx->slots[s].busy) return true;
  return false;
}

int run_pipeline(lb_ctx* ctx, Slot& sl, uint32_t n_req, uint32_t n_sets, const uint32_t* d_req_off,
                 const uint8_t* d_pks, const uint32_t* d_pk_off, const uint32_t* d_pk_idx, const uint8_t* d_msgs, const uint8_t* d_sigs,
                 const uint32_t* d_sig_off, const uint8_t* d_seed, uint8_t* d_valid, uint8_t* d_req_err,
                 uint8_t* d_set_status, Bump& ws, uint8_t* d_partial = nullptr, const g2j* d_sig_pre = nullptr,
                 const uint8_t* d_sst_pre = nullptr) {
  // d_sig_pre / d_sst_pre: signatures already decoded and validated (same-message
  // phase 2): no k_decode_sigs, d_sigs / d_sig_off unused
  const bool partial = d_partial != nullptr;
  bool lone = true;  // (no other slot busy: the GPU is this call's)
  for (int s = 0; s < ctx->n_slots; s++)
    if (&ctx->slots[s] != &sl && ctx->slots[s].busy && ctx->slots[s].lent_to != &sl) lone = false;
  // a lone call of lp_lone_max < n_sets <= lp_max_sets runs the pipeline's steps + MSM + merged-check
  // program instead of the latency path (~7.0 ms flat from ~400 sets against the latency path's
  // 7.2 / 8.0 ms at 896 / 1,024 sets, profiles/r06/orgs_probe_r06lp2.json), merged whatever its
  // request count; not when the latency-path bound was set explicitly (lb_set_latency_path, LB_LP_MAX)
  const bool lone_mid = !partial && !d_sig_pre && lone && &sl != &ctx->prio() && lp_lone_rule(ctx, n_sets) &&
                        ctx->miller_mode == 0 && ctx->tail_wave && ctx->acc_steps;
  if (!partial && !d_sig_pre && n_sets <= ctx->lp_max_sets && !lone_mid) {
    sl.h_stats[0] = sl.h_stats[1] = 0;
    return run_lp(ctx, sl, n_req, n_sets, d_req_off, d_pks, d_pk_off, d_pk_idx, d_msgs, d_sigs, d_sig_off, d_seed,
                  d_valid, d_req_err, d_set_status, ws);
  }
  const uint32_t ns = n_sets ? n_sets : 1;
  g2j* d_sig = d_sig_pre ? const_cast<g2j*>(d_sig_pre) : ws.take<g2j>(ns);
  g2j* d_rsig = ws.take<g2j>(ns);
  g2j* d_q = ws.take<g2j>(2 * (size_t)ns);
  g2j* d_h = ws.take<g2j>(ns);
  g1j* d_pk = ws.take<g1j>(ns);
  g1j* d_rpk = ws.take<g1j>(ns);
  const bool by_lines = ctx->miller_mode == 2 || (ctx->miller_mode == 0 && n_sets >= ctx->lines_min_sets) || lone_mid;
  const bool by_wave =
      !by_lines && (ctx->miller_mode == 3 || (ctx->miller_mode == 0 && n_sets <= ctx->wave_max_sets));
  fp12* d_f = by_lines ? nullptr : ws.take<fp12>(ns);  // per-set Miller values (lane / wave modes)
  // a two-phase call always merges (its partial is the merged product) and uses the wave tails
  const bool tail_wave = ctx->tail_wave || partial;
  // stored lines: set pairs [0, n_sets) (lines mode), S pairs [n_sets, n_sets + n_req) (wave tails)
  const bool merged = partial || (tail_wave && ctx->merge_min_req && n_req >= ctx->merge_min_req) || lone_mid;
  const uint32_t n_pairs = n_sets + n_req + (merged ? 1u : 0u);  // + the merged pair (-g1, S_all)
  const bool use_msm = merged && n_sets && ctx->msm_min_sets && (n_sets >= ctx->msm_min_sets || lone_mid);
  // a lone call on an otherwise idle GPU splits every request of the Miller
  // accumulation in two halves: twice the waves (one per SIMD for a 65,536-set
  // call instead of one per two SIMDs) at the price of the halves' separate
  // Fp12 squarings; with other calls in flight the idle SIMDs run their stages
  // instead and the work-efficient form is kept (LB_ACC_SPLIT=0|1 forces one)
  // steps organisation (k_steps.hip): no split (a request already has one lane per set)
  const bool steps = by_lines && tail_wave && n_sets && ctx->acc_steps;
  const bool split = by_lines && !steps && (ctx->acc_split == 1 || (ctx->acc_split < 0 && lone && n_req >= 64));
  // merged pair (-g1, S_all) with S_all from the MSM: without a split its Miller
  // value is one extra workgroup of k_miller_acc (fold; its 512 request waves
  // leave SIMDs free), otherwise its lines are stored right after the MSM, on
  // stream 0 beside stream 1's hash/lines (lines_all), and k_tail multiplies it in
  const bool fold = use_msm && by_lines && !split && !steps;
  // merged check as a round program (k_lp_mtail): S_all, its Miller value and the final
  // exponentiation from the MSM's bit sums and the 63 level products (their Horner chain folded in)
  const bool mtail = steps && use_msm && merged && ctx->mtail_lp;
  // a lone call's serial tail in its wide forms (the GPU otherwise idle: latency is what counts):
  // the merged-check program on LB_LP_MTAIL_ROWS rows, the MSM's sums over more lanes.  With other
  // calls in flight the narrow forms, whose smaller workgroups wait for less of a CU (C2 3.62 vs
  // 3.67 / 3.68 M sets/s with either wide form in every call, profiles/r06/ab_r06k/)
  const bool mt_wide = lone && ctx->wide_tail;
  const uint32_t mt_tpb = mt_wide ? LB_LP_MTAIL_ROWS * 16u : (uint32_t)LB_LP_TPB;
  const bool msm_wide = lone && ctx->msm_lanes;
  // (and its bit sums as round programs: 9 dependent one-lane additions -> 3 launches of ~10-16 rounds)
  const bool bits_lp = msm_wide && mtail && ctx->msm_bits_lp;
  if (mtail) LB_TRY(lp_ensure(ctx));
  // (steps + merged: the merged pair's lines come from a one-lane kernel before the
  // accumulation; as an extra workgroup of k_step_acc they measured 4.8 -> 8.2 ms: the
  // 1,025th wave waits for a SIMD of the 1,024 set waves, then runs the 3.4 ms line chain)
  uint32_t* d_lines =
      (by_lines || by_wave || tail_wave) ? ws.take<uint32_t>((size_t)n_pairs * LB_MILLER_LINES * 72) : nullptr;
  uint8_t* d_single = ws.take<uint8_t>(ns);
  uint8_t* d_pk_st = ws.take<uint8_t>(ns);
  uint8_t* d_sig_st = d_sst_pre ? const_cast<uint8_t*>(d_sst_pre) : d_set_status ? d_set_status : ws.take<uint8_t>(ns);
  g2a* d_S = ws.take<g2a>(n_req);
  fp12* d_fS = ws.take<fp12>(n_req);
  fp12* d_F = ws.take<fp12>(n_req);
  // (a merged call's failure path: the per-request tails' round-program inputs, k_lp_rtail)
  const bool rtail = merged && tail_wave && ctx->rtail_lp;
  if (rtail) LB_TRY(lp_ensure(ctx));
  uint32_t* d_rt_in = rtail ? ws.take<uint32_t>((size_t)(n_req ? n_req : 1) * LB_RTAIL_NIN * 16) : nullptr;
  uint32_t* d_rt_fl = rtail ? ws.take<uint32_t>(n_req ? n_req : 1) : nullptr;
  uint8_t* d_bad = ws.take<uint8_t>(n_req);
  g2a* d_Sall = ws.take<g2a>(1);
  fp12* d_Fall = ws.take<fp12>(1);
  uint8_t* d_mflag = ws.take<uint8_t>(2);  // [0] merged check passed, [1] constant 0 (req_bad of the merged pair)
  uint32_t* d_mstats = ws.take<uint32_t>(2);
  // bucket MSM workspace: keys + sorted entries (2 half-points x W windows per
  // set), histogram / cursors / offsets, chunk partials, bucket sums, G_p
  const size_t n_ent = use_msm ? 2 * (size_t)n_sets * LB_MSM_W : 0;
  // (a lone mid-size call: chunks of LB_MSM_T_LONE entries -- k_msm_chunks' chains are one lane's
  // mixed additions, 16 of them ~2.5 ms for C5; LB_MSM_SHORT=0 keeps LB_MSM_T)
  const bool msm_short = use_msm && lone && n_sets <= ctx->msm_short_max && ctx->msm_short;
  const uint32_t msm_T = msm_short ? ctx->msm_t_lone : LB_MSM_T;
  const size_t max_chunks = use_msm ? n_ent / msm_T + LB_MSM_BUCKETS : 0;
  uint32_t* d_mkeys = use_msm ? ws.take<uint32_t>(n_ent) : nullptr;
  uint32_t* d_msorted = use_msm ? ws.take<uint32_t>(n_ent) : nullptr;
  uint32_t* d_mhist = use_msm ? ws.take<uint32_t>(4 * (LB_MSM_BUCKETS + 1)) : nullptr;
  g2j* d_mcsum = use_msm ? ws.take<g2j>(max_chunks) : nullptr;
  g2j* d_mbsum = use_msm ? ws.take<g2j>(LB_MSM_BUCKETS) : nullptr;
  g2j* d_mG = use_msm ? ws.take<g2j>(LB_MSM_POS) : nullptr;
  // steps organisation: size histogram + cursors, gt, row offsets, order, meta, G, level products
  uint32_t* d_rhist = steps ? ws.take<uint32_t>(2 * ((size_t)ns + 1)) : nullptr;
  uint32_t* d_rgt = steps ? ws.take<uint32_t>((size_t)ns + 1) : nullptr;
  uint32_t* d_rowoff = steps ? ws.take<uint32_t>((size_t)ns + 1) : nullptr;
  uint32_t* d_rpos = steps ? ws.take<uint32_t>(n_req) : nullptr;
  uint32_t* d_rinv = steps ? ws.take<uint32_t>(n_req) : nullptr;
  uint32_t* d_rmeta = steps ? ws.take<uint32_t>(1) : nullptr;
  // a lone mid-size call splits every lane of the step-major accumulation (its time is the
  // one-lane latency of a lane's 68 lines: 17 or 34 lines a lane instead; LB_STEP_SPLIT forces)
  uint32_t lsplit = 1;
  if (steps) {
    lsplit = lone ? step_split_for(n_sets) : 1u;
    if (ctx->step_split) lsplit = ctx->step_split;
  }
  uint32_t* d_G = steps ? ws.take<uint32_t>(144 * (size_t)ns * lsplit) : nullptr;
  fp12* d_Fparts = steps && lsplit > 1 ? ws.take<fp12>((size_t)(n_req ? n_req : 1) * lsplit) : nullptr;
  // a lone mid-size call's signature decode as round programs (k_sm_dec_prep / k_lp_dec / k_sm_dec_finish)
  const bool dec_lp = lone && !d_sig_pre && n_sets && n_sets <= ctx->lp_dec_max && ctx->lp_decode;
  uint32_t* d_dec_in = dec_lp ? ws.take<uint32_t>((size_t)ns * 4 * 16) : nullptr;
  uint32_t* d_dec_fl = dec_lp ? ws.take<uint32_t>((size_t)ns * 3) : nullptr;
  uint32_t* d_dec_out = dec_lp ? ws.take<uint32_t>((size_t)ns * 2 * 16) : nullptr;
  uint32_t* d_dec_ofl = dec_lp ? ws.take<uint32_t>((size_t)ns * 2) : nullptr;
  uint8_t* d_dec_pre = dec_lp ? ws.take<uint8_t>(ns) : nullptr;
  if (dec_lp) LB_TRY(lp_ensure(ctx));
  // ... and, up to LB_LP_HF_MAX sets, its hash finish (k_hf_prep / k_lp_hf / k_hf_finish; above that
  // the workgroups queue: 1,536 / 2,048 sets 13.4 -> 11.0 / 11.8 ms, 4,704 (C5) 16.1 -> 17.4,
  // profiles/r06/orgs_probe_r06hf.json; LB_LP_HASH_FINISH=0: k_hash_finish)
  const bool hf_lp = lone && n_sets && n_sets <= ctx->lp_hf_max && ctx->lp_hash_finish;
  uint32_t* d_hf_in = hf_lp ? ws.take<uint32_t>((size_t)ns * 12 * 16) : nullptr;
  uint32_t* d_hf_out = hf_lp ? ws.take<uint32_t>((size_t)ns * 6 * 16) : nullptr;
  if (hf_lp) LB_TRY(lp_ensure(ctx));
  // ... and, up to LB_LP_LINES_MAX sets of the steps organisation, its lines (k_lines_prep /
  // k_lp_lines / k_lines_store; LB_LP_LINES=0: k_lines_rows)
  const bool lines_lp = steps && lone && n_sets <= ctx->lp_lines_max && ctx->lp_lines;
  uint32_t* d_ll_in = lines_lp ? ws.take<uint32_t>((size_t)ns * 9 * 16) : nullptr;
  uint32_t* d_ll_out = lines_lp ? ws.take<uint32_t>((size_t)ns * LB_LP_LINES_NOUT * 16) : nullptr;
  if (lines_lp) LB_TRY(lp_ensure(ctx));
  fp12* d_Pl = steps ? ws.take<fp12>(63) : nullptr;
  // the level products' two stages (k_level_part's partials, the first k_level_wc pass's output)
  const bool level_wc = steps && merged && ctx->level_wc;
  const uint32_t lvl_per = level_wc ? level_blocks(n_sets * lsplit, n_req, lone) * 256u : 0u;
  fp12* d_lvA = level_wc ? ws.take<fp12>(63 * (size_t)lvl_per) : nullptr;
  fp12* d_lvB = level_wc ? ws.take<fp12>(63 * (size_t)((lvl_per + LB_LVL_GROUP - 1) / LB_LVL_GROUP)) : nullptr;
  uint8_t* d_lhA = level_wc ? ws.take<uint8_t>(63 * (size_t)lvl_per) : nullptr;
  uint8_t* d_lhB = level_wc ? ws.take<uint8_t>(63 * (size_t)lvl_per) : nullptr;
  uint32_t* d_mt_in = mtail ? ws.take<uint32_t>((size_t)LB_MTAIL_NIN * 16) : nullptr;
  uint32_t* d_mt_out = mtail && partial ? ws.take<uint32_t>(12 * 16) : nullptr;
  uint32_t* d_mb_in0 = bits_lp ? ws.take<uint32_t>((size_t)LB_MSM_BITS_INST * LB_MSM_BITS_GROUP * 6 * 16) : nullptr;
  uint32_t* d_mb_in1 = bits_lp ? ws.take<uint32_t>((size_t)LB_MSM_BITS_INST * 6 * 16) : nullptr;
  uint32_t* d_mb_in2 = bits_lp ? ws.take<uint32_t>((size_t)LB_MSM_BITS_INST / 8 * 6 * 16) : nullptr;
  const Rows rows{d_rowoff, d_rinv, d_rpos, d_rmeta, lsplit};
  sl.h_stats[0] = sl.h_stats[1] = 0;
  if (ws.off > ws.cap) {
    ctx->err = "workspace overflow";
    return LB_ERR_OUT_OF_MEMORY;
  }
  LB_TRY(stream_wait(ctx, sl, 0, 1, 0));
  if (n_sets) {
    if (hf_lp && n_sets <= ctx->lp_hash_full) {  // (the whole curve part as one program per set, k_lp_hash)
      LB_STAGE("hash_finish", 1, k_hu_prep, blocks_for(n_sets, 256), 256u, n_sets, d_msgs, d_hf_in);
      LB_STAGE("hash_finish", 1, k_lp_hash, n_sets, LB_LP_NARROW_ROWS * 16u,
               ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_HASH_FULL].off, n_sets, (const uint32_t*)d_hf_in, d_hf_out);
      LB_STAGE("hash_finish", 1, k_hf_finish, blocks_for(n_sets * 6u, 256), 256u, n_sets, (const uint32_t*)d_hf_out,
               d_h);
    } else {
      LB_STAGE("hash_half", 1, k_hash_half, blocks_for(2 * n_sets), TPB, n_sets, d_msgs, d_q);
      if (hf_lp) {  // (a lone mid-size call: clear_cofactor(Q0 + Q1) as round programs, k_lp_hf)
        LB_STAGE("hash_finish", 1, k_hf_prep, blocks_for(n_sets * 12u, 256), 256u, n_sets, (const g2j*)d_q, d_hf_in);
        const bool nar = ctx->lp_narrow & 1u;
        LB_STAGE("hash_finish", 1, k_lp_hf, n_sets, (nar ? LB_LP_NARROW_ROWS : LB_LP_HF_ROWS) * 16u,
                 ctx->d_lp + LB_LP_PROGS[nar ? LB_LP_PROG_HASH_FINISH_NARROW : LB_LP_PROG_HASH_FINISH].off, n_sets,
                 (const uint32_t*)d_hf_in, d_hf_out);
        LB_STAGE("hash_finish", 1, k_hf_finish, blocks_for(n_sets * 6u, 256), 256u, n_sets, (const uint32_t*)d_hf_out,
                 d_h);
      } else {
        LB_STAGE("hash_finish", 1, k_hash_finish, blocks_for(n_sets), TPB, n_sets, d_q, d_h);
      }
    }
  }
  LB_STAGE("req_flags", 0, k_req_flags, blocks_for(n_req), TPB, n_req, d_req_off, d_single);
  if (steps) {  // size-descending order and row offsets (before stream 1's lines)
    uint32_t* d_rcur = d_rhist + (ns + 1);
    LB_HIP(hipMemsetAsync(d_rhist, 0, 2 * ((size_t)ns + 1) * sizeof(uint32_t), sl.st[0]));
    hipLaunchKernelGGL(k_rows_hist, dim3(blocks_for(n_req, 256)), dim3(256), 0, sl.st[0], n_req, d_req_off, d_rhist);
    LB_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_rows_scan, dim3(1), dim3(1024), 0, sl.st[0], n_sets, (const uint32_t*)d_rhist, d_rgt, d_rowoff,
                       d_rmeta);
    LB_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_rows_pos, dim3(blocks_for(n_req, 256)), dim3(256), 0, sl.st[0], n_req, d_req_off,
                       (const uint32_t*)d_rgt, d_rcur, d_rpos, d_rinv);
    LB_HIP(hipGetLastError());
  }
  if (n_sets) {
    const PkSource src{d_pks, d_pk_idx, ctx->d_table, ctx->table_n};
    LB_STAGE("pubkeys", 0, k_pubkeys_single, blocks_for(n_sets), TPB, n_sets, src, d_pk_off, d_pk, d_pk_st);
    if (d_pk_off)
      // one wave per set, grid-stride: enough waves that every aggregate of a
      // C4/C5-sized call (thousands of committee sets) gets its own
      LB_STAGE("pubkeys_agg", 0, k_pubkeys_agg, n_sets < 16384u ? n_sets : 16384u, TPB, n_sets, src, d_pk_off, d_pk,
               d_pk_st);
    LB_STAGE("scalar_pk", 0, k_scalar_pk, blocks_for(n_sets), TPB, n_sets, d_seed, (const g1j*)d_pk,
             (const uint8_t*)d_single, d_pk_st, d_rpk);
  }
  LB_TRY(stream_wait(ctx, sl, 0, 1, 1));
  if (steps && lines_lp) {
    // (a lone mid-size call: each slot's 68 lines as a round program, k_lp_lines)
    LB_STAGE("lines", 1, k_lines_prep, blocks_for(n_sets * 9u, 256), 256u, n_sets, rows, d_req_off, (const g1j*)d_rpk,
             (const g2j*)d_h, d_ll_in);
    LB_STAGE("lines", 1, k_lp_lines, n_sets, LB_LP_HF_ROWS * 16u, ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_LINES].off, n_sets,
             (const uint32_t*)d_ll_in, d_ll_out);
    LB_STAGE("lines", 1, k_lines_store, (uint32_t)(((size_t)n_sets * LB_MILLER_LINES * 72 + 255) / 256), 256u, n_sets,
             n_pairs, (const uint32_t*)d_ll_out, d_lines);
  } else if (steps) {
    if (ctx->lines_waves == 1)
      LB_STAGE("lines", 1, k_lines_rows<1>, blocks_for(n_sets), TPB, n_sets, n_pairs, rows, d_req_off,
               (const g1j*)d_rpk, d_h, d_lines);
    else
      LB_STAGE("lines", 1, k_lines_rows<2>, blocks_for(n_sets), TPB, n_sets, n_pairs, rows, d_req_off,
               (const g1j*)d_rpk, d_h, d_lines);
  } else if (n_sets && (by_lines || by_wave)) {
    // (small calls are latency-bound: the spill-free one-wave build unless LB_LINES_WAVES=2)
    if (ctx->lines_waves_small == 1)
      LB_STAGE("lines", 1, k_lines<1>, blocks_for(n_sets), TPB, n_sets, n_pairs, 0u, (const g1j*)d_rpk,
               (const g2j*)d_h, d_lines);
    else
      LB_STAGE("lines", 1, k_lines<2>, blocks_for(n_sets), TPB, n_sets, n_pairs, 0u, (const g1j*)d_rpk,
               (const g2j*)d_h, d_lines);
  }
  if (n_sets && by_wave)
    LB_STAGE("miller_wave", 1, k_pair_wc, n_sets, TPB, n_sets, n_pairs, (const uint32_t*)d_lines, d_f);
  else if (n_sets && !by_lines)
    LB_STAGE("miller_sets", 1, k_miller_sets, blocks_for(n_sets), TPB, n_sets, (const g1j*)d_rpk, (const g2j*)d_h,
             d_f);
  if (n_sets) {
    if (!d_sig_pre && dec_lp) {
      // (a lone mid-size call: the signatures' decode as round programs, k_lp_dec -- its one-lane
      // chain is ~5.7 ms whatever the count below the GPU's width)
      LB_STAGE("decode_sigs", 0, k_sm_dec_prep, blocks_for(n_sets, 256), 256u, n_sets, d_sigs, d_sig_off, d_dec_in,
               d_dec_fl, d_dec_pre);
      LB_STAGE("decode_sigs", 0, k_lp_dec, n_sets, LB_LP_DEC_ROWS * 16u,
               ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_SIG_DECODE].off, n_sets, (const uint32_t*)d_dec_in,
               (const uint32_t*)d_dec_fl, d_dec_out, d_dec_ofl);
      LB_STAGE("decode_sigs", 0, k_sm_dec_finish, blocks_for(n_sets, 256), 256u, n_sets, (const uint8_t*)d_dec_pre,
               (const uint32_t*)d_dec_in, (const uint32_t*)d_dec_fl, (const uint32_t*)d_dec_out,
               (const uint32_t*)d_dec_ofl, d_sig, d_sig_st, (const uint8_t*)d_single);
    } else if (!d_sig_pre) {
      LB_STAGE("decode_sigs", 0, k_decode_sigs, blocks_for(n_sets), TPB, n_sets, d_sigs, d_sig_off,
               (const uint8_t*)d_single, d_sig, d_sig_st);
    }
    if (!use_msm)
      LB_STAGE("scalar_sig", 0, k_scalar_sig, blocks_for(n_sets), TPB, n_sets, d_seed, (const g2j*)d_sig,
               (const uint8_t*)d_sig_st, d_rsig, (const uint8_t*)nullptr);
  }
  if (steps)  // request status (k_miller_acc's side reduction in the pairs organisation)
    LB_STAGE("req_status", 0, k_req_status, n_req < 4096u ? n_req : 4096u, TPB, n_req, d_req_off,
             (const uint8_t*)d_sig_st, (const uint8_t*)d_pk_st, d_bad, d_req_err);
  if (use_msm) {
    // S_all = sum r_i sig_i over the good requests' sets: one bucket MSM (k_msm.hip)
    uint32_t* d_off = d_mhist + (LB_MSM_BUCKETS + 1);
    uint32_t* d_coff = d_off + (LB_MSM_BUCKETS + 1);
    uint32_t* d_cur = d_coff + (LB_MSM_BUCKETS + 1);
    LB_HIP(hipMemsetAsync(d_mhist, 0, (LB_MSM_BUCKETS + 1) * sizeof(uint32_t), sl.st[0]));
    LB_STAGE("msm_digits", 0, k_msm_scalars, n_req, TPB, n_req, d_req_off, d_seed, (const uint64_t*)nullptr,
             (const g2j*)d_sig, (const uint8_t*)d_sig_st, (const uint8_t*)d_pk_st, d_mkeys, d_mhist);
    hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(1024), 0, sl.st[0], (const uint32_t*)d_mhist, d_off, d_coff, d_cur,
                       msm_T);
    LB_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_msm_scatter, dim3(blocks_for((uint32_t)n_ent, 256)), dim3(256), 0, sl.st[0], (uint32_t)n_ent,
                       (const uint32_t*)d_mkeys, (const uint32_t*)d_off, d_cur, d_msorted);
    LB_HIP(hipGetLastError());
    LB_STAGE("msm_chunks", 0, k_msm_chunks, blocks_for((uint32_t)max_chunks), TPB, (uint32_t)max_chunks,
             (const uint32_t*)d_off, (const uint32_t*)d_coff, (const uint32_t*)d_msorted, (const g2j*)d_sig, d_mcsum,
             msm_T);
    const uint32_t bl = msm_wide ? LB_MSM_BLANES : 1u;
    LB_STAGE("msm_buckets", 0, k_msm_buckets, blocks_for(LB_MSM_BUCKETS * bl), TPB, (const uint32_t*)d_coff,
             (const g2j*)d_mcsum, d_mbsum, bl);
    if (bits_lp) {
      // (a lone call's bit sums as three levels of round programs, 8:1 each; the last writes the
      // 33 G_p into the merged-check program's input records, so k_mtail_prep skips them)
      LB_STAGE("msm_bits", 0, k_msm_bits_prep, blocks_for(LB_MSM_BITS_INST * LB_MSM_BITS_GROUP * 6u, 256), 256u,
               (const g2j*)d_mbsum, d_mb_in0);
      constexpr uint32_t NI = LB_MSM_BITS_GROUP * 6u;
      LB_STAGE("msm_bits", 0, k_lp_msm_bits, LB_MSM_BITS_INST, LB_LP_TPB, ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_MSM_BITS0].off,
               (uint32_t)LB_MSM_BITS_INST, NI, 6u, (const uint32_t*)d_mb_in0, d_mb_in1);
      LB_STAGE("msm_bits", 0, k_lp_msm_bits, LB_MSM_BITS_INST / 8u, LB_LP_TPB,
               ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_MSM_BITS1].off, (uint32_t)LB_MSM_BITS_INST / 8u, NI, 6u,
               (const uint32_t*)d_mb_in1, d_mb_in2);
      LB_STAGE("msm_bits", 0, k_lp_msm_bits, LB_MSM_POS, LB_LP_TPB, ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_MSM_BITS2].off,
               (uint32_t)LB_MSM_POS, NI, 6u, (const uint32_t*)d_mb_in2, d_mt_in + (size_t)12 * LB_MTAIL_LEVELS * 16);
    } else {
      if (msm_wide)
        LB_STAGE("msm_bits", 0, k_msm_bits<LB_MSM_BITS_TPB>, LB_MSM_POS, LB_MSM_BITS_TPB, (const g2j*)d_mbsum, d_mG);
      else
        LB_STAGE("msm_bits", 0, k_msm_bits<TPB>, LB_MSM_POS, TPB, (const g2j*)d_mbsum, d_mG);
    }
    if (!mtail) LB_STAGE("msm_final", 0, k_msm_final, 1u, TPB, (const g2j*)d_mG, d_Sall);
    if (!fold && !mtail)
      LB_STAGE("lines_all", 0, k_lines_S, 1u, TPB, 1u, n_pairs, n_sets + n_req, (const g2a*)d_Sall, d_lines,
               (const uint8_t*)nullptr);
  } else {
    LB_STAGE("sum_tree", 0, k_sum_tree, n_req, TPB, n_req, d_req_off, (const g2j*)d_rsig, d_S, (const uint8_t*)nullptr);
    if (steps && merged) {  // S_all of the good requests and its lines, ahead of the level products
      LB_STAGE("merge", 0, k_merge, 1u, TPB, n_req, (const g2a*)d_S, (const fp12*)nullptr, (const uint8_t*)d_bad, d_Sall,
               (fp12*)nullptr, (const fp12*)nullptr);
      LB_STAGE("lines_all", 0, k_lines_S, 1u, TPB, 1u, n_pairs, n_sets + n_req, (const g2a*)d_Sall, d_lines,
               (const uint8_t*)nullptr);
    }
  }
  if (tail_wave && !merged)
    LB_STAGE("lines_S", 0, k_lines_S, blocks_for(n_req), TPB, n_req, n_pairs, n_sets, (const g2a*)d_S, d_lines,
             (const uint8_t*)nullptr);
  else if (!tail_wave)
    LB_STAGE("miller_S", 0, k_miller_S, blocks_for(n_req), TPB, n_req, (const g2a*)d_S, d_fS);
  const fp12* fS_in = tail_wave ? nullptr : (const fp12*)d_fS;
  LB_TRY(stream_wait(ctx, sl, 1, 0, 2));
  fp12* d_Fx = fold ? ws.take<fp12>(1) : nullptr;
  if (ws.off > ws.cap) {
    ctx->err = "workspace overflow";
    return LB_ERR_OUT_OF_MEMORY;
  }
  if (steps) {
#define LB_STEP_STAGE(M, W)                                                                               \
  LB_STAGE("step_acc", 0, (k_step_acc<M, W>), blocks_for(n_sets * lsplit), TPB, n_sets, n_pairs, rows, d_req_off, \
           (const uint32_t*)d_lines, d_G)
    if (ctx->step_mode == 1)
      LB_STEP_STAGE(1, 1);
    else if (ctx->step_mode == 2 && ctx->step_waves == 2)
      LB_STEP_STAGE(2, 2);
    else if (ctx->step_mode == 2)
      LB_STEP_STAGE(2, 1);
    else if (ctx->step_waves == 2)
      LB_STEP_STAGE(0, 2);
    else
      LB_STEP_STAGE(0, 1);
#undef LB_STEP_STAGE
    if (merged) {
      // (mtail: the merged pair's Miller value comes from the round program, not as lines)
      const uint32_t s_pair = mtail ? 0xffffffffu : n_sets + n_req;
      if (level_wc) {
        const dim3 g_part(lvl_per / 256u, 63);
        LB_STAGE("level_prod", 0, k_level_part, g_part, 256u, n_req, n_sets, rows, d_req_off, (const uint32_t*)d_G,
                 (const uint8_t*)d_bad, lvl_per, d_lvA, d_lhA);
        uint32_t pin = lvl_per;
        fp12 *src = d_lvA, *dst = d_lvB;
        uint8_t *sh = d_lhA, *dh = d_lhB;
        for (;;) {
          const uint32_t pout = (pin + LB_LVL_GROUP - 1) / LB_LVL_GROUP;
          const dim3 g_wc(pout, 63);
          LB_STAGE("level_wc", 0, k_level_wc, g_wc, TPB, pin, (const fp12*)src, (const uint8_t*)sh, pout, dst, dh,
                   n_pairs, s_pair, (const uint32_t*)d_lines, pout == 1 ? d_Pl : (fp12*)nullptr);
          if (pout == 1) break;
          pin = pout;
          std::swap(src, dst);
          std::swap(sh, dh);
        }
      } else {
        LB_STAGE("level_prod", 0, k_level_prod, 63u, 256u, n_req, n_sets, n_pairs, s_pair, rows, d_req_off,
                 (const uint32_t*)d_G, (const uint8_t*)d_bad, (const uint32_t*)d_lines, d_Pl);
      }
      // (mtail: the round program runs the Horner chain over the level products itself, on the
      // Miller loop's squarings of (-g1, S_all): no one-wave k_horner_all)
      if (!mtail) LB_STAGE("horner_all", 0, k_horner_all, 1u, TPB, (const fp12*)d_Pl, d_Fall);
    } else {
      LB_STAGE("req_horner", 0, k_req_horner, n_req * lsplit, TPB, n_req, n_sets, rows, d_req_off,
               (const uint32_t*)d_G, (const uint8_t*)d_bad, lsplit > 1 ? d_Fparts : d_F, (const uint8_t*)nullptr);
      if (lsplit > 1)
        LB_STAGE("req_horner", 0, k_req_join, n_req, TPB, n_req, lsplit, (const fp12*)d_Fparts, (const uint8_t*)d_bad,
                 d_F, (const uint8_t*)nullptr);
    }
  } else if (by_lines) {
    const uint32_t nr = split ? 2 * n_req : n_req;
    const uint32_t* acc_off = d_req_off;
    fp12* acc_F = d_F;
    uint8_t* acc_bad = d_bad;
    uint8_t* acc_err = d_req_err;
    if (split) {
      uint32_t* off2 = ws.take<uint32_t>(2 * (size_t)n_req + 1);
      acc_F = ws.take<fp12>(2 * (size_t)n_req);
      acc_bad = ws.take<uint8_t>(2 * (size_t)n_req);
      acc_err = ws.take<uint8_t>(2 * (size_t)n_req);
      if (ws.off > ws.cap) {
        ctx->err = "workspace overflow";
        return LB_ERR_OUT_OF_MEMORY;
      }
      hipLaunchKernelGGL(k_split_requests, dim3(blocks_for(n_req + 1)), dim3(TPB), 0, sl.st[0], n_req, d_req_off, off2);
      LB_HIP(hipGetLastError());
      acc_off = off2;
    }
    const uint32_t rpw = TPB / ctx->acc_lpr, grid = (nr + rpw - 1) / rpw + (fold ? 1u : 0u);
    const fp12* acc_fS = split ? nullptr : fS_in;
    const uint32_t halves = split ? 1u : 0u;
#define LB_ACC_STAGE(L)                                                                                       \
  LB_STAGE("miller_acc", 0, k_miller_acc<L>, grid, TPB, nr, acc_off, n_pairs, (const uint32_t*)d_lines, acc_fS, \
           (const uint8_t*)d_sig_st, (const uint8_t*)d_pk_st, acc_F, acc_bad, acc_err, halves,               \
           fold ? (const g2a*)d_Sall : (const g2a*)nullptr, d_Fx)
    if (ctx->acc_lpr == 16)
      LB_ACC_STAGE(16);
    else if (ctx->acc_lpr == 32)
      LB_ACC_STAGE(32);
    else
      LB_ACC_STAGE(64);
#undef LB_ACC_STAGE
    if (split)
      LB_STAGE("join_halves", 0, k_join_halves, blocks_for(n_req), TPB, n_req, d_req_off, (const fp12*)acc_F,
               (const uint8_t*)acc_bad, (const uint8_t*)acc_err, fS_in, d_F, d_bad, d_req_err);
  } else
    LB_STAGE("prod_tree", 0, k_prod_tree, n_req, TPB, n_req, d_req_off, (const fp12*)d_f, fS_in,
             (const uint8_t*)d_sig_st, (const uint8_t*)d_pk_st, d_F, d_bad, d_req_err);
  PipeState& ps = sl.ps;
  ps.n_req = n_req;
  ps.n_sets = n_sets;
  ps.n_pairs = n_pairs;
  ps.merged = merged;
  ps.tail_wave = tail_wave;
  ps.msm = use_msm;
  ps.d_seed = d_seed;
  ps.d_sig = d_sig;
  ps.d_sig_st = d_sig_st;
  ps.d_rsig = d_rsig;
  ps.d_req_off = d_req_off;
  ps.d_lines = d_lines;
  ps.d_S = d_S;
  ps.d_F = d_F;
  ps.d_rt_in = d_rt_in;
  ps.d_rt_fl = d_rt_fl;
  ps.d_bad = d_bad;
  ps.d_valid = d_valid;
  ps.d_mflag = d_mflag;
  ps.d_mstats = d_mstats;
  ps.steps = steps;
  ps.rows = rows;
  ps.d_G = d_G;
  ps.d_Fparts = d_Fparts;
  if (merged) {
    // merged check: one tail for the whole call; per-request tails only if it fails.
    // LB_TAIL_PRIO=1 runs its chain of one-wave kernels on a shared high-priority
    // stream instead of the slot's own (measured slower, off by default).
    hipStream_t ts = sl.st[0];
    if (ctx->tail_stream) {
      ts = ctx->tail_stream;
      LB_HIP(hipEventRecord(sl.dep[3], sl.st[0]));
      LB_HIP(hipStreamWaitEvent(ts, sl.dep[3], 0));
    }
    LB_HIP(hipMemsetAsync(d_mflag, 0, 2, ts));
    if (!steps) {  // (steps: F_all from the level products and the Horner chain, S_all's lines included)
      LB_STAGE_ON("merge", ts, k_merge, 1u, TPB, n_req, use_msm ? (const g2a*)nullptr : (const g2a*)d_S,
                  (const fp12*)d_F, (const uint8_t*)d_bad,
                  d_Sall, d_Fall, (const fp12*)d_Fx);
      if (!use_msm)  // (with the MSM: folded into k_miller_acc, or stored right after the MSM)
        LB_STAGE_ON("lines_all", ts, k_lines_S, 1u, TPB, 1u, n_pairs, n_sets + n_req, (const g2a*)d_Sall, d_lines,
                    (const uint8_t*)nullptr);
    }
    const uint32_t* merged_lines = (fold || steps) ? nullptr : (const uint32_t*)d_lines;
    if (mtail) {
      hipLaunchKernelGGL(k_mtail_prep, dim3(1), dim3(256), 0, ts, (const fp12*)d_Pl,
                         bits_lp ? (const g2j*)nullptr : (const g2j*)d_mG, d_mt_in);
      LB_HIP(hipGetLastError());
      if (partial) {  // F_all * Miller(-g1, S_all) back into d_Fall, encoded by k_partial below
        LB_STAGE_ON("mtail", ts, k_lp_mtail, 1u, mt_tpb, ctx->d_lp + LB_LP_PROGS[mt_wide ? LB_LP_PROG_MTAIL_PARTIAL_WIDE : LB_LP_PROG_MTAIL_PARTIAL].off,
                    (const uint32_t*)d_mt_in, (uint8_t*)nullptr, d_mt_out);
        hipLaunchKernelGGL(k_records_to_fp12, dim3(1), dim3(64), 0, ts, (const uint32_t*)d_mt_out, d_Fall);
        LB_HIP(hipGetLastError());
      }
    }
    if (partial) {
      // two-phase call: the merged Miller product goes to the host, which
      // combines it with the other GPUs' partials; the tails wait for its verdict
      LB_STAGE_ON("partial", ts, k_partial, 1u, TPB, n_pairs, n_sets + n_req, merged_lines,
                  (const fp12*)d_Fall, d_partial);
      LB_HIP(hipMemcpyAsync(sl.h_partial, d_partial, LB_GT_BYTES, hipMemcpyDeviceToHost, ts));
      LB_HIP(hipEventRecord(sl.partial_ev, ts));
      if (ts != sl.st[0]) {
        LB_HIP(hipEventRecord(sl.dep[4], ts));
        LB_HIP(hipStreamWaitEvent(sl.st[0], sl.dep[4], 0));
      }
      if (ctx->tp_release) {
        // the call completes on its own as if the combined check passed (every request not
        // already false valid: no per-request work) and frees its slot at once; a failed
        // combined check re-verifies the shard as a one-phase call (lb_verify_requests_finish)
        LB_HIP(hipMemsetAsync(d_mflag, 1, 1, sl.st[0]));
        return run_tails(ctx, sl);
      }
      sl.partial_pending = true;
      return LB_OK;
    }
    if (mtail)
      LB_STAGE_ON("mtail", ts, k_lp_mtail, 1u, mt_tpb, ctx->d_lp + LB_LP_PROGS[mt_wide ? LB_LP_PROG_MTAIL_CHECK_WIDE : LB_LP_PROG_MTAIL_CHECK].off,
                  (const uint32_t*)d_mt_in, d_mflag, (uint32_t*)nullptr);
    else
      LB_STAGE_ON("tail_all", ts, k_tail, 1u, TPB, 1u, n_pairs, n_sets + n_req, merged_lines,
                  (const fp12*)d_Fall, (const uint8_t*)(d_mflag + 1), d_mflag, (const uint8_t*)nullptr);
    if (ts != sl.st[0]) {
      LB_HIP(hipEventRecord(sl.dep[4], ts));
      LB_HIP(hipStreamWaitEvent(sl.st[0], sl.dep[4], 0));
    }
  }
  return run_tails(ctx, sl);
}

// lanes per set of a lone call's step-major accumulation: 4 up to 16,384 sets, 2 up to 32,768 (the
// call's lanes then fill at most one wave per SIMD), 1 above (profiles/r06/level_probe_r06x.json:
// 4,096 ... 16,384 sets 16.7-17.4 ms unsplit, 14.1-15.0 split in 4)
static uint32_t step_split_for(uint32_t n_sets) { return n_sets <= 16384u ? 4u : n_sets <= 32768u ? 2u : 1u; }

// k_level_part's workgroups per level: one request per thread (a merged call's requests are
// mostly small), and about two lanes per thread when one large request holds the call
static uint32_t level_blocks(uint32_t n_sets, uint32_t n_req, bool wide) {
  // (wide, a lone call: about one lane per thread -- the products all in the wave-cooperative
  // passes, the fastest for the call; otherwise about two, one lane product each: less work)
  const uint32_t w = wide ? (4 * n_req > n_sets / 32u ? 4 * n_req : n_sets / 32u)
                          : (n_req > n_sets / 126u ? n_req : n_sets / 126u);
  const uint32_t b = (w + 255u) / 256u;
  return b < 1u ? 1u : b > 8u ? 8u : b;
}

size_t pipeline_ws_bytes(const lb_ctx* ctx, uint32_t n_req, uint32_t n_sets) {
  size_t ns = n_sets ? n_sets : 1;
  // (+ the bucket MSM: 2 W keys + 2 W sorted entries and 2 W / T chunk partials per set)
  // (+ the steps organisation: size histogram / cursors / gt / row offsets and the lanes' G values)
  size_t per_set = sizeof(g2j) * 5 + sizeof(g1j) * 2 + sizeof(fp12) + 3 + 16 * 256 / 64 + 16 + 576 +
                   (size_t)LB_MILLER_LINES * 72 * 4 + 4 * LB_MSM_W * 4 +
                   (2 * LB_MSM_W * sizeof(g2j)) / (ns <= ctx->msm_short_max ? ctx->msm_t_lone : LB_MSM_T) + 1;
  // (+ the halves of a split Miller accumulation: 2 fp12, 2 flags, 2 offsets)
  size_t per_req = sizeof(g2a) + 8 * sizeof(fp12) + 1 + 4 + 8 + 8 + 4 * 256 / 64 + (size_t)LB_MILLER_LINES * 72 * 4 +
                   (size_t)LB_RTAIL_NIN * 64 + 4 + 2 * 256 / 64;  // (+ k_lp_rtail's records and flag)
  // (+ a lone call's bit-sum program records: 8 + 1 + 1/8 points of 6 records per level-0 instance)
  const size_t msm_fixed = (size_t)(2 * LB_MSM_BUCKETS + LB_MSM_POS) * sizeof(g2j) + 4 * (LB_MSM_BUCKETS + 1) * 4 +
                           8 * 256 + (size_t)LB_MSM_BITS_INST * (LB_MSM_BITS_GROUP + 1 + 1) * 6 * 64 + 3 * 256;
  // (+ the merged check's round-program records, k_lp_mtail)
  // (+ the level products' partials: 63 x 256 B of k_level_part, an eighth of that for the
  // first k_level_wc pass, their flags)
  // (+ the G values of a split accumulation, up to 4 lanes per set: LB_STEP_SPLIT may force 4 at
  // any size -- 3 more G per set, and 4x the lanes for the level partials)
  const size_t lvl_per = (size_t)level_blocks(n_sets * 4u, n_req, true) * 256;
  const size_t lvl = 63 * (lvl_per + (lvl_per + LB_LVL_GROUP - 1) / LB_LVL_GROUP) * sizeof(fp12) + 2 * 63 * lvl_per +
                     4 * 256;
  return ns * per_set + (size_t)(n_req + 1) * per_req + msm_fixed + 64 * sizeof(fp12) + 80 * 256 + 4096 +
         (size_t)(LB_MTAIL_NIN + 12) * 64 + 512 + lvl + ns * 3 * 576 +
         (ns <= std::max(ctx->lp_dec_max, ctx->lp_hf_max) ? ns * (6 * 64 + 5 * 4 + 1 + 18 * 64) + 7 * 256 : 0) +  // (+ a lone call's
                                                                                      // decode / hash records)
         (ns <= ctx->lp_lines_max ? ns * (9 + LB_LP_LINES_NOUT) * 64 + 2 * 256 : 0);  // (+ its line records)
}

int validate_batch(lb_ctx* ctx, const lb_request_batch* b) {
  if (!b || !b->request_offsets || !b->messages || !b->signatures || !b->sig_offsets || !b->seed ||
      (b->n_sets && !b->pubkeys && !b->pubkey_indices)) {
    ctx->err = "null pointer in lb_request_batch";
    return LB_ERR_INVALID_ARGUMENT;
  }
  return LB_OK;
}

// A host <-> device copy of a call on slot sl: on the priority slot a kernel (k_copy_bytes,
// LB_PRIO_KCOPY=0: hipMemcpyAsync), never queued on an SDMA engine behind the throughput
// calls' staging; elsewhere hipMemcpyAsync.  Host buffers are pinned (hipHostMalloc).
int slot_copy(lb_ctx* ctx, Slot& sl, void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t st) {
  if (!n) return LB_OK;
  if (ctx->prio_kcopy && &sl == &ctx->prio() && n < (1u << 30)) {
    const size_t blocks = (n / 16 + 255) / 256;
    hipLaunchKernelGGL(k_copy_bytes, dim3(blocks < 1 ? 1 : blocks > 512 ? 512 : (unsigned)blocks), dim3(256), 0, st,
                       (const uint8_t*)src, (uint8_t*)dst, (uint32_t)n);
    LB_HIP(hipGetLastError());
    return LB_OK;
  }
  LB_HIP(hipMemcpyAsync(dst, src, n, kind, st));
  return LB_OK;
}

// Copy a host-buffer call's verdicts from the device into its pinned staging
// (enqueued after the tails; the caller's buffers are filled in finish_slot).
int enqueue_host_out(lb_ctx* ctx, Slot& sl) {
  if (!sl.out_valid) return LB_OK;
  const size_t a = (sl.out_nr + 255) & ~(size_t)255;
  LB_TRY(slot_copy(ctx, sl, sl.h_out, sl.dv_valid, sl.out_nr, hipMemcpyDeviceToHost, sl.st[0]));
  LB_TRY(slot_copy(ctx, sl, sl.h_out + a, sl.dv_err, sl.out_nr, hipMemcpyDeviceToHost, sl.st[0]));
  if (sl.out_ns) LB_TRY(slot_copy(ctx, sl, sl.h_out + 2 * a, sl.dv_sst, sl.out_ns, hipMemcpyDeviceToHost, sl.st[0]));
  return LB_OK;
}

int end_call(lb_ctx* ctx, Slot& sl) {
  LB_TRY(enqueue_host_out(ctx, sl));
  LB_HIP(hipEventRecord(sl.wall1, sl.st[0]));
  LB_HIP(hipEventRecord(sl.done, sl.st[0]));
  return LB_OK;
}

// Second phase of a two-phase call: the host's combined verdict (merged_ok)
// decides whether the per-request tails run (k_lines_S / k_tail skip
// themselves when d_mflag[0] != 0).
int finish_partial(lb_ctx* ctx, Slot& sl, bool merged_ok) {
  if (!sl.partial_pending) return LB_OK;
  sl.partial_pending = false;
  if (sl.ps.n_req) {  // (an empty call has no tails)
    LB_HIP(hipMemsetAsync(sl.ps.d_mflag, merged_ok ? 1 : 0, 1, sl.st[0]));
    LB_TRY(run_tails(ctx, sl));
  }
  return end_call(ctx, sl);
}

// Wait for a slot's outstanding call and publish its stage times, stats and
// (host-buffer calls) verdicts.  A two-phase call whose host verdict never came
// runs its per-request tails (merged_ok = 0: every verdict computed alone).
int sm_advance(lb_ctx* ctx, Slot& sl, bool block);
int sm_pump(lb_ctx* ctx);

void release_borrowed(Slot& sl) {  // hand a borrowed stream back
  if (!sl.borrowed) return;
  sl.borrowed->busy = false;
  sl.borrowed->lent_to = nullptr;
  sl.st[1] = sl.st[0];
  sl.borrowed = nullptr;
}

int finish_slot(lb_ctx* ctx, Slot& sl) {
  if (sl.lent_to) return finish_slot(ctx, *sl.lent_to);  // releases this slot
  if (!sl.busy) {
    release_borrowed(sl);  // (a submission that failed after borrowing)
    return LB_OK;
  }
  LB_TRY(finish_partial(ctx, sl, false));
  while (sl.sm.active && sm_advance(ctx, sl, true) == LB_OK) {
  }  // same-message: phases 1 and 2
  if (sl.sm.err) {  // its phase 2 failed to launch (here or in another call's sm_pump)
    const int rc = sl.sm.err;
    ctx->err = sl.sm.err_msg;
    sl.sm.err = 0;
    for (int i = 0; i < 2; i++) (void)hipStreamSynchronize(sl.st[i]);
    release_borrowed(sl);
    sl.busy = false;
    return rc;
  }
  LB_HIP(hipEventSynchronize(sl.done));
  ctx->n_stages = sl.n_stages;
  for (int i = 0; i < sl.n_stages; i++) {
    float ms = 0.f;
    LB_HIP(hipEventElapsedTime(&ms, sl.ev0[i], sl.ev1[i]));
    ctx->stage_ms[i] = ms;
    ctx->stage_name[i] = sl.stage_name[i];
    ctx->stage_ops[i] = sl.stage_ops[i];
  }
  LB_HIP(hipEventElapsedTime(&ctx->wall_ms, sl.wall0, sl.wall1));
  ctx->batch_retries = sl.h_stats[0];
  ctx->batch_sigs_success = sl.h_stats[1];
  if (sl.lp_call)
    for (int i = 0; i < 4; i++) ctx->lp_clk[i] = sl.h_clk[i];
  {  // a released two-phase call: its partial outlives the slot
    TwoPhaseRec& r = ctx->tp[sl.ticket % lb_ctx::kTwoPhaseRing];
    if (sl.ticket && r.ticket == sl.ticket && !r.have_partial) {
      memcpy(r.partial, sl.h_partial, LB_GT_BYTES);
      r.have_partial = true;
    }
  }
  TicketStats& ts = ctx->tstats[sl.ticket % lb_ctx::kTicketRing];
  ts.ticket = sl.ticket;
  ts.batch_retries = sl.h_stats[0];
  ts.batch_sigs_success = sl.h_stats[1];
  ts.wall_ms = ctx->wall_ms;
  if (sl.out_valid) {
    const size_t a = (sl.out_nr + 255) & ~(size_t)255;
    memcpy(sl.out_valid, sl.h_out, sl.out_nr);
    memcpy(sl.out_err, sl.h_out + a, sl.out_nr);
    if (sl.out_sst && sl.out_ns) memcpy(sl.out_sst, sl.h_out + 2 * a, sl.out_ns);
    sl.out_valid = sl.out_err = sl.out_sst = nullptr;
  }
  release_borrowed(sl);
  sl.busy = false;
  return LB_OK;
}

// An async call on slot `sl` (single stream, just retired) while no other call is
// in flight: the lowest latency is the two-stream DAG (hash_to_G2 + lines beside
// the signature / MSM branch), so it borrows an idle slot's stream; the next call
// that wants that slot waits for this one first (finish_slot).
void borrow_idle_stream(lb_ctx* ctx, Slot& sl) {
  if (!ctx->dag || sl.st[1] != sl.st[0] || sl.borrowed || &sl == &ctx->prio()) return;
  Slot* idle = nullptr;
  for (int s = 0; s < ctx->n_slots; s++) {
    Slot& o = ctx->slots[s];
    if (&o == &sl) continue;
    if (o.busy || o.partial_pending) return;  // not alone on the GPU
    if (!idle && o.st[0] != sl.st[0]) idle = &o;
  }
  if (!idle) return;
  sl.st[1] = idle->st[0];
  sl.borrowed = idle;
  idle->busy = true;
  idle->ticket = 0;
  idle->lent_to = &sl;
}

int begin_call(lb_ctx* ctx, Slot& sl) {
  ctx->last_call_streams = sl.st[1] != sl.st[0] ? 2 : 1;
  sl.lp_call = false;
  sl.n_stages = 0;
  sl.partial_pending = false;
  sl.out_valid = sl.out_err = sl.out_sst = nullptr;
  LB_HIP(hipEventRecord(sl.wall0, sl.st[0]));
  return LB_OK;
}
// Mark the slot busy under a new ticket; a complete call also records its end
// (a two-phase call records it in finish_partial).
int end_call_async(lb_ctx* ctx, Slot& sl) {
  if (!sl.partial_pending) LB_TRY(end_call(ctx, sl));
  sl.busy = true;
  sl.ticket = ctx->next_ticket++;
  if (sl.partial_pending) {
    ctx->two_phase[ctx->two_phase_pos] = sl.ticket;
    ctx->two_phase_pos = (ctx->two_phase_pos + 1) % lb_ctx::kTwoPhaseRing;
  }
  return LB_OK;
}

Slot* slot_of_ticket(lb_ctx* ctx, uint64_t ticket) {
  for (int s = 0; s <= ctx->n_slots; s++)
    if (ctx->slots[s].busy && ctx->slots[s].ticket == ticket) return &ctx->slots[s];
  return nullptr;
}

// Synchronous verify calls run on slot 0 as the two-stream DAG.  When slot 0
// owns a single stream (the default four single-stream slots), the call
// borrows slot 1's stream (after slot 1's call in flight completes) and the
// guard hands it back when the call returns (the call is complete by then).
struct BorrowGuard {
  lb_ctx* ctx;
  bool active = false;
  ~BorrowGuard() {
    if (active) {
      ctx->slots[0].guard_st = nullptr;
      ctx->slots[0].st[1] = ctx->slots[0].st[0];
    }
  }
};
int borrow_second_stream(lb_ctx* ctx, BorrowGuard& g) {
  Slot& s0 = ctx->slots[0];
  if (ctx->dag && ctx->streams_per_slot[0] == 1 && ctx->n_slots >= 2) {
    LB_TRY(finish_slot(ctx, ctx->slots[1]));
    s0.st[1] = s0.guard_st = ctx->slots[1].st[0];
    g.active = true;
  }
  return LB_OK;
}

// Idle slot 0 for the synchronous helper entry points.
int helper_slot(lb_ctx* ctx) {
  for (int i = 0; i <= ctx->n_slots; i++) LB_TRY(finish_slot(ctx, ctx->slots[i]));
  return LB_OK;
}

// latency path: upload the round programs once (2.6 MB)
int lp_ensure(lb_ctx* ctx) {
  if (ctx->d_lp) return LB_OK;
  const size_t bytes = (size_t)LB_LP_BLOB_WORDS * 4;
  if (hipMalloc(&ctx->d_lp, bytes) != hipSuccess) {
    ctx->d_lp = nullptr;
    ctx->err = "hipMalloc latency-path programs failed";
    return LB_ERR_OUT_OF_MEMORY;
  }
  LB_HIP(hipMemcpy(ctx->d_lp, lb_lp_blob, bytes, hipMemcpyHostToDevice));
  return LB_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int lb_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Private-segment (scratch) reservation of one HIP hardware queue.  ROCr backs a
// queue's scratch for a dispatch at full-device occupancy: private bytes per lane
// x 64 lanes x 32 waves per CU x CUs, and keeps it for the queue's lifetime, so a
// process with Q queues that run the pipeline's largest-scratch kernel reserves Q
// times that.  At 24 queues the first 65,536-set calls failed with
// HSA_STATUS_ERROR_OUT_OF_RESOURCES (profiles/ab_r03/r03g_q24_fail.txt) with the
// HBM otherwise free; 16 ran, which is the cap lb_create enforces.
static std::string g_create_err = "null context";

size_t scratch_per_queue(int device, uint32_t* out_lane_bytes) {
  const void* kernels[] = {(const void*)k_miller_acc<16>, (const void*)k_miller_acc<32>,
                           (const void*)k_miller_acc<64>, (const void*)k_step_acc<0, 1>,
                           (const void*)k_step_acc<0, 2>, (const void*)k_step_acc<1, 1>, (const void*)k_step_acc<2, 1>, (const void*)k_step_acc<2, 2>, (const void*)k_lines<1>,
                           (const void*)k_lines<2>, (const void*)k_lines_rows<1>, (const void*)k_lines_rows<2>,
                           (const void*)k_pair_wc, (const void*)k_miller_sets,
                           (const void*)k_hash_half, (const void*)k_hash_finish, (const void*)k_final,
                           (const void*)k_tail, (const void*)k_req_horner, (const void*)k_req_join, (const void*)k_lp_verify,
                           (const void*)k_lp_mtail, (const void*)k_lp_final_lane, (const void*)k_gt_prod,
                           (const void*)k_lp_rtail, (const void*)k_lp_msm_bits, (const void*)k_lp_dec, (const void*)k_lp_hf, (const void*)k_lp_hash, (const void*)k_lp_lines, (const void*)k_level_prod, (const void*)k_level_part,
                           (const void*)k_level_wc,
                           (const void*)k_msm_buckets, (const void*)k_msm_bits<TPB>, (const void*)k_msm_bits<LB_MSM_BITS_TPB>,
                           (const void*)k_decode_sigs,
                           (const void*)k_scalar_pk};
  size_t lane = 0;
  for (const void* k : kernels) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k) == hipSuccess && a.localSizeBytes > lane) lane = a.localSizeBytes;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
  if (out_lane_bytes) *out_lane_bytes = (uint32_t)lane;
  return lane * 64 * 32 * (size_t)cus;
}

// The streams of every live context of this process, by kind: HIP pools the
// plain streams of one priority into at most GPU_MAX_HW_QUEUES queues PER PROCESS, so a
// second context's plain and high-priority streams share the first one's queues (up to
// that cap) while each CU-masked stream takes a queue of its own.  A latency-lane context
// (lb_create_lane, optional: the addon runs without one) is priced on the process total
// against kProcessQueueBudget, the largest process configuration seen to run: bench.py's
// process and the node addon's, 16 plain + 2 CU-masked + 4 high-priority queues (the main
// context's priority lane and aux stream, and the second context's two).
static std::mutex g_q_mu;
static int g_q_plain = 0, g_q_high = 0, g_q_masked = 0;
static constexpr int kProcessQueueBudget = 22;

static int pooled_queues(int plain, int high, int masked, int maxq) {
  return (plain < maxq ? plain : maxq) + (high < maxq ? high : maxq) + masked;
}

static int create_ctx(int device, lb_ctx** out_ctx, bool lane) {
  if (!out_ctx) return LB_ERR_INVALID_ARGUMENT;
  *out_ctx = nullptr;
  const bool lane_ctx = lane;  // (the queue guard's block below has a `lane` of its own: bytes per lane)
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0 || device < 0 || device >= n) return LB_ERR_NO_DEVICE;
  lb_ctx* ctx = new lb_ctx();
  ctx->device = device;
  ctx->lane = lane;
  bool ok = hipSetDevice(device) == hipSuccess;
  // one single-stream slot per hardware queue HIP gives this process (4 by
  // default; a host that sets GPU_MAX_HW_QUEUES=8 before HIP starts gets 8 calls
  // in flight: 2.94 vs 2.74 M sets/s once the merged check's one-wave kernels
  // left each call's queue idle at its end, profiles/ab_r03/hwq; up to 16)
  if (const char* e = getenv("GPU_MAX_HW_QUEUES")) {
    const int v = atoi(e);
    if (v > lb_ctx::kMaxSlots) {
      uint32_t lane = 0;
      const size_t per_q = scratch_per_queue(device, &lane);
      char msg[320];
      snprintf(msg, sizeof msg,
               "GPU_MAX_HW_QUEUES=%d exceeds %d: %u private bytes per lane reserve %.2f GB of scratch per "
               "hardware queue (%.1f GB for %d queues); 24 queues failed with HSA_STATUS_ERROR_OUT_OF_RESOURCES",
               v, lb_ctx::kMaxSlots, lane, per_q / 1e9, per_q * (double)v / 1e9, v);
      g_create_err = msg;
      delete ctx;
      return LB_ERR_RESOURCES;
    }
    ctx->n_slots = v < 4 ? 4 : v;
  }
  if (const char* e = getenv("LB_SLOTS")) {
    const int v = atoi(e);
    if (v >= 1 && v <= lb_ctx::kMaxSlots) ctx->n_slots = v;
  }
  if (lane) ctx->n_slots = 1;  // a latency-lane context: its priority lane (+ one slot for helpers)
  if (const char* e = getenv("LB_MILLER"))
    ctx->miller_mode = strcmp(e, "lane") == 0 ? 1 : strcmp(e, "lines") == 0 ? 2 : strcmp(e, "wave") == 0 ? 3 : 0;
  if (const char* e = getenv("LB_TAIL")) ctx->tail_wave = strcmp(e, "lane") != 0;
  if (const char* e = getenv("LB_MERGE_MIN")) ctx->merge_min_req = (uint32_t)atoi(e);
  if (const char* e = getenv("LB_MSM_MIN")) ctx->msm_min_sets = (uint32_t)atoi(e);
  if (const char* e = getenv("LB_LINES_MIN")) ctx->lines_min_sets = (uint32_t)atoi(e);
  if (const char* e = getenv("LB_LEVEL")) ctx->level_wc = atoi(e) != 0;
  if (const char* e = getenv("LB_MSM_LANES")) ctx->msm_lanes = atoi(e) != 0;
  if (const char* e = getenv("LB_WIDE_TAIL")) ctx->wide_tail = atoi(e) != 0;
  if (const char* e = getenv("LB_MSM_BITS_LP")) ctx->msm_bits_lp = atoi(e) != 0;
  if (const char* e = getenv("LB_SM_LP_DECODE")) ctx->sm_lp_decode = atoi(e) != 0;
  if (const char* e = getenv("LB_LP_DECODE")) ctx->lp_decode = atoi(e) != 0;
  if (const char* e = getenv("LB_LP_HASH_FINISH")) ctx->lp_hash_finish = atoi(e) != 0;
  if (const char* e = getenv("LB_LP_LINES")) ctx->lp_lines = atoi(e) != 0;
  if (const char* e = getenv("LB_MSM_SHORT")) ctx->msm_short = atoi(e) != 0;
  if (const char* e = getenv("LB_LP_HASH_FULL")) ctx->lp_hash_full = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_LP_NARROW")) ctx->lp_narrow = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_LP_DEC_MAX")) ctx->lp_dec_max = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_LP_HF_MAX")) ctx->lp_hf_max = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_LP_LINES_MAX")) ctx->lp_lines_max = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_MSM_SHORT_MAX")) ctx->msm_short_max = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_MSM_T_LONE")) {
    const unsigned long t = strtoul(e, nullptr, 10);
    if (t >= 1 && t <= LB_MSM_T) ctx->msm_t_lone = (uint32_t)t;
  }
  if (const char* e = getenv("LB_STEP_SPLIT")) {
    const int v = atoi(e);
    ctx->step_split = (v == 1 || v == 2 || v == 4) ? (uint32_t)v : 0u;
  }
  if (const char* e = getenv("LB_WAVE_MAX")) ctx->wave_max_sets = (uint32_t)atoi(e);
  if (const char* e = getenv("LB_MTAIL")) ctx->mtail_lp = atoi(e) != 0;
  if (const char* e = getenv("LB_RTAIL")) ctx->rtail_lp = atoi(e) != 0;
  if (const char* e = getenv("LB_TP_RELEASE")) ctx->tp_release = ctx->tp_release_cfg = atoi(e) != 0;
  if (const char* e = getenv("LB_TP_PAUSE")) ctx->tp_pause_calls = (uint32_t)atoi(e);
  if (const char* e = getenv("LB_FAULT_RERUN")) ctx->fault_rerun = atoi(e) != 0;
  if (const char* e = getenv("LB_GT_LP")) ctx->gt_lp = atoi(e) != 0;
  if (const char* e = getenv("LB_PRIO_KCOPY")) ctx->prio_kcopy = atoi(e) != 0;
  if (const char* e = getenv("LB_LP_MAX")) {
    const long v = atol(e);  // clamped like lb_set_latency_path: the product tree's 2^LB_LP_TREE_LEVELS sets
    ctx->lp_max_sets = v <= 0 ? 0u : v < (1l << LB_LP_TREE_LEVELS) ? (uint32_t)v : (1u << LB_LP_TREE_LEVELS);
    ctx->lp_explicit = true;
  }
  if (const char* e = getenv("LB_LP_LONE_MAX")) ctx->lp_lone_max = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("LB_LINES_WAVES")) ctx->lines_waves = ctx->lines_waves_small = atoi(e) == 1 ? 1 : 2;
  if (const char* e = getenv("LB_ACC_SPLIT")) ctx->acc_split = atoi(e) ? 1 : 0;
  if (const char* e = getenv("LB_ACC")) ctx->acc_steps = strcmp(e, "pairs") ? 1 : 0;
  if (const char* e = getenv("LB_DAG")) ctx->dag = atoi(e) != 0;
  if (const char* e = getenv("LB_STEP_MODE")) ctx->step_mode = atoi(e);
  if (const char* e = getenv("LB_STEP_WAVES")) ctx->step_waves = atoi(e) == 2 ? 2 : 1;
  if (const char* e = getenv("LB_STAGE_EVENTS")) ctx->stage_events = atoi(e) != 0;
  if (const char* e = getenv("LB_ACC_LPR")) {
    const int v = atoi(e);
    if (v == 64 || v == 32 || v == 16) ctx->acc_lpr = v;
  }
  for (int s = 0; s < lb_ctx::kMaxSlots; s++)
    ctx->streams_per_slot[s] = lane ? 1 : ctx->n_slots <= 2 ? 2 : (ctx->n_slots == 3 && s == 0) ? 2 : 1;
  ctx->streams_per_slot[ctx->n_slots] = 1;  // the priority lane
  // LB_SLOT0_STREAMS=1|2 overrides slot 0's two-stream DAG (the synchronous, lowest-latency slot)
  if (const char* e = getenv("LB_SLOT0_STREAMS")) ctx->streams_per_slot[0] = atoi(e) == 1 ? 1 : 2;
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
  // The priority lane's CU reservation.  A running workgroup is never
  // preempted and a priority stream only reorders dispatch, so under load a latency-path
  // call would wait for a whole CU to drain.  LB_PRIO_CUS=K (default 64 of 256; 0 = off):
  // masked streams that leave the K highest-numbered CUs to the priority lane.
  // LB_PRIO_DYN (default 1): throughput calls take them only while the priority lane has
  // been used within the last LB_PRIO_HOLD_MS (default 250), the full streams otherwise,
  // so a GPU without priority traffic keeps every CU.  Measured (profiles/r04/prio_ab/,
  // legs_ab/): 1-set / 128-set p50 under 16 calls in flight 1.2x / 1.9x idle (4-6x without),
  // C2 throughput unchanged.
  std::vector<uint32_t> cu_mask;
  {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    int k = cus >= 128 ? 64 : 0;
    if (const char* e = getenv("LB_PRIO_CUS")) k = atoi(e);
    if (lane) k = 0;  // (the reservation belongs to the throughput context: lb_mark_priority)
    if (k > 0 && k < cus) {
      cu_mask.assign((size_t)(cus + 31) / 32, 0u);
      // LB_PRIO_SPREAD=1: the K reserved CUs evenly spaced over the CU ids instead (measured
      // worse: the mask bits do not map to CUs that way)
      const char* sp = getenv("LB_PRIO_SPREAD");
      const bool spread = sp && atoi(sp) == 1;
      std::vector<char> reserved((size_t)cus, 0);
      for (int j = 0; j < k; j++) reserved[spread ? (size_t)((int64_t)(j + 1) * cus / k - 1) : (size_t)(cus - k + j)] = 1;
      for (int c = 0; c < cus; c++)
        if (!reserved[c]) cu_mask[c / 32] |= 1u << (c % 32);
      ctx->prio_cus = k;
    }
  }
  if (!cu_mask.empty()) {
    const char* dy = getenv("LB_PRIO_DYN");
    ctx->prio_dyn = !dy || atoi(dy) != 0;
    if (const char* h = getenv("LB_PRIO_HOLD_MS")) ctx->prio_hold_ms = atof(h);
    // every masked stream takes a hardware queue of a pool of its own, and every queue
    // reserves scratch (§5.1): with LB_PRIO_DYN_SLOTS=K only the first K slots get one
    // masked stream each; while the priority lane is in use new calls go to those slots
    // (default 2: 16 + 16 ran out of scratch, like 24 queues of one pool; with 4 masked
    // queues the queues of a second context or process on the same GPU -- bench.py's
    // single-stream timing context, its node leg -- slowed every later call by a third,
    // with 2 they did not)
    ctx->prio_dyn_slots = ctx->n_slots;
    int v = 2;
    if (const char* k = getenv("LB_PRIO_DYN_SLOTS")) v = atoi(k);
    if (ctx->prio_dyn && v >= 1 && v < ctx->n_slots) ctx->prio_dyn_slots = v;
  }
  // Every hardware queue this context opens reserves scratch for the largest private
  // segment it runs: price all of them, not only GPU_MAX_HW_QUEUES
  // (VERDICT r4 #7).  HIP pools the plain streams of one priority into at most
  // GPU_MAX_HW_QUEUES queues; a CU-masked stream gets a queue of its own.
  {
    int maxq = 4;
    if (const char* e = getenv("GPU_MAX_HW_QUEUES")) maxq = atoi(e) > 0 ? atoi(e) : 4;
    int plain = 0, masked = 0;
    const bool one = ctx->prio_dyn && ctx->prio_dyn_slots < ctx->n_slots;
    for (int s = 0; s < ctx->n_slots; s++) {
      const int spp = ctx->streams_per_slot[s];
      if (cu_mask.empty() || ctx->prio_dyn) plain += spp;
      if (!cu_mask.empty() && s < ctx->prio_dyn_slots) masked += one ? 1 : spp;
    }
    const char* tp = getenv("LB_TAIL_PRIO");
    const int high = 2 + (tp && atoi(tp) == 1 ? 1 : 0);  // priority lane, aux (lb_gt_check), tail stream
    const int queues = (plain < maxq ? plain : maxq) + (high < maxq ? high : maxq) + masked;
    uint32_t lane = 0;
    const size_t per_q = scratch_per_queue(device, &lane);
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
    // the largest configuration that ran: 16 plain + 2 masked + 2 high-priority queues at
    // 3,328 private bytes per lane; 24 + 2 plain (r03) and 16 + 16 masked + 2 (r04) queues
    // failed with HSA_STATUS_ERROR_OUT_OF_RESOURCES
    double budget = 20.0 * 3328 * 64 * 32 * cus;
    if (const char* e = getenv("LB_SCRATCH_BUDGET_GB")) budget = atof(e) * 1e9;
    if ((double)per_q * queues > budget) {
      char msg[400];
      snprintf(msg, sizeof msg,
               "%d hardware queues (%d plain of GPU_MAX_HW_QUEUES=%d, %d CU-masked, %d high-priority) x %u private "
               "bytes per lane x 64 x 32 x %d CUs = %.1f GB of scratch exceeds the %.1f GB budget (20 queues at "
               "3,328 B/lane ran; 16 + 16 masked failed with HSA_STATUS_ERROR_OUT_OF_RESOURCES)",
               queues, plain < maxq ? plain : maxq, maxq, masked, high < maxq ? high : maxq, lane, cus,
               per_q * (double)queues / 1e9, budget / 1e9);
      g_create_err = msg;
      delete ctx;
      return LB_ERR_RESOURCES;
    }
    std::lock_guard<std::mutex> g(g_q_mu);
    const int proc = pooled_queues(g_q_plain + plain, g_q_high + high, g_q_masked + masked, maxq);
    if (lane_ctx && proc > kProcessQueueBudget) {
      char msg[300];
      snprintf(msg, sizeof msg,
               "latency-lane context refused: the process would hold %d hardware queues (%d plain, %d high-priority "
               "streams pooled into at most GPU_MAX_HW_QUEUES=%d each, %d CU-masked), above the %d that ran",
               proc, g_q_plain + plain, g_q_high + high, maxq, g_q_masked + masked, kProcessQueueBudget);
      g_create_err = msg;
      delete ctx;
      return LB_ERR_RESOURCES;
    }
    g_q_plain += plain;
    g_q_high += high;
    g_q_masked += masked;
    ctx->q_plain = plain;
    ctx->q_high = high;
    ctx->q_masked = masked;
    ctx->hw_queues = queues;
  }
  for (int s = 0; ok && s <= ctx->n_slots; s++) {
    Slot& sl = ctx->slots[s];
    for (int i = 0; ok && i < ctx->streams_per_slot[s]; i++) {
      if (s == ctx->n_slots) {
        ok = hipStreamCreateWithPriority(&sl.st[i], hipStreamNonBlocking, prio_greatest) == hipSuccess;
      } else if (!cu_mask.empty()) {
        const bool one = ctx->prio_dyn && ctx->prio_dyn_slots < ctx->n_slots;  // one masked stream per slot
        if (s < ctx->prio_dyn_slots && !(one && i > 0))
          ok = hipExtStreamCreateWithCUMask(&sl.st_mask[i], (uint32_t)cu_mask.size(), cu_mask.data()) == hipSuccess;
        else if (one && i > 0)
          sl.st_mask[i] = sl.st_mask[0];
        if (ok && ctx->prio_dyn) ok = hipStreamCreateWithFlags(&sl.st_full[i], hipStreamNonBlocking) == hipSuccess;
        sl.st[i] = ctx->prio_dyn ? sl.st_full[i] : sl.st_mask[i];
      } else {
        ok = hipStreamCreateWithFlags(&sl.st[i], hipStreamNonBlocking) == hipSuccess;
      }
    }
    if (ctx->streams_per_slot[s] == 1) {
      sl.st_full[1] = sl.st_full[0];
      sl.st_mask[1] = sl.st_mask[0];
    }
    if (ctx->streams_per_slot[s] == 1) sl.st[1] = sl.st[0];
    for (int i = 0; ok && i < 8; i++) ok = hipEventCreateWithFlags(&sl.dep[i], hipEventDisableTiming) == hipSuccess;
    for (int i = 0; ok && i < Slot::kMaxStages; i++)
      ok = hipEventCreate(&sl.ev0[i]) == hipSuccess && hipEventCreate(&sl.ev1[i]) == hipSuccess;
    ok = ok && hipEventCreate(&sl.wall0) == hipSuccess && hipEventCreate(&sl.wall1) == hipSuccess &&
         hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&sl.partial_ev, hipEventDisableTiming) == hipSuccess &&
         hipHostMalloc(&sl.h_stats, 4 * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc(&sl.h_partial, LB_GT_BYTES, hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc(&sl.h_clk, 4 * sizeof(unsigned long long), hipHostMallocDefault) == hipSuccess;
    if (ok) sl.h_stats[0] = sl.h_stats[1] = 0;
  }
  ctx->stream = ctx->slots[0].st[0];
  // the host combine's one-wave final exponentiation must not queue behind the
  // calls in flight (their 1-wave/SIMD kernels fill every SIMD): highest priority
  ok = ok && hipStreamCreateWithPriority(&ctx->aux_stream, hipStreamNonBlocking, prio_greatest) == hipSuccess;
  {
    // off by default: one shared high-priority stream for every slot's merged check
    // measured 2.40-2.43 vs 2.56-2.57 M sets/s (profiles/ab_r02s/r02s_d_*.json)
    const char* e = getenv("LB_TAIL_PRIO");
    if (e && atoi(e) == 1)
      ok = ok && hipStreamCreateWithPriority(&ctx->tail_stream, hipStreamNonBlocking, prio_greatest) == hipSuccess;
  }
  // the latency path's round programs (2.6 MB) are uploaded here, before any call is in
  // flight: a synchronous copy on the first latency-path call would wait for the
  // throughput calls already running on blocking (CU-masked) streams
  if (ok && (ctx->lp_max_sets || ctx->mtail_lp || ctx->gt_lp || ctx->rtail_lp) && lp_ensure(ctx) != LB_OK) ok = false;
  // the priority slot's staging and workspace sized here for a latency-path call of
  // lp_max_sets sets (16 keys each by bytes): growing them later frees the old buffers,
  // and hipFree / hipHostFree synchronize the device -- the call would wait for every
  // throughput call in flight (the node leg's first 128-set priority job under load took
  // 0.9-1.5 s, profiles/r05/node_q/)
  if (ok && ctx->lp_max_sets) {
    Slot& pl = ctx->slots[ctx->n_slots];
    const size_t ns = ctx->lp_max_sets, in = ns * (32 + 192 + 16 + 16 * 96) + 65536, out = 3 * ns + 4096;
    ok = ensure_pin(ctx, pl, in + out) == LB_OK && ensure_ws(ctx, pl, in + out + pipeline_ws_bytes(ctx, ns, ns)) == LB_OK;
  }
  if (!ok) {
    lb_destroy(ctx);
    return LB_ERR_DEVICE;
  }
  *out_ctx = ctx;
  return LB_OK;
}

int lb_create(int device, lb_ctx** out_ctx) { return create_ctx(device, out_ctx, false); }

int lb_create_lane(int device, lb_ctx** out_ctx) { return create_ctx(device, out_ctx, true); }

int lb_mark_priority(lb_ctx* ctx) {
  if (!ctx) return LB_ERR_INVALID_ARGUMENT;
  ctx->last_prio_ns.store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now().time_since_epoch()).count(),
                          std::memory_order_relaxed);
  return LB_OK;
}

int lb_destroy(lb_ctx* ctx) {
  if (!ctx) return LB_OK;
  (void)hipSetDevice(ctx->device);
  for (int s = 0; s <= ctx->n_slots; s++) {
    Slot& sl = ctx->slots[s];
    for (int i = 0; i < ctx->streams_per_slot[s]; i++) {
      if (sl.st[i]) (void)hipStreamSynchronize(sl.st[i]);
      if (sl.st_full[i]) (void)hipStreamSynchronize(sl.st_full[i]);
      if (sl.st_mask[i]) (void)hipStreamSynchronize(sl.st_mask[i]);
    }
    if (sl.d_ws) (void)hipFree(sl.d_ws);
    if (sl.h_pin) (void)hipHostFree(sl.h_pin);
    for (int i = 0; i < 8; i++)
      if (sl.dep[i]) (void)hipEventDestroy(sl.dep[i]);
    for (int i = 0; i < Slot::kMaxStages; i++) {
      if (sl.ev0[i]) (void)hipEventDestroy(sl.ev0[i]);
      if (sl.ev1[i]) (void)hipEventDestroy(sl.ev1[i]);
    }
    if (sl.wall0) (void)hipEventDestroy(sl.wall0);
    if (sl.wall1) (void)hipEventDestroy(sl.wall1);
    if (sl.done) (void)hipEventDestroy(sl.done);
    if (sl.partial_ev) (void)hipEventDestroy(sl.partial_ev);
    if (sl.h_stats) (void)hipHostFree(sl.h_stats);
    if (sl.h_partial) (void)hipHostFree(sl.h_partial);
    if (sl.h_clk) (void)hipHostFree(sl.h_clk);
    for (int i = 0; i < ctx->streams_per_slot[s]; i++) {
      if (sl.st_mask[i] || sl.st_full[i]) {  // (st[] is one of these pairs)
        if (sl.st_mask[i] && !(i > 0 && sl.st_mask[i] == sl.st_mask[0])) (void)hipStreamDestroy(sl.st_mask[i]);
        if (sl.st_full[i]) (void)hipStreamDestroy(sl.st_full[i]);
      } else if (sl.st[i]) {
        (void)hipStreamDestroy(sl.st[i]);
      }
    }
  }
  if (ctx->d_table) (void)hipFree(ctx->d_table);
  if (ctx->aux_stream) {
    (void)hipStreamSynchronize(ctx->aux_stream);
    (void)hipStreamDestroy(ctx->aux_stream);
  }
  if (ctx->tail_stream) {
    (void)hipStreamSynchronize(ctx->tail_stream);
    (void)hipStreamDestroy(ctx->tail_stream);
  }
  if (ctx->d_aux) (void)hipFree(ctx->d_aux);
  if (ctx->h_aux) (void)hipHostFree(ctx->h_aux);
  if (ctx->d_lp) (void)hipFree(ctx->d_lp);
  {
    std::lock_guard<std::mutex> g(g_q_mu);
    g_q_plain -= ctx->q_plain;
    g_q_high -= ctx->q_high;
    g_q_masked -= ctx->q_masked;
  }
  delete ctx;
  return LB_OK;
}

const char* lb_last_error(const lb_ctx* ctx) {
  // (a copy per calling thread: valid until that thread's next lb_last_error)
  static thread_local std::string out;
  out = ctx ? std::string(ctx->err) : g_create_err;
  return out.c_str();
}

int lb_scratch_per_queue(int device, uint64_t* out_bytes, uint32_t* out_lane_bytes) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0 || device < 0 || device >= n) return LB_ERR_NO_DEVICE;
  if (!out_bytes) return LB_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(device) != hipSuccess) return LB_ERR_DEVICE;
  *out_bytes = scratch_per_queue(device, out_lane_bytes);
  return LB_OK;
}

int lb_slots(const lb_ctx* ctx) { return ctx ? ctx->n_slots : 0; }
int lb_hw_queues(const lb_ctx* ctx) { return ctx ? ctx->hw_queues : 0; }
int lb_last_call_streams(const lb_ctx* ctx) { return ctx ? ctx->last_call_streams : 0; }
int lb_last_latency_clocks(const lb_ctx* ctx, uint64_t* out4) {
  if (!ctx || !out4) return LB_ERR_INVALID_ARGUMENT;
  for (int i = 0; i < 4; i++) out4[i] = ctx->lp_clk[i];
  return LB_OK;
}

#ifdef LB_COUNT_OPS
// Fp products executed per stage of the last completed verify call (count build only)
int lb_opcount_stages(const lb_ctx* ctx, unsigned long long* out, int max_stages) {
  if (!ctx) return 0;
  int n = 0;
  for (int i = 0; i < ctx->n_stages && n < max_stages; i++) out[n++] = ctx->stage_ops[i];
  return n;
}
#endif

int lb_last_stage_times(const lb_ctx* ctx, float* out_ms, const char** out_names, int max_stages) {
  if (!ctx) return 0;
  int n = ctx->n_stages < max_stages ? ctx->n_stages : max_stages;
  for (int i = 0; i < n; i++) {
    if (out_ms) out_ms[i] = ctx->stage_ms[i];
    if (out_names) out_names[i] = ctx->stage_name[i];
  }
  return ctx->n_stages;
}

// the priority lane used within the last prio_hold_ms (LB_PRIO_DYN)
static bool prio_active(lb_ctx* ctx) {
  const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  return ctx->prio_dyn && (double)(now - ctx->last_prio_ns.load(std::memory_order_relaxed)) < ctx->prio_hold_ms * 1e6;
}

// A call about to run on slot sl (idle: finish_slot has retired its last call): with
// LB_PRIO_DYN, the masked streams while the priority lane is in use, else the full ones.
// The priority slot marks the lane in use.
static void pick_streams(lb_ctx* ctx, Slot& sl) {
  if (&sl == &ctx->prio()) {
    ctx->last_prio_ns.store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now().time_since_epoch()).count(),
                            std::memory_order_relaxed);
    return;
  }
  if (!ctx->prio_dyn) return;
  if (prio_active(ctx)) {
    // a slot without masked streams queues on those of slot (s mod K) -- on the GPU, not
    // in finish_slot: the submitting thread never waits longer than the round robin makes it
    const Slot& m = sl.st_mask[0] ? sl : ctx->slots[(&sl - ctx->slots) % ctx->prio_dyn_slots];
    sl.st[0] = m.st_mask[0];
    sl.st[1] = m.st_mask[1];
  } else {
    sl.st[0] = sl.st_full[0];
    sl.st[1] = sl.st_full[1];
  }
  // a synchronous call's borrowed second stream (BorrowGuard) stays: the call runs as
  // the two-stream DAG whichever stream pair slot 0 takes
  if (sl.guard_st) sl.st[1] = sl.guard_st;
}

// a two-phase call's record (LB_TP_RELEASE; the legacy mode keeps only the ticket ring)
static void tp_record(lb_ctx* ctx, uint64_t ticket, const lb_request_batch* b, bool device, uint8_t* valid,
                      uint8_t* err, uint8_t* sst) {
  if (!ctx->tp_release) return;
  // (the ticket ring too: a finish of a ticket whose record was reused -- finished or waited
  // for by then, tp_reusable -- is a no-op, not an error)
  ctx->two_phase[ctx->two_phase_pos] = ticket;
  ctx->two_phase_pos = (ctx->two_phase_pos + 1) % lb_ctx::kTwoPhaseRing;
  TwoPhaseRec& r = ctx->tp[ticket % lb_ctx::kTwoPhaseRing];
  r.ticket = ticket;
  r.device = device;
  r.finished = r.have_partial = r.failed = r.waited = false;
  r.rerun = 0;
  r.batch = *b;
  r.valid = valid;
  r.err = err;
  r.sst = sst;
  if (!b->n_requests) {  // an empty shard: its partial is 1, known now
    memset(r.partial, 0, LB_GT_BYTES);
    r.partial[47] = 1;
    r.have_partial = true;
  }
}

static TwoPhaseRec* tp_find(lb_ctx* ctx, uint64_t ticket) {
  TwoPhaseRec& r = ctx->tp[ticket % lb_ctx::kTwoPhaseRing];
  // (records exist only for calls submitted in the release mode, whatever the mode now)
  return (ticket && r.ticket == ticket) ? &r : nullptr;
}

// A record may be overwritten once nothing about its call can change: it was waited for, or
// it was finished (with a submitted re-run, if any, retired).  Before that its outputs hold
// provisional verdicts that only its record turns into final ones.
static bool tp_reusable(lb_ctx* ctx, const TwoPhaseRec& r) {
  if (!r.ticket || r.waited) return true;
  return r.finished && !r.failed && (!r.rerun || !slot_of_ticket(ctx, r.rerun));
}

static int submit_device(lb_ctx* ctx, Slot& sl, const lb_request_batch* b, uint8_t* d_valid, uint8_t* d_req_err,
                         uint8_t* d_set_status, bool partial, uint64_t* out_ticket) {
  LB_TRY(finish_slot(ctx, sl));  // at most kSlots calls in flight
  pick_streams(ctx, sl);
  if (!partial) borrow_idle_stream(ctx, sl);  // (a pending two-phase call never holds a lent slot)
  LB_TRY(ensure_ws(ctx, sl, pipeline_ws_bytes(ctx, b->n_requests, b->n_sets)));
  Bump ws{sl.d_ws, 0, sl.ws_cap};
  uint8_t* d_partial = partial ? ws.take<uint8_t>(LB_GT_BYTES) : nullptr;
  LB_TRY(begin_call(ctx, sl));
  if (b->n_requests)
    LB_TRY(run_pipeline(ctx, sl, b->n_requests, b->n_sets, b->request_offsets, b->pubkeys, b->pk_offsets,
                        b->pubkey_indices, b->messages, b->signatures, b->sig_offsets, b->seed, d_valid, d_req_err,
                        d_set_status, ws, d_partial));
  else if (partial) {  // nothing to verify: the partial is the identity (1 in Fp12)
    memset(sl.h_partial, 0, LB_GT_BYTES);
    sl.h_partial[47] = 1;
    LB_HIP(hipEventRecord(sl.partial_ev, sl.st[0]));
    sl.ps = PipeState{};
    sl.partial_pending = !ctx->tp_release;
  }
  LB_TRY(end_call_async(ctx, sl));
  *out_ticket = sl.ticket;
  if (partial) tp_record(ctx, sl.ticket, b, true, d_valid, d_req_err, d_set_status);
  return LB_OK;
}

// Host-side checks of a host-buffer batch: offsets must be monotone and start
// at 0 (a kernel must never index out of bounds).
static int check_host_batch(lb_ctx* ctx, const lb_request_batch* b) {
  const uint32_t nr = b->n_requests, ns = b->n_sets;
  if (b->request_offsets[0] != 0 || b->request_offsets[nr] != ns) {
    ctx->err = "request_offsets must start at 0 and end at n_sets";
    return LB_ERR_INVALID_ARGUMENT;
  }
  for (uint32_t k = 0; k < nr; k++)
    if (b->request_offsets[k + 1] < b->request_offsets[k]) {
      ctx->err = "request_offsets not monotone";
      return LB_ERR_INVALID_ARGUMENT;
    }
  if (b->sig_offsets[0] != 0) {
    ctx->err = "sig_offsets must start at 0";
    return LB_ERR_INVALID_ARGUMENT;
  }
  for (uint32_t i = 0; i < ns; i++)
    if (b->sig_offsets[i + 1] < b->sig_offsets[i]) {
      ctx->err = "sig_offsets not monotone";
      return LB_ERR_INVALID_ARGUMENT;
    }
  if (const uint32_t* pk_off = b->pk_offsets) {
    if (pk_off[0] != 0) {
      ctx->err = "pk_offsets must start at 0";
      return LB_ERR_INVALID_ARGUMENT;
    }
    for (uint32_t i = 0; i < ns; i++)
      if (pk_off[i + 1] < pk_off[i]) {
        ctx->err = "pk_offsets not monotone";
        return LB_ERR_INVALID_ARGUMENT;
      }
  }
  return LB_OK;
}

// Host-buffer call on slot `sl`: inputs staged through the slot's pinned
// buffer (one H2D copy), the pipeline, verdicts copied back into pinned memory
// on the slot's stream and into the caller's buffers when the call retires.
// LB_HOST_TRACE=1: host-side phases of every host-buffer submission on stderr (ms)
static bool host_trace() {
  static const int on = [] {
    const char* e = getenv("LB_HOST_TRACE");
    return e && atoi(e) ? 1 : 0;
  }();
  return on != 0;
}
static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

static int submit_host(lb_ctx* ctx, Slot& sl, const lb_request_batch* b, uint8_t* out_valid, uint8_t* out_req_err,
                       uint8_t* out_set_status, bool partial, uint64_t* out_ticket) {
  const auto t0 = std::chrono::steady_clock::now();
  double t_check = 0, t_finish = 0, t_stage = 0, t_pipe = 0;
  const uint32_t nr = b->n_requests, ns = b->n_sets;
  LB_TRY(check_host_batch(ctx, b));
  t_check = ms_since(t0);
  const uint32_t* pk_off = b->pk_offsets;
  const size_t n_pk = pk_off ? pk_off[ns] : ns;
  const bool by_index = b->pubkey_indices != nullptr;
  // mixed package: rows of `pubkeys` named by flagged indices (every row < n_rows is staged)
  size_t n_rows = 0;
  if (by_index && b->pubkeys)
    for (size_t k = 0; k < n_pk; k++) {
      const uint32_t j = b->pubkey_indices[k];
      if ((j & LB_PK_ROW_FLAG) && (size_t)(j & LB_PK_ROW_MASK) + 1 > n_rows) n_rows = (j & LB_PK_ROW_MASK) + 1;
    }
  const size_t sig_bytes = b->sig_offsets[ns];
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t sz_req = sizeof(uint32_t) * (nr + 1), sz_pko = pk_off ? sizeof(uint32_t) * (ns + 1) : 0,
               sz_pk = n_pk * (by_index ? sizeof(uint32_t) : 96), sz_msg = (size_t)ns * 32,
               sz_sigo = sizeof(uint32_t) * (ns + 1), sz_sig = sig_bytes, sz_seed = 32, sz_rows = n_rows * 96;
  const size_t in_bytes =
      al(sz_req) + al(sz_pko) + al(sz_pk) + al(sz_msg) + al(sz_sigo) + al(sz_sig) + al(sz_seed) + al(sz_rows);
  const size_t out_bytes = al(nr ? nr : 1) * 2 + al(ns ? ns : 1);
  LB_TRY(finish_slot(ctx, sl));
  pick_streams(ctx, sl);
  t_finish = ms_since(t0);
  if (!partial) borrow_idle_stream(ctx, sl);
  LB_TRY(ensure_pin(ctx, sl, in_bytes + out_bytes));
  LB_TRY(ensure_ws(ctx, sl, in_bytes + out_bytes + pipeline_ws_bytes(ctx, nr, ns)));
  Bump ws{sl.d_ws, 0, sl.ws_cap};
  char* h = sl.h_pin;
  size_t ho = 0;
  auto stage = [&](const void* src, size_t n) {
    if (n) memcpy(h + ho, src, n);
    ho += al(n);
  };
  stage(b->request_offsets, sz_req);
  if (pk_off) stage(pk_off, sz_pko);
  stage(by_index ? (const void*)b->pubkey_indices : (const void*)b->pubkeys, sz_pk);
  stage(b->messages, sz_msg);
  stage(b->sig_offsets, sz_sigo);
  stage(b->signatures, sz_sig);
  stage(b->seed, sz_seed);
  if (n_rows) stage(b->pubkeys, sz_rows);
  t_stage = ms_since(t0);
  char* d_in = ws.take<char>(in_bytes);
  uint8_t* d_valid = ws.take<uint8_t>(nr ? nr : 1);
  uint8_t* d_err = ws.take<uint8_t>(nr ? nr : 1);
  uint8_t* d_sst = ws.take<uint8_t>(ns ? ns : 1);
  uint8_t* d_partial = partial ? ws.take<uint8_t>(LB_GT_BYTES) : nullptr;
  LB_TRY(begin_call(ctx, sl));
  sl.dv_valid = d_valid;
  sl.dv_err = d_err;
  sl.dv_sst = d_sst;
  sl.h_out = h + in_bytes;
  sl.out_valid = out_valid;
  sl.out_err = out_req_err;
  sl.out_sst = out_set_status;
  sl.out_nr = nr;
  sl.out_ns = out_set_status ? ns : 0;
  LB_TRY(slot_copy(ctx, sl, d_in, h, in_bytes, hipMemcpyHostToDevice, sl.st[0]));
  size_t o = 0;
  auto dptr = [&](size_t n) {
    char* p = d_in + o;
    o += al(n);
    return p;
  };
  const uint32_t* d_req = (const uint32_t*)dptr(sz_req);
  const uint32_t* d_pko = pk_off ? (const uint32_t*)dptr(sz_pko) : nullptr;
  const uint8_t* d_pks = (const uint8_t*)dptr(sz_pk);
  const uint8_t* d_msg = (const uint8_t*)dptr(sz_msg);
  const uint32_t* d_sigo = (const uint32_t*)dptr(sz_sigo);
  const uint8_t* d_sig = (const uint8_t*)dptr(sz_sig);
  const uint8_t* d_seed = (const uint8_t*)dptr(sz_seed);
  const uint8_t* d_rows = n_rows ? (const uint8_t*)dptr(sz_rows) : nullptr;
  if (nr) {
    LB_TRY(run_pipeline(ctx, sl, nr, ns, d_req, by_index ? d_rows : d_pks, d_pko,
                        by_index ? (const uint32_t*)d_pks : nullptr, d_msg, d_sig, d_sigo, d_seed, d_valid, d_err, d_sst,
                        ws, d_partial));
    t_pipe = ms_since(t0);
  } else if (partial) {
    memset(sl.h_partial, 0, LB_GT_BYTES);
    sl.h_partial[47] = 1;
    LB_HIP(hipEventRecord(sl.partial_ev, sl.st[0]));
    sl.ps = PipeState{};
    sl.partial_pending = !ctx->tp_release;
  }
  LB_TRY(end_call_async(ctx, sl));
  *out_ticket = sl.ticket;
  if (partial) tp_record(ctx, sl.ticket, b, false, out_valid, out_req_err, out_set_status);
  if (host_trace())
    fprintf(stderr, "lb_host_trace sets=%u check=%.3f finish_slot=%.3f stage=%.3f pipeline=%.3f total=%.3f dag=%d slot=%d\n",
            ns, t_check, t_finish, t_stage, t_pipe, ms_since(t0), sl.st[1] != sl.st[0] ? 1 : 0,
            (int)(&sl - ctx->slots));
  return LB_OK;
}

static void fill_stats(lb_ctx* ctx, uint64_t ticket, lb_verify_stats* stats) {
  if (!stats) return;
  const TicketStats& ts = ctx->tstats[ticket % lb_ctx::kTicketRing];
  if (ts.ticket == ticket) {
    stats->batch_retries = ts.batch_retries;
    stats->batch_sigs_success = ts.batch_sigs_success;
    stats->device_ms = ts.wall_ms;
  } else {  // more than kTicketRing calls retired since: the stats are gone
    *stats = lb_verify_stats{0, 0, 0.0};
  }
}

// Round robin over the slots, passing over a slot whose two-phase call still
// waits for the host's combined verdict (reusing it would retire that call with
// merged_ok = 0: correct verdicts, but every request's tail re-run); only when
// every slot holds a pending partial is the next one taken anyway.
static Slot& next_async_slot(lb_ctx* ctx) {  // internal: not part of the C ABI
  int s = ctx->next_slot;
  for (int k = 0; k < ctx->n_slots; k++) {
    const int c = (ctx->next_slot + k) % ctx->n_slots;
    if (!ctx->slots[c].partial_pending) {
      s = c;
      break;
    }
  }
  ctx->next_slot = (s + 1) % ctx->n_slots;
  return ctx->slots[s];
}

int lb_verify_requests_device_async(lb_ctx* ctx, const lb_request_batch* b, uint8_t* d_valid, uint8_t* d_req_err,
                                    uint8_t* d_set_status, uint64_t* out_ticket) {
  if (!ctx || !out_ticket) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(validate_batch(ctx, b));
  if (!d_valid || !d_req_err) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  return submit_device(ctx, next_async_slot(ctx), b, d_valid, d_req_err, d_set_status, false, out_ticket);
}

int lb_verify_requests_async(lb_ctx* ctx, const lb_request_batch* b, uint8_t* out_valid, uint8_t* out_req_err,
                             uint8_t* out_set_status, uint64_t* out_ticket) {
  if (!ctx || !out_ticket) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(validate_batch(ctx, b));
  if (!out_valid || !out_req_err) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  return submit_host(ctx, next_async_slot(ctx), b, out_valid, out_req_err, out_set_status, false, out_ticket);
}

int lb_verify_requests_partial_async(lb_ctx* ctx, const lb_request_batch* b, uint32_t flags, uint8_t* out_valid,
                                     uint8_t* out_req_err, uint8_t* out_set_status, uint64_t* out_ticket) {
  if (!ctx || !out_ticket) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(validate_batch(ctx, b));
  if (!out_valid || !out_req_err) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  ctx->tp_release = ctx->tp_release_cfg && ctx->tp_pause == 0;
  if (ctx->tp_pause) ctx->tp_pause--;
  if (ctx->tp_release && !tp_reusable(ctx, ctx->tp[ctx->next_ticket % lb_ctx::kTwoPhaseRing])) {
    // (the ticket this call would take is end_call_async's next_ticket: no ticket is issued
    // in between)
    ctx->err = "two-phase ring full: the call " +
               std::to_string(ctx->tp[ctx->next_ticket % lb_ctx::kTwoPhaseRing].ticket) +
               " is neither finished nor waited for (" + std::to_string(lb_ctx::kTwoPhaseRing) +
               "-entry ring by ticket): finish or wait for older two-phase calls first";
    return LB_ERR_RESOURCES;
  }
  Slot& sl = next_async_slot(ctx);
  if (flags & LB_BATCH_DEVICE)
    return submit_device(ctx, sl, b, out_valid, out_req_err, out_set_status, true, out_ticket);
  return submit_host(ctx, sl, b, out_valid, out_req_err, out_set_status, true, out_ticket);
}

int lb_partial_wait(lb_ctx* ctx, uint64_t ticket, uint8_t* out576) {
  if (!ctx || !out576) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  Slot* sl = slot_of_ticket(ctx, ticket);
  if (TwoPhaseRec* r = tp_find(ctx, ticket)) {  // released: on its slot, or saved when it retired
    if (!r->have_partial && sl) {
      LB_HIP(hipEventSynchronize(sl->partial_ev));
      memcpy(out576, sl->h_partial, LB_GT_BYTES);
      return LB_OK;
    }
    if (r->have_partial) {
      memcpy(out576, r->partial, LB_GT_BYTES);
      return LB_OK;
    }
  }
  if (!sl || !sl->partial_pending) {
    ctx->err = "ticket is not a pending two-phase call";
    return LB_ERR_INVALID_ARGUMENT;
  }
  LB_HIP(hipEventSynchronize(sl->partial_ev));
  memcpy(out576, sl->h_partial, LB_GT_BYTES);
  return LB_OK;
}

int lb_partial_poll(lb_ctx* ctx, uint64_t ticket, int32_t* out_ready) {
  if (!ctx || !out_ready) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  Slot* sl = slot_of_ticket(ctx, ticket);
  if (TwoPhaseRec* r = tp_find(ctx, ticket)) {
    if (r->have_partial) {
      *out_ready = 1;
      return LB_OK;
    }
    if (sl) {
      const hipError_t q = hipEventQuery(sl->partial_ev);
      if (q == hipErrorNotReady) {
        *out_ready = 0;
        return LB_OK;
      }
      LB_HIP(q);
      *out_ready = 1;
      return LB_OK;
    }
  }
  if (!sl || !sl->partial_pending) {
    ctx->err = "ticket is not a pending two-phase call";
    return LB_ERR_INVALID_ARGUMENT;
  }
  const hipError_t q = hipEventQuery(sl->partial_ev);
  if (q == hipErrorNotReady) {
    *out_ready = 0;
    return LB_OK;
  }
  LB_HIP(q);
  *out_ready = 1;
  return LB_OK;
}

int lb_verify_requests_finish(lb_ctx* ctx, uint64_t ticket, int merged_ok) {
  if (!ctx) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  if (TwoPhaseRec* r = tp_find(ctx, ticket)) {
    if (r->finished) return LB_OK;
    r->finished = true;
    if (merged_ok) return LB_OK;  // its verdicts (every request not already false valid) stand
    // the combined check failed: the shard again as a one-phase call -- its own merged check
    // fails and every request is verified alone (worker.ts:74-85) -- into the same outputs,
    // after the released call has retired (its verdicts must not land after the re-run's)
    // (a failure from here on leaves the outputs provisional: the record says so, and
    // lb_wait returns the error instead of them)
    r->failed = true;
    ctx->tp_pause = ctx->tp_pause_calls;  // (the next two-phase calls: legacy mode)
    if (Slot* sl = slot_of_ticket(ctx, ticket)) LB_TRY(finish_slot(ctx, *sl));
    if (ctx->fault_rerun) {  // (fault injection for the tests: the re-run's submission fails)
      ctx->err = "LB_FAULT_RERUN: the failed combine's re-verification was not submitted";
      return LB_ERR_DEVICE;
    }
    const lb_request_batch b = r->batch;
    uint8_t *v = r->valid, *e = r->err, *st = r->sst;
    const bool device = r->device;
    uint64_t t2 = 0;
    LB_TRY(device ? submit_device(ctx, next_async_slot(ctx), &b, v, e, st, false, &t2)
                  : submit_host(ctx, next_async_slot(ctx), &b, v, e, st, false, &t2));
    if (TwoPhaseRec* r2 = tp_find(ctx, ticket)) {
      r2->rerun = t2;
      r2->failed = false;
    }
    return LB_OK;
  }
  Slot* sl = slot_of_ticket(ctx, ticket);
  if (!sl || !sl->partial_pending) {
    // a two-phase call another call's slot reuse already resumed (with merged_ok
    // = 0: every request re-verified alone, so its verdicts stand): nothing to do
    for (int i = 0; ticket != 0 && i < lb_ctx::kTwoPhaseRing; i++)
      if (ctx->two_phase[i] == ticket) return LB_OK;
    // older than every two-phase ticket the ring still holds (the ring wrapped): whether
    // it was a two-phase call is no longer known, but any retired call's verdicts are
    // final, so finishing it is a no-op rather than an error
    const uint64_t oldest = ctx->two_phase[ctx->two_phase_pos];  // (0 until the ring wraps)
    if (ticket != 0 && oldest != 0 && ticket < oldest && ticket < ctx->next_ticket) return LB_OK;
    ctx->err = "ticket is not a two-phase call";
    return LB_ERR_INVALID_ARGUMENT;
  }
  if (!merged_ok && ctx->tp_release_cfg) ctx->tp_pause = ctx->tp_pause_calls;  // (failures go on: stay legacy)
  return finish_partial(ctx, *sl, merged_ok != 0);
}

int lb_gt_check(lb_ctx* ctx, uint32_t n, const uint8_t* partials576, int32_t* out_is_one) {
  if (!ctx || !out_is_one || (n && !partials576)) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  // (+ the combined product's 12 records for the round-program final exponentiation)
  const size_t need = (((size_t)n * LB_GT_BYTES + 255) & ~(size_t)255) + 256 + 12 * 64;
  if (ctx->gt_lp) LB_TRY(lp_ensure(ctx));
  if (need > ctx->aux_cap) {
    LB_HIP(hipStreamSynchronize(ctx->aux_stream));
    if (ctx->d_aux) LB_HIP(hipFree(ctx->d_aux));
    if (ctx->h_aux) LB_HIP(hipHostFree(ctx->h_aux));
    ctx->d_aux = nullptr;
    ctx->h_aux = nullptr;
    ctx->aux_cap = 0;
    const size_t cap = need < 16 * LB_GT_BYTES + 256 + 12 * 64 ? 16 * LB_GT_BYTES + 256 + 12 * 64 : need;
    if (hipMalloc(&ctx->d_aux, cap) != hipSuccess || hipHostMalloc(&ctx->h_aux, cap, hipHostMallocDefault) != hipSuccess) {
      ctx->err = "gt_check buffers";
      return LB_ERR_OUT_OF_MEMORY;
    }
    ctx->aux_cap = cap;
  }
  uint8_t* d_out = ctx->d_aux;
  uint8_t* d_in = ctx->d_aux + 256;
  if (n) {
    memcpy(ctx->h_aux + 256, partials576, (size_t)n * LB_GT_BYTES);
    LB_HIP(hipMemcpyAsync(d_in, ctx->h_aux + 256, (size_t)n * LB_GT_BYTES, hipMemcpyHostToDevice, ctx->aux_stream));
  }
  if (ctx->gt_lp) {
    // the product (one wave), then the final exponentiation as a round program on one
    // workgroup (~420 rounds) instead of the one-wave chain
    uint32_t* d_rec = reinterpret_cast<uint32_t*>(ctx->d_aux + 256 + (((size_t)n * LB_GT_BYTES + 255) & ~(size_t)255));
    hipLaunchKernelGGL(k_gt_prod, dim3(1), dim3(TPB), 0, ctx->aux_stream, n, (const uint8_t*)d_in, d_rec, d_out);
    LB_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_lp_final_lane, dim3(1), dim3(LB_LP_TPB), 0, ctx->aux_stream,
                       (const uint32_t*)(ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_FINAL_LANE].off), (const uint32_t*)d_rec,
                       d_out);
    LB_HIP(hipGetLastError());
  } else {
    hipLaunchKernelGGL(k_gt_check, dim3(1), dim3(TPB), 0, ctx->aux_stream, n, (const uint8_t*)d_in, d_out);
    LB_HIP(hipGetLastError());
  }
  LB_HIP(hipMemcpyAsync(ctx->h_aux, d_out, 2, hipMemcpyDeviceToHost, ctx->aux_stream));
  LB_HIP(hipStreamSynchronize(ctx->aux_stream));
  if (ctx->h_aux[1]) {
    ctx->err = "partial with a coefficient >= p";
    return LB_ERR_INVALID_ARGUMENT;
  }
  *out_is_one = ctx->h_aux[0] ? 1 : 0;
  return LB_OK;
}

int lb_poll(lb_ctx* ctx, uint64_t ticket, int32_t* out_done) {
  if (!ctx || !out_done) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  *out_done = 1;
  if (TwoPhaseRec* r = tp_find(ctx, ticket)) {
    if (!r->finished) {  // (lb_wait would first finish it with merged_ok = 0)
      *out_done = 0;
      return LB_OK;
    }
    if (r->rerun) ticket = r->rerun;
  }
  Slot* sl = slot_of_ticket(ctx, ticket);
  if (!sl) return LB_OK;  // retired
  // (a same-message package's phase 1 still running: sm_pump above found it unfinished;
  // in phase 2 its retries' end event decides)
  if (sl->partial_pending || (sl->sm.active && sl->sm.phase == 1)) {
    *out_done = 0;
    return LB_OK;
  }
  const hipError_t q = hipEventQuery(sl->done);
  if (q == hipErrorNotReady) {
    *out_done = 0;
    return LB_OK;
  }
  LB_HIP(q);
  return LB_OK;
}

int lb_wait(lb_ctx* ctx, uint64_t ticket, lb_verify_stats* stats) {
  if (!ctx) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  bool rerun = false;
  if (TwoPhaseRec* r = tp_find(ctx, ticket)) {
    // waited for without a combined verdict: as before, each request verified alone
    if (!r->finished) {
      const int rc = lb_verify_requests_finish(ctx, ticket, 0);
      if (rc != LB_OK) {
        if (TwoPhaseRec* r2 = tp_find(ctx, ticket)) r2->waited = true;
        return rc;
      }
    }
    TwoPhaseRec* r2 = tp_find(ctx, ticket);
    if (r2 && r2->failed) {  // the failed combine's re-run never ran: the outputs are not verdicts
      const uint64_t own = ticket;
      if (Slot* sl = slot_of_ticket(ctx, own)) LB_TRY(finish_slot(ctx, *sl));
      r2->waited = true;
      ctx->err = "two-phase call " + std::to_string(own) +
                 ": the combined check failed and its re-verification could not be submitted; its outputs are not "
                 "verdicts";
      return LB_ERR_DEVICE;
    }
    if (r2) r2->waited = true;
    if (r2 && r2->rerun) {
      ticket = r2->rerun;
      rerun = true;
    }
  }
  if (Slot* sl = slot_of_ticket(ctx, ticket)) LB_TRY(finish_slot(ctx, *sl));
  fill_stats(ctx, ticket, stats);
  // a re-run after a failed combined check: the shard's batch failed once and every request
  // was verified alone (worker.ts:74-85 counts that as one retry of the merged batch)
  if (rerun && stats) {
    stats->batch_retries = 1;
    stats->batch_sigs_success = 0;
  }
  return LB_OK;
}

int lb_verify_requests_device(lb_ctx* ctx, const lb_request_batch* b, uint8_t* d_valid, uint8_t* d_req_err,
                              uint8_t* d_set_status, lb_verify_stats* stats) {
  if (!ctx) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(validate_batch(ctx, b));
  if (!d_valid || !d_req_err) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  uint64_t t = 0;
  if (b->n_sets <= ctx->lp_max_sets && !(lp_lone_rule(ctx, b->n_sets) && !any_slot_busy(ctx))) {
    // latency path: the priority lane, beside any calls in flight
    LB_TRY(submit_device(ctx, ctx->prio(), b, d_valid, d_req_err, d_set_status, false, &t));
    return lb_wait(ctx, t, stats);
  }
  BorrowGuard g{ctx};
  LB_TRY(borrow_second_stream(ctx, g));
  LB_TRY(submit_device(ctx, ctx->slots[0], b, d_valid, d_req_err, d_set_status, false, &t));  // slot 0: DAG
  return lb_wait(ctx, t, stats);
}

int lb_verify_requests(lb_ctx* ctx, const lb_request_batch* b, uint8_t* out_valid, uint8_t* out_req_err,
                       uint8_t* out_set_status, lb_verify_stats* stats) {
  if (!ctx) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(validate_batch(ctx, b));
  if (!out_valid || !out_req_err) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  if (b->n_requests == 0) {
    if (stats) *stats = lb_verify_stats{0, 0, 0.0};
    return LB_OK;
  }
  uint64_t t = 0;
  if (b->n_sets <= ctx->lp_max_sets && !(lp_lone_rule(ctx, b->n_sets) && !any_slot_busy(ctx))) {
    // latency path: the priority lane, beside any calls in flight
    LB_TRY(submit_host(ctx, ctx->prio(), b, out_valid, out_req_err, out_set_status, false, &t));
    return lb_wait(ctx, t, stats);
  }
  BorrowGuard g{ctx};  // synchronous host API: slot 0 (two-stream DAG, lowest latency)
  LB_TRY(borrow_second_stream(ctx, g));
  LB_TRY(submit_host(ctx, ctx->slots[0], b, out_valid, out_req_err, out_set_status, false, &t));
  return lb_wait(ctx, t, stats);
}

int lb_verify_requests_priority_async(lb_ctx* ctx, const lb_request_batch* b, uint8_t* out_valid,
                                      uint8_t* out_req_err, uint8_t* out_set_status, uint64_t* out_ticket) {
  if (!ctx || !out_ticket) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(validate_batch(ctx, b));
  if (!out_valid || !out_req_err) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  return submit_host(ctx, ctx->prio(), b, out_valid, out_req_err, out_set_status, false, out_ticket);
}
// ---- helpers for small host-buffer calls ----------------------------------
static int upload(lb_ctx* ctx, Bump& ws, const void* src, size_t n, void** out) {
  char* d = ws.take<char>(n ? n : 1);
  if (n) LB_HIP(hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, ctx->stream));
  *out = d;
  return LB_OK;
}

int lb_hash_to_g2(lb_ctx* ctx, uint32_t n, const uint8_t* messages, uint8_t* out192) {
  if (!ctx || (n && (!messages || !out192))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (32 + sizeof(g2a) + 192) + 4096));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void* d_msg;
  LB_TRY(upload(ctx, ws, messages, (size_t)n * 32, &d_msg));
  g2a* d_h = ws.take<g2a>(n);
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 192);
  LB_LAUNCH(k_hash, blocks_for(n), TPB, n, (const uint8_t*)d_msg, d_h);
  LB_LAUNCH(k_g2a_serialize, blocks_for(n), TPB, n, (const g2a*)d_h, d_out);
  LB_HIP(hipMemcpyAsync(out192, d_out, (size_t)n * 192, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_decode_signatures(lb_ctx* ctx, uint32_t n, const uint8_t* sigs, const uint32_t* sig_off, uint8_t* out_status,
                         uint8_t* out192) {
  if (!ctx || (n && (!sigs || !sig_off || !out_status))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  for (uint32_t i = 0; i < n; i++)
    if (sig_off[i + 1] < sig_off[i]) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  const size_t nb = sig_off[n];
  LB_TRY(ensure_ws(ctx, nb + (size_t)n * (4 + sizeof(g2j) + 1 + 192) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_s, *d_o;
  LB_TRY(upload(ctx, ws, sigs, nb, &d_s));
  LB_TRY(upload(ctx, ws, sig_off, sizeof(uint32_t) * (n + 1), &d_o));
  g2j* d_sig = ws.take<g2j>(n);
  uint8_t* d_st = ws.take<uint8_t>(n);
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 192);
  LB_LAUNCH(k_decode_sigs, blocks_for(n), TPB, n, (const uint8_t*)d_s, (const uint32_t*)d_o, (const uint8_t*)nullptr,
            d_sig, d_st);
  LB_LAUNCH(k_g2_serialize, blocks_for(n), TPB, n, (const g2j*)d_sig, d_out);
  LB_HIP(hipMemcpyAsync(out_status, d_st, n, hipMemcpyDeviceToHost, ctx->stream));
  if (out192) LB_HIP(hipMemcpyAsync(out192, d_out, (size_t)n * 192, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_aggregate_pubkeys(lb_ctx* ctx, uint32_t n, const uint8_t* pks, uint8_t* out96, uint8_t* out_status) {
  if (!ctx || !out96 || (n && !pks)) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) {
    ctx->err = "EMPTY_AGGREGATE_ARRAY";
    return LB_ERR_INVALID_ARGUMENT;
  }
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * 96 + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void* d_p;
  LB_TRY(upload(ctx, ws, pks, (size_t)n * 96, &d_p));
  uint32_t off[2] = {0, n};
  void* d_off;
  LB_TRY(upload(ctx, ws, off, sizeof(off), &d_off));
  g1j* d_pk = ws.take<g1j>(1);
  uint8_t* d_st = ws.take<uint8_t>(1);
  uint8_t* d_out = ws.take<uint8_t>(96);
  const PkSource src{(const uint8_t*)d_p, nullptr, nullptr, 0};
  LB_LAUNCH(k_pubkeys_single, 1, TPB, 1u, src, (const uint32_t*)d_off, d_pk, d_st);
  LB_LAUNCH(k_pubkeys_agg, 1, TPB, 1u, src, (const uint32_t*)d_off, d_pk, d_st);
  LB_LAUNCH(k_g1_serialize, 1, TPB, 1u, (const g1j*)d_pk, d_out);
  uint8_t st = 0;
  LB_HIP(hipMemcpyAsync(out96, d_out, 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipMemcpyAsync(&st, d_st, 1, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  if (st == LB_ST_PK_INFINITY) st = LB_ST_OK;  // an infinite aggregate is a valid encoding (0x40...)
  if (out_status) *out_status = st;
  return LB_OK;
}

int lb_pubkeys_from_bytes(lb_ctx* ctx, uint32_t n, const uint8_t* pks, uint32_t pk_len, uint8_t* out96,
                          uint8_t* out_status) {
  if (!ctx || (n && (!pks || !out96 || !out_status)) || (pk_len != 48 && pk_len != 96)) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (pk_len + 96 + 1) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void* d_in;
  LB_TRY(upload(ctx, ws, pks, (size_t)n * pk_len, &d_in));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 96);
  uint8_t* d_st = ws.take<uint8_t>(n);
  LB_LAUNCH(k_pubkey_validate, blocks_for(n), TPB, n, (const uint8_t*)d_in, pk_len, d_out, d_st);
  LB_HIP(hipMemcpyAsync(out96, d_out, (size_t)n * 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipMemcpyAsync(out_status, d_st, n, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

// ---- device-resident pubkey table (index2pubkey mirror) ------------------------
int lb_pubkey_table_append(lb_ctx* ctx, uint32_t n, const uint8_t* pks, uint32_t pk_len, int32_t* out_bad_index) {
  if (!ctx || (n && !pks) || (pk_len != 48 && pk_len != 96)) return LB_ERR_INVALID_ARGUMENT;
  if (out_bad_index) *out_bad_index = -1;
  if (n == 0) return LB_OK;
  if ((uint64_t)ctx->table_n + n > 0x7fffffffu) {
    ctx->err = "pubkey table full";
    return LB_ERR_INVALID_ARGUMENT;
  }
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));  // calls in flight read the table
  const uint32_t need = ctx->table_n + n;
  if (need > ctx->table_cap) {
    uint64_t cap = (uint64_t)ctx->table_cap * 2;
    if (cap < need) cap = need;
    if (cap < 4096) cap = 4096;
    if (cap > 0x7fffffffu) cap = 0x7fffffffu;
    g1a* d = nullptr;
    if (hipMalloc(&d, sizeof(g1a) * cap) != hipSuccess) {
      ctx->err = "hipMalloc pubkey table failed";
      return LB_ERR_OUT_OF_MEMORY;
    }
    if (ctx->table_n)
      LB_HIP(hipMemcpyAsync(d, ctx->d_table, sizeof(g1a) * ctx->table_n, hipMemcpyDeviceToDevice, ctx->stream));
    LB_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->d_table) LB_HIP(hipFree(ctx->d_table));
    ctx->d_table = d;
    ctx->table_cap = (uint32_t)cap;
  }
  // decode straight into the table tail, in chunks that bound the staging workspace;
  // table_n only advances once every key decoded
  const uint32_t chunk = 1u << 20;
  std::vector<uint8_t> st;
  for (uint32_t first = 0; first < n; first += chunk) {
    const uint32_t m = n - first < chunk ? n - first : chunk;
    LB_TRY(ensure_ws(ctx, (size_t)m * (pk_len + 1) + 4096));
    Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
    void* d_in;
    LB_TRY(upload(ctx, ws, pks + (size_t)first * pk_len, (size_t)m * pk_len, &d_in));
    uint8_t* d_st = ws.take<uint8_t>(m);
    LB_LAUNCH(k_table_decode, blocks_for(m), TPB, m, (const uint8_t*)d_in, pk_len, ctx->d_table + ctx->table_n + first,
              d_st);
    st.resize(m);
    LB_HIP(hipMemcpyAsync(st.data(), d_st, m, hipMemcpyDeviceToHost, ctx->stream));
    LB_HIP(hipStreamSynchronize(ctx->stream));
    for (uint32_t i = 0; i < m; i++)
      if (st[i] != LB_ST_OK) {
        if (out_bad_index) *out_bad_index = (int32_t)(first + i);
        ctx->err = "pubkey fails PublicKey.fromBytes (bad encoding / not on curve)";
        return LB_ERR_INVALID_ARGUMENT;
      }
  }
  ctx->table_n = need;
  return LB_OK;
}

int lb_pubkey_table_size(const lb_ctx* ctx, uint32_t* out_n) {
  if (!ctx || !out_n) return LB_ERR_INVALID_ARGUMENT;
  *out_n = ctx->table_n;
  return LB_OK;
}

int lb_pubkey_table_truncate(lb_ctx* ctx, uint32_t n) {
  if (!ctx || n > ctx->table_n) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  ctx->table_n = n;
  return LB_OK;
}

int lb_pubkey_table_read(lb_ctx* ctx, uint32_t first, uint32_t n, uint8_t* out96) {
  if (!ctx || (n && !out96) || (uint64_t)first + n > ctx->table_n) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * 96 + 4096));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 96);
  LB_LAUNCH(k_g1a_serialize, blocks_for(n), TPB, n, (const g1a*)(ctx->d_table + first), d_out);
  LB_HIP(hipMemcpyAsync(out96, d_out, (size_t)n * 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_aggregate_pubkeys_indexed(lb_ctx* ctx, uint32_t n, const uint32_t* indices, uint8_t* out96,
                                 uint8_t* out_status) {
  if (!ctx || !out96 || (n && !indices)) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) {
    ctx->err = "EMPTY_AGGREGATE_ARRAY";
    return LB_ERR_INVALID_ARGUMENT;
  }
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * 4 + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void* d_idx;
  LB_TRY(upload(ctx, ws, indices, (size_t)n * 4, &d_idx));
  uint32_t off[2] = {0, n};
  void* d_off;
  LB_TRY(upload(ctx, ws, off, sizeof(off), &d_off));
  g1j* d_pk = ws.take<g1j>(1);
  uint8_t* d_st = ws.take<uint8_t>(1);
  uint8_t* d_out = ws.take<uint8_t>(96);
  const PkSource src{nullptr, (const uint32_t*)d_idx, ctx->d_table, ctx->table_n};
  LB_LAUNCH(k_pubkeys_single, 1, TPB, 1u, src, (const uint32_t*)d_off, d_pk, d_st);
  LB_LAUNCH(k_pubkeys_agg, 1, TPB, 1u, src, (const uint32_t*)d_off, d_pk, d_st);
  LB_LAUNCH(k_g1_serialize, 1, TPB, 1u, (const g1j*)d_pk, d_out);
  uint8_t st = 0;
  LB_HIP(hipMemcpyAsync(out96, d_out, 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipMemcpyAsync(&st, d_st, 1, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  if (st == LB_ST_PK_INFINITY) st = LB_ST_OK;  // an infinite aggregate is a valid encoding (0x40...)
  if (out_status) *out_status = st;
  return LB_OK;
}

// ---- signing roots -----------------------------------------------------------
static int signing_roots(lb_ctx* ctx, uint32_t n, uint32_t m, const uint8_t* in, size_t in_per_obj,
                         const uint8_t* domains, uint32_t dstride, uint8_t* out32) {
  if (!ctx || (n && (!in || !domains || !out32)) || (dstride != 0 && dstride != 32)) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  const size_t n_dom = dstride ? n : 1;
  LB_TRY(ensure_ws(ctx, (size_t)n * (in_per_obj + 32) + n_dom * 32 + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_in, *d_dom;
  LB_TRY(upload(ctx, ws, in, (size_t)n * in_per_obj, &d_in));
  LB_TRY(upload(ctx, ws, domains, n_dom * 32, &d_dom));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 32);
  if (m == 0)
    LB_LAUNCH(k_signing_root_att, blocks_for(n), TPB, n, (const uint8_t*)d_in, (const uint8_t*)d_dom, dstride, d_out);
  else
    LB_LAUNCH(k_signing_root_chunks, blocks_for(n), TPB, n, m, (const uint8_t*)d_in, (const uint8_t*)d_dom, dstride,
              d_out);
  LB_HIP(hipMemcpyAsync(out32, d_out, (size_t)n * 32, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_signing_roots_attestation(lb_ctx* ctx, uint32_t n, const uint8_t* data128, const uint8_t* domains,
                                 uint32_t domain_stride, uint8_t* out32) {
  return signing_roots(ctx, n, 0, data128, 128, domains, domain_stride, out32);
}

int lb_signing_roots_attestation_device(lb_ctx* ctx, uint32_t n, const uint8_t* d_data, const uint8_t* d_domains,
                                        uint32_t dstride, uint8_t* d_out) {
  if (!ctx || (n && (!d_data || !d_domains || !d_out)) || (dstride != 0 && dstride != 32))
    return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_LAUNCH(k_signing_root_att, blocks_for(n), TPB, n, d_data, d_domains, dstride, d_out);
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_signing_roots_chunks(lb_ctx* ctx, uint32_t n, uint32_t m, const uint8_t* chunks, const uint8_t* domains,
                            uint32_t domain_stride, uint8_t* out32) {
  if (m < 1 || m > 16) return LB_ERR_INVALID_ARGUMENT;
  return signing_roots(ctx, n, m, chunks, (size_t)m * 32, domains, domain_stride, out32);
}

int lb_aggregate_signatures(lb_ctx* ctx, uint32_t n, const uint8_t* sigs, const uint32_t* sig_off, uint8_t* out192,
                            int32_t* out_bad_index) {
  if (!ctx || !out192 || !out_bad_index || (n && (!sigs || !sig_off))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) {
    ctx->err = "EMPTY_AGGREGATE_ARRAY";
    return LB_ERR_INVALID_ARGUMENT;
  }
  for (uint32_t i = 0; i < n; i++)
    if (sig_off[i + 1] < sig_off[i]) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  const size_t nb = sig_off[n];
  LB_TRY(ensure_ws(ctx, nb + (size_t)n * (4 + sizeof(g2j) + 1) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_s, *d_o;
  LB_TRY(upload(ctx, ws, sigs, nb, &d_s));
  LB_TRY(upload(ctx, ws, sig_off, sizeof(uint32_t) * (n + 1), &d_o));
  g2j* d_sig = ws.take<g2j>(n);
  uint8_t* d_st = ws.take<uint8_t>(n);
  g2j* d_sum = ws.take<g2j>(1);
  uint8_t* d_out = ws.take<uint8_t>(192);
  LB_LAUNCH(k_decode_sigs, blocks_for(n), TPB, n, (const uint8_t*)d_s, (const uint32_t*)d_o, (const uint8_t*)nullptr,
            d_sig, d_st);
  LB_LAUNCH(k_jac_sum<fp2>, 1, 256, n, (const g2j*)d_sig, d_sum);
  LB_LAUNCH(k_g2_serialize, 1, TPB, 1u, (const g2j*)d_sum, d_out);
  std::vector<uint8_t> st(n);
  LB_HIP(hipMemcpyAsync(st.data(), d_st, n, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipMemcpyAsync(out192, d_out, 192, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  *out_bad_index = -1;
  for (uint32_t i = 0; i < n; i++)
    if (st[i] != LB_ST_OK) {
      *out_bad_index = (int32_t)i;
      break;
    }
  return LB_OK;
}

// Same-message jobs, batched (BlsMultiThreadWorkerPool.verifySignatureSetsSameMessage
// jobs: jobItemWorkReq sameMessage, jobItem.ts:64-86, the worker's verify of
// the aggregated set, index.ts:455-489, and the per-set retry of failed jobs,
// index.ts:473-484,557-568 / jobItemSameMessageToMultiSet, jobItem.ts:93-125).
// Phase 1 (sm_submit): every signature decoded + validated ONCE, pubkeys and
// signatures summed per job, every job's aggregated set verified as a 1-set
// request of ONE merged call.  Phase 2 (sm_complete, when the call retires and
// only if a job failed): the sets of the failed jobs, each its own 1-set
// request, through the same pipeline on the same slot -- signatures from the
// phase-1 decode (k_sm_retry_gather), pubkeys / messages from the phase-1
// uploads: nothing re-packed or re-uploaded but the retry index list.
}  // extern "C"

// phase-2 inputs: retry r = set rset[r] of job rjob[r] as a 1-set request
__global__ void __launch_bounds__(TPB) k_sm_retry_gather(uint32_t n, const uint32_t* __restrict__ rset,
                                                         const uint32_t* __restrict__ rjob,
                                                         const g2j* __restrict__ sig, const uint8_t* __restrict__ sst,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint32_t* __restrict__ pk_index, g2j* __restrict__ out_sig,
                                                         uint8_t* __restrict__ out_st, uint8_t* __restrict__ out_msg,
                                                         uint32_t* __restrict__ out_idx, uint32_t* __restrict__ out_req) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t i = rset[r], j = rjob[r];
  const g2j g = sig[i];
  uint8_t st = sst[i];
  // a 1-set request: core verify rejects the infinite signature (k_decode_sigs' single-set rule)
  if (st == LB_ST_OK && jac_is_inf(g)) st = LB_ST_ZERO_SIGNATURE;
  out_sig[r] = g;
  out_st[r] = st;
  for (int k = 0; k < 32; k++) out_msg[(size_t)r * 32 + k] = msgs[(size_t)j * 32 + k];
  // the set's key: its validator index, or row i of the package's 96-byte keys
  out_idx[r] = pk_index ? pk_index[i] : (i | LB_PK_ROW_FLAG);
  out_req[r] = r;
  if (r == n - 1) out_req[n] = n;
}

namespace {

int sm_validate(lb_ctx* ctx, const lb_same_message_batch* b) {
  const uint32_t nj = b->n_jobs, ns = b->n_sets;
  if (!b->job_offsets || !b->sig_offsets || !b->messages || !b->seed || (ns && !b->signatures) ||
      (ns && !b->pubkeys && !b->pubkey_indices)) {
    ctx->err = "null pointer in lb_same_message_batch";
    return LB_ERR_INVALID_ARGUMENT;
  }
  if (b->job_offsets[0] != 0 || b->job_offsets[nj] != ns || b->sig_offsets[0] != 0) {
    ctx->err = "job_offsets / sig_offsets must start at 0 (job_offsets end at n_sets)";
    return LB_ERR_INVALID_ARGUMENT;
  }
  for (uint32_t j = 0; j < nj; j++)
    if (b->job_offsets[j + 1] < b->job_offsets[j]) {
      ctx->err = "job_offsets not monotone";
      return LB_ERR_INVALID_ARGUMENT;
    }
  for (uint32_t i = 0; i < ns; i++)
    if (b->sig_offsets[i + 1] < b->sig_offsets[i]) {
      ctx->err = "sig_offsets not monotone";
      return LB_ERR_INVALID_ARGUMENT;
    }
  return LB_OK;
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// phase-2 device reserve: the retry pipeline over at most every set, its gathered inputs
size_t sm_phase2_bytes(const lb_ctx* ctx, uint32_t ns) {
  const size_t n = ns ? ns : 1;
  return pipeline_ws_bytes(ctx, ns, ns) + n * (2 * 4 + sizeof(g2j) + 1 + 32 + 4 + 4 + 2) + 16 * 256;
}

// Phase 1 on slot `sl` (already retired by the caller); the call stays busy
// until finish_slot, which runs sm_complete.
int sm_submit(lb_ctx* ctx, Slot& sl, const lb_same_message_batch* b, uint8_t* out_valid, uint8_t* out_job_fast) {
  const uint32_t nj = b->n_jobs, ns = b->n_sets;
  const bool by_index = b->pubkey_indices != nullptr;
  // mixed package (indices AND rows): rows of `pubkeys` named by flagged indices, as in
  // lb_request_batch (every row < n_rows is staged)
  size_t n_rows = 0;
  if (by_index && b->pubkeys)
    for (uint32_t i = 0; i < ns; i++) {
      const uint32_t j = b->pubkey_indices[i];
      if ((j & LB_PK_ROW_FLAG) && (size_t)(j & LB_PK_ROW_MASK) + 1 > n_rows) n_rows = (j & LB_PK_ROW_MASK) + 1;
    }
  const size_t sz_joff = sizeof(uint32_t) * (nj + 1), sz_pk = (size_t)ns * (by_index ? 4 : 96),
               sz_sigo = sizeof(uint32_t) * (ns + 1), sz_sig = b->sig_offsets[ns], sz_msg = (size_t)nj * 32,
               sz_seed = 32, sz_areq = sizeof(uint32_t) * (nj + 1), sz_asig = sizeof(uint32_t) * (nj + 1),
               sz_rows = n_rows * 96;
  const size_t in_bytes = al256(sz_joff) + al256(sz_pk) + al256(sz_sigo) + al256(sz_sig) + al256(sz_msg) +
                          al256(sz_seed) + al256(sz_areq) + al256(sz_asig) + al256(sz_rows);
  const size_t ns1 = ns ? ns : 1;
  const size_t res_bytes = 4 * al256(nj), retry_bytes = 2 * al256(4 * ns1) + 2 * al256(ns1);
  const size_t extra = ns1 * (sizeof(g2j) + 1) + (size_t)nj * (sizeof(g1j) + 1 + 96 + 192 + 1 + 2) + 16 * 256;
  LB_TRY(ensure_pin(ctx, sl, in_bytes + res_bytes + retry_bytes));
  // (+ a small package's decode records: 4 + 2 records, 5 flags and a status per signature)
  const size_t dec_bytes = ns <= LB_SM_DEC_MAX ? (size_t)ns * (6 * 64 + 5 * 4 + 1) + 6 * 256 : 0;
  LB_TRY(ensure_ws(ctx, sl, in_bytes + extra + pipeline_ws_bytes(ctx, nj, nj) + sm_phase2_bytes(ctx, ns) + dec_bytes));
  Bump ws{sl.d_ws, 0, sl.ws_cap};
  char* h = sl.h_pin;
  size_t ho = 0;
  auto stage = [&](const void* src, size_t n) {
    char* p = h + ho;
    if (n && src) memcpy(p, src, n);
    ho += al256(n);
    return p;
  };
  const uint32_t* h_joff = (const uint32_t*)stage(b->job_offsets, sz_joff);
  stage(by_index ? (const void*)b->pubkey_indices : (const void*)b->pubkeys, sz_pk);
  stage(b->sig_offsets, sz_sigo);
  stage(b->signatures, sz_sig);
  stage(b->messages, sz_msg);
  stage(b->seed, sz_seed);
  uint32_t* areq = (uint32_t*)stage(nullptr, sz_areq);
  uint32_t* asig = (uint32_t*)stage(nullptr, sz_asig);
  if (n_rows) stage(b->pubkeys, sz_rows);
  for (uint32_t j = 0; j <= nj; j++) {
    areq[j] = j;        // every job one request of one (aggregated) set
    asig[j] = 192 * j;  // Signature.aggregate(...).toBytes(uncompressed)
  }
  char* d_in = ws.take<char>(in_bytes);
  size_t o = 0;
  auto dptr = [&](size_t n) {
    char* p = d_in + o;
    o += al256(n);
    return p;
  };
  const uint32_t* d_joff = (const uint32_t*)dptr(sz_joff);
  const uint8_t* d_pks = (const uint8_t*)dptr(sz_pk);
  const uint32_t* d_sigo = (const uint32_t*)dptr(sz_sigo);
  const uint8_t* d_sigs = (const uint8_t*)dptr(sz_sig);
  const uint8_t* d_msgs = (const uint8_t*)dptr(sz_msg);
  const uint8_t* d_seed = (const uint8_t*)dptr(sz_seed);
  const uint32_t* d_areq = (const uint32_t*)dptr(sz_areq);
  const uint32_t* d_asig = (const uint32_t*)dptr(sz_asig);
  const uint8_t* d_rows = n_rows ? (const uint8_t*)dptr(sz_rows) : nullptr;
  g2j* d_sig = ws.take<g2j>(ns1);
  uint8_t* d_sst = ws.take<uint8_t>(ns1);
  g1j* d_jpk = ws.take<g1j>(nj);
  uint8_t* d_jpkst = ws.take<uint8_t>(nj);
  uint8_t* d_pk96 = ws.take<uint8_t>((size_t)nj * 96);
  uint8_t* d_sig192 = ws.take<uint8_t>((size_t)nj * 192);
  uint8_t* d_jbad = ws.take<uint8_t>(nj);
  uint8_t* d_valid = ws.take<uint8_t>(nj);
  uint8_t* d_err = ws.take<uint8_t>(nj);
  LB_TRY(begin_call(ctx, sl));
  LB_HIP(hipMemcpyAsync(d_in, h, in_bytes, hipMemcpyHostToDevice, sl.st[0]));
  if (ns && ns <= LB_SM_DEC_MAX && ctx->sm_lp_decode) {
    // a small package: each signature's decode as a round program on an 8-row workgroup (~540
    // rounds) instead of k_decode_sigs' one-lane chain (~4 ms); the same outputs and statuses
    LB_TRY(lp_ensure(ctx));
    uint32_t* d_dec_in = ws.take<uint32_t>((size_t)ns * 4 * 16);
    uint32_t* d_dec_fl = ws.take<uint32_t>((size_t)ns * 3);
    uint32_t* d_dec_out = ws.take<uint32_t>((size_t)ns * 2 * 16);
    uint32_t* d_dec_ofl = ws.take<uint32_t>((size_t)ns * 2);
    uint8_t* d_dec_pre = ws.take<uint8_t>(ns);
    if (ws.off > ws.cap) {
      ctx->err = "workspace overflow";
      return LB_ERR_OUT_OF_MEMORY;
    }
    LB_STAGE("sm_decode", 0, k_sm_dec_prep, blocks_for(ns, 256), 256u, ns, d_sigs, d_sigo, d_dec_in, d_dec_fl,
             d_dec_pre);
    LB_STAGE("sm_decode", 0, k_lp_dec, ns, LB_LP_DEC_ROWS * 16u, ctx->d_lp + LB_LP_PROGS[LB_LP_PROG_SIG_DECODE].off, ns,
             (const uint32_t*)d_dec_in, (const uint32_t*)d_dec_fl, d_dec_out, d_dec_ofl);
    LB_STAGE("sm_decode", 0, k_sm_dec_finish, blocks_for(ns, 256), 256u, ns, (const uint8_t*)d_dec_pre,
             (const uint32_t*)d_dec_in, (const uint32_t*)d_dec_fl, (const uint32_t*)d_dec_out,
             (const uint32_t*)d_dec_ofl, d_sig, d_sst, (const uint8_t*)nullptr);
  } else if (ns) {
    LB_STAGE("sm_decode", 0, k_decode_sigs, blocks_for(ns), TPB, ns, d_sigs, d_sigo, (const uint8_t*)nullptr, d_sig,
             d_sst);
  }
  const PkSource src{by_index ? d_rows : d_pks, by_index ? (const uint32_t*)d_pks : nullptr, ctx->d_table,
                     ctx->table_n};
  const uint32_t agg_grid = nj < 16384u ? nj : 16384u;
  LB_STAGE("sm_pubkeys", 0, k_pubkeys_single, blocks_for(nj), TPB, nj, src, d_joff, d_jpk, d_jpkst);
  LB_STAGE("sm_pubkeys_agg", 0, k_pubkeys_agg, agg_grid, TPB, nj, src, d_joff, d_jpk, d_jpkst);
  LB_STAGE("sm_aggregate", 0, k_same_message_agg, agg_grid, TPB, nj, d_joff, (const g2j*)d_sig, (const uint8_t*)d_sst,
           (const g1j*)d_jpk, d_pk96, d_sig192, d_jbad);
  LB_TRY(run_pipeline(ctx, sl, nj, nj, d_areq, d_pk96, nullptr, nullptr, d_msgs, d_sig192, d_asig, d_seed, d_valid,
                      d_err, nullptr, ws));
  char* h_res = h + in_bytes;
  LB_HIP(hipMemcpyAsync(h_res, d_valid, nj, hipMemcpyDeviceToHost, sl.st[0]));
  LB_HIP(hipMemcpyAsync(h_res + al256(nj), d_err, nj, hipMemcpyDeviceToHost, sl.st[0]));
  LB_HIP(hipMemcpyAsync(h_res + 2 * al256(nj), d_jbad, nj, hipMemcpyDeviceToHost, sl.st[0]));
  LB_HIP(hipMemcpyAsync(h_res + 3 * al256(nj), d_jpkst, nj, hipMemcpyDeviceToHost, sl.st[0]));
  SmState& m = sl.sm;
  m.active = true;
  m.phase = 1;
  m.by_index = by_index;
  m.nj = nj;
  m.ns = ns;
  m.out_valid = out_valid;
  m.out_job_fast = out_job_fast;
  m.h_joff = h_joff;
  m.h_res = (const uint8_t*)h_res;
  m.h_rset = (uint32_t*)(h_res + res_bytes);
  m.h_rout = (uint8_t*)(h_res + res_bytes + 2 * al256(4 * ns1));
  m.d_pks = d_pks;
  m.d_rows = d_rows;
  m.d_sig = d_sig;
  m.d_sst = d_sst;
  m.d_msgs = d_msgs;
  m.d_seed = d_seed;
  m.ws_off = ws.off;
  return end_call_async(ctx, sl);
}

// Progress of a same-message call.  Phase 1 done: verdicts of the jobs whose
// aggregate passed, and phase 2 -- the sets of the other jobs, each its own
// 1-set request -- enqueued on the same slot at once (sm_pump launches it from
// any later library call, so it need not wait for the caller's lb_wait).
// Phase 2 done: its verdicts.  block = false: return at once when the phase's
// work is still in flight.
int sm_advance_launch(lb_ctx* ctx, Slot& sl, bool block);

// One step of a same-message call; a failure ends the call (sm.active cleared) and
// stays on its slot for its own ticket's wait to report.
int sm_advance(lb_ctx* ctx, Slot& sl, bool block) {
  const int rc = sm_advance_launch(ctx, sl, block);
  if (rc != LB_OK) {
    sl.sm.active = false;
    sl.sm.phase = 0;
    sl.sm.err = rc;
    sl.sm.err_msg = ctx->err;
  }
  return rc;
}

int sm_advance_launch(lb_ctx* ctx, Slot& sl, bool block) {
  SmState& m = sl.sm;
  if (!m.active) return LB_OK;
  if (!block) {
    const hipError_t q = hipEventQuery(sl.done);
    if (q == hipErrorNotReady) return LB_OK;
    if (q != hipSuccess) LB_HIP(q);
  }
  LB_HIP(hipEventSynchronize(sl.done));
  const uint32_t nj = m.nj, ns = m.ns;
  if (m.phase == 2) {
    for (uint32_t r = 0; r < m.nr; r++)
      m.out_valid[m.h_rset[r]] = (m.h_rout[r] && m.h_rout[al256(ns) + r] == LB_REQ_OK) ? 1 : 0;
  } else {
    const uint8_t *v = m.h_res, *e = v + al256(nj), *jb = v + 2 * al256(nj), *pst = v + 3 * al256(nj);
    uint32_t fast_sets = 0, retried_jobs = 0, nr = 0;
    for (uint32_t j = 0; j < nj; j++) {
      // fast path: aggregated set valid, every signature validated, pubkeys aggregated
      const bool fast = v[j] && e[j] == LB_REQ_OK && !jb[j] && pst[j] == LB_ST_OK;
      if (m.out_job_fast) m.out_job_fast[j] = fast ? 1 : 0;
      const uint32_t a = m.h_joff[j], b = m.h_joff[j + 1];
      if (fast) {
        for (uint32_t i = a; i < b; i++) m.out_valid[i] = 1;
        fast_sets += b - a;
      } else if (b > a) {
        retried_jobs++;
        for (uint32_t i = a; i < b; i++) {
          m.h_rset[nr] = i;
          m.h_rset[(size_t)ns + nr] = j;
          nr++;
        }
      }
    }
    m.nr = nr;
    m.retried_jobs = retried_jobs;
    m.fast_sets = fast_sets;
    if (nr) {
      Bump ws{sl.d_ws, m.ws_off, sl.ws_cap};
      uint32_t* d_rset = ws.take<uint32_t>(2 * (size_t)ns);
      g2j* d_rsig = ws.take<g2j>(nr);
      uint8_t* d_rst = ws.take<uint8_t>(nr);
      uint8_t* d_rmsg = ws.take<uint8_t>((size_t)nr * 32);
      uint32_t* d_ridx = ws.take<uint32_t>(nr);
      uint32_t* d_rreq = ws.take<uint32_t>((size_t)nr + 1);
      uint8_t* d_rvalid = ws.take<uint8_t>(nr);
      uint8_t* d_rerr = ws.take<uint8_t>(nr);
      if (ws.off > ws.cap) {
        ctx->err = "workspace overflow";
        return LB_ERR_OUT_OF_MEMORY;
      }
      LB_HIP(hipMemcpyAsync(d_rset, m.h_rset, sizeof(uint32_t) * 2 * (size_t)ns, hipMemcpyHostToDevice, sl.st[0]));
      hipLaunchKernelGGL(k_sm_retry_gather, dim3(blocks_for(nr)), dim3(TPB), 0, sl.st[0], nr, (const uint32_t*)d_rset,
                         (const uint32_t*)(d_rset + ns), m.d_sig, m.d_sst, m.d_msgs,
                         m.by_index ? (const uint32_t*)m.d_pks : (const uint32_t*)nullptr, d_rsig, d_rst, d_rmsg,
                         d_ridx, d_rreq);
      LB_HIP(hipGetLastError());
      LB_TRY(run_pipeline(ctx, sl, nr, nr, d_rreq, m.by_index ? m.d_rows : m.d_pks, nullptr, d_ridx, d_rmsg, nullptr,
                          nullptr, m.d_seed, d_rvalid, d_rerr, nullptr, ws, nullptr, d_rsig, d_rst));
      LB_HIP(hipMemcpyAsync(m.h_rout, d_rvalid, nr, hipMemcpyDeviceToHost, sl.st[0]));
      LB_HIP(hipMemcpyAsync(m.h_rout + al256(ns), d_rerr, nr, hipMemcpyDeviceToHost, sl.st[0]));
      LB_TRY(end_call(ctx, sl));
      m.phase = 2;
      return LB_OK;
    }
  }
  // the package's worker bookkeeping (index.ts:557-568): jobs retried set by set,
  // sets verified by a passing aggregate (after phase 2's own merged-check stats)
  sl.h_stats[0] = m.retried_jobs;
  sl.h_stats[1] = m.fast_sets;
  m.active = false;
  m.phase = 0;
  return LB_OK;
}

// Launch the phase 2 of every same-message call whose phase 1 has completed
// (called from every async entry point and lb_wait: no blocking).
int sm_pump(lb_ctx* ctx) {
  for (int s = 0; s <= ctx->n_slots; s++) {
    Slot& sl = ctx->slots[s];
    // (another call's failure is not this caller's: it stays on that slot's ticket)
    if (sl.busy && sl.sm.active && sl.sm.phase == 1) (void)sm_advance(ctx, sl, false);
  }
  return LB_OK;
}

}  // namespace

extern "C" {

int lb_verify_same_message_batch_async(lb_ctx* ctx, const lb_same_message_batch* b, uint8_t* out_valid,
                                       uint8_t* out_job_fast, uint64_t* out_ticket) {
  if (!ctx || !b || !out_ticket || (b->n_sets && !out_valid)) return LB_ERR_INVALID_ARGUMENT;
  LB_TRY(sm_validate(ctx, b));
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(sm_pump(ctx));
  Slot& sl = next_async_slot(ctx);
  LB_TRY(finish_slot(ctx, sl));
  pick_streams(ctx, sl);
  if (b->n_jobs == 0) {  // nothing to verify: a call that completes at once
    LB_TRY(begin_call(ctx, sl));
    LB_TRY(end_call_async(ctx, sl));
    *out_ticket = sl.ticket;
    return LB_OK;
  }
  borrow_idle_stream(ctx, sl);
  LB_TRY(sm_submit(ctx, sl, b, out_valid, out_job_fast));
  *out_ticket = sl.ticket;
  return LB_OK;
}

// Synchronous form: slot 0 as the two-stream DAG (lowest latency).
int lb_verify_same_message_batch(lb_ctx* ctx, const lb_same_message_batch* b, uint8_t* out_valid,
                                 uint8_t* out_job_fast, lb_verify_stats* stats) {
  if (!ctx || !b || (b->n_sets && !out_valid)) return LB_ERR_INVALID_ARGUMENT;
  if (stats) *stats = lb_verify_stats{0, 0, 0.0};
  if (b->n_jobs == 0) return LB_OK;
  LB_TRY(sm_validate(ctx, b));
  LB_HIP(hipSetDevice(ctx->device));
  BorrowGuard g{ctx};
  LB_TRY(borrow_second_stream(ctx, g));
  Slot& sl = ctx->slots[0];
  LB_TRY(finish_slot(ctx, sl));
  pick_streams(ctx, sl);
  LB_TRY(sm_submit(ctx, sl, b, out_valid, out_job_fast));
  const uint64_t t = sl.ticket;
  LB_TRY(finish_slot(ctx, sl));
  fill_stats(ctx, t, stats);
  return LB_OK;
}

int lb_verify_same_message(lb_ctx* ctx, uint32_t n, const uint8_t* pks, const uint8_t* sigs, const uint32_t* sig_off,
                           const uint8_t* message, const uint8_t* seed, uint8_t* out_valid,
                           uint32_t* out_used_fast_path) {
  if (!ctx || (n && (!pks || !sigs || !sig_off || !message || !seed || !out_valid))) return LB_ERR_INVALID_ARGUMENT;
  if (out_used_fast_path) *out_used_fast_path = 0;
  if (n == 0) return LB_OK;
  const uint32_t job_off[2] = {0, n};
  lb_same_message_batch b{};
  b.n_jobs = 1;
  b.n_sets = n;
  b.job_offsets = job_off;
  b.pubkeys = pks;
  b.signatures = sigs;
  b.sig_offsets = sig_off;
  b.messages = message;
  b.seed = seed;
  uint8_t fast = 0;
  LB_TRY(lb_verify_same_message_batch(ctx, &b, out_valid, &fast, nullptr));
  if (out_used_fast_path) *out_used_fast_path = fast;
  return LB_OK;
}

int lb_pairing(lb_ctx* ctx, uint32_t n, const uint8_t* g1_96, const uint8_t* g2_192, uint8_t* out576) {
  if (!ctx || (n && (!g1_96 || !g2_192 || !out576))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (96 + 192 + 576) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d1, *d2;
  LB_TRY(upload(ctx, ws, g1_96, (size_t)n * 96, &d1));
  LB_TRY(upload(ctx, ws, g2_192, (size_t)n * 192, &d2));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 576);
  LB_LAUNCH(k_pairing, blocks_for(n), TPB, n, (const uint8_t*)d1, (const uint8_t*)d2, d_out);
  LB_HIP(hipMemcpyAsync(out576, d_out, (size_t)n * 576, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_batch_scalars(lb_ctx* ctx, const uint8_t* seed, uint32_t first, uint32_t n, uint64_t* out) {
  if (!ctx || !seed || (n && !out)) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * 8 + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void* d_seed;
  LB_TRY(upload(ctx, ws, seed, 32, &d_seed));
  uint64_t* d_out = ws.take<uint64_t>(n);
  LB_LAUNCH(k_scalars, blocks_for(n), TPB, (const uint8_t*)d_seed, first, n, d_out);
  LB_HIP(hipMemcpyAsync(out, d_out, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_g1_mul(lb_ctx* ctx, uint32_t n, const uint8_t* in96, const uint64_t* k, uint8_t* out96) {
  if (!ctx || (n && (!in96 || !k || !out96))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (96 * 2 + 8) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_in, *d_k;
  LB_TRY(upload(ctx, ws, in96, (size_t)n * 96, &d_in));
  LB_TRY(upload(ctx, ws, k, (size_t)n * 8, &d_k));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 96);
  LB_LAUNCH(k_g1_mul, blocks_for(n), TPB, n, (const uint8_t*)d_in, (const uint64_t*)d_k, d_out);
  LB_HIP(hipMemcpyAsync(out96, d_out, (size_t)n * 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_g2_mul(lb_ctx* ctx, uint32_t n, const uint8_t* in192, const uint64_t* k, uint8_t* out192) {
  if (!ctx || (n && (!in192 || !k || !out192))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (192 * 2 + 8) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_in, *d_k;
  LB_TRY(upload(ctx, ws, in192, (size_t)n * 192, &d_in));
  LB_TRY(upload(ctx, ws, k, (size_t)n * 8, &d_k));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 192);
  LB_LAUNCH(k_g2_mul, blocks_for(n), TPB, n, (const uint8_t*)d_in, (const uint64_t*)d_k, d_out);
  LB_HIP(hipMemcpyAsync(out192, d_out, (size_t)n * 192, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

// sum_i (a_i + b_i lambda) P_i through the merged check's bucket MSM (k_msm.hip),
// a_i / b_i = the low / high 32 bits of raw[i]: the MSM alone, for tests.
int lb_g2_msm(lb_ctx* ctx, uint32_t n, const uint8_t* in192, const uint64_t* raw, uint8_t* out192) {
  if (!ctx || !out192 || (n && (!in192 || !raw))) return LB_ERR_INVALID_ARGUMENT;
  if (n > (1u << 28)) {
    ctx->err = "lb_g2_msm: too many points";
    return LB_ERR_INVALID_ARGUMENT;
  }
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  const uint32_t ns = n ? n : 1;
  const size_t n_ent = 2 * (size_t)ns * LB_MSM_W, max_chunks = n_ent / LB_MSM_T + LB_MSM_BUCKETS;
  LB_TRY(ensure_ws(ctx, (size_t)ns * (192 + 8 + sizeof(g2j) + 1) + 2 * n_ent * 4 + max_chunks * sizeof(g2j) +
                            (LB_MSM_BUCKETS + LB_MSM_POS) * sizeof(g2j) + 4 * (LB_MSM_BUCKETS + 1) * 4 + 64 * 256));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_in = nullptr, *d_raw = nullptr;
  if (n) {
    LB_TRY(upload(ctx, ws, in192, (size_t)n * 192, &d_in));
    LB_TRY(upload(ctx, ws, raw, (size_t)n * 8, &d_raw));
  }
  g2j* d_pts = ws.take<g2j>(ns);
  uint8_t* d_st = ws.take<uint8_t>(ns);
  uint32_t* d_req = ws.take<uint32_t>(2);
  uint32_t* d_keys = ws.take<uint32_t>(n_ent);
  uint32_t* d_sorted = ws.take<uint32_t>(n_ent);
  uint32_t* d_hist = ws.take<uint32_t>(4 * (LB_MSM_BUCKETS + 1));
  g2j* d_csum = ws.take<g2j>(max_chunks);
  g2j* d_bsum = ws.take<g2j>(LB_MSM_BUCKETS);
  g2j* d_G = ws.take<g2j>(LB_MSM_POS);
  g2a* d_S = ws.take<g2a>(1);
  uint8_t* d_out = ws.take<uint8_t>(192);
  if (ws.off > ws.cap) {
    ctx->err = "workspace overflow";
    return LB_ERR_OUT_OF_MEMORY;
  }
  uint32_t* d_off = d_hist + (LB_MSM_BUCKETS + 1);
  uint32_t* d_coff = d_off + (LB_MSM_BUCKETS + 1);
  uint32_t* d_cur = d_coff + (LB_MSM_BUCKETS + 1);
  const uint32_t req[2] = {0, n};
  LB_HIP(hipMemcpyAsync(d_req, req, sizeof(req), hipMemcpyHostToDevice, ctx->stream));
  LB_HIP(hipMemsetAsync(d_hist, 0, (LB_MSM_BUCKETS + 1) * sizeof(uint32_t), ctx->stream));
  if (n) {
    LB_LAUNCH(k_msm_load, blocks_for(n), TPB, n, (const uint8_t*)d_in, d_pts, d_st);
    LB_LAUNCH(k_msm_scalars, 1u, TPB, 1u, (const uint32_t*)d_req, (const uint8_t*)nullptr, (const uint64_t*)d_raw,
              (const g2j*)d_pts, (const uint8_t*)d_st, (const uint8_t*)nullptr, d_keys, d_hist);
  }
  LB_LAUNCH(k_msm_scan, 1u, 1024u, (const uint32_t*)d_hist, d_off, d_coff, d_cur, LB_MSM_T);
  if (n) LB_LAUNCH(k_msm_scatter, blocks_for((uint32_t)n_ent, 256), 256u, (uint32_t)n_ent, (const uint32_t*)d_keys,
                   (const uint32_t*)d_off, d_cur, d_sorted);
  LB_LAUNCH(k_msm_chunks, blocks_for((uint32_t)max_chunks), TPB, (uint32_t)max_chunks, (const uint32_t*)d_off,
            (const uint32_t*)d_coff, (const uint32_t*)d_sorted, (const g2j*)d_pts, d_csum, LB_MSM_T);
  LB_LAUNCH(k_msm_buckets, blocks_for(LB_MSM_BUCKETS * LB_MSM_BLANES), TPB, (const uint32_t*)d_coff,
            (const g2j*)d_csum, d_bsum, LB_MSM_BLANES);
  LB_LAUNCH(k_msm_bits<LB_MSM_BITS_TPB>, LB_MSM_POS, LB_MSM_BITS_TPB, (const g2j*)d_bsum, d_G);
  LB_LAUNCH(k_msm_final, 1u, TPB, (const g2j*)d_G, d_S);
  LB_LAUNCH(k_g2a_serialize, 1u, TPB, 1u, (const g2a*)d_S, d_out);
  LB_HIP(hipMemcpyAsync(out192, d_out, 192, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

// Round program on n instances, one workgroup each (tests, timing): prog_words
// == nullptr runs the embedded program `prog` (LB_LP_PROG_*), else the caller's
// encoded program (lodestar_amd/lpgen) of n_words words.  in16: n x n_in records
// of 16 words (canonical Montgomery limbs), in_flags: n x n_inflag words; out16:
// n x n_out records, out_flags: n x n_outflag words; *out_ms: kernel time;
// stamps (optional): s_memtime after each round of instance 0.
static int lp_program_run(lb_ctx* ctx, const uint32_t* d_prog, uint32_t n, uint32_t n_in, uint32_t n_inflag,
                          uint32_t n_out, uint32_t n_outflag, uint32_t n_rounds, const uint32_t* in16,
                          const uint32_t* in_flags, uint32_t* out16, uint32_t* out_flags, float* out_ms,
                          uint64_t* stamps, Bump& ws) {
  const size_t in_w = (size_t)n * n_in * 16, fl_w = (size_t)n * n_inflag + 1, out_w = (size_t)n * n_out * 16,
               ofl_w = (size_t)n * n_outflag + 1;
  void* d_in = nullptr;
  LB_TRY(upload(ctx, ws, in16, in_w * 4, &d_in));
  uint32_t* d_fl = ws.take<uint32_t>(fl_w);
  if (n_inflag) LB_HIP(hipMemcpyAsync(d_fl, in_flags, (fl_w - 1) * 4, hipMemcpyHostToDevice, ctx->stream));
  uint32_t* d_out = ws.take<uint32_t>(out_w);
  uint32_t* d_ofl = ws.take<uint32_t>(ofl_w);
  unsigned long long* d_st = stamps ? ws.take<unsigned long long>((size_t)(n_rounds + 1) * LB_LP_STAMPS) : nullptr;
  if (ws.off > ws.cap) {
    ctx->err = "workspace overflow";
    return LB_ERR_OUT_OF_MEMORY;
  }
  hipEvent_t e0, e1;
  LB_HIP(hipEventCreate(&e0));
  LB_HIP(hipEventCreate(&e1));
  LB_HIP(hipEventRecord(e0, ctx->stream));
  LB_LAUNCH(k_lp_program, n, LB_LP_TPB, d_prog, n, (const uint32_t*)d_in, n_in * 16u, (const uint32_t*)d_fl, n_inflag,
            d_out, n_out * 16u, d_ofl, n_outflag, d_st);
  LB_HIP(hipEventRecord(e1, ctx->stream));
  LB_HIP(hipMemcpyAsync(out16, d_out, out_w * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (n_outflag) LB_HIP(hipMemcpyAsync(out_flags, d_ofl, (ofl_w - 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (stamps)
    LB_HIP(hipMemcpyAsync(stamps, d_st, (size_t)n_rounds * LB_LP_STAMPS * 8, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (out_ms) *out_ms = ms;
  return LB_OK;
}

int lb_lp_program_run(lb_ctx* ctx, uint32_t prog, const uint32_t* prog_words, size_t n_words, uint32_t n,
                      const uint32_t* in16, const uint32_t* in_flags, uint32_t* out16, uint32_t* out_flags,
                      float* out_ms, uint64_t* stamps) {
  if (!ctx || n == 0 || !in16 || !out16) return LB_ERR_INVALID_ARGUMENT;
  if (!prog_words && prog >= LB_LP_NPROGS) return LB_ERR_INVALID_ARGUMENT;
  // (the wide merged-check programs are compiled for k_lp_mtail's LB_LP_MTAIL_ROWS rows, more
  // than k_lp_program's workgroup runs)
  if (!prog_words && LB_LP_MTAIL_ROWS > LB_LP_ROWS &&
      (prog == LB_LP_PROG_MTAIL_CHECK_WIDE || prog == LB_LP_PROG_MTAIL_PARTIAL_WIDE))
    return LB_ERR_INVALID_ARGUMENT;
  if (prog_words && (n_words < LB_LP_HDR || prog_words[0] != 0x4C500004u)) return LB_ERR_INVALID_ARGUMENT;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  const uint32_t* hw = prog_words ? prog_words : lb_lp_blob + LB_LP_PROGS[prog].off;
  const uint32_t n_rounds = hw[1], n_in = hw[5], n_inflag = hw[6], n_out = hw[7], n_outflag = hw[8];
  if ((n_inflag && !in_flags) || (n_outflag && !out_flags)) return LB_ERR_INVALID_ARGUMENT;
  const size_t io = 4 * ((size_t)n * (n_in + n_out) * 16 + (size_t)n * (n_inflag + n_outflag) + 2) +
                    8 * (size_t)(n_rounds + 1) * LB_LP_STAMPS;
  LB_TRY(ensure_ws(ctx, io + (prog_words ? 4 * n_words : 0) + 16384));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  const uint32_t* d_prog;
  if (prog_words) {
    void* d = nullptr;
    LB_TRY(upload(ctx, ws, prog_words, n_words * 4, &d));
    d_prog = (const uint32_t*)d;
  } else {
    LB_TRY(lp_ensure(ctx));
    d_prog = ctx->d_lp + LB_LP_PROGS[prog].off;
  }
  return lp_program_run(ctx, d_prog, n, n_in, n_inflag, n_out, n_outflag, n_rounds, in16, in_flags, out16, out_flags,
                        out_ms, stamps, ws);
}

int lb_set_latency_path(lb_ctx* ctx, uint32_t max_sets) {
  if (!ctx) return LB_ERR_INVALID_ARGUMENT;
  // (k_lp_verify's product tree has LB_LP_TREE_LEVELS levels of arrival counters: a
  // request longer than 2^levels sets would count past them)
  ctx->lp_max_sets = max_sets < (1u << LB_LP_TREE_LEVELS) ? max_sets : (1u << LB_LP_TREE_LEVELS);
  ctx->lp_explicit = true;
  return LB_OK;
}

int lb_sk_to_pk(lb_ctx* ctx, uint32_t n, const uint8_t* sk32, uint8_t* out96) {
  if (!ctx || (n && (!sk32 || !out96))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (32 + 96) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void* d_k;
  LB_TRY(upload(ctx, ws, sk32, (size_t)n * 32, &d_k));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 96);
  LB_LAUNCH(k_sk_to_pk, blocks_for(n), TPB, n, (const uint8_t*)d_k, d_out);
  LB_HIP(hipMemcpyAsync(out96, d_out, (size_t)n * 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

int lb_sign(lb_ctx* ctx, uint32_t n, const uint8_t* sk32, const uint8_t* messages, uint8_t* out96) {
  if (!ctx || (n && (!sk32 || !messages || !out96))) return LB_ERR_INVALID_ARGUMENT;
  if (n == 0) return LB_OK;
  LB_HIP(hipSetDevice(ctx->device));
  LB_TRY(helper_slot(ctx));
  LB_TRY(ensure_ws(ctx, (size_t)n * (32 + 32 + 96) + 8192));
  Bump ws{ctx->slots[0].d_ws, 0, ctx->slots[0].ws_cap};
  void *d_k, *d_m;
  LB_TRY(upload(ctx, ws, sk32, (size_t)n * 32, &d_k));
  LB_TRY(upload(ctx, ws, messages, (size_t)n * 32, &d_m));
  uint8_t* d_out = ws.take<uint8_t>((size_t)n * 96);
  LB_LAUNCH(k_sign, blocks_for(n), TPB, n, (const uint8_t*)d_k, (const uint8_t*)d_m, d_out);
  LB_HIP(hipMemcpyAsync(out96, d_out, (size_t)n * 96, hipMemcpyDeviceToHost, ctx->stream));
  LB_HIP(hipStreamSynchronize(ctx->stream));
  return LB_OK;
}

}  // extern "C"
