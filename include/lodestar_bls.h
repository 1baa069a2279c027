/*
 * lodestar_bls.h -- C ABI of the MI355X-native BLS12-381 signature-set verifier.
 *
 * This is the drop-in boundary for Lodestar's BLS hot path
 * (packages/beacon-node/src/chain/bls).  Every entry point takes plain
 * pointers and sizes; no torch or HIP types cross the boundary.  Lodestar binds
 * it through the N-API addon lodestar_amd/napi/addon.cc.
 *
 * Reference interfaces replaced (paths relative to packages/beacon-node/src/):
 *   lb_verify_requests      <- worker verifyManySignatureSets(BlsWorkReq[]) -> BlsWorkResult
 *                              chain/bls/multithread/worker.ts:30-108, types.ts:8-39,
 *                              with verifySignatureSetsMaybeBatch semantics (chain/bls/maybeBatch.ts:16-46)
 *                              and main-thread pubkey aggregation fused in
 *                              (chain/bls/utils.ts:6-21, chain/bls/multithread/jobItem.ts:55-63)
 *   lb_verify_same_message  <- BlsMultiThreadWorkerPool.verifySignatureSetsSameMessage job path:
 *                              jobItemWorkReq sameMessage (jobItem.ts:64-86) + retry
 *                              (index.ts:473-484,557-568, jobItem.ts:93-125); also
 *                              BlsSingleThreadVerifier.verifySignatureSetsSameMessage (singleThread.ts:37-81)
 *   lb_aggregate_pubkeys    <- bls.PublicKey.aggregate(pks).toBytes(uncompressed)
 *                              (chain/bls/utils.ts:13, jobItem.ts:59,80)
 *   lb_aggregate_signatures <- Signature.fromBytes(validate) x n + bls.Signature.aggregate(sigs).toBytes()
 *                              (jobItem.ts:73,81)
 *   lb_create / lb_destroy  <- BlsMultiThreadWorkerPool constructor / close() (index.ts:132-153,244-265)
 *   lb_verify_requests_partial_async .. lb_gt_check  <- the pool's fan-out over workers
 *                              (index.ts:191-205) as a multi-GPU combine of Fp12 partials
 *   lb_verify_same_message_batch <- every same-message job of a worker package
 *                              (jobItem.ts:64-125, index.ts:455-489,557-568)
 *
 * The Lodestar-side binding is the N-API addon lodestar_amd/napi/addon.cc
 * (INTEGRATION.md).
 * Threading: a context is bound to one GPU and is not thread-safe; use one
 * context per host submission thread (one process per GPU for multi-GPU).
 */
#ifndef LODESTAR_BLS_H
#define LODESTAR_BLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (return values) ------------------------------------- */
#define LB_OK 0
#define LB_ERR_INVALID_ARGUMENT (-1) /* API misuse: NULL pointer, bad offsets  */
#define LB_ERR_DEVICE (-2)           /* HIP runtime failure (maps to Promise rejection, index.ts:503-512) */
#define LB_ERR_NO_DEVICE (-3)        /* no GPU / bad ordinal                      */
#define LB_ERR_OUT_OF_MEMORY (-4)
#define LB_ERR_RESOURCES (-5)        /* lb_create: more hardware queues than the scratch reservation allows;
                                        lb_verify_requests_partial_async: 256 unfinished two-phase calls */

/* ---- per-request error codes (lb_verify_requests out_request_error) ----- */
#define LB_REQ_OK 0
#define LB_REQ_EMPTY_AGGREGATE 1 /* aggregate set with zero pubkeys: the reference REJECTS
                                    the job (EMPTY_AGGREGATE_ARRAY thrown in jobItemWorkReq,
                                    index.ts:403-409) instead of returning false */
#define LB_REQ_BAD_PUBKEY 2      /* pubkey bytes that PublicKey.fromBytes would throw on
                                    (worker.ts:110-116 -> the worker call rejects) */

/* ---- per-set decode status (optional outputs) -------------------------- */
#define LB_SET_OK 0
#define LB_SET_BAD_ENCODING 1
#define LB_SET_NOT_ON_CURVE 2
#define LB_SET_NOT_IN_GROUP 3
#define LB_SET_PK_INFINITY 4
#define LB_SET_EMPTY_AGGREGATE 5

/* Sizes */
#define LB_PUBKEY_BYTES 96      /* uncompressed affine G1 (PointFormat.uncompressed, index.ts:144) */
#define LB_PUBKEY_COMPRESSED 48
#define LB_SIG_COMPRESSED 96
#define LB_SIG_UNCOMPRESSED 192
#define LB_MESSAGE_BYTES 32
#define LB_SEED_BYTES 32
#define LB_GT_BYTES 576 /* an Fp12 value: 12 x 48-byte big-endian Fp */

typedef struct lb_ctx lb_ctx;

/* Create a context on HIP device `device` (one per process per GPU). */
int lb_create(int device, lb_ctx** out_ctx);
/* A latency-lane context on the same GPU: one slot plus the priority lane, no CU-masked
 * streams.  A host that must never make a priority call wait behind its submission
 * thread's staging of throughput packages (the reference verifies verifyOnMainThread sets
 * at once and unshifts priority jobs, BN/chain/bls/multithread/index.ts:174-187,544-555)
 * drives lb_verify_requests_priority_async on this context from a thread of its own and
 * calls lb_mark_priority on the throughput context, whose calls then leave the reserved
 * CUs free (LB_PRIO_CUS).  Its pubkey table is its own: append the same keys to both. */
int lb_create_lane(int device, lb_ctx** out_ctx);
/* Mark the priority lane in use now (LB_PRIO_DYN: calls submitted within LB_PRIO_HOLD_MS
 * take the CU-masked streams).  The one entry point that may be called on a context
 * while another thread uses it. */
int lb_mark_priority(lb_ctx* ctx);
/* Release device memory and streams.  Safe on NULL. */
int lb_destroy(lb_ctx* ctx);
/* Human-readable message for the last error on this context (never NULL); with
 * ctx == NULL, why the last lb_create failed. */
const char* lb_last_error(const lb_ctx* ctx);
/* Calls the context keeps in flight on the async entry points (one per HIP hardware
 * queue of the process: GPU_MAX_HW_QUEUES, 4 by default, up to 16; LB_SLOTS overrides):
 * the capacity a host keeps busy (the pool's worker count, multithread/index.ts:47).
 * lb_create refuses GPU_MAX_HW_QUEUES > 16 with LB_ERR_RESOURCES: every queue reserves
 * scratch for the largest private segment at full occupancy (lb_scratch_per_queue). */
int lb_slots(const lb_ctx* ctx);
/* HIP hardware queues the context opens: its plain streams (pooled into at most
 * GPU_MAX_HW_QUEUES queues), its CU-masked streams (one queue each) and its
 * high-priority streams (priority lane, lb_gt_check's aux stream).  lb_create prices
 * all of them against the scratch budget (LB_SCRATCH_BUDGET_GB, default that of the
 * largest configuration seen to run: 20 queues at 3,328 private bytes per lane) and
 * refuses a configuration above it with LB_ERR_RESOURCES. */
int lb_hw_queues(const lb_ctx* ctx);
/* Distinct streams the last submitted verify call runs on (2: the two-stream DAG). */
int lb_last_call_streams(const lb_ctx* ctx);
/* Clock stamps of the last retired latency-path call (diagnostics): [0] s_memrealtime
 * (100 MHz) and [1] s_memtime (shader clock) when its first workgroup started, [2] / [3]
 * when request 0's verdict was written -- the kernel's own duration and the shader clock
 * it ran at, apart from any wait before its dispatch. */
int lb_last_latency_clocks(const lb_ctx* ctx, uint64_t* out4);
/* Number of visible HIP devices (0 when none). */
int lb_device_count(void);
/* Scratch one hardware queue reserves for the library's kernels: the largest
 * private segment per lane (*out_lane_bytes, optional) x 64 lanes x 32 waves per
 * CU x CUs (*out_bytes). */
int lb_scratch_per_queue(int device, uint64_t* out_bytes, uint32_t* out_lane_bytes);
/* Calls (lb_verify_requests*, same-message packages' aggregated sets) of at most
 * max_sets sets run the latency path: one workgroup per set executing the
 * verification as a round program of row-cooperative Fp products (~2 ms for one
 * set instead of ~17 ms), each request verified on its own; larger calls run the
 * throughput pipeline (merged check, bucket MSM, step-major Miller accumulation).
 * Default 1024 (LB_LP_MAX); 0 disables it.  The reference's analogue is the
 * main-thread path for latency-critical callers (BN/chain/bls/multithread/index.ts:174-187). */
int lb_set_latency_path(lb_ctx* ctx, uint32_t max_sets);

/*
 * A batch of verification requests.  A request is one BlsWorkReq (one
 * verifySignatureSets job of <= 128 sets); it gets ONE verdict = the AND over
 * its sets, exactly as verifySignatureSetsMaybeBatch returns it:
 *   - 0 sets                 -> false ("Empty signature set" caught)
 *   - any signature that fails Signature.fromBytes(validate=true) -> false
 *   - infinite (aggregated) pubkey -> false
 *   - 1 set: core verify (pubkey G1 check, infinite signature -> false)
 *   - >= 2 sets: random-scalar batch verification with 2^64 possible scalars
 *     per set, drawn from the deterministic DRBG
 *       w_i = LE64(SHA-256(seed || LE32(i))[0..8]) (0 -> 1),
 *       r_i = (w_i mod 2^32) + (w_i >> 32) * lambda (mod r), lambda = -x^2,
 *     i = the set's index in this call (blst draws 8 random bytes per set; the
 *     lambda split lets the GPU multiply with two 32-bit halves, GLV).
 *   Requests that are not already false are first checked together (one merged
 *   product, the worker's merged batch, worker.ts:41-96); each request is
 *   re-verified alone only when the merged check fails, so a merged failure
 *   never changes any request's verdict.
 * Set i's pubkeys are pubkeys[pk_offsets[i] .. pk_offsets[i+1]) (96-byte
 * uncompressed each); more than one -> aggregated on the GPU (the reference
 * aggregates on the main thread before dispatch).
 */
typedef struct {
  uint32_t n_requests;
  uint32_t n_sets;
  const uint32_t* request_offsets; /* n_requests + 1, sets of request k: [off[k], off[k+1]) */
  const uint8_t* request_batchable; /* n_requests, opts.batchable (may be NULL)              */
  const uint8_t* pubkeys;          /* pk_offsets[n_sets] x 96 bytes                          */
  const uint32_t* pk_offsets;      /* n_sets + 1 (NULL => exactly one pubkey per set)        */
  const uint8_t* messages;         /* n_sets x 32 bytes (signing roots)                      */
  const uint8_t* signatures;       /* concatenated signature bytes                           */
  const uint32_t* sig_offsets;     /* n_sets + 1 byte offsets into signatures                */
  const uint8_t* seed;             /* 32 bytes of batch randomness seed                      */
  /* Optional (NULL => use `pubkeys`): pk_offsets[n_sets] (or n_sets) u32 validator
   * indices into the context's device-resident pubkey table (lb_pubkey_table_append);
   * `pubkeys` is then ignored and may be NULL.  An index >= the table size makes
   * its request LB_REQ_BAD_PUBKEY (the reference would index index2pubkey out of range).
   * Mixed packages (e.g. a capella block: validator-index keys plus the BLS-change
   * keys that are not in the table): with BOTH pubkey_indices and pubkeys given, an
   * entry with LB_PK_ROW_FLAG set names row (entry & LB_PK_ROW_MASK) of `pubkeys`;
   * with LB_PK_ROW48_FLAG also set, that 96-byte row holds a 48-byte COMPRESSED
   * encoding in its first 48 bytes (decompressed on the GPU: a @chainsafe/bls
   * PublicKey serialized compressed, PublicKey.fromBytes(48 B) semantics). */
  const uint32_t* pubkey_indices;
} lb_request_batch;
#define LB_PK_ROW_FLAG 0x80000000u
#define LB_PK_ROW48_FLAG 0x40000000u
#define LB_PK_ROW_MASK 0x3fffffffu

typedef struct {
  uint32_t batch_retries;      /* the DEVICE's merged check: 1 when it failed and requests were
                                  re-verified alone, else 0 (0 below LB_MERGE_MIN requests).  The
                                  reference counts per 16-request chunk of batchable requests
                                  (worker.ts:54,75); the hosts derive that figure from the verdicts
                                  (verifier.worker_batch_stats, js workerBatchStats) for the metric */
  uint32_t batch_sigs_success; /* sets verified inside a passing merged check (worker.ts:71)   */
  double device_ms;            /* wall time of the device pipeline for this call              */
} lb_verify_stats;

/*
 * Host-buffer entry point: stages inputs through pinned memory onto the
 * device, runs the pipeline, copies verdicts back.  out_request_valid[k] is
 * 1/0; out_request_error[k] is LB_REQ_*; out_set_status (optional, n_sets) is
 * LB_SET_*; stats optional.  Returns LB_OK or a negative LB_ERR_*.
 */
int lb_verify_requests(lb_ctx* ctx, const lb_request_batch* batch, uint8_t* out_request_valid,
                       uint8_t* out_request_error, uint8_t* out_set_status, lb_verify_stats* stats);

/*
 * Device-resident variant: every pointer in `batch` and every output pointer
 * is device memory already resident in HBM (used by bench.py to time the
 * kernels without PCIe).  Runs on the context's stream and synchronises it
 * before returning.
 */
int lb_verify_requests_device(lb_ctx* ctx, const lb_request_batch* batch, uint8_t* d_out_request_valid,
                              uint8_t* d_out_request_error, uint8_t* d_out_set_status, lb_verify_stats* stats);

/*
 * Asynchronous variants: enqueue the call and return a ticket; lb_wait(ticket)
 * blocks until it is complete and reports THAT call's stats.  One call is in
 * flight per slot (LB_SLOTS, default 4 = one per HIP hardware queue, each with
 * its own stream, workspace and pinned staging), so the tail of one call
 * overlaps the per-set stages of the next -- the way the reference pool keeps
 * several worker packages in flight (index.ts:362-519).  Submitting more calls
 * than slots first waits for the oldest call of the reused slot.
 *   lb_verify_requests_device_async: every pointer is device memory (bench.py).
 *   lb_verify_requests_async: host buffers, staged through the slot's pinned
 *     buffer; the outputs are written when the call retires (lb_wait, or a
 *     later call reusing the slot).  The caller keeps every buffer valid until
 *     lb_wait returns.
 */
int lb_verify_requests_device_async(lb_ctx* ctx, const lb_request_batch* batch, uint8_t* d_out_request_valid,
                                    uint8_t* d_out_request_error, uint8_t* d_out_set_status, uint64_t* out_ticket);
int lb_verify_requests_async(lb_ctx* ctx, const lb_request_batch* batch, uint8_t* out_request_valid,
                             uint8_t* out_request_error, uint8_t* out_set_status, uint64_t* out_ticket);
/* The priority lane: like lb_verify_requests_async, but on a slot of its own whose
 * stream runs at the device's highest priority, outside the round robin of the
 * calls in flight -- for priority jobs and verifyOnMainThread callers (the
 * reference puts them at the queue front / on the main thread, index.ts:174-187,
 * 327-357, 544-555).  Calls of at most lb_set_latency_path's size take the latency
 * path.  One priority call in flight: a second first waits for the first.  The
 * synchronous lb_verify_requests uses this lane for calls of that size too. */
int lb_verify_requests_priority_async(lb_ctx* ctx, const lb_request_batch* batch, uint8_t* out_request_valid,
                                      uint8_t* out_request_error, uint8_t* out_set_status, uint64_t* out_ticket);
int lb_wait(lb_ctx* ctx, uint64_t ticket, lb_verify_stats* stats);
/* Non-blocking completion test of an async call: *out_done = 1 when lb_wait(ticket)
 * would return without waiting (the call's device work is complete, or it has
 * retired), 0 while it runs (also launches a finished same-message phase 1's
 * retries).  Lets a submission thread keep submitting while calls run (the N-API
 * addon's worker loop) instead of blocking on the oldest call. */
int lb_poll(lb_ctx* ctx, uint64_t ticket, int32_t* out_done);

/*
 * Multi-GPU combine (BASELINE north_star: "the per-GPU
 * partial Fp12 Miller-loop products (576 B each) are combined on the host").
 * The batch equation is multiplicative across shards, so each GPU verifies its
 * shard of requests up to its merged Miller product
 *     P_g = prod_{k in shard, not already false} F_k * Miller(-g1, sum_k S_k)
 * and stops there (two-phase call).  The host gathers the partials, checks
 * final_exp(prod_g P_g) == 1 ONCE (lb_gt_check, on any one GPU), and resumes
 * every shard with the verdict: merged_ok = 1 -> every request that is not
 * already false is valid, no further work; merged_ok = 0 -> each shard runs its
 * per-request tails (each request verified alone, as worker.ts:74-85 does after
 * a failed merged batch).  Either way the per-request verdicts are those of
 * lb_verify_requests.  Reference analogue of the fan-out: the pool's chunking
 * across workers, chain/bls/multithread/index.ts:191-205.
 *
 *   lb_verify_requests_partial_async(flags)  enqueue (LB_BATCH_DEVICE: every
 *                                           pointer, outputs included, is device memory)
 *   lb_partial_wait(ticket, out576)          block until the shard's partial is ready
 *   lb_gt_check(n, partials, out_is_one)     final_exp(prod of n partials) == 1
 *   lb_verify_requests_finish(ticket, ok)    resume the shard with the verdict
 *   lb_wait(ticket)                          verdicts (and stats) of the shard
 * A partial is 12 big-endian canonical Fp coefficients (c0.c0.c0 ... c1.c2.c1,
 * the lb_pairing order); an empty shard's partial is 1.  A two-phase call that
 * is waited for without lb_verify_requests_finish resumes with merged_ok = 0.
 *
 * Contract of the default flow (LB_TP_RELEASE=1: the call frees its slot once its
 * partial is out, instead of holding it through the host's combine):
 *   - the outputs are PROVISIONAL until lb_wait(ticket) returns LB_OK: the released
 *     call writes "valid" for every request not already false before the combined
 *     check has run (into device outputs at once, into host outputs when it
 *     retires).  Only lb_wait's return makes them verdicts;
 *   - every input buffer (host or device) must stay valid and unchanged until
 *     lb_wait returns: a failed combined check (merged_ok = 0) re-verifies the shard
 *     from the caller's buffers as a one-phase call into the same outputs;
 *   - lb_wait returns an error, never verdicts, when that re-verification could not
 *     be submitted (lb_verify_requests_finish returned the error first);
 *   - at most 256 two-phase calls can be unfinished: the context keeps one record per
 *     ticket in a 256-entry ring, and lb_verify_requests_partial_async refuses a call
 *     with LB_ERR_RESOURCES (nothing enqueued) while its ring entry still holds a call
 *     that is neither finished nor waited for, instead of overwriting it.
 * LB_TP_RELEASE=0 (legacy): the call holds its slot until finish; its outputs are
 * written only by the per-request tails or the verdict, i.e. never provisional.
 * After a failed combined check (merged_ok = 0) the context submits its next 32
 * two-phase calls (LB_TP_PAUSE) in the legacy mode: a re-run repeats the whole shard,
 * the legacy mode only its per-request tails, so a stream of failing batches costs
 * the tails alone while a clean stream keeps the release.
 */
#define LB_BATCH_DEVICE 1u
int lb_verify_requests_partial_async(lb_ctx* ctx, const lb_request_batch* batch, uint32_t flags,
                                     uint8_t* out_request_valid, uint8_t* out_request_error, uint8_t* out_set_status,
                                     uint64_t* out_ticket);
int lb_partial_wait(lb_ctx* ctx, uint64_t ticket, uint8_t* out576);
/* Non-blocking: *out_ready = 1 when lb_partial_wait(ticket) would return at once
 * (a host's resolver thread polls it, so the combine never stalls submission). */
int lb_partial_poll(lb_ctx* ctx, uint64_t ticket, int32_t* out_ready);
/* lb_gt_check touches only the context's own combine buffers and its aux stream (not
 * the slots): one thread may run it while another submits and retires calls on the
 * same context (bench.py's resolver thread does); two lb_gt_check at once may not. */
int lb_gt_check(lb_ctx* ctx, uint32_t n, const uint8_t* partials576, int32_t* out_is_one);
int lb_verify_requests_finish(lb_ctx* ctx, uint64_t ticket, int merged_ok);

/*
 * verifySignatureSetsSameMessage for one job (<= 128 sets in the reference,
 * any n here): out_valid[i] per set.  Fast path: every signature validates,
 * aggregate pubkeys and signatures (plain sums, as the reference does) and
 * core-verify once; otherwise / on failure every set is core-verified alone.
 * n == 0 -> nothing written (the reference returns []).
 */
int lb_verify_same_message(lb_ctx* ctx, uint32_t n, const uint8_t* pubkeys /* n x 96 */,
                           const uint8_t* signatures, const uint32_t* sig_offsets /* n + 1 */,
                           const uint8_t* message /* 32 */, const uint8_t* seed /* 32 */, uint8_t* out_valid,
                           uint32_t* out_used_fast_path);

/*
 * Many same-message jobs in one call (the dominant gossip load: one job per
 * attestation-data group, chunked to <= 128 sets by verifySignatureSetsSameMessage,
 * index.ts:218-242).  Job j = sets [job_offsets[j], job_offsets[j+1]) over
 * messages[32 j .. 32 j + 32).  Every signature is decoded and validated once
 * on the GPU, each job's pubkeys and signatures are summed (plain sums, as
 * jobItemWorkReq does, jobItem.ts:64-86) and all jobs' aggregated sets are
 * verified together as 1-set requests of one merged call; the sets of a job
 * whose aggregate fails (or that holds a signature failing
 * Signature.fromBytes(validate=true)) are re-verified each alone
 * (jobItemSameMessageToMultiSet, jobItem.ts:93-125).  out_valid: n_sets
 * verdicts; out_job_fast (optional): 1 where the job's aggregate passed.
 * stats (optional): batch_retries = jobs retried set by set,
 * batch_sigs_success = sets verified by a passing aggregate.
 */
typedef struct {
  uint32_t n_jobs;
  uint32_t n_sets;
  const uint32_t* job_offsets;     /* n_jobs + 1                                    */
  const uint8_t* pubkeys;          /* n_sets x 96 (uncompressed), or NULL with ...  */
  const uint32_t* pubkey_indices;  /* n_sets validator indices (device pubkey table); with
                                      both given, a mixed package as in lb_request_batch
                                      (LB_PK_ROW_FLAG / LB_PK_ROW48_FLAG rows of pubkeys) */
  const uint8_t* signatures;       /* concatenated signature bytes                  */
  const uint32_t* sig_offsets;     /* n_sets + 1                                    */
  const uint8_t* messages;         /* n_jobs x 32                                   */
  const uint8_t* seed;             /* 32                                            */
} lb_same_message_batch;
int lb_verify_same_message_batch(lb_ctx* ctx, const lb_same_message_batch* batch, uint8_t* out_valid,
                                 uint8_t* out_job_fast, lb_verify_stats* stats);
/* The same, asynchronous, on the ring of calls in flight (like lb_verify_requests_async):
 * the inputs are staged before it returns; out_valid / out_job_fast are written when the
 * call retires (lb_wait(ticket, stats), or when its slot is reused).  The per-set retry of
 * failed jobs runs on the same slot from the device-resident decoded signatures (no second
 * request batch, no re-upload); the pool's packages in flight across workers
 * (BN/chain/bls/multithread/index.ts:362-519). */
int lb_verify_same_message_batch_async(lb_ctx* ctx, const lb_same_message_batch* batch, uint8_t* out_valid,
                                       uint8_t* out_job_fast, uint64_t* out_ticket);

/* Sum of n uncompressed pubkeys -> 96-byte uncompressed encoding.  n == 0 ->
 * LB_ERR_INVALID_ARGUMENT (EMPTY_AGGREGATE_ARRAY). *out_status = LB_SET_*. */
int lb_aggregate_pubkeys(lb_ctx* ctx, uint32_t n, const uint8_t* pubkeys, uint8_t* out96, uint8_t* out_status);

/* Validate-deserialize n signatures and sum them -> 192-byte uncompressed
 * encoding.  *out_bad_index = index of the first invalid signature or -1. */
int lb_aggregate_signatures(lb_ctx* ctx, uint32_t n, const uint8_t* signatures, const uint32_t* sig_offsets,
                            uint8_t* out192, int32_t* out_bad_index);

/* PublicKey.fromBytes(bytes, CoordType.affine, validate=true) for n keys of pk_len
 * (48 compressed / 96 uncompressed) bytes: out96 = the uncompressed encoding,
 * out_status[i] = LB_SET_OK, or LB_SET_BAD_ENCODING / NOT_ON_CURVE / NOT_IN_GROUP /
 * PK_INFINITY for a key the reference's fromBytes would throw on (out96 then holds
 * the infinity encoding).  Used for the fromBlsPubkey of BLS-to-execution changes
 * (state-transition/src/signatureSets/blsToExecutionChange.ts:30). */
int lb_pubkeys_from_bytes(lb_ctx* ctx, uint32_t n, const uint8_t* pubkeys, uint32_t pk_len, uint8_t* out96,
                          uint8_t* out_status);
/* ---- device-resident pubkey table ----------------------
 * Mirror of the beacon node's index2pubkey cache
 * (state-transition/src/cache/pubkeyCache.ts:56-77 syncPubkeys, held in
 * epochCache.ts:765): validators' pubkeys are decoded ONCE into HBM (affine,
 * Montgomery form, ~100 B per key; 2M validators ~200 MB of the 288 GB), so
 * aggregate sets ship 4-byte validator indices instead of 96-byte points and
 * the main-thread aggregation (chain/bls/utils.ts:13, jobItem.ts:80) moves to
 * the GPU.
 *
 * Append n keys (pk_len = 48 compressed, as the state holds them, or 96
 * uncompressed) at indices [size, size + n).  Decode semantics are those of
 * PublicKey.fromBytes without validation (syncPubkeys: "Do not do any
 * validation here"): a key that fails to decode makes the whole call fail with
 * LB_ERR_INVALID_ARGUMENT, nothing is appended and *out_bad_index (optional)
 * names the first bad key, else -1.  Waits for calls in flight. */
int lb_pubkey_table_append(lb_ctx* ctx, uint32_t n, const uint8_t* pubkeys, uint32_t pk_len, int32_t* out_bad_index);
/* Number of keys in the table. */
int lb_pubkey_table_size(const lb_ctx* ctx, uint32_t* out_n);
/* Table entries [first, first + n) re-encoded as 96-byte uncompressed points. */
int lb_pubkey_table_read(lb_ctx* ctx, uint32_t first, uint32_t n, uint8_t* out96);
/* Truncate the table to n keys (n <= size). */
int lb_pubkey_table_truncate(lb_ctx* ctx, uint32_t n);
/* lb_aggregate_pubkeys over table entries: sum of table[indices[0..n)] ->
 * 96-byte uncompressed (committee aggregation from validator indices).
 * n == 0 -> LB_ERR_INVALID_ARGUMENT (EMPTY_AGGREGATE_ARRAY); an index out of
 * range -> *out_status = LB_SET_BAD_ENCODING. */
int lb_aggregate_pubkeys_indexed(lb_ctx* ctx, uint32_t n, const uint32_t* indices, uint8_t* out96,
                                 uint8_t* out_status);

/* ---- signing roots (the step before the verifier) --------
 * computeSigningRoot(type, obj, domain) = hash_tree_root(SigningData{hash_tree_root(obj), domain})
 * (state-transition/src/util/signingRoot.ts:7-13), SSZ merkleization on the GPU.
 * domains: n x 32 bytes (domain_stride 32) or one shared domain (domain_stride 0).
 *
 * Attestations: data = n x 128-byte SSZ phase0.AttestationData (slot, index,
 * beacon_block_root, source, target) -> n x 32-byte signing roots, as
 * getAttestationDataSigningRoot (signatureSets/indexedAttestation.ts:10-19). */
int lb_signing_roots_attestation(lb_ctx* ctx, uint32_t n, const uint8_t* data128, const uint8_t* domains,
                                 uint32_t domain_stride, uint8_t* out32);
/* Device-resident variant: data128, domains and out32 are device pointers (e.g.
 * out32 = the `messages` buffer of a following lb_verify_requests_device call,
 * so signing roots never leave HBM).  Synchronises before returning. */
int lb_signing_roots_attestation_device(lb_ctx* ctx, uint32_t n, const uint8_t* d_data128, const uint8_t* d_domains,
                                        uint32_t domain_stride, uint8_t* d_out32);
/* Any container given as its m (1..16) field roots per object (n x m x 32 bytes;
 * basic fields packed little-endian into a zero-padded chunk): merkleize, then SigningData. */
int lb_signing_roots_chunks(lb_ctx* ctx, uint32_t n, uint32_t m, const uint8_t* chunks, const uint8_t* domains,
                            uint32_t domain_stride, uint8_t* out32);

/* ---- stage-level entry points (parity tests against the CPU oracle) ----- */
/* hash_to_G2(msg_i) -> 192-byte uncompressed affine encoding each */
int lb_hash_to_g2(lb_ctx* ctx, uint32_t n, const uint8_t* messages, uint8_t* out192);
/* Signature.fromBytes(validate=true): status + 192-byte uncompressed re-encoding */
int lb_decode_signatures(lb_ctx* ctx, uint32_t n, const uint8_t* signatures, const uint32_t* sig_offsets,
                         uint8_t* out_status, uint8_t* out192);
/* e(P_i, Q_i) after the final exponentiation (f^(3(p^12-1)/r)), 576 bytes each
 * (12 big-endian Fp coefficients, c0.c0.c0 ... c1.c2.c1 order) */
int lb_pairing(lb_ctx* ctx, uint32_t n, const uint8_t* g1_96, const uint8_t* g2_192, uint8_t* out576);
/* batch scalars r_i, i in [first, first + n) */
int lb_batch_scalars(lb_ctx* ctx, const uint8_t* seed, uint32_t first, uint32_t n, uint64_t* out);
/* [k_i] P_i on G1 and G2 (uncompressed in/out) */
int lb_g1_mul(lb_ctx* ctx, uint32_t n, const uint8_t* g1_96, const uint64_t* k, uint8_t* out96);
int lb_g2_mul(lb_ctx* ctx, uint32_t n, const uint8_t* g2_192, const uint64_t* k, uint8_t* out192);
/* sum_i (a_i + b_i lambda) P_i, a_i / b_i = low / high 32 bits of raw[i], lambda = -x^2: the
 * merged check's bucket MSM alone (uncompressed in/out; an undecodable point gives infinity).
 * Replaces nothing in the reference: the sum blst's mul_n_aggregate accumulates inside
 * verifyMultipleSignatures (BN/chain/bls/maybeBatch.ts:19-26), exposed for tests. */
int lb_g2_msm(lb_ctx* ctx, uint32_t n, const uint8_t* g2_192, const uint64_t* raw, uint8_t* out192);

/* The latency path's round programs alone (prog: 0 set_single, 1 set_batch, 2 fp12
 * product, 3 final exponentiation == 1; or, with prog_words != NULL, a caller-encoded
 * program of n_words words), one workgroup per instance: in16 = n x n_in records of 16
 * words (canonical Montgomery limbs), in_flags n x n_inflag words; out16 / out_flags
 * likewise; *out_ms = kernel time; stamps (optional, n_rounds): s_memtime after each
 * round of instance 0.  Replaces nothing in the reference: the stages of blst's verify
 * behind BN/chain/bls/maybeBatch.ts:19-38, exposed for parity tests and timing. */
int lb_lp_program_run(lb_ctx* ctx, uint32_t prog, const uint32_t* prog_words, size_t n_words, uint32_t n,
                      const uint32_t* in16, const uint32_t* in_flags, uint32_t* out16, uint32_t* out_flags,
                      float* out_ms, uint64_t* stamps);

/* ---- synthetic data generation (bench / tests) ---------------------------- */
/* SecretKey.fromBytes(sk).toPublicKey().toBytes(uncompressed) and
 * SecretKey.sign(msg).toBytes() (compressed), as the reference's own perf/unit
 * tests build their inputs (test/perf/bls/bls.test.ts:19-40).  sk32 = 32-byte
 * big-endian secret keys (< r). */
int lb_sk_to_pk(lb_ctx* ctx, uint32_t n, const uint8_t* sk32, uint8_t* out96);
int lb_sign(lb_ctx* ctx, uint32_t n, const uint8_t* sk32, const uint8_t* messages, uint8_t* out96);

/* ---- profiling ----------------------------------------------------------- */
/* Per-stage device time (ms) of the last lb_verify_* call, measured with HIP
 * events on the context's stream.  Writes up to max_stages values and their
 * names; returns the number of stages. */
int lb_last_stage_times(const lb_ctx* ctx, float* out_ms, const char** out_names, int max_stages);

#ifdef __cplusplus
}
#endif
#endif /* LODESTAR_BLS_H */
