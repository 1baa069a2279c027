// N-API addon: the Lodestar-side binding of the MI355X BLS verifier C ABI
// (include/lodestar_bls.h).  This is what a BlsGpuVerifier beside
// BlsMultiThreadWorkerPool (packages/beacon-node/src/chain/bls, chosen at
// BN/chain/chain.ts:206-208) requires: it replaces the worker boundary
// workerApi.verifyManySignatureSets(workReqs) (chain/bls/multithread/index.ts:444,
// worker.ts:24-30) with one call per package on a GPU.
//
// Threading: JS calls arrive on the main thread; their
// offsets are copied there (the reference structured-clones its requests to the
// worker, index.ts:444), the bulk arrays of verifyRequests are read in place (kept
// alive by references until the promise settles: the caller must not modify them
// meanwhile), and the task goes to ONE host submission thread per GPU, which owns
// the lb_ctx (not thread-safe) and keeps up to `capacity` calls in flight
// (lb_verify_requests_async + lb_wait).  Completions come back to the event
// loop through a threadsafe function; the event loop never blocks on the GPU.
// Every native method returns a Promise; bad arguments and device errors
// reject it (a malformed signature is a verdict, never an error).
//
// Exports:
//   deviceCount() -> number
//   validateRequests(batch) -> {nRequests, nSets, nPubkeys, byIndex}   (marshalling dry run, no device)
//   new Context(device, {capacity?}) (throws Error{code: "LB_ERR_NO_DEVICE", ...} without a GPU)
//     .verifyRequests(batch, {priority?}) -> Promise<{valid, errors, setStatus, batchRetries,
//                                        batchSigsSuccess, deviceMs, workerStartNs, workerEndNs}>
//         (priority: the device's priority lane -- started at once, beside the calls in
//          flight, retired as soon as it completes; lb_verify_requests_priority_async)
//     .verifyRequestsPartial(batch) -> Promise<{id, partial: Uint8Array(576)}>  (two-phase, multi-GPU)
//     .finish(id, mergedOk) -> Promise<result of verifyRequests>
//     .gtCheck(Uint8Array n*576) -> Promise<boolean>
//     .verifySameMessage({jobOffsets, pubkeys|pubkeyIndices, signatures, sigOffsets, messages, seed})
//         -> Promise<{valid, jobFast, retriedJobs, fastSets, deviceMs}>
//     .syncPubkeys(Uint8Array keys, pkLen) -> Promise<number>          (index2pubkey mirror)
//     .aggregatePubkeys(Uint8Array n*96 | Uint32Array indices) -> Promise<Uint8Array(96)>
//     .close() -> Promise<void>                                      (waits for calls in flight)
//   batch = {requestOffsets: Uint32Array, pubkeys?: Uint8Array, pubkeyIndices?: Uint32Array,
//            pkOffsets?: Uint32Array, messages: Uint8Array, signatures: Uint8Array,
//            sigOffsets: Uint32Array, seed: Uint8Array(32), batchable?: Uint8Array}
#define NAPI_VERSION 8
#include <node_api.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lodestar_bls.h"

namespace {

#define NAPI_OK(call)                       \
  do {                                      \
    if ((call) != napi_ok) return nullptr;  \
  } while (0)

struct ArgError {
  std::string msg;
};

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ---- marshalling --------------------------------------------------------------
bool has_prop(napi_env env, napi_value obj, const char* name, napi_value* out) {
  bool has = false;
  if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return false;
  if (napi_get_named_property(env, obj, name, out) != napi_ok) return false;
  napi_valuetype t;
  napi_typeof(env, *out, &t);
  return t != napi_undefined && t != napi_null;
}

template <class T>
void typed(napi_env env, napi_value v, napi_typedarray_type want, const char* name, std::vector<T>& out) {
  bool is = false;
  napi_is_typedarray(env, v, &is);
  if (!is) throw ArgError{std::string(name) + " must be a typed array"};
  napi_typedarray_type t;
  size_t len = 0;
  void* data = nullptr;
  napi_value ab;
  size_t off = 0;
  napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
  if (t != want && !(want == napi_uint8_array && t == napi_uint8_clamped_array))
    throw ArgError{std::string(name) + (want == napi_uint8_array ? " must be a Uint8Array" : " must be a Uint32Array")};
  out.resize(len);
  if (len) memcpy(out.data(), data, len * sizeof(T));
}

template <class T>
void req_typed(napi_env env, napi_value obj, const char* name, napi_typedarray_type want, std::vector<T>& out) {
  napi_value v;
  if (!has_prop(env, obj, name, &v)) throw ArgError{std::string("missing ") + name};
  typed(env, v, want, name, out);
}

template <class T>
bool opt_typed(napi_env env, napi_value obj, const char* name, napi_typedarray_type want, std::vector<T>& out) {
  napi_value v;
  if (!has_prop(env, obj, name, &v)) return false;
  typed(env, v, want, name, out);
  return true;
}

// A typed array read in place (no copy on the JS thread): the caller's buffer, kept
// alive by a reference the JS thread releases when the task settles.  Used for the
// bulk inputs of verifyRequests (messages, signatures, pubkeys, pubkeyIndices: ~8 MB
// for a 65,536-set package, ~1 ms of main-thread memcpy); the caller must not modify
// them until the promise settles (packRequests' arrays are fresh and private).
template <class T>
struct View {
  const T* p = nullptr;
  size_t n = 0;
  std::vector<T> own;  // a copy instead (empty-array placeholder)
  const T* data() const { return p ? p : own.data(); }
  size_t size() const { return p ? n : own.size(); }
  bool empty() const { return size() == 0; }
};

template <class T>
void typed_view(napi_env env, napi_value v, napi_typedarray_type want, const char* name, View<T>& out,
                std::vector<napi_ref>& refs) {
  bool is = false;
  napi_is_typedarray(env, v, &is);
  if (!is) throw ArgError{std::string(name) + " must be a typed array"};
  napi_typedarray_type t;
  size_t len = 0;
  void* data = nullptr;
  napi_value ab;
  size_t off = 0;
  napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
  if (t != want && !(want == napi_uint8_array && t == napi_uint8_clamped_array))
    throw ArgError{std::string(name) + (want == napi_uint8_array ? " must be a Uint8Array" : " must be a Uint32Array")};
  napi_ref r = nullptr;
  if (len && napi_create_reference(env, v, 1, &r) == napi_ok) {
    refs.push_back(r);
    out.p = static_cast<const T*>(data);
    out.n = len;
  } else {
    out.p = nullptr;
    out.own.assign(static_cast<const T*>(data), static_cast<const T*>(data) + len);
  }
}

void check_offsets(const std::vector<uint32_t>& off, size_t n, uint32_t last, const char* name) {
  if (off.size() != n + 1) throw ArgError{std::string(name) + ": wrong length"};
  if (off[0] != 0) throw ArgError{std::string(name) + " must start at 0"};
  for (size_t i = 0; i < n; i++)
    if (off[i + 1] < off[i]) throw ArgError{std::string(name) + " not monotone"};
  if (last != UINT32_MAX && off[n] != last) throw ArgError{std::string(name) + ": wrong end"};
}

// ---- tasks ---------------------------------------------------------------------
enum class Kind { Verify, Partial, Finish, SameMessage, SyncPubkeys, AggPubkeys, GtCheck, Close };

struct Task {
  Kind kind = Kind::Verify;
  napi_deferred deferred = nullptr;
  // inputs (copied on the JS thread)
  std::vector<uint32_t> req_off, pk_off, sig_off, pk_idx, job_off;
  std::vector<uint8_t> pubkeys, messages, signatures, seed, batchable;
  // verifyRequests: the bulk inputs read in place (see View); refs released on the JS thread
  View<uint8_t> v_pubkeys, v_messages, v_signatures;
  View<uint32_t> v_pk_idx;
  std::vector<napi_ref> refs;
  bool has_pk_off = false, by_index = false, has_batchable = false, mixed = false;
  bool prio = false;  // verifyRequests(batch, {priority: true}): the device's priority lane
  uint32_t n_req = 0, n_sets = 0, n_jobs = 0, pk_len = 0, n_keys = 0;
  int merged_ok = 0;
  uint64_t partial_id = 0;
  // outputs
  std::vector<uint8_t> valid, err, sst, job_fast, out_bytes;
  lb_verify_stats stats{0, 0, 0.0};
  int32_t i32 = 0;
  uint32_t u32 = 0;
  uint64_t ticket = 0;
  uint64_t t_start = 0, t_end = 0, t_submitted = 0, t_retire = 0;
  uint64_t clk[4] = {};  // latency-lane calls: lb_last_latency_clocks
  // latency-lane calls with LB_STAGE_EVENTS=1: the call's stage times (lb_last_stage_times)
  float stage_ms[16] = {};
  const char* stage_names[16] = {};
  int n_stage = 0;
  int rc = LB_OK;
  std::string errmsg;
  Task* target = nullptr;  // Finish: the two-phase call it resumes
};

void parse_requests(napi_env env, napi_value obj, Task& t) {
  napi_valuetype ty;
  napi_typeof(env, obj, &ty);
  if (ty != napi_object) throw ArgError{"batch must be an object"};
  req_typed(env, obj, "requestOffsets", napi_uint32_array, t.req_off);
  if (t.req_off.empty()) throw ArgError{"requestOffsets: wrong length"};
  t.n_req = (uint32_t)t.req_off.size() - 1;
  t.n_sets = t.req_off.back();
  check_offsets(t.req_off, t.n_req, UINT32_MAX, "requestOffsets");
  napi_value mv, sv;
  if (!has_prop(env, obj, "messages", &mv)) throw ArgError{"missing messages"};
  typed_view(env, mv, napi_uint8_array, "messages", t.v_messages, t.refs);
  if (t.v_messages.size() != (size_t)t.n_sets * 32) throw ArgError{"messages: 32 bytes per set"};
  if (!has_prop(env, obj, "signatures", &sv)) throw ArgError{"missing signatures"};
  typed_view(env, sv, napi_uint8_array, "signatures", t.v_signatures, t.refs);
  req_typed(env, obj, "sigOffsets", napi_uint32_array, t.sig_off);
  check_offsets(t.sig_off, t.n_sets, (uint32_t)t.v_signatures.size(), "sigOffsets");
  req_typed(env, obj, "seed", napi_uint8_array, t.seed);
  if (t.seed.size() != 32) throw ArgError{"seed must be 32 bytes"};
  t.has_pk_off = opt_typed(env, obj, "pkOffsets", napi_uint32_array, t.pk_off);
  if (t.has_pk_off) check_offsets(t.pk_off, t.n_sets, UINT32_MAX, "pkOffsets");
  const size_t n_pk = t.has_pk_off ? t.pk_off[t.n_sets] : t.n_sets;
  napi_value iv, kv;
  t.by_index = has_prop(env, obj, "pubkeyIndices", &iv);
  const bool has_keys = has_prop(env, obj, "pubkeys", &kv);
  if (has_keys) typed_view(env, kv, napi_uint8_array, "pubkeys", t.v_pubkeys, t.refs);
  if (t.by_index) {
    typed_view(env, iv, napi_uint32_array, "pubkeyIndices", t.v_pk_idx, t.refs);
    if (t.v_pk_idx.size() != n_pk) throw ArgError{"pubkeyIndices: one index per pubkey"};
    // mixed package: rows of `pubkeys` named by indices with LB_PK_ROW_FLAG set
    size_t rows = 0;
    const uint32_t* ix = t.v_pk_idx.data();
    for (size_t q = 0; q < n_pk; q++)
      if ((ix[q] & LB_PK_ROW_FLAG) && (size_t)(ix[q] & LB_PK_ROW_MASK) + 1 > rows) rows = (ix[q] & LB_PK_ROW_MASK) + 1;
    t.mixed = has_keys;
    if (rows && (!t.mixed || t.v_pubkeys.size() < rows * LB_PUBKEY_BYTES))
      throw ArgError{"pubkeyIndices name pubkey rows that `pubkeys` does not hold"};
  } else {
    if (!has_keys && n_pk) throw ArgError{"missing pubkeys (or pubkeyIndices)"};
    if (t.v_pubkeys.size() != n_pk * LB_PUBKEY_BYTES) throw ArgError{"pubkeys: 96 bytes per pubkey"};
  }
  t.has_batchable = opt_typed(env, obj, "batchable", napi_uint8_array, t.batchable);
  if (t.has_batchable && t.batchable.size() != t.n_req) throw ArgError{"batchable: one flag per request"};
  // (empty arrays: one placeholder byte / index, so every pointer is valid)
  if (t.v_signatures.empty()) t.v_signatures.own.assign(1, 0);
  if (t.v_messages.empty()) t.v_messages.own.assign(1, 0);
  if (t.v_pubkeys.empty()) t.v_pubkeys.own.assign(1, 0);
  if (t.v_pk_idx.empty()) t.v_pk_idx.own.assign(1, 0);
}

void release_refs(napi_env env, Task* t) {
  for (napi_ref r : t->refs) napi_delete_reference(env, r);
  t->refs.clear();
}

lb_request_batch batch_of(Task& t) {
  lb_request_batch b{};
  b.n_requests = t.n_req;
  b.n_sets = t.n_sets;
  b.request_offsets = t.req_off.data();
  b.request_batchable = t.has_batchable ? t.batchable.data() : nullptr;
  b.pubkeys = (!t.by_index || t.mixed) ? t.v_pubkeys.data() : nullptr;
  b.pk_offsets = t.has_pk_off ? t.pk_off.data() : nullptr;
  b.messages = t.v_messages.data();
  b.signatures = t.v_signatures.data();
  b.sig_offsets = t.sig_off.data();
  b.seed = t.seed.data();
  b.pubkey_indices = t.by_index ? t.v_pk_idx.data() : nullptr;
  return b;
}

void alloc_outputs(Task& t) {
  t.valid.assign(t.n_req ? t.n_req : 1, 0);
  t.err.assign(t.n_req ? t.n_req : 1, 0);
  t.sst.assign(t.n_sets ? t.n_sets : 1, 0);
}

// ---- the per-GPU context ---------------------------------------------------------
struct Context {
  lb_ctx* ctx = nullptr;
  int device = 0;
  int capacity = 4;
  napi_env env = nullptr;
  napi_threadsafe_function tsfn = nullptr;
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Task*> queue;
  bool closing = false;   // no new work accepted
  bool finalizing = false;
  bool joined = false;
  int pending = 0;        // JS thread only: tasks not yet completed
  uint64_t next_partial = 1;
  std::map<uint64_t, Task*> partials;  // worker thread only
  // The latency lane (LB_PRIO_THREAD, default on): priority verify calls run on a context
  // of their own (lb_create_lane) driven by a thread of their own, so they never wait for
  // the submission thread's staging of throughput packages or its retiring of calls
  // (the reference's verifyOnMainThread / priority unshift,
  // BN/chain/bls/multithread/index.ts:174-187,544-555).  Its pubkey table mirrors ctx's.
  lb_ctx* lctx = nullptr;
  // false once the lane's pubkey table failed to follow ctx's: from then on
  // priority calls go back to ctx (the submission thread), never to a table that resolves
  // indices differently
  std::atomic<bool> lane_ok{true};
  std::thread lane;
  std::mutex lmu;
  std::condition_variable lcv;
  std::deque<Task*> lqueue;
  bool lane_stop = false;
};

void complete(Context* c, Task* t) {
  if (c->finalizing) {
    delete t;
    return;
  }
  napi_call_threadsafe_function(c->tsfn, t, napi_tsfn_blocking);
}

void fail(Task* t, int rc, lb_ctx* ctx) {
  t->rc = rc;
  t->errmsg = ctx ? lb_last_error(ctx) : "no context";
}

// The lane thread: owns c->lctx.  Priority verify calls one at a time (the priority slot
// admits one), and the second half of every pubkey-table append (the main worker appends
// to ctx first, then hands the task here).
void lane_loop(Context* c) {
  for (;;) {
    Task* t = nullptr;
    {
      std::unique_lock<std::mutex> lk(c->lmu);
      c->lcv.wait(lk, [&] { return !c->lqueue.empty() || c->lane_stop; });
      if (c->lqueue.empty()) break;  // stopped and drained
      t = c->lqueue.front();
      c->lqueue.pop_front();
    }
    if (c->finalizing) {
      delete t;
      continue;
    }
    if (t->kind == Kind::SyncPubkeys) {
      // (ctx's table, the authoritative one, already holds the keys: the task succeeds; a
      // lane that cannot follow is retired instead of left out of sync)
      int32_t bad = -1;
      uint32_t n = 0;
      if (c->lane_ok && (lb_pubkey_table_append(c->lctx, t->n_keys, t->pubkeys.data(), t->pk_len, &bad) != LB_OK ||
                         lb_pubkey_table_size(c->lctx, &n) != LB_OK || n != t->u32)) {
        c->lane_ok = false;
        fprintf(stderr, "lodestar_bls: latency lane retired (its pubkey table could not follow: %s); priority "
                        "calls run on the main context\n", lb_last_error(c->lctx));
      }
      complete(c, t);
      continue;
    }
    if (!c->lane_ok) {  // a priority call queued here before the lane retired: back to ctx
      {
        std::lock_guard<std::mutex> lk(c->mu);
        auto it = c->queue.begin();
        while (it != c->queue.end() && (*it)->prio) ++it;
        c->queue.insert(it, t);
      }
      c->cv.notify_all();
      continue;
    }
    t->t_start = now_ns();
    alloc_outputs(*t);
    lb_request_batch b = batch_of(*t);
    int rc = lb_verify_requests_priority_async(c->lctx, &b, t->valid.data(), t->err.data(), t->sst.data(), &t->ticket);
    t->t_submitted = now_ns();
    if (rc == LB_OK) {
      t->t_retire = now_ns();
      rc = lb_wait(c->lctx, t->ticket, &t->stats);
      if (rc == LB_OK) {
        lb_last_latency_clocks(c->lctx, t->clk);
        t->n_stage = lb_last_stage_times(c->lctx, t->stage_ms, t->stage_names, 16);
        if (t->n_stage > 16) t->n_stage = 16;
      }
    }
    if (rc != LB_OK) fail(t, rc, c->lctx);
    t->t_end = now_ns();
    complete(c, t);
  }
  lb_destroy(c->lctx);
  c->lctx = nullptr;
}

// stop the lane thread after it has drained its queue (worker thread, before lb_destroy)
void lane_join(Context* c) {
  if (!c->lane.joinable()) return;
  {
    std::lock_guard<std::mutex> lk(c->lmu);
    c->lane_stop = true;
  }
  c->lcv.notify_one();
  c->lane.join();
}

// A queued task the worker can start now: a priority call always (its lane is
// separate from the calls in flight), close always, anything else when a slot is free.
bool startable(Context* c, size_t n_inflight) {
  if (c->queue.empty()) return false;
  const Task* f = c->queue.front();
  return f->prio || f->kind == Kind::Close || (int)n_inflight < c->capacity;
}

// Worker thread: owns c->ctx.
void worker_loop(Context* c) {
  std::deque<Task*> inflight;  // submitted, waiting for lb_wait
  std::deque<Task*> prio;      // priority-lane calls in flight (retired as soon as done)
  for (;;) {
    Task* t = nullptr;
    // a finished priority call retires before anything else is started: with packages
    // startable back to back (each ~3 ms of staging in lb_verify_requests_async), its
    // verdict would otherwise wait behind all of them
    if (!prio.empty()) {
      Task* w = prio.front();
      int32_t done = 0;
      if (lb_poll(c->ctx, w->ticket, &done) == LB_OK && done) {
        prio.pop_front();
        w->t_retire = now_ns();
        const int rc = lb_wait(c->ctx, w->ticket, &w->stats);
        if (rc != LB_OK) fail(w, rc, c->ctx);
        w->t_end = now_ns();
        complete(c, w);
        continue;
      }
    }
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv.wait(lk, [&] { return !c->queue.empty() || !inflight.empty() || !prio.empty() || c->finalizing; });
      if (startable(c, inflight.size())) {
        t = c->queue.front();
        c->queue.pop_front();
      } else if (inflight.empty() && prio.empty() && c->finalizing) {
        break;
      }
    }
    if (!t && !prio.empty()) {  // a finished priority call retires ahead of everything
      Task* w = prio.front();
      int32_t done = 1;
      if (c->finalizing || (lb_poll(c->ctx, w->ticket, &done) == LB_OK && done)) {
        prio.pop_front();
        w->t_retire = now_ns();
        const int rc = lb_wait(c->ctx, w->ticket, &w->stats);
        if (rc != LB_OK) fail(w, rc, c->ctx);
        w->t_end = now_ns();
        complete(c, w);
        continue;
      }
      if (inflight.empty()) {
        std::unique_lock<std::mutex> lk(c->mu);
        c->cv.wait_for(lk, std::chrono::microseconds(50), [&] { return startable(c, 0) || c->finalizing; });
        continue;
      }
    }
    if (!t) {  // retire the oldest call in flight
      Task* w = inflight.front();
      Task* owner = w->kind == Kind::Finish ? w->target : w;
      if (!c->finalizing) {
        // never block on it: the JS thread may queue the next package (blocking here held
        // every new package back until the oldest call finished: ~12 of 16 calls in
        // flight, 2.3 M sets/s through node), or a priority call that must start now
        int32_t done = 1;
        if (lb_poll(c->ctx, owner->ticket, &done) == LB_OK && !done) {
          std::unique_lock<std::mutex> lk(c->mu);
          c->cv.wait_for(lk, std::chrono::microseconds(prio.empty() ? 200 : 50),
                         [&] { return startable(c, inflight.size()) || c->finalizing; });
          continue;
        }
      }
      inflight.pop_front();
      owner->t_retire = now_ns();
      const int rc = lb_wait(c->ctx, owner->ticket, &owner->stats);
      if (rc != LB_OK) fail(w, rc, c->ctx);
      if (w->kind == Kind::Finish) {
        w->valid.swap(owner->valid);
        w->err.swap(owner->err);
        w->sst.swap(owner->sst);
        w->stats = owner->stats;
        w->n_req = owner->n_req;
        w->n_sets = owner->n_sets;
        w->t_start = owner->t_start;
        w->refs.swap(owner->refs);  // its inputs' references, released on the JS thread
        c->partials.erase(owner->partial_id);
        delete owner;
      }
      w->t_end = now_ns();
      complete(c, w);
      continue;
    }
    t->t_start = now_ns();
    switch (t->kind) {
      case Kind::Verify: {
        alloc_outputs(*t);
        lb_request_batch b = batch_of(*t);
        const int rc = t->prio ? lb_verify_requests_priority_async(c->ctx, &b, t->valid.data(), t->err.data(),
                                                                   t->sst.data(), &t->ticket)
                               : lb_verify_requests_async(c->ctx, &b, t->valid.data(), t->err.data(),
                                                          t->sst.data(), &t->ticket);
        t->t_submitted = now_ns();
        if (rc != LB_OK) {
          fail(t, rc, c->ctx);
          complete(c, t);
        } else {
          (t->prio ? prio : inflight).push_back(t);
        }
        break;
      }
      case Kind::Partial: {
        // the two-phase call stays in the map (its outputs are written when it
        // retires); the JS promise resolves with its partial
        Task* call = new Task(std::move(*t));
        call->deferred = nullptr;
        alloc_outputs(*call);
        lb_request_batch b = batch_of(*call);
        int rc = lb_verify_requests_partial_async(c->ctx, &b, 0, call->valid.data(), call->err.data(),
                                                  call->sst.data(), &call->ticket);
        t->out_bytes.assign(LB_GT_BYTES, 0);
        if (rc == LB_OK) rc = lb_partial_wait(c->ctx, call->ticket, t->out_bytes.data());
        if (rc != LB_OK) {
          fail(t, rc, c->ctx);
          t->refs.swap(call->refs);
          delete call;
        } else {
          call->partial_id = t->partial_id;
          c->partials[t->partial_id] = call;
        }
        complete(c, t);
        break;
      }
      case Kind::Finish: {
        auto it = c->partials.find(t->partial_id);
        if (it == c->partials.end()) {
          t->rc = LB_ERR_INVALID_ARGUMENT;
          t->errmsg = "unknown or already finished two-phase call";
          complete(c, t);
          break;
        }
        t->target = it->second;
        // (a released call -- LB_TP_RELEASE, the default -- holds provisional verdicts until this
        // finish; a failed finish, e.g. the failed combine's re-run not submitted, rejects the
        // promise: the call still retires through lb_wait below, whose error is kept)
        {
          const int rc = lb_verify_requests_finish(c->ctx, t->target->ticket, t->merged_ok);
          if (rc != LB_OK) fail(t, rc, c->ctx);
        }
        inflight.push_back(t);
        break;
      }
      case Kind::SameMessage: {
        lb_same_message_batch b{};
        b.n_jobs = t->n_jobs;
        b.n_sets = t->n_sets;
        b.job_offsets = t->job_off.data();
        b.pubkeys = (t->by_index && !t->mixed) ? nullptr : t->pubkeys.data();
        b.pubkey_indices = t->by_index ? t->pk_idx.data() : nullptr;
        b.signatures = t->signatures.data();
        b.sig_offsets = t->sig_off.data();
        b.messages = t->messages.data();
        b.seed = t->seed.data();
        t->valid.assign(t->n_sets ? t->n_sets : 1, 0);
        t->job_fast.assign(t->n_jobs ? t->n_jobs : 1, 0);
        // in flight like a verify call (the package's per-set retries run when it retires)
        const int rc =
            lb_verify_same_message_batch_async(c->ctx, &b, t->valid.data(), t->job_fast.data(), &t->ticket);
        if (rc != LB_OK) {
          fail(t, rc, c->ctx);
          t->t_end = now_ns();
          complete(c, t);
        } else {
          inflight.push_back(t);
        }
        break;
      }
      case Kind::SyncPubkeys: {
        int32_t bad = -1;
        const int rc = lb_pubkey_table_append(c->ctx, t->n_keys, t->pubkeys.data(), t->pk_len, &bad);
        if (rc != LB_OK) {
          fail(t, rc, c->ctx);
          if (bad >= 0) t->errmsg += " (pubkey " + std::to_string(bad) + ")";
        } else {
          lb_pubkey_table_size(c->ctx, &t->u32);
          if (c->lctx && c->lane_ok) {  // the same keys into the latency lane's table, then resolve
            {
              std::lock_guard<std::mutex> lk(c->lmu);
              c->lqueue.push_back(t);
            }
            c->lcv.notify_one();
            break;
          }
        }
        complete(c, t);
        break;
      }
      case Kind::AggPubkeys: {
        t->out_bytes.assign(LB_PUBKEY_BYTES, 0);
        uint8_t st = 0;
        const int rc = t->by_index
                           ? lb_aggregate_pubkeys_indexed(c->ctx, t->n_keys, t->pk_idx.data(), t->out_bytes.data(), &st)
                           : lb_aggregate_pubkeys(c->ctx, t->n_keys, t->pubkeys.data(), t->out_bytes.data(), &st);
        if (rc != LB_OK)
          fail(t, rc, c->ctx);
        else if (st != LB_SET_OK) {
          t->rc = LB_ERR_INVALID_ARGUMENT;
          t->errmsg = "invalid pubkey";
        }
        complete(c, t);
        break;
      }
      case Kind::GtCheck: {
        const int rc = lb_gt_check(c->ctx, t->n_keys, t->out_bytes.data(), &t->i32);
        if (rc != LB_OK) fail(t, rc, c->ctx);
        complete(c, t);
        break;
      }
      case Kind::Close: {
        for (Task* w : prio) {
          const int rc = lb_wait(c->ctx, w->ticket, &w->stats);
          if (rc != LB_OK) fail(w, rc, c->ctx);
          complete(c, w);
        }
        prio.clear();
        while (!inflight.empty()) {  // never destroy the context under a call in flight
          Task* w = inflight.front();
          inflight.pop_front();
          Task* owner = w->kind == Kind::Finish ? w->target : w;
          const int rc = lb_wait(c->ctx, owner->ticket, &owner->stats);
          if (rc != LB_OK) fail(w, rc, c->ctx);
          if (w->kind == Kind::Finish) {
            w->valid.swap(owner->valid);
            w->err.swap(owner->err);
            w->sst.swap(owner->sst);
            w->stats = owner->stats;
            w->n_req = owner->n_req;
            w->n_sets = owner->n_sets;
            w->refs.swap(owner->refs);
            c->partials.erase(owner->partial_id);
            delete owner;
          }
          complete(c, w);
        }
        for (auto& kv : c->partials) delete kv.second;
        c->partials.clear();
        lane_join(c);  // (its queued priority calls complete first)
        lb_destroy(c->ctx);
        c->ctx = nullptr;
        complete(c, t);
        return;
      }
    }
  }
  // finalizer path (Context garbage-collected without close())
  for (Task* w : prio) {
    lb_wait(c->ctx, w->ticket, nullptr);
    delete w;
  }
  for (Task* w : inflight) {
    Task* owner = w->kind == Kind::Finish ? w->target : w;
    lb_wait(c->ctx, owner->ticket, nullptr);
    delete w;
  }
  for (auto& kv : c->partials) delete kv.second;
  lane_join(c);
  lb_destroy(c->ctx);
  c->ctx = nullptr;
}

// ---- JS side -----------------------------------------------------------------------
napi_value make_u8(napi_env env, const uint8_t* p, size_t n) {
  napi_value ab, arr;
  void* data = nullptr;
  NAPI_OK(napi_create_arraybuffer(env, n, &data, &ab));
  if (n) memcpy(data, p, n);
  NAPI_OK(napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &arr));
  return arr;
}

void set_num(napi_env env, napi_value obj, const char* k, double v) {
  napi_value x;
  napi_create_double(env, v, &x);
  napi_set_named_property(env, obj, k, x);
}

napi_value make_error(napi_env env, int rc, const std::string& msg) {
  const char* code = rc == LB_ERR_INVALID_ARGUMENT ? "LB_ERR_INVALID_ARGUMENT"
                     : rc == LB_ERR_DEVICE         ? "LB_ERR_DEVICE"
                     : rc == LB_ERR_NO_DEVICE      ? "LB_ERR_NO_DEVICE"
                     : rc == LB_ERR_OUT_OF_MEMORY  ? "LB_ERR_OUT_OF_MEMORY"
                     : rc == LB_ERR_RESOURCES      ? "LB_ERR_RESOURCES"
                                                   : "LB_ERR";
  napi_value c, m, e;
  napi_create_string_utf8(env, code, NAPI_AUTO_LENGTH, &c);
  napi_create_string_utf8(env, msg.c_str(), NAPI_AUTO_LENGTH, &m);
  napi_create_error(env, c, m, &e);
  return e;
}

napi_value verify_result(napi_env env, Task* t) {
  napi_value o;
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "valid", make_u8(env, t->valid.data(), t->n_req));
  napi_set_named_property(env, o, "errors", make_u8(env, t->err.data(), t->n_req));
  napi_set_named_property(env, o, "setStatus", make_u8(env, t->sst.data(), t->n_sets));
  set_num(env, o, "batchRetries", t->stats.batch_retries);
  set_num(env, o, "batchSigsSuccess", t->stats.batch_sigs_success);
  set_num(env, o, "deviceMs", t->stats.device_ms);
  set_num(env, o, "workerStartNs", (double)t->t_start);
  set_num(env, o, "workerEndNs", (double)t->t_end);
  set_num(env, o, "workerSubmittedNs", (double)t->t_submitted);  // lb_verify_requests_async returned
  set_num(env, o, "workerRetireNs", (double)t->t_retire);        // lb_wait called on it
  if (t->clk[2] > t->clk[0]) {  // latency lane: the kernel's own time and shader clock
    const double rt = (double)(t->clk[2] - t->clk[0]);
    set_num(env, o, "kernelMs", rt / 1e5);
    set_num(env, o, "kernelClockMHz", (double)(t->clk[3] - t->clk[1]) / rt * 100.0);
  }
  if (t->n_stage > 0) {
    napi_value st;
    napi_create_object(env, &st);
    for (int i = 0; i < t->n_stage; i++)
      if (t->stage_names[i]) set_num(env, st, t->stage_names[i], t->stage_ms[i]);
    napi_set_named_property(env, o, "stageMs", st);
  }
  return o;
}

void call_js(napi_env env, napi_value /*cb*/, void* context, void* data) {
  Context* c = static_cast<Context*>(context);
  Task* t = static_cast<Task*>(data);
  if (env == nullptr) {  // environment tearing down
    delete t;
    return;
  }
  release_refs(env, t);
  napi_value result = nullptr;
  if (t->rc != LB_OK) {
    napi_reject_deferred(env, t->deferred, make_error(env, t->rc, t->errmsg));
  } else {
    switch (t->kind) {
      case Kind::Verify:
      case Kind::Finish:
        result = verify_result(env, t);
        break;
      case Kind::Partial: {
        napi_create_object(env, &result);
        set_num(env, result, "id", (double)t->partial_id);
        napi_set_named_property(env, result, "partial", make_u8(env, t->out_bytes.data(), LB_GT_BYTES));
        break;
      }
      case Kind::SameMessage:
        napi_create_object(env, &result);
        napi_set_named_property(env, result, "valid", make_u8(env, t->valid.data(), t->n_sets));
        napi_set_named_property(env, result, "jobFast", make_u8(env, t->job_fast.data(), t->n_jobs));
        set_num(env, result, "retriedJobs", t->stats.batch_retries);
        set_num(env, result, "fastSets", t->stats.batch_sigs_success);
        set_num(env, result, "deviceMs", t->stats.device_ms);
        set_num(env, result, "workerStartNs", (double)t->t_start);
        set_num(env, result, "workerEndNs", (double)t->t_end);
        break;
      case Kind::SyncPubkeys:
        napi_create_uint32(env, t->u32, &result);
        break;
      case Kind::AggPubkeys:
        result = make_u8(env, t->out_bytes.data(), LB_PUBKEY_BYTES);
        break;
      case Kind::GtCheck:
        napi_get_boolean(env, t->i32 != 0, &result);
        break;
      case Kind::Close:
        napi_get_undefined(env, &result);
        break;
    }
    napi_resolve_deferred(env, t->deferred, result);
  }
  const bool closed = t->kind == Kind::Close;
  delete t;
  if (--c->pending == 0 && !closed) napi_unref_threadsafe_function(env, c->tsfn);
  if (closed) {
    if (c->worker.joinable()) c->worker.join();
    c->joined = true;
    napi_release_threadsafe_function(c->tsfn, napi_tsfn_release);
    c->tsfn = nullptr;
  }
}

Context* unwrap(napi_env env, napi_callback_info info, size_t* argc, napi_value* argv) {
  napi_value self;
  napi_get_cb_info(env, info, argc, argv, &self, nullptr);
  void* p = nullptr;
  napi_unwrap(env, self, &p);
  return static_cast<Context*>(p);
}

// Queue a task; returns its promise (rejected at once when the context is closed).
napi_value submit(napi_env env, Context* c, Task* t) {
  napi_value promise;
  napi_create_promise(env, &t->deferred, &promise);
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->closing) {
      napi_reject_deferred(env, t->deferred, make_error(env, LB_ERR_INVALID_ARGUMENT, "QUEUE_ERROR_QUEUE_ABORTED: context closed"));
      release_refs(env, t);
      delete t;
      return promise;
    }
    if (t->kind == Kind::Close) c->closing = true;
    if (t->prio && t->kind == Kind::Verify && c->lctx && c->lane_ok) {
      // the latency lane: its own thread and context; the throughput context's calls
      // submitted from now on leave the reserved CUs free (lb_mark_priority)
      lb_mark_priority(c->ctx);
      {
        std::lock_guard<std::mutex> lk2(c->lmu);
        c->lqueue.push_back(t);
      }
      if (c->pending++ == 0) napi_ref_threadsafe_function(env, c->tsfn);
      c->lcv.notify_one();
      return promise;
    }
    if (t->prio) {  // ahead of every queued non-priority task, behind earlier priority ones
      auto it = c->queue.begin();
      while (it != c->queue.end() && (*it)->prio) ++it;
      c->queue.insert(it, t);
    } else {
      c->queue.push_back(t);
    }
  }
  if (c->pending++ == 0) napi_ref_threadsafe_function(env, c->tsfn);
  c->cv.notify_one();
  return promise;
}

napi_value rejected(napi_env env, const std::string& msg) {
  napi_deferred d;
  napi_value promise, m, e;
  napi_create_promise(env, &d, &promise);
  napi_create_string_utf8(env, msg.c_str(), NAPI_AUTO_LENGTH, &m);
  napi_create_type_error(env, nullptr, m, &e);
  napi_reject_deferred(env, d, e);
  return promise;
}

napi_value m_verify(napi_env env, napi_callback_info info, Kind kind) {
  size_t argc = 2;
  napi_value argv[2];
  Context* c = unwrap(env, info, &argc, argv);
  if (!c) return rejected(env, "not a Context");
  Task* t = new Task();
  t->kind = kind;
  try {
    if (argc < 1) throw ArgError{"verifyRequests(batch[, {priority}])"};
    parse_requests(env, argv[0], *t);
    napi_value pv;
    napi_valuetype ty = napi_undefined;
    if (argc >= 2) napi_typeof(env, argv[1], &ty);
    if (kind == Kind::Verify && ty == napi_object && has_prop(env, argv[1], "priority", &pv)) {
      bool b = false;
      napi_get_value_bool(env, pv, &b);
      t->prio = b;
    }
  } catch (const ArgError& e) {
    release_refs(env, t);
    delete t;
    return rejected(env, e.msg);
  }
  if (kind == Kind::Partial) t->partial_id = c->next_partial++;
  return submit(env, c, t);
}
napi_value VerifyRequests(napi_env env, napi_callback_info info) { return m_verify(env, info, Kind::Verify); }
napi_value VerifyRequestsPartial(napi_env env, napi_callback_info info) { return m_verify(env, info, Kind::Partial); }

napi_value Finish(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  Context* c = unwrap(env, info, &argc, argv);
  if (!c || argc < 2) return rejected(env, "finish(id, mergedOk)");
  double id = 0;
  bool ok = false;
  if (napi_get_value_double(env, argv[0], &id) != napi_ok || napi_get_value_bool(env, argv[1], &ok) != napi_ok)
    return rejected(env, "finish(id: number, mergedOk: boolean)");
  Task* t = new Task();
  t->kind = Kind::Finish;
  t->partial_id = (uint64_t)id;
  t->merged_ok = ok ? 1 : 0;
  return submit(env, c, t);
}

napi_value GtCheck(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  Context* c = unwrap(env, info, &argc, argv);
  Task* t = new Task();
  t->kind = Kind::GtCheck;
  try {
    if (!c || argc < 1) throw ArgError{"gtCheck(partials: Uint8Array)"};
    typed(env, argv[0], napi_uint8_array, "partials", t->out_bytes);
    if (t->out_bytes.size() % LB_GT_BYTES) throw ArgError{"partials: 576 bytes each"};
    t->n_keys = (uint32_t)(t->out_bytes.size() / LB_GT_BYTES);
    if (t->out_bytes.empty()) t->out_bytes.push_back(0);
  } catch (const ArgError& e) {
    delete t;
    return rejected(env, e.msg);
  }
  return submit(env, c, t);
}

napi_value VerifySameMessage(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  Context* c = unwrap(env, info, &argc, argv);
  Task* t = new Task();
  t->kind = Kind::SameMessage;
  try {
    if (!c || argc < 1) throw ArgError{"verifySameMessage(batch)"};
    napi_value o = argv[0];
    req_typed(env, o, "jobOffsets", napi_uint32_array, t->job_off);
    if (t->job_off.empty()) throw ArgError{"jobOffsets: wrong length"};
    t->n_jobs = (uint32_t)t->job_off.size() - 1;
    t->n_sets = t->job_off.back();
    check_offsets(t->job_off, t->n_jobs, UINT32_MAX, "jobOffsets");
    req_typed(env, o, "signatures", napi_uint8_array, t->signatures);
    req_typed(env, o, "sigOffsets", napi_uint32_array, t->sig_off);
    check_offsets(t->sig_off, t->n_sets, (uint32_t)t->signatures.size(), "sigOffsets");
    req_typed(env, o, "messages", napi_uint8_array, t->messages);
    if (t->messages.size() != (size_t)t->n_jobs * 32) throw ArgError{"messages: 32 bytes per job"};
    req_typed(env, o, "seed", napi_uint8_array, t->seed);
    if (t->seed.size() != 32) throw ArgError{"seed must be 32 bytes"};
    t->by_index = opt_typed(env, o, "pubkeyIndices", napi_uint32_array, t->pk_idx);
    if (t->by_index) {
      if (t->pk_idx.size() != t->n_sets) throw ArgError{"pubkeyIndices: one per set"};
      // mixed package: rows of `pubkeys` named by indices with LB_PK_ROW_FLAG set
      size_t rows = 0;
      for (uint32_t j : t->pk_idx)
        if ((j & LB_PK_ROW_FLAG) && (size_t)(j & LB_PK_ROW_MASK) + 1 > rows) rows = (j & LB_PK_ROW_MASK) + 1;
      t->mixed = opt_typed(env, o, "pubkeys", napi_uint8_array, t->pubkeys);
      if (rows && (!t->mixed || t->pubkeys.size() < rows * LB_PUBKEY_BYTES))
        throw ArgError{"pubkeyIndices name pubkey rows that `pubkeys` does not hold"};
    } else {
      if (!opt_typed(env, o, "pubkeys", napi_uint8_array, t->pubkeys) && t->n_sets)
        throw ArgError{"missing pubkeys (or pubkeyIndices)"};
      if (t->pubkeys.size() != (size_t)t->n_sets * LB_PUBKEY_BYTES) throw ArgError{"pubkeys: 96 bytes per set"};
    }
    for (auto* v : {&t->signatures, &t->messages, &t->pubkeys}) if (v->empty()) v->push_back(0);
    if (t->pk_idx.empty()) t->pk_idx.push_back(0);
  } catch (const ArgError& e) {
    delete t;
    return rejected(env, e.msg);
  }
  return submit(env, c, t);
}

napi_value SyncPubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  Context* c = unwrap(env, info, &argc, argv);
  Task* t = new Task();
  t->kind = Kind::SyncPubkeys;
  try {
    if (!c || argc < 2) throw ArgError{"syncPubkeys(keys: Uint8Array, pkLen: 48 | 96)"};
    typed(env, argv[0], napi_uint8_array, "keys", t->pubkeys);
    napi_get_value_uint32(env, argv[1], &t->pk_len);
    if (t->pk_len != 48 && t->pk_len != 96) throw ArgError{"pkLen must be 48 or 96"};
    if (t->pubkeys.size() % t->pk_len) throw ArgError{"keys: a whole number of keys"};
    t->n_keys = (uint32_t)(t->pubkeys.size() / t->pk_len);
    if (t->pubkeys.empty()) t->pubkeys.push_back(0);
  } catch (const ArgError& e) {
    delete t;
    return rejected(env, e.msg);
  }
  return submit(env, c, t);
}

napi_value AggregatePubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  Context* c = unwrap(env, info, &argc, argv);
  Task* t = new Task();
  t->kind = Kind::AggPubkeys;
  try {
    if (!c || argc < 1) throw ArgError{"aggregatePubkeys(keys: Uint8Array | indices: Uint32Array)"};
    napi_typedarray_type ty;
    size_t len;
    void* d;
    napi_value ab;
    size_t off;
    bool is = false;
    napi_is_typedarray(env, argv[0], &is);
    if (!is) throw ArgError{"aggregatePubkeys expects a typed array"};
    napi_get_typedarray_info(env, argv[0], &ty, &len, &d, &ab, &off);
    t->by_index = ty == napi_uint32_array;
    if (t->by_index) {
      typed(env, argv[0], napi_uint32_array, "indices", t->pk_idx);
      t->n_keys = (uint32_t)t->pk_idx.size();
    } else {
      typed(env, argv[0], napi_uint8_array, "keys", t->pubkeys);
      if (t->pubkeys.size() % LB_PUBKEY_BYTES) throw ArgError{"keys: 96 bytes each"};
      t->n_keys = (uint32_t)(t->pubkeys.size() / LB_PUBKEY_BYTES);
    }
    if (t->n_keys == 0) throw ArgError{"EMPTY_AGGREGATE_ARRAY"};
  } catch (const ArgError& e) {
    delete t;
    return rejected(env, e.msg);
  }
  return submit(env, c, t);
}

napi_value Close(napi_env env, napi_callback_info info) {
  size_t argc = 0;
  Context* c = unwrap(env, info, &argc, nullptr);
  if (!c) return rejected(env, "not a Context");
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->closing) {  // second close(): already resolved or pending
      napi_deferred d;
      napi_value p, u;
      napi_create_promise(env, &d, &p);
      napi_get_undefined(env, &u);
      napi_resolve_deferred(env, d, u);
      return p;
    }
  }
  Task* t = new Task();
  t->kind = Kind::Close;
  return submit(env, c, t);
}

void finalize_ctx(napi_env env, void* data, void* /*hint*/) {
  Context* c = static_cast<Context*>(data);
  if (!c->joined) {
    {
      std::lock_guard<std::mutex> lk(c->mu);
      c->finalizing = true;
      c->closing = true;
      for (Task* t : c->queue) {
        release_refs(env, t);
        delete t;
      }
      c->queue.clear();
    }
    {
      std::lock_guard<std::mutex> lk(c->lmu);
      for (Task* t : c->lqueue) {
        release_refs(env, t);
        delete t;
      }
      c->lqueue.clear();
    }
    c->cv.notify_one();
    if (c->worker.joinable()) c->worker.join();
    if (c->tsfn) napi_release_threadsafe_function(c->tsfn, napi_tsfn_abort);
  }
  delete c;
}

napi_value New(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], self;
  napi_get_cb_info(env, info, &argc, argv, &self, nullptr);
  int32_t device = 0;
  if (argc >= 1) napi_get_value_int32(env, argv[0], &device);
  int32_t capacity = 0;  // default: the library's calls in flight (lb_slots)
  napi_value v;
  if (argc >= 2 && has_prop(env, argv[1], "capacity", &v)) napi_get_value_int32(env, v, &capacity);
  lb_ctx* ctx = nullptr;
  const int rc = lb_create(device, &ctx);
  if (rc != LB_OK) {
    napi_throw(env, make_error(env, rc, "lb_create(" + std::to_string(device) + ") failed: " + lb_last_error(nullptr)));
    return nullptr;
  }
  if (capacity <= 0) capacity = lb_slots(ctx);
  Context* c = new Context();
  c->ctx = ctx;
  c->device = device;
  c->capacity = capacity < 1 ? 1 : capacity;
  c->env = env;
  {
    const char* e = getenv("LB_PRIO_THREAD");
    if (!(e && atoi(e) == 0) && lb_create_lane(device, &c->lctx) != LB_OK) c->lctx = nullptr;  // (then: no lane)
  }
  napi_value name;
  napi_create_string_utf8(env, "lodestar_bls_gpu", NAPI_AUTO_LENGTH, &name);
  napi_create_threadsafe_function(env, nullptr, nullptr, name, 0, 1, nullptr, nullptr, c, call_js, &c->tsfn);
  napi_unref_threadsafe_function(env, c->tsfn);  // idle contexts do not keep the process alive
  c->worker = std::thread(worker_loop, c);
  if (c->lctx) c->lane = std::thread(lane_loop, c);
  napi_wrap(env, self, c, finalize_ctx, nullptr, nullptr);
  napi_value dev, cap;
  napi_create_int32(env, device, &dev);
  napi_set_named_property(env, self, "device", dev);
  napi_create_int32(env, c->capacity, &cap);
  napi_set_named_property(env, self, "capacity", cap);
  return self;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
  napi_value r;
  napi_create_int32(env, lb_device_count(), &r);
  return r;
}

// Marshalling dry run (no device): the same checks verifyRequests applies.
napi_value ValidateRequests(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  Task t;
  try {
    if (argc < 1) throw ArgError{"validateRequests(batch)"};
    parse_requests(env, argv[0], t);
  } catch (const ArgError& e) {
    release_refs(env, &t);
    napi_throw_type_error(env, nullptr, e.msg.c_str());
    return nullptr;
  }
  release_refs(env, &t);
  napi_value o;
  napi_create_object(env, &o);
  set_num(env, o, "nRequests", t.n_req);
  set_num(env, o, "nSets", t.n_sets);
  set_num(env, o, "nPubkeys", t.has_pk_off ? t.pk_off[t.n_sets] : t.n_sets);
  napi_value b;
  napi_get_boolean(env, t.by_index, &b);
  napi_set_named_property(env, o, "byIndex", b);
  return o;
}

napi_value Init(napi_env env, napi_value exports) {
  // 16 HIP hardware queues for this process: the library keeps one call in flight per
  // queue (lb_slots), 3.03 vs 2.74 M sets/s over HIP's default 4 (profiles/ab_r03/hwq2).
  // Before the first HIP call (lb_create).  A GPU_MAX_HW_QUEUES the host already set
  // wins; LB_HW_QUEUES picks another count, clamped to [1, 16] -- lb_create refuses
  // more (each queue reserves scratch for the largest private segment).
  int nq = 16;
  if (const char* q = getenv("LB_HW_QUEUES")) nq = atoi(q) < 1 ? 1 : atoi(q) > 16 ? 16 : atoi(q);
  char qs[8];
  snprintf(qs, sizeof qs, "%d", nq);
  setenv("GPU_MAX_HW_QUEUES", qs, 0);
  // no per-stage timing events in the library (nothing on the JS side reads them; they
  // are two HIP calls per kernel on the submission thread); LB_STAGE_EVENTS=1 keeps them
  setenv("LB_STAGE_EVENTS", "0", 0);
  napi_property_descriptor methods[] = {
      {"verifyRequests", nullptr, VerifyRequests, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"verifyRequestsPartial", nullptr, VerifyRequestsPartial, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"finish", nullptr, Finish, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"gtCheck", nullptr, GtCheck, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"verifySameMessage", nullptr, VerifySameMessage, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"syncPubkeys", nullptr, SyncPubkeys, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"aggregatePubkeys", nullptr, AggregatePubkeys, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"close", nullptr, Close, nullptr, nullptr, nullptr, napi_default, nullptr},
  };
  napi_value cls;
  napi_define_class(env, "Context", NAPI_AUTO_LENGTH, New, nullptr, sizeof(methods) / sizeof(methods[0]), methods,
                    &cls);
  napi_set_named_property(env, exports, "Context", cls);
  napi_value f;
  napi_create_function(env, "deviceCount", NAPI_AUTO_LENGTH, DeviceCount, nullptr, &f);
  napi_set_named_property(env, exports, "deviceCount", f);
  napi_create_function(env, "validateRequests", NAPI_AUTO_LENGTH, ValidateRequests, nullptr, &f);
  napi_set_named_property(env, exports, "validateRequests", f);
  napi_value sz;
  napi_create_int32(env, LB_GT_BYTES, &sz);
  napi_set_named_property(env, exports, "GT_BYTES", sz);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
