"use strict";
/**
 * BlsGpuVerifier: IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:25-68)
 * over MI355X GPUs, through the N-API addon (lodestar_amd/napi/addon.cc).  It is
 * what chain.ts:206-208 would construct beside BlsMultiThreadWorkerPool; its
 * scheduling is the pool's (chain/bls/multithread/index.ts:114-580) with GPUs in
 * place of worker threads:
 *
 *  - verifySignatureSets(sets, opts) -> Promise<boolean>            (index.ts:163-213)
 *  - verifySignatureSetsSameMessage(sets, message, opts) -> boolean[] (index.ts:218-242)
 *  - close() / canAcceptWork()                                       (index.ts:244-265,155-161)
 *  - sets chunked to <= 128 per job (chunkifyMaximizeChunkSize, utils.ts:4-19)
 *  - batchable jobs buffered up to 100 ms or > 32 sig sets (index.ts:327-343),
 *    priority jobs to the queue front (index.ts:544-555)
 *  - an aggregate set with zero pubkeys rejects its job (index.ts:403-409)
 *  - a same-message job that fails is retried set by set (index.ts:473-484,557-568)
 *    -- on the GPU, inside the same batched call (lb_verify_same_message_batch)
 *
 * What changes for a GPU: a package may hold up to maxSetsPerDispatch (65,536)
 * sig sets, because the GPU wants tens of thousands of sets per call; every job
 * keeps its own verdict (per-request verdicts on the device), so merging never
 * changes a verdict (worker.ts:74-85 guarantees the same on CPU by re-verifying).
 * Each GPU takes up to `capacity` packages at once (the addon's in-flight slots).
 *
 * Sets: {type: "single", pubkey, signingRoot, signature} or
 *       {type: "aggregate", pubkeys, signingRoot, signature}
 * (ISignatureSet, state-transition/src/util/signatureSets.ts:5-24).  A pubkey is:
 *  - a @chainsafe/bls PublicKey, as every reference set builder passes one out of
 *    index2pubkey (state-transition/src/signatureSets/indexedAttestation.ts:27,
 *    proposer.ts:28, randao.ts:30, ...).  One mirrored by syncPubkeys (the index2pubkey
 *    mirror of state-transition/src/cache/pubkeyCache.ts:56-77) ships as its 4-byte
 *    validator index (an identity map, no serialization on the main thread); any other
 *    is serialized with toBytes(PointFormat.uncompressed) as the reference does
 *    (BN/chain/bls/multithread/index.ts:144, jobItem.ts:59);
 *  - a Uint8Array: the 96-byte uncompressed or the 48-byte compressed encoding
 *    (compressed keys are decompressed on the GPU: LB_PK_ROW48_FLAG rows);
 *  - {index}: a validator index into the device pubkey table.
 */
const crypto = require("crypto");
const path = require("path");

const MAX_SIGNATURE_SETS_PER_JOB = 128; // index.ts:57
const MAX_BUFFERED_SIGS = 32; // index.ts:66
const MAX_BUFFER_WAIT_MS = 100; // index.ts:75
const MAX_JOBS_CAN_ACCEPT_WORK = 512; // index.ts:80
// one priority-lane package: at most this many sets (the library's latency path,
// lb_set_latency_path's default 1024, runs calls up to that size)
const MAX_PRIORITY_LANE_SETS = 1024;
const BATCHABLE_MIN_PER_CHUNK = 16; // worker.ts:17
// a package of more sets is packed in slices of this many, yielding to the event loop
const PACK_SLICE_SETS = 8192;
const LB_PK_ROW_FLAG = 0x80000000;
const LB_PK_ROW48_FLAG = 0x40000000; // the row holds a 48-byte compressed encoding
const LB_PK_ROW_MASK = 0x3fffffff;
// @chainsafe/bls PointFormat (the reference passes PointFormat.uncompressed to toBytes,
// BN/chain/bls/multithread/index.ts:144 -> jobItem.ts:59,80)
const PointFormat = {compressed: "compressed", uncompressed: "uncompressed"};
const LB_REQ_EMPTY_AGGREGATE = 1;
const LB_REQ_BAD_PUBKEY = 2;
const GT_BYTES = 576;

const QueueErrorCode = {QUEUE_ABORTED: "QUEUE_ERROR_QUEUE_ABORTED"};

class QueueError extends Error {
  constructor(code) {
    super(code);
    this.type = {code};
  }
}

/** The pool's job queue: push / unshift / shift in O(1) (a package takes 512 jobs from a
 * queue that can hold ~50k under load; Array.prototype.shift on that moved the whole
 * array per job). */
class JobQueue {
  constructor() {
    this.a = [];
    this.h = 0;
  }
  get length() {
    return this.a.length - this.h;
  }
  at(i) {
    return this.a[this.h + i];
  }
  push(x) {
    this.a.push(x);
  }
  unshift(x) {
    if (this.h > 0) this.a[--this.h] = x;
    else this.a.unshift(x);
  }
  shift() {
    if (this.h >= this.a.length) return undefined;
    const x = this.a[this.h];
    this.a[this.h++] = undefined;
    if (this.h > 1024 && this.h * 2 > this.a.length) {
      this.a = this.a.slice(this.h);
      this.h = 0;
    }
    return x;
  }
  clear() {
    const rest = this.a.slice(this.h);
    this.a = [];
    this.h = 0;
    return rest;
  }
}

function loadAddon() {
  return require(path.join(__dirname, "..", "napi", "lodestar_bls.node"));
}

/** utils.ts:4-19 */
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
}

/** (batchRetries, batchSigsSuccess) of one package as the reference worker counts them
 * (worker.ts:41-85): batchable requests chunked by >= 16, one retry per failed chunk. */
function workerBatchStats(requestSizes, batchable, valid) {
  const idx = [];
  for (let k = 0; k < batchable.length; k++) if (batchable[k]) idx.push(k);
  let retries = 0;
  let sigsOk = 0;
  if (idx.length === 0) return {retries, sigsOk};
  for (const chunk of chunkifyMaximizeChunkSize(idx, BATCHABLE_MIN_PER_CHUNK)) {
    const n = chunk.reduce((s, k) => s + requestSizes[k], 0);
    if (n > 0 && chunk.every((k) => valid[k])) sigsOk += n;
    else retries++;
  }
  return {retries, sigsOk};
}

function concat(arrays, total) {
  const out = new Uint8Array(total);
  let o = 0;
  for (const a of arrays) {
    out.set(a, o);
    o += a.length;
  }
  return out;
}

/** Requests (arrays of sets) -> the addon's batch (lb_request_batch layout).  Two passes:
 * count, then fill typed arrays allocated once (no per-set or per-key objects: a 65,536-set
 * package was ~75 ms of main-thread JS with intermediate arrays, the node leg's bound).
 * keyMap (optional WeakMap PublicKey -> validator index, BlsGpuVerifier.syncPubkeys) turns
 * mirrored key objects into indices; every other key is serialized once (first pass). */
function packRequests(requests, seed, keyMap) {
  const it = packRequestsGen(requests, seed, keyMap, Infinity);
  let r = it.next();
  while (!r.done) r = it.next();
  return r.value;
}

/** packRequests in slices of `slice` sets with the event loop turning between them: a
 * 65,536-set package is ~4 ms of main-thread work, and a priority call's completion
 * (or a gossip handler) must not wait for all of it (VERDICT r4 #2).  `timing`
 * (optional): timing.mainThreadS receives the sum of the synchronous slices alone -- the
 * main thread's own share, without the turns spent on other work in between (ADVICE r5). */
async function packRequestsAsync(requests, seed, keyMap, slice = 8192, timing = null) {
  const it = packRequestsGen(requests, seed, keyMap, slice);
  let busy = 0n;
  let t0 = process.hrtime.bigint();
  let r = it.next();
  busy += process.hrtime.bigint() - t0;
  while (!r.done) {
    await new Promise((res) => setImmediate(res));
    t0 = process.hrtime.bigint();
    r = it.next();
    busy += process.hrtime.bigint() - t0;
  }
  if (timing) timing.mainThreadS = Number(busy) / 1e9;
  return r.value;
}

function* packRequestsGen(requests, seed, keyMap, slice) {
  // pass 1: sizes; pass 2: every key's index (one identity-map lookup per key) or its
  // encoding; pass 3: the arrays.  Between slices of `slice` sets the caller may yield.
  let nSets = 0;
  let nKeys = 0;
  let sigBytes = 0;
  for (const req of requests) {
    for (const s of req) {
      nKeys += s.type === "aggregate" ? (s.pubkeys || []).length : 1;
      if (!(s.signingRoot instanceof Uint8Array) || s.signingRoot.length !== 32)
        throw new TypeError("signingRoot must be 32 bytes");
      sigBytes += s.signature.length;
      nSets++;
    }
  }
  // the final index words, written here: a table index, or a flagged row of the keys shipped
  // by their encodings (LB_PK_ROW_FLAG | LB_PK_ROW48_FLAG for a compressed one | row)
  const keyIx = new Uint32Array(nKeys);
  const rowKeys = []; // encodings of the keys shipped as rows, in order
  let nIdx = 0;
  let nComp = 0;
  let k = 0;
  let sinceYield = 0;
  const sym = keyMap ? keyMap.lbIndexSymbol : undefined;
  const lookKey = (pk) => {
    const ix = keyIndex(pk, keyMap);
    if (ix >= 0) {
      keyIx[k++] = ix;
      nIdx++;
      return;
    }
    const b = keyBytes(pk);
    if (b.length === 48) nComp++;
    keyIx[k++] = (LB_PK_ROW_FLAG | (b.length === 48 ? LB_PK_ROW48_FLAG : 0) | rowKeys.length) >>> 0;
    rowKeys.push(b);
  };
  for (const req of requests) {
    for (const s of req) {
      if (s.type === "aggregate") {
        const ks = s.pubkeys || [];
        for (let q = 0; q < ks.length; q++) {
          // (a mirrored key object: its index as a property read, no call)
          const pk = ks[q];
          const ix = sym !== undefined && pk !== null && typeof pk === "object" ? pk[sym] : undefined;
          if (ix !== undefined) {
            keyIx[k++] = ix;
            nIdx++;
          } else lookKey(pk);
        }
      } else lookKey(s.pubkey);
    }
    if ((sinceYield += req.length) >= slice) {
      sinceYield = 0;
      yield;
    }
  }
  const reqOff = new Uint32Array(requests.length + 1);
  const pkOff = new Uint32Array(nSets + 1);
  const sigOff = new Uint32Array(nSets + 1);
  const messages = new Uint8Array(32 * nSets);
  const signatures = new Uint8Array(sigBytes);
  // all keys by validator index; a mixed package (a capella block's BLS-change keys beside
  // validator keys, or compressed keys): indices plus flagged indices naming rows of the
  // shipped keys (LB_PK_ROW_FLAG, LB_PK_ROW48_FLAG for a compressed row); no index and no
  // compressed key: the 96-byte encodings
  const mixed = nIdx > 0 || nComp > 0;
  const idx = mixed ? keyIx : null;
  const rows = rowKeys.length > 0 ? new Uint8Array(96 * rowKeys.length) : null;
  for (let r = 0; r < rowKeys.length; r++) rows.set(rowKeys[r], 96 * r);
  let i = 0;
  let so = 0;
  k = 0;
  for (let r = 0; r < requests.length; r++) {
    for (const s of requests[r]) {
      k += s.type === "aggregate" ? (s.pubkeys || []).length : 1;
      pkOff[i + 1] = k;
      messages.set(s.signingRoot, 32 * i);
      signatures.set(s.signature, so);
      so += s.signature.length;
      sigOff[i + 1] = so;
      i++;
    }
    reqOff[r + 1] = i;
    if ((sinceYield += requests[r].length) >= slice) {
      sinceYield = 0;
      yield;
    }
  }
  const batch = {requestOffsets: reqOff, pkOffsets: pkOff, messages, signatures, sigOffsets: sigOff, seed};
  if (idx) batch.pubkeyIndices = idx;
  if (rows) batch.pubkeys = rows;
  return batch;
}

/** A key's validator index, or -1 for a key shipped by its bytes (a 96- or 48-byte
 * encoding, or a PublicKey object that syncPubkeys has not mirrored). */
function keyIndex(pk, keyMap) {
  if (pk instanceof Uint8Array) {
    if (pk.length !== 96 && pk.length !== 48) throw new TypeError("pubkey: 96-byte uncompressed or 48-byte compressed encoding");
    return -1;
  }
  if (pk && typeof pk === "object") {
    if (keyMap) {
      // the index the key's own object carries (a symbol property of this key map, set by
      // syncPubkeys: one inline-cached property read per key), else the identity map
      const sym = keyMap.lbIndexSymbol;
      if (sym !== undefined) {
        const ix = pk[sym];
        if (ix !== undefined) return ix;
      }
      const ix = keyMap.get(pk);
      if (ix !== undefined) return ix;
    }
    if (typeof pk.index === "number") return pk.index;
    if (typeof pk.toBytes === "function") return -1;
  }
  throw new TypeError("pubkey: a PublicKey (toBytes(format)), Uint8Array(96 | 48) or {index}");
}

/** The encoding of a key shipped by its bytes: a PublicKey serialized as the reference does,
 * toBytes(PointFormat.uncompressed) (index.ts:144, jobItem.ts:59); an implementation that
 * returns its compressed form instead is taken as such (decompressed on the GPU). */
function keyBytes(pk) {
  const b = pk instanceof Uint8Array ? pk : pk.toBytes(PointFormat.uncompressed);
  if (!(b instanceof Uint8Array) || (b.length !== 96 && b.length !== 48))
    throw new TypeError("pubkey: toBytes() must return a 96-byte uncompressed or 48-byte compressed encoding");
  return b;
}

/** Same-message jobs -> the addon's lb_same_message_batch layout (keys as packRequests:
 * mirrored key objects by index; the rest by their encodings). */
function packSameMessage(jobs, seed, keyMap) {
  let nSets = 0;
  let nIdx = 0;
  let nComp = 0;
  let sigBytes = 0;
  const rowKeys = [];
  for (const job of jobs) {
    for (const s of job.sets) {
      if (keyIndex(s.publicKey, keyMap) >= 0) nIdx++;
      else {
        const b = keyBytes(s.publicKey);
        if (b.length === 48) nComp++;
        rowKeys.push(b);
      }
      sigBytes += s.signature.length;
      nSets++;
    }
  }
  // every key by index, every key by its 96 bytes, or a mixed package (flagged rows)
  const mixed = nIdx > 0 || nComp > 0;
  const jobOff = new Uint32Array(jobs.length + 1);
  const sigOff = new Uint32Array(nSets + 1);
  const signatures = new Uint8Array(sigBytes);
  const messages = new Uint8Array(32 * jobs.length);
  const idx = mixed ? new Uint32Array(nSets) : null;
  const pks = rowKeys.length > 0 ? new Uint8Array(96 * rowKeys.length) : null;
  let i = 0;
  let so = 0;
  let row = 0;
  for (let j = 0; j < jobs.length; j++) {
    messages.set(jobs[j].message, 32 * j);
    for (const s of jobs[j].sets) {
      const ix = keyIndex(s.publicKey, keyMap);
      if (ix >= 0) idx[i] = ix;
      else {
        const b = rowKeys[row];
        pks.set(b, 96 * row);
        if (idx) idx[i] = (LB_PK_ROW_FLAG | (b.length === 48 ? LB_PK_ROW48_FLAG : 0) | row) >>> 0;
        row++;
      }
      signatures.set(s.signature, so);
      so += s.signature.length;
      sigOff[i + 1] = so;
      i++;
    }
    jobOff[j + 1] = i;
  }
  const batch = {jobOffsets: jobOff, signatures, sigOffsets: sigOff, messages, seed};
  if (idx) batch.pubkeyIndices = idx;
  if (pks) batch.pubkeys = pks;
  return batch;
}

/** The reference's metric names (metrics/metrics/lodestar.ts:379-510), in-process. */
class PoolMetrics {
  constructor() {
    this.values = new Map();
    this.hist = new Map();
  }
  key(name, labels) {
    const l = labels ? Object.keys(labels).sort().map((k) => `${k}="${labels[k]}"`).join(",") : "";
    return l ? `${name}{${l}}` : name;
  }
  inc(name, v = 1, labels) {
    const k = this.key(name, labels);
    this.values.set(k, (this.values.get(k) || 0) + v);
  }
  set(name, v, labels) {
    this.values.set(this.key(name, labels), v);
  }
  observe(name, v, labels) {
    const k = this.key(name, labels);
    const h = this.hist.get(k) || {count: 0, sum: 0};
    h.count++;
    h.sum += v;
    this.hist.set(k, h);
  }
  get(name, labels) {
    return this.values.get(this.key(name, labels)) || 0;
  }
}

const P = "lodestar_bls_thread_pool_";
const M = {
  AGGREGATED_PUBKEYS: "lodestar_bls_aggregated_pubkeys_total",
  JOBS_WORKER_TIME: P + "time_seconds_sum",
  SUCCESS_JOBS_SETS: P + "success_jobs_signature_sets_count",
  ERROR_AGGREGATE_SETS: P + "error_aggregate_signature_sets_count",
  ERROR_JOBS_SETS: P + "error_jobs_signature_sets_count",
  JOB_WAIT_TIME: P + "queue_job_wait_time_seconds",
  QUEUE_LENGTH: P + "queue_length",
  WORKERS_BUSY: P + "workers_busy",
  JOB_GROUPS_STARTED: P + "job_groups_started_total",
  JOBS_STARTED: P + "jobs_started_total",
  SIG_SETS_STARTED: P + "sig_sets_started_total",
  BATCH_RETRIES: P + "batch_retries_total",
  BATCH_SIGS_SUCCESS: P + "batch_sigs_success_total",
  SAME_MESSAGE_RETRY_JOBS: P + "same_message_jobs_retries_total",
  SAME_MESSAGE_RETRY_SETS: P + "same_message_sets_retries_total",
  LATENCY_TO_WORKER: P + "latency_to_worker",
  LATENCY_FROM_WORKER: P + "latency_from_worker",
  MAIN_THREAD_TIME: P + "main_thread_time_seconds",
  TIME_PER_SIG_SET: "lodestar_bls_worker_thread_time_per_sigset_seconds",
  TOTAL_SIG_SETS: P + "sig_sets_total",
  PRIORITIZED_SIG_SETS: P + "prioritized_sig_sets_total",
  BATCHABLE_SIG_SETS: P + "batchable_sig_sets_total",
  // lodestar.ts:486,491: the main thread's share of deserialization / aggregation.  Both run on
  // the GPU here; what stays on the main thread is packing the keys and signature bytes
  SIG_DESERIALIZATION_MAIN_THREAD: P + "signature_deserialization_main_thread_time_seconds",
  PUBKEYS_AGGREGATION_MAIN_THREAD: P + "pubkeys_aggregation_main_thread_time_seconds",
  // lodestar.ts:500,505 (single-thread mode)
  SINGLE_THREAD_TIME: "lodestar_bls_single_thread_time_seconds",
  SINGLE_THREAD_TIME_PER_SIGSET: "lodestar_bls_single_thread_time_per_sigset_seconds",
};

/** Append keys to every backend's pubkey table; PublicKey objects are serialized with
 * toBytes(format) and mapped to their table index in keyMap.  Returns the table size. */
/** A mirrored key object also carries its table index under a symbol of its verifier's key
 * map (non-enumerable, read-only; frozen objects keep the WeakMap entry only): packing reads
 * it as a plain property instead of a WeakMap lookup (~3x fewer ns per key on 488-key
 * aggregates). */
function markKey(keyMap, k, index) {
  if (keyMap.lbIndexSymbol === undefined) keyMap.lbIndexSymbol = Symbol("lodestar-amd key index");
  try {
    Object.defineProperty(k, keyMap.lbIndexSymbol, {value: index, enumerable: false, writable: false, configurable: false});
  } catch (e) {
    // (frozen / sealed / already marked: the WeakMap entry serves)
  }
}

async function syncKeyTables(backends, keyMap, keys, pkLen) {
  if (pkLen !== 48 && pkLen !== 96) throw new TypeError("syncPubkeys: pkLen 48 or 96");
  const fmt = pkLen === 96 ? PointFormat.uncompressed : PointFormat.compressed;
  const enc = keys.map((k) => (k instanceof Uint8Array ? k : k.toBytes(fmt)));
  for (const b of enc)
    if (!(b instanceof Uint8Array) || b.length !== pkLen) throw new TypeError(`syncPubkeys: ${pkLen}-byte keys`);
  const blob = concat(enc, keys.length * pkLen);
  const sizes = await Promise.all(backends.map((b) => b.syncPubkeys(blob, pkLen)));
  if (new Set(sizes).size !== 1) throw new Error(`pubkey tables out of sync: ${sizes}`);
  const base = sizes[0] - keys.length;
  keys.forEach((k, i) => {
    if (!(k instanceof Uint8Array) && k && typeof k === "object") {
      keyMap.set(k, base + i);
      markKey(keyMap, k, base + i);
    }
  });
  return sizes[0];
}

function hrNowNs() {
  const [s, ns] = process.hrtime();
  return s * 1e9 + ns;
}

class BlsGpuVerifier {
  /**
   * @param {object} o
   * @param {number[]} [o.devices]  GPU ordinals, one addon Context each (default [0])
   * @param {object[]} [o.backends] Context-like objects instead (tests: mocks)
   * @param {boolean} [o.blsVerifyAllMultiThread]
   * @param {number} [o.maxSetsPerDispatch]
   * @param {number} [o.prefetch] packages per GPU queued beyond its calls in flight (default 0;
   *   4 measured 2.32 vs 2.48 M sets/s in the node leg: the queue only grew)
   * @param {() => Uint8Array} [o.seedSource] 32-byte batch-randomness seed per call
   * @param {boolean} [o.priorityLane] priority jobs and verifyOnMainThread calls go to the
   *   device's priority lane (lb_verify_requests_priority_async: its own high-priority
   *   stream beside the calls in flight) instead of waiting for a free slot (default true)
   */
  constructor(o = {}) {
    if (o.backends) this.backends = o.backends;
    else {
      const addon = loadAddon();
      // capacity: the library's calls in flight per GPU (lb_slots) unless given
      this.backends = (o.devices || [0]).map((d) => new addon.Context(d, o.capacity ? {capacity: o.capacity} : {}));
    }
    if (this.backends.length === 0) throw new Error("at least one GPU backend is required");
    this.blsVerifyAllMultiThread = Boolean(o.blsVerifyAllMultiThread);
    this.maxSetsPerDispatch = o.maxSetsPerDispatch || 65536;
    this.seedSource = o.seedSource || (() => new Uint8Array(crypto.randomBytes(32)));
    this.metrics = new PoolMetrics();
    this.priorityLane = o.priorityLane === undefined ? true : Boolean(o.priorityLane);
    this.prioBusy = this.backends.map(() => false);  // one priority package in flight per GPU
    this.jobs = new JobQueue();
    this.buffered = null;
    this.idle = [];
    // per GPU: the addon's calls in flight plus `prefetch` packages packed ahead and queued
    // in the addon, so a slot that frees starts its next call at once instead of after the
    // main thread has packed it (node leg: ~11.5 of 16 calls in flight without)
    const prefetch = o.prefetch === undefined ? 0 : o.prefetch;
    this.capacity = 0;  // the GPUs' calls in flight (the pool's "workers")
    const per = this.backends.map((b) => b.capacity || 4);
    per.forEach((c) => (this.capacity += c));
    // tokens interleaved over the GPUs (the calls in flight first, then the prefetch)
    for (let k = 0; k < Math.max(...per); k++) per.forEach((c, i) => k < c && this.idle.push(i));
    for (let k = 0; k < prefetch; k++) per.forEach((c, i) => this.idle.push(i));
    this.tokens = this.idle.length;
    this.running = new Set();
    this.closed = false;
    // PublicKey object -> validator index in the GPUs' pubkey tables (syncPubkeys): sets
    // built from index2pubkey ship 4-byte indices, never serialized keys
    this.keyMap = new WeakMap();
    this.tableSize = 0;
    this.mirror = null;  // syncIndex2pubkey: {base, n} of the index2pubkey mirror in the tables
  }

  canAcceptWork() {
    return this.idle.length > 0 && this.jobs.length < MAX_JOBS_CAN_ACCEPT_WORK;
  }

  /** Append keys to the pubkey table of every GPU (the index2pubkey mirror,
   * pubkeyCache.ts:56-77) and return the table size.  keys: @chainsafe/bls PublicKey
   * objects (serialized once here with toBytes(format); each object then maps to its
   * table index, so sets built from it ship the index) or pkLen-byte encodings
   * (48 compressed, as the state holds them, or 96 uncompressed). */
  async syncPubkeys(keys, pkLen = 48) {
    this.tableSize = await syncKeyTables(this.backends, this.keyMap, keys, pkLen);
    return this.tableSize;
  }

  /** pubkeyCache.syncPubkeys (pubkeyCache.ts:56-77) for the GPUs: mirror the entries of
   * index2pubkey (PublicKey objects) not mirrored yet -- index2pubkey[i] maps to table
   * entry base + i, where base is the table size at the first call -- and return the
   * number of entries mirrored.  Call it wherever the node calls syncPubkeys. */
  async syncIndex2pubkey(index2pubkey) {
    if (!this.mirror) this.mirror = {base: this.tableSize, n: 0};
    const m = this.mirror;
    if (this.tableSize !== m.base + m.n) throw new Error("the pubkey table grew outside syncIndex2pubkey");
    if (index2pubkey.length > m.n) {
      await this.syncPubkeys(index2pubkey.slice(m.n), 48);
      m.n = index2pubkey.length;
    }
    return m.n;
  }

  async verifySignatureSets(sets, opts = {}) {
    const m = this.metrics;
    m.inc(M.AGGREGATED_PUBKEYS, sets.reduce((s, x) => s + (x.type === "aggregate" ? (x.pubkeys || []).length : 0), 0));
    m.inc(M.TOTAL_SIG_SETS, sets.length);
    if (opts.priority) m.inc(M.PRIORITIZED_SIG_SETS, sets.length);
    if (opts.batchable) m.inc(M.BATCHABLE_SIG_SETS, sets.length);
    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      // index.ts:174-187: verified at once, bypassing the queue (the GPU call does
      // not block the event loop, unlike blst on the reference's main thread)
      const t0 = process.hrtime();
      try {
        const d0 = this.trace ? hrNowNs() : 0;
        const batch = packRequests([sets], this.seedSource(), this.keyMap);
        const packed = this.trace ? hrNowNs() : 0;
        const r = await this.backends[0].verifyRequests(batch, this.priorityLane ? {priority: true} : undefined);
        this.lastMainThreadResult = r;  // (diagnostics: deviceMs, the lane's kernelMs / kernelClockMHz)
        if (this.trace)
          this.trace.push({main: true, dispatchNs: d0, packedNs: packed, submittedNs: packed, backNs: hrNowNs(),
                           workerStartNs: r.workerStartNs, workerEndNs: r.workerEndNs, deviceMs: r.deviceMs,
                           workerSubmittedNs: r.workerSubmittedNs, workerRetireNs: r.workerRetireNs});
        return this.requestVerdict(r, 0);
      } finally {
        const [s, ns] = process.hrtime(t0);
        m.observe(M.MAIN_THREAD_TIME, s + ns / 1e9);
      }
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map(
        (chunk) => new Promise((resolve, reject) => this.queueBlsWork({type: "default", resolve, reject, opts, sets: chunk, added: Date.now()}))
      )
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((v) => v === true);
  }

  async verifySignatureSetsSameMessage(sets, message, opts = {}) {
    if (!(message instanceof Uint8Array) || message.length !== 32) throw new TypeError("message must be 32 bytes");
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map(
        (chunk) =>
          new Promise((resolve, reject) =>
            this.queueBlsWork({type: "sameMessage", resolve, reject, opts, sets: chunk, message, added: Date.now()})
          )
      )
    );
    return results.flat();
  }

  async close() {
    if (this.buffered) {
      clearTimeout(this.buffered.timeout);
      for (const job of this.buffered.jobs.concat(this.buffered.prioritizedJobs))
        job.reject(new QueueError(QueueErrorCode.QUEUE_ABORTED));
      this.buffered = null;
    }
    for (const job of this.jobs.clear()) job.reject(new QueueError(QueueErrorCode.QUEUE_ABORTED));
    this.closed = true;
    await Promise.all([...this.running].map((p) => p.catch(() => undefined)));
    await Promise.all(this.backends.map((b) => (b.close ? b.close() : undefined)));
  }

  // ---- scheduling (index.ts:308-568) --------------------------------------------
  queueBlsWork(job) {
    if (this.closed) throw new QueueError(QueueErrorCode.QUEUE_ABORTED);
    const sigSets = job.type === "default" ? job.sets.length : 1; // jobItemSigSets, jobItem.ts:39-46
    if (job.opts.batchable) {
      if (!this.buffered) {
        this.buffered = {jobs: [], prioritizedJobs: [], sigCount: 0, timeout: setTimeout(this.runBufferedJobs, MAX_BUFFER_WAIT_MS)};
      }
      (job.opts.priority ? this.buffered.prioritizedJobs : this.buffered.jobs).push(job);
      this.buffered.sigCount += sigSets;
      if (this.buffered.sigCount > MAX_BUFFERED_SIGS) {
        clearTimeout(this.buffered.timeout);
        this.runBufferedJobs();
      }
    } else {
      if (job.opts.priority) this.jobs.unshift(job);
      else this.jobs.push(job);
      // a priority job with a free priority lane starts now (its package is packed and
      // handed to the addon in this call) instead of after setTimeout(runJob, 0)
      if (job.opts.priority && job.type === "default" && this.priorityLane && !this.closed && this.runPriority()) {
        if (this.jobs.length > 0) this.scheduleRun();
        return;
      }
      this.scheduleRun();
    }
  }

  runBufferedJobs = () => {
    if (!this.buffered) return;
    for (const job of this.buffered.jobs) this.jobs.push(job);
    for (const job of this.buffered.prioritizedJobs) this.jobs.unshift(job);
    this.buffered = null;
    this.scheduleRun();
  };

  /** @param {number} skip leading jobs left in the queue (priority jobs waiting for the lane) */
  prepareWork(skip = 0) {
    const jobs = [];
    let total = 0;
    const held = [];
    for (let q = 0; q < skip; q++) held.push(this.jobs.shift());
    while (total < this.maxSetsPerDispatch && this.jobs.length > 0) {
      const job = this.jobs.shift();
      jobs.push(job);
      total += job.type === "default" ? job.sets.length : 1;
    }
    for (let q = held.length - 1; q >= 0; q--) this.jobs.unshift(held[q]);
    return jobs;
  }

  leadingPriorityJobs() {
    let n = 0;
    while (n < this.jobs.length && this.jobs.at(n).opts.priority && this.jobs.at(n).type === "default") n++;
    return n;
  }

  /** setTimeout(runJob, 0) as the reference does after every queue change (index.ts:386,
   * 453, 515), at most one pending: a package of 512 jobs queued at once schedules one run. */
  scheduleRun() {
    if (this.runScheduled) return;
    this.runScheduled = true;
    setTimeout(this.runJobScheduled, 0);
  }

  runJobScheduled = () => {
    this.runScheduled = false;
    this.runJob();
  };

  /** Leading priority verify jobs (up to MAX_PRIORITY_LANE_SETS sets) as one package on
   * a GPU whose priority lane is free: they start now, beside the packages in flight,
   * instead of waiting for a slot (the reference's queue-front insertion,
   * index.ts:327-357,544-555, plus head-of-line isolation on the device). */
  runPriority() {
    const g = this.prioBusy.indexOf(false);
    if (g < 0) return false;
    const jobs = [];
    let total = 0;
    while (this.jobs.length > 0) {
      const j = this.jobs.at(0);
      if (!j.opts.priority || j.type !== "default") break;
      if (jobs.length && total + j.sets.length > MAX_PRIORITY_LANE_SETS) break;
      jobs.push(this.jobs.shift());
      total += j.sets.length;
    }
    if (jobs.length === 0) return false;
    this.prioBusy[g] = true;
    this.metrics.inc(M.JOB_GROUPS_STARTED);
    this.metrics.inc(M.JOBS_STARTED, jobs.length, {type: "default"});
    this.metrics.inc(M.SIG_SETS_STARTED, total, {type: "default"});
    const now = Date.now();
    for (const j of jobs) this.metrics.observe(M.JOB_WAIT_TIME, (now - j.added) / 1000);
    const p = this.dispatch(g, jobs, true).finally(() => {
      this.prioBusy[g] = false;
      this.running.delete(p);
      if (this.jobs.length > 0) this.scheduleRun();
    });
    this.running.add(p);
    return true;
  }

  runJob = () => {
    if (this.closed || this.jobs.length === 0) return;
    let skip = 0;
    if (this.priorityLane && this.leadingPriorityJobs() > 0) {
      if (this.runPriority()) {
        if (this.jobs.length > 0) this.scheduleRun();
        return;
      }
      skip = this.leadingPriorityJobs();  // the lanes are busy: they wait for one, the rest go on
    }
    if (this.idle.length === 0 || this.jobs.length <= skip) return;
    const jobs = this.prepareWork(skip);
    if (jobs.length === 0) return;
    const bi = this.idle.shift();
    const m = this.metrics;
    m.inc(M.JOB_GROUPS_STARTED);
    for (const type of ["default", "sameMessage"]) {
      m.inc(M.JOBS_STARTED, jobs.filter((j) => j.type === type).length, {type});
      m.inc(M.SIG_SETS_STARTED, jobs.filter((j) => j.type === type).reduce((s, j) => s + j.sets.length, 0), {type});
    }
    const now = Date.now();
    for (const j of jobs) m.observe(M.JOB_WAIT_TIME, (now - j.added) / 1000);
    m.set(M.WORKERS_BUSY, Math.min(this.capacity, this.tokens - this.idle.length));
    m.set(M.QUEUE_LENGTH, this.jobs.length);
    const p = this.dispatch(bi, jobs).finally(() => this.running.delete(p));
    this.running.add(p);
    if (this.idle.length > 0 && this.jobs.length > 0) this.scheduleRun();
  };

  requestVerdict(r, k) {
    if (r.errors[k] === LB_REQ_EMPTY_AGGREGATE) throw new Error("EMPTY_AGGREGATE_ARRAY");
    if (r.errors[k] === LB_REQ_BAD_PUBKEY) throw new Error("invalid pubkey encoding");
    return r.valid[k] === 1;
  }

  async dispatch(bi, jobs, priority = false) {
    const backend = this.backends[bi];
    const m = this.metrics;
    const dispatchNs = hrNowNs();
    const def = jobs.filter((j) => j.type === "default");
    const same = jobs.filter((j) => j.type === "sameMessage");
    let outs;
    try {
      const waits = [];
      if (def.length) {
        // the main thread's share of pubkey aggregation (jobItem.ts:55-63 / utils.ts:12):
        // packing the keys; the sum itself runs on the GPU
        // (large packages pack in slices, the event loop turning between them; the
        // histogram takes the main thread's own share)
        const t0 = process.hrtime();
        const reqs = def.map((j) => j.sets);
        const nSets = def.reduce((s, j) => s + j.sets.length, 0);
        const sliced = !(priority || nSets <= PACK_SLICE_SETS);
        const timing = {mainThreadS: 0};
        const batch = !sliced ? packRequests(reqs, this.seedSource(), this.keyMap)
          : await packRequestsAsync(reqs, this.seedSource(), this.keyMap, PACK_SLICE_SETS, timing);
        const [s0, ns0] = process.hrtime(t0);
        if (def.some((j) => j.sets.some((x) => x.type === "aggregate")))
          m.observe(M.PUBKEYS_AGGREGATION_MAIN_THREAD, sliced ? timing.mainThreadS : s0 + ns0 / 1e9);
        const packedNs = hrNowNs();
        waits.push(priority ? backend.verifyRequests(batch, {priority: true}) : backend.verifyRequests(batch));
        if (this.trace) this.trace.push({dispatchNs, packedNs, submittedNs: hrNowNs(), inFlight: this.running.size, prio: priority});
      }
      if (same.length) {
        // jobItem.ts:72-74 times Signature.fromBytes on the main thread; here the bytes are
        // only packed (every signature is decoded once, on the GPU)
        const t0 = process.hrtime();
        const batch = packSameMessage(same, this.seedSource(), this.keyMap);
        const [s0, ns0] = process.hrtime(t0);
        m.observe(M.SIG_DESERIALIZATION_MAIN_THREAD, s0 + ns0 / 1e9);
        waits.push(backend.verifySameMessage(batch));
      }
      outs = await Promise.all(waits);
    } catch (e) {
      // device failure rejects every job of the package (index.ts:503-512)
      if (!priority) this.idle.push(bi);
      m.set(M.WORKERS_BUSY, Math.min(this.capacity, this.tokens - this.idle.length));
      for (const job of jobs) job.reject(e);
      this.scheduleRun();
      return;
    }
    const backNs = hrNowNs();
    if (priority && def.length) this.lastPriorityResult = outs[0];  // (diagnostics, as lastMainThreadResult)
    if (this.trace && def.length) {
      for (let q = this.trace.length - 1; q >= 0; q--)
        if (this.trace[q].dispatchNs === dispatchNs) {
          this.trace[q].backNs = backNs;
          this.trace[q].workerStartNs = outs[0].workerStartNs;
          this.trace[q].workerEndNs = outs[0].workerEndNs;
          this.trace[q].deviceMs = outs[0].deviceMs;
          this.trace[q].workerSubmittedNs = outs[0].workerSubmittedNs;
          this.trace[q].workerRetireNs = outs[0].workerRetireNs;
          break;
        }
    }
    if (!priority) this.idle.push(bi);
    m.set(M.WORKERS_BUSY, Math.min(this.capacity, this.tokens - this.idle.length));
    let k = 0;
    let success = 0;
    let errors = 0;
    const started = jobs.reduce((s, j) => s + j.sets.length, 0);
    const observeWorker = (r) => {
      if (!r.workerEndNs) return;
      const sec = (r.workerEndNs - r.workerStartNs) / 1e9;
      m.inc(M.JOBS_WORKER_TIME, sec, {workerId: bi});
      if (started) m.observe(M.TIME_PER_SIG_SET, sec / started);
      m.observe(M.LATENCY_TO_WORKER, Math.max(0, (r.workerStartNs - dispatchNs) / 1e9));
      m.observe(M.LATENCY_FROM_WORKER, Math.max(0, (backNs - r.workerEndNs) / 1e9));
    };
    if (def.length) {
      const r = outs[k++];
      observeWorker(r);
      const ok = [];
      def.forEach((job, n) => {
        try {
          const v = this.requestVerdict(r, n);
          ok.push(v);
          job.resolve(v);
          success += job.sets.length;
        } catch (e) {
          ok.push(false);
          if (r.errors[n] === LB_REQ_EMPTY_AGGREGATE) m.inc(M.ERROR_AGGREGATE_SETS, job.sets.length, {type: "default"});
          job.reject(e);
          errors += job.sets.length;
        }
      });
      const st = workerBatchStats(def.map((j) => j.sets.length), def.map((j) => Boolean(j.opts.batchable)), ok);
      m.inc(M.BATCH_RETRIES, st.retries);
      m.inc(M.BATCH_SIGS_SUCCESS, st.sigsOk);
    }
    if (same.length) {
      const r = outs[k++];
      observeWorker(r);
      let at = 0;
      same.forEach((job, n) => {
        const verdicts = Array.from(r.valid.subarray(at, at + job.sets.length), (v) => v === 1);
        at += job.sets.length;
        if (!r.jobFast[n] && job.sets.length) {
          m.inc(M.SAME_MESSAGE_RETRY_JOBS); // index.ts:566-567
          m.inc(M.SAME_MESSAGE_RETRY_SETS, job.sets.length);
        }
        success += 1;
        job.resolve(verdicts);
      });
      const st = workerBatchStats(same.map(() => 1), same.map((j) => Boolean(j.opts.batchable)), Array.from(r.jobFast, (f) => f === 1));
      m.inc(M.BATCH_RETRIES, st.retries);
      m.inc(M.BATCH_SIGS_SUCCESS, st.sigsOk);
    }
    m.inc(M.SUCCESS_JOBS_SETS, success);
    m.inc(M.ERROR_JOBS_SETS, errors);
    this.scheduleRun();
  }
}

/** BlsSingleThreadVerifier (chain/bls/singleThread.ts:10-89) on one GPU: no queue,
 * no buffering, every call goes straight to the device. */
class BlsGpuSingleThreadVerifier {
  constructor(o = {}) {
    this.backend = o.backend || new (loadAddon().Context)(o.device || 0);
    this.seedSource = o.seedSource || (() => new Uint8Array(crypto.randomBytes(32)));
    this.metrics = o.metrics || new PoolMetrics();
    this.keyMap = new WeakMap();
    this.tableSize = 0;
    this.mirror = null;
  }
  /** as BlsGpuVerifier.syncPubkeys / syncIndex2pubkey, on this verifier's one GPU */
  async syncPubkeys(keys, pkLen = 48) {
    this.tableSize = await syncKeyTables([this.backend], this.keyMap, keys, pkLen);
    return this.tableSize;
  }
  async syncIndex2pubkey(index2pubkey) {
    return BlsGpuVerifier.prototype.syncIndex2pubkey.call(this, index2pubkey);
  }
  /** singleThread.ts:27-35 times the verification (mainThreadDurationInThreadPool); the
   * single-thread histograms of lodestar.ts:498-508 get the same duration, and per set. */
  observe(t0, nSets) {
    const [s, ns] = process.hrtime(t0);
    const sec = s + ns / 1e9;
    this.metrics.observe(M.MAIN_THREAD_TIME, sec);
    this.metrics.observe(M.SINGLE_THREAD_TIME, sec);
    if (nSets > 0) this.metrics.observe(M.SINGLE_THREAD_TIME_PER_SIGSET, sec / nSets);
  }
  async verifySignatureSets(sets) {
    const t0 = process.hrtime();
    const r = await this.backend.verifyRequests(packRequests([sets], this.seedSource(), this.keyMap));
    if (r.errors[0] === LB_REQ_EMPTY_AGGREGATE) throw new Error("EMPTY_AGGREGATE_ARRAY");
    if (r.errors[0] === LB_REQ_BAD_PUBKEY) throw new Error("invalid pubkey encoding");
    this.observe(t0, sets.length); // counted only for runs without an exception, as the reference
    return r.valid[0] === 1;
  }
  async verifySignatureSetsSameMessage(sets, message) {
    if (sets.length === 0) throw new Error("EMPTY_AGGREGATE_ARRAY"); // PublicKey.aggregate([]) throws (singleThread.ts:43)
    const t0 = process.hrtime();
    const r = await this.backend.verifySameMessage(packSameMessage([{sets, message}], this.seedSource(), this.keyMap));
    this.observe(t0, sets.length);
    return Array.from(r.valid.subarray(0, sets.length), (v) => v === 1);
  }
  async close() {
    if (this.backend.close) await this.backend.close();
  }
  canAcceptWork() {
    return true;
  }
}

/** Contiguous shards of whole requests balanced by set count (sharding.py:shard_requests). */
function shardRequests(sizes, nShards) {
  const total = sizes.reduce((a, b) => a + b, 0);
  const bounds = [0];
  let acc = 0;
  let k = 1;
  sizes.forEach((s, i) => {
    acc += s;
    while (k < nShards && acc * nShards >= total * k && bounds[bounds.length - 1] <= i) {
      bounds.push(i + 1);
      k++;
    }
  });
  while (bounds.length < nShards) bounds.push(sizes.length);
  bounds.push(sizes.length);
  const out = [];
  for (let j = 0; j < nShards; j++) out.push([bounds[j], bounds[j + 1]]);
  return out;
}

/** One call over several GPUs (SURVEY §8e): each shard runs to its 576-byte Fp12
 * partial, the host combines them with ONE final exponentiation (gtCheck on the GPU of
 * the largest shard, not always the first) and resumes every shard with the verdict.
 * A shard that fails in phase 1 fails the call after the others are resumed.
 * Returns {valid, errors, mergedOk}. */
async function verifyRequestsSharded(backends, requests, seedSource) {
  return combineShards(
    backends,
    requests.map((r) => r.length),
    (lo, hi) => packRequests(requests.slice(lo, hi), seedSource())
  );
}

/** Requests [lo, hi) of a packed call ({requestOffsets, pkOffsets, pubkeyIndices |
 * pubkeys, messages, signatures, sigOffsets}) as a call of their own, offsets rebased. */
function slicePacked(p, lo, hi, seed) {
  const a = p.requestOffsets[lo];
  const b = p.requestOffsets[hi];
  const ka = p.pkOffsets[a];
  const kb = p.pkOffsets[b];
  const sa = p.sigOffsets[a];
  const sb = p.sigOffsets[b];
  const rebase = (arr, x, y, base) => {
    const o = arr.slice(x, y);
    if (base !== 0) for (let q = 0; q < o.length; q++) o[q] -= base;
    return o;
  };
  const out = {
    requestOffsets: rebase(p.requestOffsets, lo, hi + 1, a),
    pkOffsets: rebase(p.pkOffsets, a, b + 1, ka),
    messages: p.messages.subarray(32 * a, 32 * b),
    signatures: p.signatures.subarray(sa, sb),
    sigOffsets: rebase(p.sigOffsets, a, b + 1, sa),
    seed,
  };
  if (p.pubkeyIndices && p.pubkeys) {
    // mixed package: keep the rows this slice names (LB_PK_ROW_FLAG), renumbered from 0
    const idx = Uint32Array.from(p.pubkeyIndices.subarray(ka, kb));
    const rows = [];
    for (let q = 0; q < idx.length; q++)
      if (idx[q] & LB_PK_ROW_FLAG) {
        rows.push(idx[q] & LB_PK_ROW_MASK);
        idx[q] = (LB_PK_ROW_FLAG | (idx[q] & LB_PK_ROW48_FLAG) | (rows.length - 1)) >>> 0;
      }
    out.pubkeyIndices = idx;
    if (rows.length) {
      out.pubkeys = new Uint8Array(96 * rows.length);
      rows.forEach((r, q) => out.pubkeys.set(p.pubkeys.subarray(96 * r, 96 * r + 96), 96 * q));
    }
  } else if (p.pubkeyIndices) out.pubkeyIndices = p.pubkeyIndices.subarray(ka, kb);
  else out.pubkeys = p.pubkeys.subarray(96 * ka, 96 * kb);
  return out;
}

/** verifyRequestsSharded for a call already packed (a gossip replay of ~1M sets
 * without one JS object per set or key). */
async function verifyPackedSharded(backends, packed, seedSource) {
  const nReq = packed.requestOffsets.length - 1;
  const sizes = [];
  for (let k = 0; k < nReq; k++) sizes.push(packed.requestOffsets[k + 1] - packed.requestOffsets[k]);
  return combineShards(backends, sizes, (lo, hi) => slicePacked(packed, lo, hi, seedSource()));
}

async function combineShards(backends, sizes, packShard) {
  const nReq = sizes.length;
  const shards = shardRequests(sizes, backends.length)
    .map(([lo, hi], g) => [lo, hi, g])
    .filter(([lo, hi]) => hi > lo);
  const settled = await Promise.allSettled(
    shards.map(([lo, hi, g]) => backends[g].verifyRequestsPartial(packShard(lo, hi)))
  );
  const failed = settled.find((x) => x.status === "rejected");
  if (failed) {
    await Promise.allSettled(
      settled.map((x, i) => (x.status === "fulfilled" ? backends[shards[i][2]].finish(x.value.id, false) : null))
    );
    throw failed.reason;
  }
  const calls = settled.map((x) => x.value);
  const partials = concat(
    calls.map((c) => c.partial),
    GT_BYTES * calls.length
  );
  let big = 0;
  shards.forEach(([lo, hi], i) => {
    if (hi - lo > shards[big][1] - shards[big][0]) big = i;
  });
  const mergedOk = calls.length === 0 ? true : await backends[shards[big][2]].gtCheck(partials);
  const res = await Promise.all(calls.map((c, i) => backends[shards[i][2]].finish(c.id, mergedOk)));
  const valid = new Uint8Array(nReq);
  const errors = new Uint8Array(nReq);
  shards.forEach(([lo], g) => {
    valid.set(res[g].valid, lo);
    errors.set(res[g].errors, lo);
  });
  return {valid, errors, mergedOk};
}

module.exports = {
  BlsGpuVerifier,
  BlsGpuSingleThreadVerifier,
  QueueError,
  QueueErrorCode,
  PoolMetrics,
  METRICS: M,
  chunkifyMaximizeChunkSize,
  workerBatchStats,
  packRequests,
  packRequestsAsync,
  packSameMessage,
  shardRequests,
  slicePacked,
  verifyRequestsSharded,
  verifyPackedSharded,
  loadAddon,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
  MAX_JOBS_CAN_ACCEPT_WORK,
  MAX_PRIORITY_LANE_SETS,
  PointFormat,
  LB_PK_ROW_FLAG,
  LB_PK_ROW48_FLAG,
};
