"use strict";
// BlsGpuVerifier scheduling semantics with a mock backend (the pattern of the
// reference's test/mocks/mockedBls.ts), on node without a GPU:
// chunking, buffering, priority, same-message flattening, rejection rules,
// close(), metrics, the worker's batch accounting and the sharded combine.
const assert = require("assert");
const path = require("path");
const V = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "bls_gpu_verifier.js"));

const GOOD = new Uint8Array(96).fill(1);
const BAD = new Uint8Array(96).fill(2);
const PK = new Uint8Array(96);

class MockBackend {
  constructor(capacity = 1) {
    this.capacity = capacity;
    this.dispatches = [];
    this.sameCalls = [];
    this.closed = false;
    this.partials = new Map();
    this.nextId = 1;
  }
  verdicts(b) {
    const nReq = b.requestOffsets.length - 1;
    const valid = new Uint8Array(nReq);
    const errors = new Uint8Array(nReq);
    const sizes = [];
    for (let k = 0; k < nReq; k++) {
      const a = b.requestOffsets[k];
      const e = b.requestOffsets[k + 1];
      sizes.push(e - a);
      let ok = e > a;
      for (let i = a; i < e; i++) {
        if (b.pkOffsets && b.pkOffsets[i + 1] === b.pkOffsets[i]) errors[k] = 1;
        if (b.signatures[b.sigOffsets[i]] !== 1) ok = false;
      }
      valid[k] = ok ? 1 : 0;
    }
    return {valid, errors, sizes};
  }
  async verifyRequests(b, opts) {
    assert(!this.closed);
    const {valid, errors, sizes} = this.verdicts(b);
    this.dispatches.push(sizes);
    const prio = Boolean(opts && opts.priority);
    (this.log || (this.log = [])).push({sizes, prio, t: Date.now()});
    await new Promise((r) => setTimeout(r, prio ? 1 : this.delayMs || 1));
    return {valid, errors, setStatus: new Uint8Array(0), batchRetries: 0, batchSigsSuccess: 0, deviceMs: 0};
  }
  async verifySameMessage(b) {
    const nJobs = b.jobOffsets.length - 1;
    const nSets = b.jobOffsets[nJobs];
    const valid = new Uint8Array(nSets);
    const jobFast = new Uint8Array(nJobs);
    for (let i = 0; i < nSets; i++) valid[i] = b.signatures[b.sigOffsets[i]] === 1 ? 1 : 0;
    for (let j = 0; j < nJobs; j++) {
      this.sameCalls.push(b.jobOffsets[j + 1] - b.jobOffsets[j]);
      jobFast[j] = valid.subarray(b.jobOffsets[j], b.jobOffsets[j + 1]).every((v) => v === 1) ? 1 : 0;
    }
    return {valid, jobFast, retriedJobs: 0, fastSets: 0, deviceMs: 0};
  }
  // two-phase protocol (addon Context.verifyRequestsPartial / gtCheck / finish)
  async verifyRequestsPartial(b) {
    const v = this.verdicts(b);
    const id = this.nextId++;
    this.partials.set(id, v);
    const partial = new Uint8Array(576);
    partial[0] = v.valid.every((x) => x === 1) ? 1 : 0;
    return {id, partial};
  }
  async gtCheck(partials) {
    for (let i = 0; i < partials.length; i += 576) if (partials[i] !== 1) return false;
    return true;
  }
  async finish(id, ok) {
    const v = this.partials.get(id);
    this.partials.delete(id);
    this.lastFinish = ok;
    return {valid: v.valid, errors: v.errors};
  }
  async close() {
    this.closed = true;
  }
}

function sets(n, bad = new Set()) {
  const out = [];
  for (let i = 0; i < n; i++)
    out.push({type: "single", pubkey: PK, signingRoot: new Uint8Array(32).fill(i % 256), signature: bad.has(i) ? BAD : GOOD});
  return out;
}
const seed = () => new Uint8Array(32);

const tests = [];
function test(name, fn) {
  tests.push([name, fn]);
}

test("chunkify matches the reference", () => {
  const r = (n, m) => V.chunkifyMaximizeChunkSize(Array.from({length: n}, (_, i) => i), m).map((c) => c.length);
  assert.deepStrictEqual(r(300, 128), [150, 150]);
  assert.deepStrictEqual(r(100, 128), [100]);
  assert.deepStrictEqual(r(0, 128), [0]);
});

test("valid and invalid calls", async () => {
  const b = new MockBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed});
  assert.strictEqual(await v.verifySignatureSets(sets(3)), true);
  assert.strictEqual(await v.verifySignatureSets(sets(3, new Set([1]))), false);
  await v.close();
});

test("large call chunked into jobs of <= 128", async () => {
  const b = new MockBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed});
  assert.strictEqual(await v.verifySignatureSets(sets(300)), true);
  assert.deepStrictEqual(b.dispatches.flat().sort(), [150, 150]);
  await v.close();
});

test("batchable calls buffered into one package", async () => {
  const b = new MockBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed});
  const opts = {batchable: true};
  const r = await Promise.all([
    v.verifySignatureSets(sets(3), opts),
    v.verifySignatureSets(sets(4), opts),
    v.verifySignatureSets(sets(2, new Set([0])), opts),
  ]);
  assert.deepStrictEqual(r, [true, true, false]);
  assert.deepStrictEqual(b.dispatches, [[3, 4, 2]]);
  await v.close();
});

test("batchable waits for the buffer timeout, > 32 sigs flushes at once", async () => {
  const v = new V.BlsGpuVerifier({backends: [new MockBackend()], seedSource: seed});
  let t0 = Date.now();
  await v.verifySignatureSets(sets(2), {batchable: true});
  assert(Date.now() - t0 >= V.MAX_BUFFER_WAIT_MS * 0.9);
  t0 = Date.now();
  await v.verifySignatureSets(sets(33), {batchable: true});
  assert(Date.now() - t0 < V.MAX_BUFFER_WAIT_MS / 2);
  await v.close();
});

test("priority jobs run first", async () => {
  const b = new MockBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed, maxSetsPerDispatch: 1});
  const hold = v.idle;
  v.idle = [];
  const f1 = v.verifySignatureSets(sets(2));
  const f2 = v.verifySignatureSets(sets(5), {priority: true});
  await new Promise((r) => setTimeout(r, 5));
  v.idle = hold;
  v.runJob();
  await Promise.all([f1, f2]);
  assert.deepStrictEqual(b.dispatches[0], [5]);
  await v.close();
});

test("priority job takes the priority lane ahead of queued packages", async () => {
  // one slot, busy with a slow package, two more packages queued: the priority job
  // starts at once on the lane (verifyRequests(batch, {priority: true})) and resolves
  // before the queued packages; verifyOnMainThread takes the lane too
  const b = new MockBackend(1);
  b.delayMs = 40;
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed, maxSetsPerDispatch: 1});
  const done = [];
  const normal = [0, 1, 2].map((i) => v.verifySignatureSets(sets(3 + i)).then(() => done.push("n" + i)));
  await new Promise((r) => setTimeout(r, 5));
  const t0 = Date.now();
  const p = v.verifySignatureSets(sets(7), {priority: true}).then((ok) => done.push("p") && ok);
  const m = v.verifySignatureSets(sets(1), {verifyOnMainThread: true}).then((ok) => done.push("m") && ok);
  assert.strictEqual(await p, true);
  assert.strictEqual(await m, true);
  assert(Date.now() - t0 < 30, "priority work waited for a slot");
  await Promise.all(normal);
  assert(done.indexOf("p") < done.indexOf("n1") && done.indexOf("m") < done.indexOf("n1"), done.join());
  const prio = b.log.filter((x) => x.prio).map((x) => x.sizes[0]);
  assert.deepStrictEqual(prio.sort(), [1, 7]);
  // without the lane: the reference's queue-front order through the slots
  const b2 = new MockBackend(1);
  const v2 = new V.BlsGpuVerifier({backends: [b2], seedSource: seed, priorityLane: false});
  await v2.verifySignatureSets(sets(2), {priority: true});
  assert(b2.log.every((x) => !x.prio));
  await v.close();
  await v2.close();
});

test("slicePacked keeps a mixed package's rows, renumbered", () => {
  const F = 0x80000000;
  const rows = new Uint8Array(96 * 3);
  for (let r = 0; r < 3; r++) rows.fill(10 + r, 96 * r, 96 * r + 96);
  const p = {
    requestOffsets: Uint32Array.from([0, 2, 4]),
    pkOffsets: Uint32Array.from([0, 1, 2, 3, 4]),
    pubkeyIndices: Uint32Array.from([5, (F | 0) >>> 0, (F | 2) >>> 0, 9]),
    pubkeys: rows,
    messages: new Uint8Array(128),
    signatures: new Uint8Array(384),
    sigOffsets: Uint32Array.from([0, 96, 192, 288, 384]),
  };
  const q = V.slicePacked(p, 1, 2, new Uint8Array(32));
  assert.deepStrictEqual(Array.from(q.pubkeyIndices), [(F | 0) >>> 0, 9]);
  assert.strictEqual(q.pubkeys.length, 96);
  assert.strictEqual(q.pubkeys[0], 12);
  const q0 = V.slicePacked(p, 0, 1, new Uint8Array(32));
  assert.deepStrictEqual(Array.from(q0.pubkeyIndices), [5, (F | 0) >>> 0]);
  assert.strictEqual(q0.pubkeys[0], 10);
});

test("empty aggregate rejects the job; empty sets are false", async () => {
  const v = new V.BlsGpuVerifier({backends: [new MockBackend()], seedSource: seed});
  await assert.rejects(
    v.verifySignatureSets([{type: "aggregate", pubkeys: [], signingRoot: new Uint8Array(32), signature: GOOD}]),
    /EMPTY_AGGREGATE_ARRAY/
  );
  assert.strictEqual(await v.verifySignatureSets([]), false);
  await v.close();
});

test("same-message chunks flatten; one package, one device call", async () => {
  const b = new MockBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed});
  const pairs = [];
  for (let i = 0; i < 300; i++) pairs.push({publicKey: PK, signature: i === 299 ? BAD : GOOD});
  const out = await v.verifySignatureSetsSameMessage(pairs, new Uint8Array(32));
  assert.deepStrictEqual(out, Array(299).fill(true).concat([false]));
  assert.deepStrictEqual(b.sameCalls.sort(), [150, 150]);
  assert.deepStrictEqual(await v.verifySignatureSetsSameMessage([], new Uint8Array(32)), []);
  assert.strictEqual(v.metrics.get(V.METRICS.SAME_MESSAGE_RETRY_JOBS), 1);
  await v.close();
});

test("close rejects queued jobs and new work, waits for packages in flight", async () => {
  const b = new MockBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed});
  const f = v.verifySignatureSets(sets(2), {batchable: true});
  await v.close();
  await assert.rejects(f, (e) => e instanceof V.QueueError);
  await assert.rejects(v.verifySignatureSets(sets(1)), (e) => e instanceof V.QueueError);
  assert(b.closed);
});

test("canAcceptWork and several GPUs share the load", async () => {
  const bs = [new MockBackend(2), new MockBackend(2)];
  const v = new V.BlsGpuVerifier({backends: bs, seedSource: seed, maxSetsPerDispatch: 128});
  assert(v.canAcceptWork());
  assert.strictEqual(v.capacity, 4);
  const r = await Promise.all(Array.from({length: 6}, () => v.verifySignatureSets(sets(128))));
  assert(r.every((x) => x));
  assert(bs.every((b) => b.dispatches.length > 0));
  await v.close();
});

test("pubkeys by validator index ship as indices", () => {
  const s1 = {type: "single", pubkey: {index: 4}, signingRoot: new Uint8Array(32), signature: GOOD};
  const s2 = {type: "aggregate", pubkeys: [{index: 1}, {index: 2}], signingRoot: new Uint8Array(32), signature: GOOD};
  const b = V.packRequests([[s1, s2]], new Uint8Array(32));
  assert.deepStrictEqual(Array.from(b.pubkeyIndices), [4, 1, 2]);
  assert.deepStrictEqual(Array.from(b.pkOffsets), [0, 1, 3]);
  assert.strictEqual(b.pubkeys, undefined);
  assert.throws(() => V.packRequests([[{...s1, signingRoot: new Uint8Array(31)}]], new Uint8Array(32)), TypeError);
});

test("worker batch accounting (worker.ts:41-85)", () => {
  const w = V.workerBatchStats;
  assert.deepStrictEqual(w(Array(10).fill(3), Array(10).fill(true), Array(10).fill(true)), {retries: 0, sigsOk: 30});
  const v = Array(40).fill(true);
  v[25] = false;
  assert.deepStrictEqual(w(Array(40).fill(2), Array(40).fill(true), v), {retries: 1, sigsOk: 40});
  assert.deepStrictEqual(w([5, 5], [false, false], [false, true]), {retries: 0, sigsOk: 0});
});

test("metrics carry the reference's names", async () => {
  const v = new V.BlsGpuVerifier({backends: [new MockBackend()], seedSource: seed});
  await v.verifySignatureSets(sets(300), {batchable: true, priority: true});
  const M = V.METRICS;
  assert.strictEqual(v.metrics.get(M.TOTAL_SIG_SETS), 300);
  assert.strictEqual(v.metrics.get(M.BATCHABLE_SIG_SETS), 300);
  assert.strictEqual(v.metrics.get(M.SIG_SETS_STARTED, {type: "default"}), 300);
  assert.strictEqual(v.metrics.get(M.BATCH_SIGS_SUCCESS), 300);
  assert.strictEqual(v.metrics.get(M.JOBS_STARTED, {type: "default"}), 2);
  await v.close();
});

test("sharded call combines the shards' partials", async () => {
  const reqs = [];
  for (let k = 0; k < 9; k++) reqs.push(sets(k % 4 + 1));
  let bs = [new MockBackend(), new MockBackend(), new MockBackend()];
  let r = await V.verifyRequestsSharded(bs, reqs, seed);
  assert.strictEqual(r.mergedOk, true);
  assert(Array.from(r.valid).every((x) => x === 1));
  assert(bs.every((b) => b.lastFinish === true));
  reqs[5] = sets(2, new Set([1]));
  bs = [new MockBackend(), new MockBackend()];
  r = await V.verifyRequestsSharded(bs, reqs, seed);
  assert.strictEqual(r.mergedOk, false);
  assert.deepStrictEqual(Array.from(r.valid), [1, 1, 1, 1, 1, 0, 1, 1, 1]);
});

test("single-thread verifier", async () => {
  const v = new V.BlsGpuSingleThreadVerifier({backend: new MockBackend(), seedSource: seed});
  assert.strictEqual(await v.verifySignatureSets(sets(2)), true);
  assert.deepStrictEqual(await v.verifySignatureSetsSameMessage([{publicKey: PK, signature: BAD}], new Uint8Array(32)), [false]);
  await assert.rejects(v.verifySignatureSetsSameMessage([], new Uint8Array(32)), /EMPTY_AGGREGATE_ARRAY/);
  assert(v.canAcceptWork());
});

// A @chainsafe/bls PublicKey as the reference's set builders hand it over
// (index2pubkey[i], state-transition/src/signatureSets/indexedAttestation.ts:27):
// toBytes(format) returns the COMPRESSED encoding unless format is "uncompressed"
// (PointFormat, the reference passes PointFormat.uncompressed, index.ts:144).
class MockPublicKey {
  constructor(b, ignoreFormat = false) {
    this.unc = new Uint8Array(96).fill(b);
    this.unc[0] = b & 0x1f;
    this.comp = new Uint8Array(48).fill(b);
    this.comp[0] = 0x80 | (b & 0x1f);
    this.ignoreFormat = ignoreFormat;
    this.formats = [];
  }
  toBytes(format) {
    this.formats.push(format);
    return format === "uncompressed" && !this.ignoreFormat ? this.unc : this.comp;
  }
}

test("PublicKey objects (unmapped) are serialized once with PointFormat.uncompressed", () => {
  const ks = [1, 2, 3, 4].map((b) => new MockPublicKey(b));
  const s1 = {type: "single", pubkey: ks[0], signingRoot: new Uint8Array(32), signature: GOOD};
  const s2 = {type: "aggregate", pubkeys: [ks[1], ks[2], ks[3]], signingRoot: new Uint8Array(32), signature: GOOD};
  const b = V.packRequests([[s1, s2]], new Uint8Array(32), new WeakMap());
  assert.strictEqual(b.pubkeyIndices, undefined);
  assert.deepStrictEqual(Array.from(b.pkOffsets), [0, 1, 4]);
  assert.strictEqual(b.pubkeys.length, 4 * 96);
  ks.forEach((k, i) => {
    assert.deepStrictEqual(k.formats, ["uncompressed"]);
    assert.deepStrictEqual(Array.from(b.pubkeys.subarray(96 * i, 96 * i + 96)), Array.from(k.unc));
  });
  // the old boolean form would have produced the compressed 48 bytes and thrown
  assert.strictEqual(new MockPublicKey(7).toBytes(false).length, 48);
});

test("compressed keys (48-byte bytes, or toBytes ignoring the format) ship as flagged rows", () => {
  const F = 0x80000000;
  const F48 = 0x40000000;
  const raw48 = new MockPublicKey(5).comp;
  const obj48 = new MockPublicKey(6, true);
  const unc = new MockPublicKey(7);
  const sets_ = [
    {type: "single", pubkey: raw48, signingRoot: new Uint8Array(32), signature: GOOD},
    {type: "aggregate", pubkeys: [obj48, unc, {index: 9}], signingRoot: new Uint8Array(32), signature: GOOD},
  ];
  const b = V.packRequests([sets_], new Uint8Array(32));
  assert.deepStrictEqual(Array.from(b.pubkeyIndices), [(F | F48 | 0) >>> 0, (F | F48 | 1) >>> 0, (F | 2) >>> 0, 9]);
  assert.deepStrictEqual(Array.from(b.pubkeys.subarray(0, 48)), Array.from(raw48));
  assert.deepStrictEqual(Array.from(b.pubkeys.subarray(96, 144)), Array.from(obj48.comp));
  assert.deepStrictEqual(Array.from(b.pubkeys.subarray(192, 288)), Array.from(unc.unc));
  // slicing keeps the compressed flag while renumbering rows
  const q = V.slicePacked({...b, requestOffsets: Uint32Array.from([0, 1, 2])}, 1, 2, new Uint8Array(32));
  assert.deepStrictEqual(Array.from(q.pubkeyIndices), [(F | F48 | 0) >>> 0, (F | 1) >>> 0, 9]);
  // same-message packages: the same mixed layout
  const sm = V.packSameMessage([{sets: [{publicKey: raw48, signature: GOOD}, {publicKey: unc, signature: GOOD}],
    message: new Uint8Array(32)}], new Uint8Array(32));
  assert.deepStrictEqual(Array.from(sm.pubkeyIndices), [(F | F48 | 0) >>> 0, (F | 1) >>> 0]);
  assert.throws(() => V.packRequests([[{...sets_[0], pubkey: new Uint8Array(47)}]], new Uint8Array(32)), TypeError);
});

class TableBackend extends MockBackend {
  constructor() {
    super(2);
    this.table = 0;
    this.synced = [];
  }
  async syncPubkeys(blob, pkLen) {
    this.synced.push({n: blob.length / pkLen, pkLen, first: blob[0]});
    this.table += blob.length / pkLen;
    return this.table;
  }
  async verifyRequests(b, opts) {
    this.lastBatch = b;
    return super.verifyRequests(b, opts);
  }
  async verifySameMessage(b) {
    this.lastSame = b;
    return super.verifySameMessage(b);
  }
}

test("index2pubkey objects mirrored by syncPubkeys ship as validator indices", async () => {
  const bs = [new TableBackend(), new TableBackend()];
  const v = new V.BlsGpuVerifier({backends: bs, seedSource: seed});
  const index2pubkey = Array.from({length: 600}, (_, i) => new MockPublicKey(1 + (i % 200)));
  assert.strictEqual(await v.syncIndex2pubkey(index2pubkey.slice(0, 500)), 500);
  assert.strictEqual(await v.syncIndex2pubkey(index2pubkey), 600);  // incremental: 100 more
  assert.deepStrictEqual(bs[0].synced.map((x) => [x.n, x.pkLen]), [[500, 48], [100, 48]]);
  assert.deepStrictEqual(index2pubkey[0].formats, ["compressed"]);  // serialized once, at sync
  // a C4-shaped aggregate (488 keys of a committee) + a single set, built from index2pubkey
  const committee = Array.from({length: 488}, (_, i) => index2pubkey[(i * 7) % 600]);
  const r = await v.verifySignatureSets([
    {type: "aggregate", pubkeys: committee, signingRoot: new Uint8Array(32), signature: GOOD},
    {type: "single", pubkey: index2pubkey[42], signingRoot: new Uint8Array(32), signature: GOOD},
  ]);
  assert.strictEqual(r, true);
  const b = bs.find((x) => x.lastBatch).lastBatch;
  assert.strictEqual(b.pubkeys, undefined);
  assert.deepStrictEqual(Array.from(b.pubkeyIndices.subarray(0, 3)), [0, 7, 14]);
  assert.strictEqual(b.pubkeyIndices[488], 42);
  assert(index2pubkey.every((k) => k.formats.length === 1), "a mirrored key was serialized again");
  // an unmirrored key beside mirrored ones: a mixed package (its row, serialized uncompressed)
  const stranger = new MockPublicKey(250);
  await v.verifySignatureSets([{type: "aggregate", pubkeys: [index2pubkey[3], stranger], signingRoot: new Uint8Array(32), signature: GOOD}]);
  const b2 = bs.map((x) => x.lastBatch).filter(Boolean).pop();
  assert.deepStrictEqual(Array.from(b2.pubkeyIndices), [3, 0x80000000]);
  assert.deepStrictEqual(stranger.formats, ["uncompressed"]);
  // same-message sets from index2pubkey: by index
  await v.verifySignatureSetsSameMessage([{publicKey: index2pubkey[5], signature: GOOD}, {publicKey: index2pubkey[6], signature: GOOD}],
    new Uint8Array(32));
  const sm = bs.map((x) => x.lastSame).filter(Boolean).pop();
  assert.deepStrictEqual(Array.from(sm.pubkeyIndices), [5, 6]);
  assert.strictEqual(sm.pubkeys, undefined);
  await v.close();
  // the single-thread verifier keeps the same map
  const st = new V.BlsGpuSingleThreadVerifier({backend: new TableBackend(), seedSource: seed});
  await st.syncIndex2pubkey(index2pubkey.slice(0, 10));
  await st.verifySignatureSets([{type: "single", pubkey: index2pubkey[4], signingRoot: new Uint8Array(32), signature: GOOD}]);
  assert.deepStrictEqual(Array.from(st.backend.lastBatch.pubkeyIndices), [4]);
});

test("mirrored key objects: index as a hidden per-verifier property; frozen keys via the map", async () => {
  const b = new TableBackend();
  const v = new V.BlsGpuVerifier({backends: [b], seedSource: seed});
  const keys = Array.from({length: 6}, (_, i) => new MockPublicKey(10 + i));
  Object.freeze(keys[2]);  // (cannot take the property: the identity map serves)
  const before = Object.keys(keys[0]);
  await v.syncIndex2pubkey(keys);
  assert.deepStrictEqual(Object.keys(keys[0]), before, "the index property must not be enumerable");
  await v.verifySignatureSets([{type: "aggregate", pubkeys: [keys[5], keys[2], keys[0]], signingRoot: new Uint8Array(32), signature: GOOD}]);
  assert.deepStrictEqual(Array.from(b.lastBatch.pubkeyIndices), [5, 2, 0]);
  // a second verifier (its own table) maps the same objects to its own indices
  const b2 = new TableBackend();
  const v2 = new V.BlsGpuVerifier({backends: [b2], seedSource: seed});
  await v2.syncPubkeys([keys[4], keys[3]], 48);
  await v2.verifySignatureSets([{type: "aggregate", pubkeys: [keys[3], keys[4]], signingRoot: new Uint8Array(32), signature: GOOD}]);
  assert.deepStrictEqual(Array.from(b2.lastBatch.pubkeyIndices), [1, 0]);
  await v.close();
  await v2.close();
});

test("packRequestsAsync (sliced, yielding) packs exactly what packRequests packs", async () => {
  const reqs = [];
  for (let r = 0; r < 40; r++) {
    const req = [];
    for (let q = 0; q < 1 + (r % 5); q++)
      req.push(q % 3 === 2
        ? {type: "aggregate", pubkeys: [{index: r}, new MockPublicKey(1 + q), new MockPublicKey(9, true)],
           signingRoot: new Uint8Array(32).fill(r), signature: GOOD}
        : {type: "single", pubkey: q % 2 ? {index: q} : new MockPublicKey(3 + r), signingRoot: new Uint8Array(32).fill(q),
           signature: r === 7 ? new Uint8Array(192).fill(1) : GOOD});
    reqs.push(req);
  }
  const a = V.packRequests(reqs, new Uint8Array(32));
  const b = await V.packRequestsAsync(reqs, new Uint8Array(32), undefined, 7);
  for (const key of Object.keys(a)) assert.deepStrictEqual(Array.from(b[key]), Array.from(a[key]), key);
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try {
      await fn();
      console.log("ok   " + name);
    } catch (e) {
      failed++;
      console.log("FAIL " + name + "\n" + (e && e.stack));
    }
  }
  console.log(`${tests.length - failed} passed, ${failed} failed`);
  process.exit(failed ? 1 : 0);
})();
