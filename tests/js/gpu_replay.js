"use strict";
// GPU replay through the N-API addon (node): every verdict scenario of
// tests/golden/vectors.json (the reference's bls.test.ts / multithread.test.ts
// tables plus the edge cases) through BlsGpuVerifier on cuda:0, merged
// (batchable) and one job at a time; the same-message scenarios; the
// single-thread verifier; the device pubkey table by index; aggregatePubkeys
// bit-exact; and a sharded call over two contexts with the Fp12-partial combine.
// Exit code 0 iff everything matches.  Run: node tests/js/gpu_replay.js
const assert = require("assert");
const fs = require("fs");
const path = require("path");
const ROOT = path.join(__dirname, "..", "..");
const V = require(path.join(ROOT, "lodestar_amd", "js", "bls_gpu_verifier.js"));
const addon = V.loadAddon();
const VEC = JSON.parse(fs.readFileSync(path.join(ROOT, "tests", "golden", "vectors.json"), "utf8"));
const hex = (h) => new Uint8Array(Buffer.from(h, "hex"));
const seed = () => new Uint8Array(32);

function toSets(req) {
  return req.map((s) =>
    s.pks.length === 1
      ? {type: "single", pubkey: hex(s.pks[0]), signingRoot: hex(s.msg), signature: hex(s.sig)}
      : {type: "aggregate", pubkeys: s.pks.map(hex), signingRoot: hex(s.msg), signature: hex(s.sig)}
  );
}

async function outcome(p) {
  try {
    return await p;
  } catch (e) {
    return /EMPTY_AGGREGATE_ARRAY/.test(e.message) ? null : "error: " + e.message;
  }
}

(async () => {
  const report = {};
  assert(addon.deviceCount() >= 1, "no GPU visible");
  const v = new V.BlsGpuVerifier({devices: [0], seedSource: seed});
  for (const sc of VEC.verify_requests) {
    for (const batchable of [false, true]) {
      const got = await Promise.all(sc.requests.map((r) => outcome(v.verifySignatureSets(toSets(r), {batchable}))));
      assert.deepStrictEqual(got, sc.expect, `${sc.name} batchable=${batchable}`);
    }
  }
  report.verify_requests = VEC.verify_requests.length;
  for (const sc of VEC.same_message) {
    const sets = sc.pubkeys.map((p, i) => ({publicKey: hex(p), signature: hex(sc.signatures[i])}));
    const got = await v.verifySignatureSetsSameMessage(sets, hex(sc.message), {batchable: true});
    assert.deepStrictEqual(got, sc.expect, sc.name);
  }
  report.same_message = VEC.same_message.length;
  // verifyOnMainThread path (index.ts:174-187)
  const first = VEC.verify_requests[0];
  assert.strictEqual(await v.verifySignatureSets(toSets(first.requests[0]), {verifyOnMainThread: true}), first.expect[0]);
  await v.close();

  // single-thread verifier (singleThread.ts)
  const st = new V.BlsGpuSingleThreadVerifier({device: 0, seedSource: seed});
  for (const sc of VEC.verify_requests)
    for (let k = 0; k < sc.requests.length; k++)
      assert.deepStrictEqual(await outcome(st.verifySignatureSets(toSets(sc.requests[k]))), sc.expect[k], "st " + sc.name);
  for (const sc of VEC.same_message) {
    const sets = sc.pubkeys.map((p, i) => ({publicKey: hex(p), signature: hex(sc.signatures[i])}));
    assert.deepStrictEqual(await st.verifySignatureSetsSameMessage(sets, hex(sc.message)), sc.expect, "st " + sc.name);
  }
  await st.close();

  // aggregatePubkeys bit-exact + the device pubkey table by index
  const ctx = new addon.Context(0);
  const ap = VEC.aggregate_pubkeys;
  const keys = ap.pubkeys.map(hex);
  const agg = await ctx.aggregatePubkeys(Buffer.concat(keys.map((k) => Buffer.from(k))));
  assert.strictEqual(Buffer.from(agg).toString("hex"), ap.out);
  const n = await ctx.syncPubkeys(Buffer.concat(keys.map((k) => Buffer.from(k))), 96);
  assert.strictEqual(n, keys.length);
  const aggIdx = await ctx.aggregatePubkeys(Uint32Array.from(keys.map((_, i) => i)));
  assert.strictEqual(Buffer.from(aggIdx).toString("hex"), ap.out);
  await assert.rejects(ctx.verifyRequests({}), TypeError);
  await ctx.close();
  await assert.rejects(ctx.verifyRequests({}), /closed|TypeError|missing/);
  report.aggregate_pubkeys = true;

  // sharded call over two contexts: partials combined with one final exponentiation
  const reqs = [];
  const want = [];
  for (const sc of VEC.verify_requests)
    sc.requests.forEach((r, k) => {
      if (sc.expect[k] !== null) {
        reqs.push(toSets(r));
        want.push(sc.expect[k] ? 1 : 0);
      }
    });
  const ctxs = [new addon.Context(0), new addon.Context(0)];
  const r = await V.verifyRequestsSharded(ctxs, reqs, seed);
  assert.deepStrictEqual(Array.from(r.valid), want);
  assert.strictEqual(r.mergedOk, false);
  const goodOnly = reqs.filter((_, i) => want[i] === 1);
  const r2 = await V.verifyRequestsSharded(ctxs, goodOnly, seed);
  assert.strictEqual(r2.mergedOk, true);
  assert(Array.from(r2.valid).every((x) => x === 1));
  await Promise.all(ctxs.map((c) => c.close()));
  report.sharded = {requests: reqs.length, mergedOkAllValid: r2.mergedOk};
  console.log(JSON.stringify(report));
})().catch((e) => {
  console.error(e && e.stack);
  process.exit(1);
});
