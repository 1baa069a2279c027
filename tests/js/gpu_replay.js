"use strict";
// GPU replay through the N-API addon (node): every verdict scenario of
// tests/golden/vectors.json (the reference's bls.test.ts / multithread.test.ts
// tables plus the edge cases) through BlsGpuVerifier on cuda:0, merged
// (batchable) and one job at a time; the same-message scenarios; the
// single-thread verifier; the device pubkey table by index; aggregatePubkeys
// bit-exact; and a sharded call over two contexts with the Fp12-partial combine.
// Every scenario is replayed again with the keys as @chainsafe/bls-shaped PublicKey
// objects (unmapped, compressed-only, raw 48-byte, mirrored into the pubkey table).
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

// Keys as the reference's set builders pass them: @chainsafe/bls PublicKey objects out of
// index2pubkey (state-transition/src/signatureSets/indexedAttestation.ts:27), whose
// toBytes(format) is COMPRESSED unless format is "uncompressed" (the reference passes
// PointFormat.uncompressed, BN/chain/bls/multithread/index.ts:144).  Built here from the
// vectors' 96-byte encodings (compression in BigInt arithmetic); keys no PublicKey object
// could hold (off the curve, bad flags) stay raw bytes.
const P = BigInt("0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab");
const big = (u8) => BigInt("0x" + Buffer.from(u8).toString("hex"));
function keyObjectable(unc) {
  if (unc.length !== 96) return false;
  if (unc[0] & 0x80) return false;
  if (unc[0] & 0x40) return (unc[0] & 0x3f) === 0 && unc.subarray(1).every((b) => b === 0);
  if (unc[0] & 0x20) return false;
  const x = big(unc.subarray(0, 48));
  const y = big(unc.subarray(48, 96));
  return x < P && y < P && (y * y - (x * x * x + 4n)) % P === 0n;
}
function compressG1(unc) {
  const c = new Uint8Array(48);
  if (unc[0] & 0x40) {
    c[0] = 0xc0;
    return c;
  }
  c.set(unc.subarray(0, 48));
  c[0] |= 0x80;
  if (2n * big(unc.subarray(48, 96)) > P) c[0] |= 0x20;  // y lexicographically largest
  return c;
}
class PublicKey {
  constructor(unc, compressedOnly = false) {
    this.unc = unc;
    this.comp = compressG1(unc);
    this.compressedOnly = compressedOnly;
  }
  toBytes(format) {
    return format === "uncompressed" && !this.compressedOnly ? this.unc : this.comp;
  }
}
function keyFactory(kind) {
  const cache = new Map();
  return (h) => {
    const unc = hex(h);
    if (!keyObjectable(unc)) return unc;
    if (!cache.has(h)) cache.set(h, kind === "raw48" ? compressG1(unc) : new PublicKey(unc, kind === "object48"));
    return cache.get(h);
  };
}
function toSetsWith(req, mk) {
  return req.map((s) =>
    s.pks.length === 1
      ? {type: "single", pubkey: mk(s.pks[0]), signingRoot: hex(s.msg), signature: hex(s.sig)}
      : {type: "aggregate", pubkeys: s.pks.map(mk), signingRoot: hex(s.msg), signature: hex(s.sig)}
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

  // every verdict scenario with the keys as PublicKey objects: unmapped (serialized with
  // toBytes("uncompressed")), objects that only give their compressed form and raw 48-byte
  // keys (decompressed on the GPU), and mirrored by syncPubkeys (shipped as indices)
  report.public_key_objects = {};
  for (const kind of ["object", "object48", "raw48", "mirrored"]) {
    const mk = keyFactory(kind === "mirrored" ? "object" : kind);
    const vk = new V.BlsGpuVerifier({devices: [0], seedSource: seed});
    if (kind === "mirrored") {
      const objs = [];
      const seen = new Set();
      for (const sc of VEC.verify_requests)
        for (const r of sc.requests)
          for (const st of r)
            for (const h of st.pks) {
              const k = mk(h);
              if (k instanceof PublicKey && !(k.unc[0] & 0x40) && !seen.has(h)) {
                seen.add(h);
                objs.push(k);
              }
            }
      for (const sc of VEC.same_message)
        for (const h of sc.pubkeys) {
          const k = mk(h);
          if (k instanceof PublicKey && !(k.unc[0] & 0x40) && !seen.has(h)) {
            seen.add(h);
            objs.push(k);
          }
        }
      assert.strictEqual(await vk.syncIndex2pubkey(objs), objs.length);
      // the packages really ship indices for them
      const probe = V.packRequests([[{type: "single", pubkey: objs[0], signingRoot: new Uint8Array(32), signature: new Uint8Array(96)}]],
        seed(), vk.keyMap);
      assert.deepStrictEqual(Array.from(probe.pubkeyIndices), [0]);
    }
    for (const sc of VEC.verify_requests)
      for (const batchable of [false, true]) {
        const got = await Promise.all(sc.requests.map((r) => outcome(vk.verifySignatureSets(toSetsWith(r, mk), {batchable}))));
        assert.deepStrictEqual(got, sc.expect, `${kind}: ${sc.name} batchable=${batchable}`);
      }
    for (const sc of VEC.same_message) {
      const sets = sc.pubkeys.map((p, i) => ({publicKey: mk(p), signature: hex(sc.signatures[i])}));
      assert.deepStrictEqual(await vk.verifySignatureSetsSameMessage(sets, hex(sc.message), {batchable: true}), sc.expect,
        `${kind}: ${sc.name}`);
    }
    const f0 = VEC.verify_requests[0];
    assert.strictEqual(await vk.verifySignatureSets(toSetsWith(f0.requests[0], mk), {verifyOnMainThread: true}), f0.expect[0]);
    await vk.close();
    report.public_key_objects[kind] = VEC.verify_requests.length + VEC.same_message.length;
  }

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
