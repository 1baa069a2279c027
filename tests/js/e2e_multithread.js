"use strict";
// The reference's e2e pool test (BNT/e2e/chain/bls/multithread.test.ts:85-129) replayed
// through BlsGpuVerifier -> N-API addon -> the GPU, while a background load keeps 16
// C2-sized packages (512 jobs x 128 sets) in flight through the same verifier:
//   - 8 concurrent verifySignatureSets + verifySignatureSetsSameMessage calls submitted
//     synchronously, asynchronously (5 ms apart) and batchable, each with priority true
//     and false: every call valid;
//   - "first is invalid": a batchable 32-zero-byte signature (priority true / false)
//     queued ahead of 8 batchable valid calls: false, and the 8 stay true.
// Keys are @chainsafe/bls-shaped PublicKey objects (toBytes(format): compressed unless
// "uncompressed"), built from tests/golden/e2e_multithread.json.  The reference starts a
// fresh pool per case; here one verifier carries every case and the load, so priority
// work is checked against queued packages.
// usage: node tests/js/e2e_multithread.js LOAD_DIR   (LOAD_DIR: pks.bin msgs.bin sigs.bin)
const assert = require("assert");
const fs = require("fs");
const path = require("path");
const ROOT = path.join(__dirname, "..", "..");
const V = require(path.join(ROOT, "lodestar_amd", "js", "bls_gpu_verifier.js"));
const FX = JSON.parse(fs.readFileSync(path.join(ROOT, "tests", "golden", "e2e_multithread.json"), "utf8"));
const hex = (h) => new Uint8Array(Buffer.from(h, "hex"));

class PublicKey {
  constructor(unc, comp) {
    this.unc = unc;
    this.comp = comp;
  }
  toBytes(format) {
    return format === "uncompressed" ? this.unc : this.comp;
  }
}

const sets = FX.sets.map((s) => ({
  type: "single",
  pubkey: new PublicKey(hex(s.pk_uncompressed), hex(s.pk_compressed)),
  signingRoot: hex(s.message),
  signature: hex(s.signature),
}));
const sameMessage = hex(FX.same_message);
const sameMessageSets = FX.same_message_sets.map((s, i) => ({publicKey: sets[i].pubkey, signature: hex(s.signature)}));
const sleep = (ms) => new Promise((r) => setTimeout(r, ms));

async function main() {
  const dir = process.argv[2];
  const pks = fs.readFileSync(path.join(dir, "pks.bin"));
  const msgs = fs.readFileSync(path.join(dir, "msgs.bin"));
  const sigs = fs.readFileSync(path.join(dir, "sigs.bin"));
  const nLoad = pks.length / 96;
  const v = new V.BlsGpuVerifier({devices: [0]});
  // the load's keys in the device table (by index); the table's keys are not mirrored
  const keys = [];
  for (let i = 0; i < nLoad; i++) keys.push(new Uint8Array(pks.buffer, pks.byteOffset + 96 * i, 96));
  await v.syncPubkeys(keys, 96);
  const loadJob = (j) => {
    const out = [];
    for (let q = 0; q < 128; q++) {
      const i = (j * 128 + q) % nLoad;
      out.push({type: "single", pubkey: {index: i}, signingRoot: msgs.subarray(32 * i, 32 * i + 32),
                signature: sigs.subarray(96 * i, 96 * i + 96)});
    }
    return out;
  };
  // background: 16 packages' worth of jobs outstanding until the cases are done
  const TARGET = 16 * 512;
  let outstanding = 0;
  let stop = false;
  let loadDone = 0;
  let loadBad = 0;
  let next = 0;
  const loadPromises = [];
  const refill = () => {
    while (!stop && outstanding < TARGET) {
      outstanding++;
      const p = v.verifySignatureSets(loadJob(next++)).then((ok) => {
        outstanding--;
        loadDone++;
        if (ok !== true) loadBad++;
        refill();
      });
      loadPromises.push(p);
    }
  };
  refill();
  await sleep(50);  // packages on the GPU before the first case

  const report = {cases: [], load_jobs_done: 0};
  async function testMany(name, sleepMs, opts) {
    const t0 = Date.now();
    const arr = [];
    for (let i = 0; i < 8; i++) {
      arr.push(v.verifySignatureSets(sets, opts));
      arr.push(v.verifySignatureSetsSameMessage(sameMessageSets, sameMessage, opts));
      if (sleepMs) await sleep(sleepMs);
    }
    const res = await Promise.all(arr);
    res.forEach((r, i) => {
      if (i % 2 === 0) assert.strictEqual(r, true, `${name}: call ${i}`);
      else assert.deepStrictEqual(r, [true, true, true], `${name}: same-message call ${i}`);
    });
    report.cases.push({name, ms: Date.now() - t0, calls: res.length, loadJobsOutstanding: outstanding});
  }
  for (const priority of [true, false]) await testMany(`synchronously priority=${priority}`, 0, {priority});
  for (const priority of [true, false]) await testMany(`asynchronously priority=${priority}`, 5, {priority});
  for (const priority of [true, false])
    await testMany(`batched priority=${priority}`, 5, {batchable: true, priority});
  for (const priority of [true, false]) {
    const t0 = Date.now();
    const invalidSet = {...sets[0], signature: hex(FX.invalid_signature)};
    const isInvalid = v.verifySignatureSets([invalidSet], {batchable: true, priority});
    const valid = [];
    for (let i = 0; i < 8; i++) valid.push(v.verifySignatureSets(sets, {batchable: true}));
    assert.strictEqual(await isInvalid, false, `first is invalid priority=${priority}`);
    (await Promise.all(valid)).forEach((r, i) => assert.strictEqual(r, true, `first invalid: valid call ${i}`));
    report.cases.push({name: `batched, first is invalid priority=${priority}`, ms: Date.now() - t0,
                       loadJobsOutstanding: outstanding});
  }
  stop = true;
  await Promise.all(loadPromises);
  assert.strictEqual(loadBad, 0, "a load job was not valid");
  report.load_jobs_done = loadDone;
  report.load_sets_done = loadDone * 128;
  await v.close();
  console.log(JSON.stringify(report));
}

main().catch((e) => {
  console.error(e && e.stack);
  process.exit(1);
});
