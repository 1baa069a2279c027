"use strict";
// CPU-only ceiling of the JS host (VERDICT r3 next #6): BlsGpuVerifier over N mock
// contexts that answer at once (all valid, a 1 ms device time each), so the rate
// is what the main thread alone sustains: chunking, queueing, packing into the C-ABI
// layout, dispatch, per-job resolution.  Two inputs:
//   objects: ISignatureSet objects (pubkeys by validator index), the IBlsVerifier path;
//   packed:  calls already in the C-ABI layout (verifyPackedSharded), the shape a gossip
//            replay or a network layer that packs on arrival takes.
// Usage: node tools/js_host_bench.js [contexts=8] [rounds=16]
const path = require("path");
const V = require(path.join(__dirname, "..", "lodestar_amd", "js", "bls_gpu_verifier.js"));

const nCtx = parseInt(process.argv[2] || "8", 10);
const rounds = parseInt(process.argv[3] || "16", 10);
const N = 65536;

class InstantBackend {
  constructor() {
    this.capacity = 16;
    this.sets = 0;
  }
  async verifyRequests(b) {
    const nReq = b.requestOffsets.length - 1;
    this.sets += b.requestOffsets[nReq];
    await new Promise((r) => setTimeout(r, 1));
    return {valid: new Uint8Array(nReq).fill(1), errors: new Uint8Array(nReq), setStatus: new Uint8Array(0),
      batchRetries: 0, batchSigsSuccess: 0, deviceMs: 1};
  }
  async verifyRequestsPartial(b) {
    const nReq = b.requestOffsets.length - 1;
    this.sets += b.requestOffsets[nReq];
    return {id: nReq, partial: new Uint8Array(576).fill(1)};
  }
  async gtCheck() {
    return true;
  }
  async finish(id) {
    return {valid: new Uint8Array(id).fill(1), errors: new Uint8Array(id)};
  }
}

const ms = () => Number(process.hrtime.bigint()) / 1e6;

(async () => {
  const sig = new Uint8Array(96 * N);
  const roots = new Uint8Array(32 * N);
  const jobs = [];
  for (let j = 0; j < N / 128; j++) {
    const js = [];
    for (let k = 0; k < 128; k++) {
      const i = 128 * j + k;
      js.push({type: "single", pubkey: {index: i}, signingRoot: roots.subarray(32 * i, 32 * i + 32),
        signature: sig.subarray(96 * i, 96 * i + 96)});
    }
    jobs.push(js);
  }
  const out = {contexts: nCtx, rounds, sets_per_round: N};
  // objects through the pool
  {
    const backends = Array.from({length: nCtx}, () => new InstantBackend());
    const v = new V.BlsGpuVerifier({backends, seedSource: () => new Uint8Array(32)});
    await Promise.all(jobs.map((js) => v.verifySignatureSets(js)));  // warm-up
    const t0 = ms();
    const all = [];
    for (let r = 0; r < rounds; r++) for (const js of jobs) all.push(v.verifySignatureSets(js));
    const ok = (await Promise.all(all)).every((x) => x === true);
    const el = ms() - t0;
    out.objects_sets_per_s = Math.round((rounds * N * 1000) / el);
    out.objects_all_valid = ok;
    // the packing alone (main thread), per 65,536-set package
    const tp = ms();
    for (let r = 0; r < 4; r++) V.packRequests(jobs, new Uint8Array(32));
    out.pack_ms_per_package = +((ms() - tp) / 4).toFixed(3);
    await v.close();
  }
  // packed calls sharded over the contexts (two-phase combine)
  {
    const backends = Array.from({length: nCtx}, () => new InstantBackend());
    const packed = V.packRequests(jobs, new Uint8Array(32));
    await V.verifyPackedSharded(backends, packed, () => new Uint8Array(32));
    const t0 = ms();
    let ok = true;
    for (let r = 0; r < rounds; r++) {
      const res = await V.verifyPackedSharded(backends, packed, () => new Uint8Array(32));
      ok = ok && res.mergedOk && res.valid.every((x) => x === 1);
    }
    const el = ms() - t0;
    out.packed_sets_per_s = Math.round((rounds * N * 1000) / el);
    out.packed_all_valid = ok;
  }
  out.node = process.version;
  process.stdout.write(JSON.stringify(out) + "\n");
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
