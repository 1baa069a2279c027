"use strict";
// The C4 composition through the N-API addon (node): a packed gossip replay of
// ~1M sets sharded over N contexts (all on cuda:0 here; one per GPU in Lodestar)
// by verifyPackedSharded -- every shard to its 576-byte Fp12 partial, ONE
// combined final exponentiation, every shard resumed with the verdict.
// Usage: node tests/js/c4_sharded.js DIR N_CONTEXTS  (DIR holds the raw arrays
// written by tests/test_gpu_c4_composition.py); prints one JSON line.
const fs = require("fs");
const path = require("path");
const ROOT = path.join(__dirname, "..", "..");
const V = require(path.join(ROOT, "lodestar_amd", "js", "bls_gpu_verifier.js"));

const dir = process.argv[2];
const nCtx = parseInt(process.argv[3] || "8", 10);
const u32 = (name) => {
  const b = fs.readFileSync(path.join(dir, name));
  return new Uint32Array(b.buffer, b.byteOffset, b.length / 4);
};
const u8 = (name) => {
  const b = fs.readFileSync(path.join(dir, name));
  return new Uint8Array(b.buffer, b.byteOffset, b.length);
};

(async () => {
  const addon = V.loadAddon();
  const packed = {
    requestOffsets: u32("req_off.bin"),
    pkOffsets: u32("pk_off.bin"),
    pubkeyIndices: u32("idx.bin"),
    messages: u8("msgs.bin"),
    signatures: u8("sigs.bin"),
    sigOffsets: u32("sig_off.bin"),
  };
  const keys = u8("keys.bin");
  const ctxs = [];
  for (let g = 0; g < nCtx; g++) ctxs.push(new addon.Context(0, {capacity: 2}));
  const sizes = await Promise.all(ctxs.map((c) => c.syncPubkeys(keys, 96)));
  const t0 = process.hrtime.bigint();
  const r = await V.verifyPackedSharded(ctxs, packed, () => new Uint8Array(32));
  const ms = Number(process.hrtime.bigint() - t0) / 1e6;
  await Promise.all(ctxs.map((c) => c.close()));
  process.stdout.write(
    JSON.stringify({
      valid: Buffer.from(r.valid).toString("hex"),
      errors: Buffer.from(r.errors).toString("hex"),
      mergedOk: r.mergedOk,
      tableSizes: sizes,
      ms,
    }) + "\n"
  );
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
