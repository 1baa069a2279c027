"use strict";
// The N-API addon on a host without a GPU: it loads, exports the boundary,
// marshals and validates a batch (validateRequests dry run), and a Context
// refuses to open with code LB_ERR_NO_DEVICE -- the error a Lodestar caller
// would see as a rejected verifier construction.
const assert = require("assert");
const path = require("path");
const addon = require(path.join(__dirname, "..", "..", "lodestar_amd", "napi", "lodestar_bls.node"));

assert.strictEqual(typeof addon.Context, "function");
assert.strictEqual(typeof addon.deviceCount(), "number");
assert.strictEqual(addon.GT_BYTES, 576);
for (const m of ["verifyRequests", "verifyRequestsPartial", "finish", "gtCheck", "verifySameMessage", "syncPubkeys",
                 "aggregatePubkeys", "close"])
  assert.strictEqual(typeof addon.Context.prototype[m], "function", m);

const ok = {
  requestOffsets: new Uint32Array([0, 2, 3]),
  pkOffsets: new Uint32Array([0, 1, 4, 5]),
  pubkeys: new Uint8Array(5 * 96),
  messages: new Uint8Array(3 * 32),
  signatures: new Uint8Array(96 + 192 + 96),
  sigOffsets: new Uint32Array([0, 96, 288, 384]),
  seed: new Uint8Array(32),
  batchable: new Uint8Array([1, 0]),
};
assert.deepStrictEqual(addon.validateRequests(ok), {nRequests: 2, nSets: 3, nPubkeys: 5, byIndex: false});
assert.deepStrictEqual(
  addon.validateRequests({...ok, pubkeys: undefined, pubkeyIndices: new Uint32Array([7, 1, 2, 3, 9])}),
  {nRequests: 2, nSets: 3, nPubkeys: 5, byIndex: true}
);
const bad = [
  [{...ok, messages: new Uint8Array(95)}, /32 bytes per set/],
  [{...ok, seed: new Uint8Array(31)}, /seed/],
  [{...ok, sigOffsets: new Uint32Array([0, 96, 90, 384])}, /not monotone/],
  [{...ok, sigOffsets: new Uint32Array([0, 96, 288, 380])}, /wrong end/],
  [{...ok, requestOffsets: new Uint32Array([1, 2, 3])}, /start at 0/],
  [{...ok, pubkeys: new Uint8Array(10)}, /96 bytes per pubkey/],
  [{...ok, pubkeys: undefined}, /missing pubkeys/],
  [{...ok, pubkeyIndices: new Uint32Array(2), pubkeys: undefined}, /one index per pubkey/],
  [{...ok, requestOffsets: [0, 2, 3]}, /typed array/],
  [{...ok, messages: new Uint32Array(24)}, /Uint8Array/],
  [{...ok, batchable: new Uint8Array(3)}, /one flag per request/],
  [{...ok, signatures: undefined}, /missing signatures/],
];
for (const [b, re] of bad) assert.throws(() => addon.validateRequests(b), (e) => e instanceof TypeError && re.test(e.message));

if (addon.deviceCount() === 0) {
  assert.throws(() => new addon.Context(0), (e) => e.code === "LB_ERR_NO_DEVICE");
  // BlsGpuVerifier construction surfaces the same error
  const V = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "bls_gpu_verifier.js"));
  assert.throws(() => new V.BlsGpuVerifier({devices: [0]}), (e) => e.code === "LB_ERR_NO_DEVICE");
}
console.log("addon ok");
