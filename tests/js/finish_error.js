"use strict";
// A failing lb_verify_requests_finish rejects the addon's finish() promise instead of
// resolving with a released two-phase call's provisional verdicts (napi/addon.cc
// Kind::Finish; include/lodestar_bls.h, "Contract of the default flow").  Run by
// tests/test_gpu_twophase.py with LB_FAULT_RERUN=1: the failed combine's re-verification
// is reported as not submitted.  Inputs: DIR/{pks,msgs,sigs}.bin, 4 sets, set 1 invalid.
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const ROOT = path.join(__dirname, "..", "..");
const addon = require(path.join(ROOT, "lodestar_amd", "napi", "lodestar_bls.node"));
const dir = process.argv[2];
const rd = (n) => new Uint8Array(fs.readFileSync(path.join(dir, n + ".bin")));

(async () => {
  const pks = rd("pks"), msgs = rd("msgs"), sigs = rd("sigs");
  const n = msgs.length / 32;
  assert.strictEqual(n, 4);
  const ctx = new addon.Context(0);
  const sigOffsets = new Uint32Array(n + 1).map((_, i) => 96 * i);
  const batch = {requestOffsets: new Uint32Array([0, 2, 4]), pubkeys: pks, messages: msgs, signatures: sigs,
                 sigOffsets, seed: new Uint8Array(32)};
  const part = await ctx.verifyRequestsPartial(batch);
  const gtOk = await ctx.gtCheck(part.partial);
  let rejected = false, code = null, message = null;
  try {
    await ctx.finish(part.id, gtOk);
  } catch (e) {
    rejected = true;
    code = e.code;
    message = e.message;
  }
  // the context stays usable: a one-phase call afterwards gives the real verdicts
  const r = await ctx.verifyRequests(batch);
  assert.deepStrictEqual(Array.from(r.valid), [0, 1]);
  await ctx.close();
  console.log(JSON.stringify({gt_ok: gtOk, rejected, code, message}));
})().catch((e) => {
  console.error(e && e.stack);
  process.exit(1);
});
