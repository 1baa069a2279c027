"use strict";
// The path Lodestar takes, timed: BlsGpuVerifier (JS host) -> N-API addon ->
// lb_verify_requests_async, pubkeys by validator index (the index2pubkey mirror).
// Usage: node tools/bench_node.js DIR ROUNDS   (DIR: pks.bin n x 96, msgs.bin n x 32,
// sigs.bin n x 96 of bench.py's workload).  Prints one JSON line:
//   sets_per_s  ROUNDS x (n / 128) verifySignatureSets jobs of 128 sets, all queued at
//               once (the pool packs up to 65,536 sets per package, capacity packages
//               in flight), JS packing + addon + PCIe included;
//   p50_ms_128set  one verifySignatureSets of 128 sets on an idle verifier (before the
//                  throughput phase; *_after_throughput: the same after it);
//   p50_ms_1set    one verifyOnMainThread set (gossip block proposer signature,
//                  BN/chain/validation/block.ts:146 -> index.ts:174-187).
const fs = require("fs");
const path = require("path");
const ROOT = path.join(__dirname, "..");
const V = require(path.join(ROOT, "lodestar_amd", "js", "bls_gpu_verifier.js"));

const dir = process.argv[2];
const rounds = parseInt(process.argv[3] || "4", 10);
const rd = (name) => new Uint8Array(fs.readFileSync(path.join(dir, name)));

function median(xs) {
  const s = xs.slice().sort((a, b) => a - b);
  return s[Math.floor(s.length / 2)];
}

class PublicKey {  // @chainsafe/bls-shaped: compressed unless "uncompressed"
  constructor(unc, comp) {
    this.unc = unc;
    this.comp = comp;
  }
  toBytes(format) {
    return format === "uncompressed" ? this.unc : this.comp;
  }
}

async function c4Leg(dir, n, pks, msgs, sigs) {
  const pkc = rd("pks_c.bin");
  const aggIdx = new Uint32Array(rd("agg_idx.bin").buffer);
  const aggMsg = rd("agg_msgs.bin");
  const aggSig = rd("agg_sigs.bin");
  const nAgg = aggMsg.length / 32;
  const k = aggIdx.length / nAgg;
  const index2pubkey = [];
  for (let i = 0; i < n; i++) index2pubkey.push(new PublicKey(pks.subarray(96 * i, 96 * i + 96), pkc.subarray(48 * i, 48 * i + 48)));
  const tSync = Number(process.hrtime.bigint()) / 1e6;
  // a fresh verifier: its own tables mirror index2pubkey from entry 0
  const w = new V.BlsGpuVerifier({devices: [0]});
  await w.syncIndex2pubkey(index2pubkey);
  const syncMs = Number(process.hrtime.bigint()) / 1e6 - tSync;
  const single = (i) => ({type: "single", pubkey: index2pubkey[i], signingRoot: msgs.subarray(32 * i, 32 * i + 32),
                          signature: sigs.subarray(96 * i, 96 * i + 96)});
  const triples = [];
  for (let a = 0; a < nAgg; a++) {
    const keys = [];
    for (let q = 0; q < k; q++) keys.push(index2pubkey[aggIdx[a * k + q]]);
    triples.push([single((2 * a) % n), single((2 * a + 1) % n),
                  {type: "aggregate", pubkeys: keys, signingRoot: aggMsg.subarray(32 * a, 32 * a + 32),
                   signature: aggSig.subarray(96 * a, 96 * a + 96)}]);
  }
  // a round in C4's proportions (SURVEY §8d: 901,696 single attestations beside 32,768
  // AggregateAndProof triples): 220 jobs of 128 single sets + the triples
  const singleJobs = [];
  for (let j = 0; j < 220; j++) singleJobs.push(Array.from({length: 128}, (_, q) => single((j * 128 + q) % n)));
  const roundSets = 220 * 128 + 3 * triples.length;
  const run = async (verifier, reps) => {
    const m = verifier.metrics;
    const h0 = m.hist.get(V.METRICS.PUBKEYS_AGGREGATION_MAIN_THREAD) || {count: 0, sum: 0};
    const c0 = h0.count;
    const s0 = h0.sum;
    const t0 = Number(process.hrtime.bigint()) / 1e6;
    const all = [];
    for (let r = 0; r < reps; r++) {
      for (const js of singleJobs) all.push(verifier.verifySignatureSets(js, {batchable: true}));
      for (const t of triples) all.push(verifier.verifySignatureSets(t, {batchable: true}));
    }
    const okAll = (await Promise.all(all)).every((x) => x === true);
    const el = Number(process.hrtime.bigint()) / 1e6 - t0;
    const h = m.hist.get(V.METRICS.PUBKEYS_AGGREGATION_MAIN_THREAD) || {count: 0, sum: 0};
    return {sets_per_s: Math.round((reps * roundSets * 1000) / el),
            keys_per_s: Math.round((reps * (220 * 128 + nAgg * (k + 2)) * 1000) / el),
            pack_ms_per_package: h.count > c0 ? +(((h.sum - s0) / (h.count - c0)) * 1e3).toFixed(3) : null,
            packages: h.count - c0, rounds: reps, all_valid: okAll};
  };
  await run(w, 2);  // warm-up
  const mirrored = await run(w, 32);
  await w.close();
  // the same calls on a verifier whose tables do not hold the keys: every key serialized
  const u = new V.BlsGpuVerifier({devices: [0]});
  await run(u, 1);
  const unmirrored = await run(u, 4);
  await u.close();
  return {sets_per_round: roundSets, triples_per_round: triples.length, keys_per_aggregate: k,
          sync_index2pubkey_ms: +syncMs.toFixed(1), mirrored, unmirrored,
          api: "verifySignatureSets([selection proof, aggregator sig, aggregate of " + k +
               " keys], {batchable}) with index2pubkey PublicKey objects"};
}

(async () => {
  const pks = rd("pks.bin");
  const msgs = rd("msgs.bin");
  const sigs = rd("sigs.bin");
  const n = msgs.length / 32;
  // LB_JS_PREFETCH: packages packed ahead per GPU (BlsGpuVerifier prefetch; default 0)
  const prefetch = process.env.LB_JS_PREFETCH ? parseInt(process.env.LB_JS_PREFETCH, 10) : undefined;
  const v = new V.BlsGpuVerifier({devices: [0], prefetch});
  const tableSize = await v.syncPubkeys(Array.from({length: n}, (_, i) => pks.subarray(96 * i, 96 * i + 96)), 96);
  const set = (i) => ({
    type: "single",
    pubkey: {index: i},
    signingRoot: msgs.subarray(32 * i, 32 * i + 32),
    signature: sigs.subarray(96 * i, 96 * i + 96),
  });
  const jobs = [];
  for (let j = 0; j < n / 128; j++) jobs.push(Array.from({length: 128}, (_, k) => set(128 * j + k)));
  const ms = () => Number(process.hrtime.bigint()) / 1e6;
  // warm-up: one package; the latency loop below runs on this fresh verifier; then one package
  // per further call in flight, so every library slot has allocated its pinned staging and
  // workspace for a 65,536-set call before the timed phase (a slot's first large call
  // reallocates both: ~45 ms on the submission thread, LB_HOST_TRACE=1)
  let ok = (await Promise.all(jobs.map((js) => v.verifySignatureSets(js)))).every((x) => x === true);
  // latency on an idle verifier, before the throughput phase
  const pre128 = [];
  const pre1 = [];
  const clkPre = [];
  const clkAfter = [];
  // where a lone call's time goes: the lane's device time (first to last event of the call),
  // the kernel's own time and shader clock (s_memrealtime / s_memtime inside k_lp_verify)
  const clockSummary = (rs) => {
    const f = (k) => {
      const xs = rs.filter((r) => r && r[k] !== undefined).map((r) => r[k]);
      return xs.length ? +median(xs).toFixed(3) : null;
    };
    return {device_ms: f("deviceMs"), kernel_ms: f("kernelMs"), kernel_clock_mhz: f("kernelClockMHz")};
  };
  if (process.env.LB_JS_TRACE === "1") v.trace = [];
  for (let r = 0; r < 11; r++) {
    let t = Number(process.hrtime.bigint()) / 1e6;
    ok = ok && (await v.verifySignatureSets(jobs[r % jobs.length])) === true;
    pre128.push(Number(process.hrtime.bigint()) / 1e6 - t);
    t = Number(process.hrtime.bigint()) / 1e6;
    ok = ok && (await v.verifySignatureSets([set(r)], {verifyOnMainThread: true})) === true;
    pre1.push(Number(process.hrtime.bigint()) / 1e6 - t);
    clkPre.push(v.lastMainThreadResult);
  }
  const latSummary = (tr) => {
    const avg = (f) => +(tr.reduce((s, x) => s + f(x), 0) / Math.max(tr.length, 1) / 1e6).toFixed(3);
    return {
      calls: tr.length,
      pack_ms: avg((x) => Number(x.packedNs - x.dispatchNs)),
      to_worker_ms: avg((x) => (x.workerStartNs ? Number(x.workerStartNs) - Number(x.submittedNs) : 0)),
      worker_ms: avg((x) => (x.workerEndNs ? Number(x.workerEndNs) - Number(x.workerStartNs) : 0)),
      submit_ms: avg((x) => (x.workerSubmittedNs ? x.workerSubmittedNs - x.workerStartNs : 0)),
      until_retire_ms: avg((x) => (x.workerRetireNs ? x.workerRetireNs - x.workerSubmittedNs : 0)),
      from_worker_ms: avg((x) => (x.workerEndNs ? Number(x.backNs) - Number(x.workerEndNs) : 0)),
      device_ms: +(tr.reduce((s, x) => s + (x.deviceMs || 0), 0) / Math.max(tr.length, 1)).toFixed(3),
    };
  };
  let latTrace = null;
  if (v.trace) {
    const tr = v.trace.filter((x) => x.backNs);
    const avg = (f) => +(tr.reduce((s, x) => s + f(x), 0) / Math.max(tr.length, 1) / 1e6).toFixed(3);
    latTrace = {
      calls: tr.length,
      pack_ms: avg((x) => Number(x.packedNs - x.dispatchNs)),
      to_worker_ms: avg((x) => (x.workerStartNs ? Number(x.workerStartNs) - Number(x.submittedNs) : 0)),
      worker_ms: avg((x) => (x.workerEndNs ? Number(x.workerEndNs) - Number(x.workerStartNs) : 0)),
      from_worker_ms: avg((x) => (x.workerEndNs ? Number(x.backNs) - Number(x.workerEndNs) : 0)),
      device_ms: +(tr.reduce((s, x) => s + (x.deviceMs || 0), 0) / Math.max(tr.length, 1)).toFixed(3),
    };
    v.trace = [];
  }
  // the remaining slots' first 65,536-set calls, before the timed phase
  const warm = [];
  for (let r = 1; r < v.capacity; r++) for (const js of jobs) warm.push(v.verifySignatureSets(js));
  ok = ok && (await Promise.all(warm)).every((x) => x === true);
  if (v.trace) v.trace = [];
  const t0 = ms();
  const all = [];
  for (let r = 0; r < rounds; r++) for (const js of jobs) all.push(v.verifySignatureSets(js));
  ok = ok && (await Promise.all(all)).every((x) => x === true);
  const el = ms() - t0;
  let trace = null;
  if (v.trace) {
    // per package: main-thread packing, the addon call, dispatch -> results back; gaps
    // between consecutive dispatches; packages already in flight when one was dispatched
    const tr = v.trace.filter((x) => x.backNs);
    const avg = (f) => +(tr.reduce((s, x) => s + f(x), 0) / tr.length / 1e6).toFixed(3);
    const gaps = tr.slice(1).map((x, q) => Number(x.dispatchNs - tr[q].dispatchNs) / 1e6);
    trace = {
      packages: tr.length,
      pack_ms: avg((x) => Number(x.packedNs - x.dispatchNs)),
      addon_call_ms: avg((x) => Number(x.submittedNs - x.packedNs)),
      dispatch_to_back_ms: avg((x) => Number(x.backNs - x.dispatchNs)),
      dispatch_gap_ms_p50: +median(gaps).toFixed(3),
      in_flight_avg: +(tr.reduce((s, x) => s + x.inFlight, 0) / tr.length).toFixed(2),
      // addon side: queued -> picked up by the submission thread, picked up -> retired,
      // retired -> results on the JS thread; the call's own device time (first to last event)
      to_worker_ms: avg((x) => (x.workerStartNs ? Number(x.workerStartNs) - Number(x.submittedNs) : 0)),
      worker_ms: avg((x) => (x.workerEndNs ? Number(x.workerEndNs) - Number(x.workerStartNs) : 0)),
      from_worker_ms: avg((x) => (x.workerEndNs ? Number(x.backNs) - Number(x.workerEndNs) : 0)),
      device_ms: +(tr.reduce((s, x) => s + (x.deviceMs || 0), 0) / tr.length).toFixed(3),
      // inside the worker: lb_verify_requests_async itself, submitted -> lb_wait called, lb_wait
      submit_ms: avg((x) => (x.workerSubmittedNs ? x.workerSubmittedNs - x.workerStartNs : 0)),
      until_retire_ms: avg((x) => (x.workerRetireNs ? x.workerRetireNs - x.workerSubmittedNs : 0)),
      wait_ms: avg((x) => (x.workerRetireNs ? x.workerEndNs - x.workerRetireNs : 0)),
    };
    v.trace = null;
  }
  // latency under load: packages kept queued (every slot busy with a 65,536-set call and
  // LOAD_PACKAGES packages' jobs waiting in the JS queue, refilled as they retire);
  // meanwhile one 1-set verifyOnMainThread call and one 128-set priority job at a time
  // take the device's priority lane (BlsGpuVerifier priorityLane -> addon {priority} ->
  // the addon's latency-lane thread and context -> the library's priority slot)
  const loadPackages = Math.max(8, rounds >> 2);
  const loadJobs = loadPackages * jobs.length;
  let outstanding = 0;
  let stop = false;
  let nextJob = 0;
  let loadBad = 0;
  let loadDoneJobs = 0;
  const loadAll = [];
  const refill = () => {
    while (!stop && outstanding < loadJobs) {
      outstanding++;
      loadAll.push(v.verifySignatureSets(jobs[nextJob++ % jobs.length]).then((x) => {
        outstanding--;
        loadDoneJobs++;
        if (x !== true) loadBad++;
        refill();
      }));
    }
  };
  refill();
  await new Promise((r) => setTimeout(r, 300));  // the pipe full
  // onset: a verifyOnMainThread set arriving after >= 600 ms without priority traffic (every
  // call in flight on the full streams, the CU reservation lapsed): the first block of a
  // slot under gossip load.  A priority call's workgroups cannot preempt the throughput
  // waves already on the GPU, so it waits for CUs to drain (DESIGN.md §7).
  const onset1 = [];
  const clkOnset = [];  // per sample: where its time went (device time vs the kernel's own clock)
  const onsetSamples = parseInt(process.env.LB_NODE_ONSET_SAMPLES || "20", 10);
  for (let r = 0; r < onsetSamples; r++) {
    await new Promise((res) => setTimeout(res, 600));
    const t = ms();
    ok = ok && (await v.verifySignatureSets([set(r + 3)], {verifyOnMainThread: true})) === true;
    onset1.push(ms() - t);
    clkOnset.push(v.lastMainThreadResult);
  }
  // steady state: priority traffic every ~10 ms (the reservation held)
  const load1 = [];
  const load128 = [];
  const detail1 = [];
  const detail128 = [];
  const tLoad = ms();
  const loadJobs0 = loadDoneJobs;
  const samples = parseInt(process.env.LB_NODE_LOAD_SAMPLES || "25", 10);
  if (process.env.LB_JS_TRACE === "1") v.trace = [];
  // (the first priority calls after the onset still find the calls submitted before it on the
  // full streams: 300 ms of warm-up traffic, not sampled)
  for (const tEnd = ms() + 300; ms() < tEnd;) {
    ok = ok && (await v.verifySignatureSets([set(1)], {verifyOnMainThread: true})) === true;
    await new Promise((res) => setTimeout(res, 10));
  }
  for (let r = 0; r < samples; r++) {
    let t = ms();
    ok = ok && (await v.verifySignatureSets([set(r + 7)], {verifyOnMainThread: true})) === true;
    load1.push(ms() - t);
    const lr = v.lastMainThreadResult || {};
    detail1.push([+load1[load1.length - 1].toFixed(2), +(((lr.workerEndNs || 0) - (lr.workerStartNs || 0)) / 1e6).toFixed(2),
                  +(lr.deviceMs || 0).toFixed(2), +(lr.kernelMs || 0).toFixed(2)]);
    t = ms();
    ok = ok && (await v.verifySignatureSets(jobs[(r + 3) % jobs.length], {priority: true})) === true;
    load128.push(ms() - t);
    const pr = v.lastPriorityResult || {};
    detail128.push([+load128[load128.length - 1].toFixed(2), +(((pr.workerEndNs || 0) - (pr.workerStartNs || 0)) / 1e6).toFixed(2),
                    +(pr.deviceMs || 0).toFixed(2), +(pr.kernelMs || 0).toFixed(2), pr.stageMs || null]);
    await new Promise((res) => setTimeout(res, 10));
  }
  const loadRate = ((loadDoneJobs - loadJobs0) * 128 * 1000) / (ms() - tLoad);
  let loadTrace = null;
  if (v.trace) {  // the priority calls' phases under load (the packages' own entries left out)
    loadTrace = {set1: latSummary(v.trace.filter((x) => x.main && x.backNs)),
                 set128: latSummary(v.trace.filter((x) => !x.main && x.backNs && x.inFlight !== undefined && x.prio))};
    v.trace = null;
  }
  stop = true;
  await Promise.all(loadAll);
  ok = ok && loadBad === 0;
  const lat128 = [];
  const lat1 = [];
  if (process.env.LB_JS_TRACE === "1") v.trace = [];
  for (let r = 0; r < 11; r++) {
    let t = ms();
    ok = ok && (await v.verifySignatureSets(jobs[r % jobs.length])) === true;
    lat128.push(ms() - t);
    t = ms();
    ok = ok && (await v.verifySignatureSets([set(r)], {verifyOnMainThread: true})) === true;
    lat1.push(ms() - t);
    clkAfter.push(v.lastMainThreadResult);
  }
  let latTraceAfter = null;
  if (v.trace) {
    latTraceAfter = {
      set128: latSummary(v.trace.filter((x) => x.backNs && !x.main)),
      set1: latSummary(v.trace.filter((x) => x.backNs && x.main)),
    };
    v.trace = null;
  }
  // C4-shaped AggregateAndProof triples (BN/chain/validation/aggregateAndProof.ts:200: a
  // selection proof, the aggregator's signature, the aggregate attestation of ~488
  // committee keys), keys as @chainsafe/bls-shaped PublicKey objects out of index2pubkey:
  // mirrored (syncIndex2pubkey: shipped as 4-byte indices) and not (serialized with
  // toBytes("uncompressed") per key, as the reference does, index.ts:144)
  // (after closing v: one verifier's contexts at a time, every context's hardware queues
  // reserve scratch, DESIGN.md §5.1)
  await v.close();
  let c4 = null;
  if (fs.existsSync(path.join(dir, "agg_idx.bin"))) c4 = await c4Leg(dir, n, pks, msgs, sigs);
  process.stdout.write(
    JSON.stringify({
      sets_per_s: Math.round((rounds * n * 1000) / el),
      rounds,
      sets_per_round: n,
      p50_ms_128set: +median(pre128).toFixed(3),
      p50_ms_1set: +median(pre1).toFixed(3),
      // the same after the throughput phase (a process that has just run 96 packages)
      p50_ms_128set_after_throughput: +median(lat128).toFixed(3),
      p50_ms_1set_after_throughput: +median(lat1).toFixed(3),
      lane_1set_clocks: {fresh: clockSummary(clkPre), after_throughput: clockSummary(clkAfter)},
      // while every slot is busy with a 65,536-set package (priority lane)
      under_load_onset: {ms_1set: onset1.map((x) => +x.toFixed(2)), p50_ms_1set: +median(onset1).toFixed(3),
                         max_ms_1set: +Math.max(...onset1).toFixed(3),
                         ratio_p50_vs_idle: +(median(onset1) / median(pre1)).toFixed(2),
                         ratio_max_vs_idle: +(Math.max(...onset1) / median(pre1)).toFixed(2),
                         samples: onset1.length, gap_ms: 600,
                         // device_ms: the call's first to last event on the lane's stream; kernel_ms: k_lp_verify's
                         // own clock from its first workgroup's start -- device - kernel = waiting for CUs
                         device_ms: clkOnset.map((r) => (r && r.deviceMs !== undefined ? +r.deviceMs.toFixed(2) : null)),
                         kernel_ms: clkOnset.map((r) => (r && r.kernelMs !== undefined ? +r.kernelMs.toFixed(2) : null))},
      under_load: {
        p50_ms_1set_main_thread: load1.length ? +median(load1).toFixed(3) : null,
        p50_ms_128set_priority: load128.length ? +median(load128).toFixed(3) : null,
        ratio_1set_vs_idle: load1.length ? +(median(load1) / median(pre1)).toFixed(2) : null,
        ratio_128set_vs_idle: load128.length ? +(median(load128) / median(pre128)).toFixed(2) : null,
        samples: load1.length,
        ...(process.env.LB_JS_TRACE === "1"
          ? {ms_1set: load1.map((x) => +x.toFixed(2)), ms_128set: load128.map((x) => +x.toFixed(2)),
             detail_1set_total_lane_device_kernel_ms: detail1,
             detail_128set_total_lane_device_kernel_ms_stages: detail128} : {}),
        load_packages_queued: loadPackages,
        background_sets_per_s: Math.round(loadRate),
      },
      ...(trace ? {trace} : {}),
      ...(latTrace ? {latency_trace: latTrace} : {}),
      ...(latTraceAfter ? {latency_trace_after_throughput: latTraceAfter} : {}),
      ...(loadTrace ? {latency_trace_under_load: loadTrace} : {}),
      ...(c4 ? {c4_public_key_objects: c4} : {}),
      all_valid: ok,
      table_size: tableSize,
      capacity: v.capacity,
      api: "BlsGpuVerifier.verifySignatureSets -> N-API addon -> lb_verify_requests_async (validator indices)",
    }) + "\n"
  );
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
