"""Gossip batch-size study: same-message packages on one MI355X.

The reference groups gossip attestations by AttestationData into chunks of
MIN_SIGNATURE_SETS_TO_BATCH_VERIFY = 32 .. MAX_GOSSIP_ATTESTATION_BATCH_SIZE = 128
sets (BN/network/processor/gossipQueues/index.ts:21-26,90-91); every chunk is one
verifySignatureSetsSameMessage job, and the pool packs jobs into worker packages
(multithread/index.ts:455-489).  On the GPU every job of a package is one
aggregated set of one device call, so the question is how throughput, latency
and the cost of one bad signature depend on the job size and the package size.

Measured (lb_verify_same_message_batch_async, pubkeys by validator index):
* job size {32, 64, 128, 256, 512} at 65,536 sets per package: sets/s with 8
  packages in flight, p50 of a lone package, and the same with ONE invalid set
  per package (its job is re-verified set by set on the same slot);
* package size {1,024, 4,096, 16,384, 65,536} sets at job size 128: p50 and
  sets/s -- the latency a gossip buffer threshold buys.

Usage (GPU box): python tools/gossip_study.py > profiles/gossip_study_r03.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("LB_HW_QUEUES", "16")

import workloads as W  # noqa: E402


def main():
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from lodestar_amd.native import Device
    dev = Device(0)
    nbuf = dev.slots()
    keys = W.make_keys(dev, 65536)
    assert dev.pubkey_table_append(keys.pks) == 65536
    seed = bytes(32)
    out = {"device": "MI355X", "slots": nbuf, "job_size": [], "package_size": []}

    def run(jobs, reps):
        prep = dev.prepare_same_message(jobs, seed, by_index=True)
        lat = []
        for _ in range(5):
            t = time.perf_counter()
            res = dev.wait_same_message(dev.verify_same_message_prepared_async(prep))
            lat.append((time.perf_counter() - t) * 1e3)
        fast_all = all(res[1])
        t = time.perf_counter()
        pend = []
        for _ in range(reps):
            pend.append(dev.verify_same_message_prepared_async(prep))
            if len(pend) >= nbuf:
                dev.wait_same_message(pend.pop(0))
        for p in pend:
            dev.wait_same_message(p)
        el = time.perf_counter() - t
        n = sum(len(s) for _, s, _ in jobs)
        return {"p50_ms": round(float(np.median(lat)), 3), "sets_per_s": round(n * reps / el, 1),
                "all_fast": fast_all}

    for size in (32, 64, 128, 256, 512):
        jobs, expect = W.same_message_jobs(dev, keys, n_jobs=65536 // size, per_job=size, seed=size)
        r = run(jobs, 16)
        bad = [list(j) for j in jobs]
        bad[len(bad) // 2] = (jobs[len(jobs) // 2][0], [bytes([10]) * 96] + list(jobs[len(jobs) // 2][1][1:]),
                              jobs[len(jobs) // 2][2])
        rb = run([tuple(b) for b in bad], 16)
        out["job_size"].append({"sets_per_job": size, "jobs": len(jobs), "valid": r,
                                "one_invalid_set": {"p50_ms": rb["p50_ms"], "sets_per_s": rb["sets_per_s"],
                                                    "retried_sets": size}})
        print(json.dumps(out["job_size"][-1]), file=sys.stderr, flush=True)
    for total in (1024, 4096, 16384, 65536):
        jobs, _ = W.same_message_jobs(dev, keys, n_jobs=total // 128, per_job=128, seed=total)
        r = run(jobs, max(16, 2 * 65536 // total))
        out["package_size"].append({"sets": total, "jobs": total // 128, **r})
        print(json.dumps(out["package_size"][-1]), file=sys.stderr, flush=True)
    dev.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
