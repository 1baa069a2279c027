"""Small-call latency on one GPU (the run `rocprofv3 --kernel-trace --stats` wraps for
profiles/r04/): lone 1-set and 128-set requests through lb_verify_requests (host
buffers; the latency path on the priority lane), p50 wall time and the stage
times of the last call (k_pubkeys_*, k_lp_prep, k_lp_verify).
Usage: python tools/lp_bench.py [reps]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    from bench import make_workload
    from lodestar_amd.native import Device, pack_blobs
    dev = Device(0)
    # LB_LP_BENCH_SIZES: request sizes (default 1,128); calls of several 128-set requests
    # above 128 (e.g. 1024 = 8 requests: more workgroups than one per CU for a 512 one)
    sizes = [int(x) for x in os.environ.get("LB_LP_BENCH_SIZES", "1,128").split(",")]
    n = max(sizes)
    sks, pks, msgs, sigs = make_workload(dev, n, 0, hashlib.sha256(b"lp-bench").digest())
    seed = hashlib.sha256(b"lp-seed").digest()
    out = {}
    for k in sizes:
        name = "%dset" % k
        req = np.array(list(range(0, k, 128)) + [k] if k > 128 else [0, k], np.uint32)
        blob, offs = pack_blobs(sigs[:k])
        args = (req, np.frombuffer(b"".join(pks[:k]), np.uint8), None, np.frombuffer(b"".join(msgs[:k]), np.uint8),
                blob, offs, seed)
        r = dev.verify_requests(*args)
        assert r.valid.all(), name
        lat = []
        for _ in range(reps):
            t0 = time.perf_counter()
            dev.verify_requests(*args)
            lat.append((time.perf_counter() - t0) * 1e3)
        out[name] = {"p50_ms": round(float(np.median(lat)), 3), "min_ms": round(float(np.min(lat)), 3),
                     "stages_ms": {s: round(ms, 3) for s, ms in dev.last_stage_times()}}
        print(name, json.dumps(out[name]), flush=True)
    dev.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
