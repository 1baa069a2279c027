"""Library host path in steady state (no JS): one thread keeps 16 host-buffer calls of
65,536 sets in flight (pubkeys by validator index, as the node leg), submitting a new call
as soon as the oldest retires; times every lb_verify_requests_async and lb_wait.
Usage: python tools/host_probe.py [calls]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")


def main():
    import numpy as np

    from bench import make_workload
    from lodestar_amd.native import Device
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    dev = Device(0)
    n = 65536
    sks, pks, msgs, sigs = make_workload(dev, n, 0, hashlib.sha256(b"lodestar-mi355x-bench").digest())
    dev.pubkey_table_append(pks)
    idx = np.arange(n, dtype=np.uint32)
    mg = np.frombuffer(b"".join(msgs), np.uint8)
    blob = np.frombuffer(b"".join(sigs), np.uint8)
    so = np.arange(0, 96 * (n + 1), 96, dtype=np.uint32)
    ro = np.arange(0, n + 1, 128, dtype=np.uint32)
    seed = hashlib.sha256(b"batch-rand").digest()
    out = {}
    for events in ("1", "0"):
        os.environ["LB_STAGE_EVENTS"] = events
        d2 = Device(0)
        d2.pubkey_table_append(pks)
        sub, wt, pend = [], [], []
        for _ in range(16):  # warm
            pend.append(d2.verify_requests_async(ro, None, None, mg, blob, so, seed, pk_indices=idx))
        for pc in pend:
            d2.wait_call(pc)
        pend = []
        t0 = time.perf_counter()
        for _ in range(calls):
            if len(pend) >= 16:
                t1 = time.perf_counter()
                assert d2.wait_call(pend.pop(0)).valid.all()
                wt.append(time.perf_counter() - t1)
            t1 = time.perf_counter()
            pend.append(d2.verify_requests_async(ro, None, None, mg, blob, so, seed, pk_indices=idx))
            sub.append(time.perf_counter() - t1)
        for pc in pend:
            d2.wait_call(pc)
        el = time.perf_counter() - t0
        d2.close()
        out["events" + events] = {"sets_per_s": round(n * calls / el), "submit_ms_avg": round(1e3 * float(np.mean(sub)), 3),
                                  "submit_ms_p50": round(1e3 * float(np.median(sub)), 3),
                                  "wait_ms_avg": round(1e3 * float(np.mean(wt)), 3) if wt else None}
        print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
