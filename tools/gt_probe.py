"""lb_gt_check alone on an idle GPU: one two-phase call's 576-byte partial, then the
host combine's final exponentiation timed 20 times (LB_GT_LP=1: the round program,
k_gt_prod + final_exp_lane; 0: the one-wave chain).  Usage: python tools/gt_probe.py"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from bench import make_workload
    from lodestar_amd.native import Device, pack_blobs
    dev = Device(0)
    n = 256
    sks, pks, msgs, sigs = make_workload(dev, n, 0, hashlib.sha256(b"gt-probe").digest())
    blob, offs = pack_blobs(sigs)
    req = np.array([0, 128, 256], np.uint32)
    pc = dev.verify_requests_async(req, np.frombuffer(b"".join(pks), np.uint8), None,
                                   np.frombuffer(b"".join(msgs), np.uint8), blob, offs, bytes(32), partial=True)
    part = dev.partial_wait(pc)
    ok = dev.gt_check([part])
    lat = []
    for _ in range(20):
        t = time.perf_counter()
        ok = dev.gt_check([part]) and ok
        lat.append((time.perf_counter() - t) * 1e3)
    dev.verify_finish(pc, ok)
    r = dev.wait_call(pc)
    dev.close()
    print(json.dumps({"gt_lp": os.environ.get("LB_GT_LP", "default"), "ok": bool(ok), "valid": [int(v) for v in r.valid],
                      "p50_ms": round(float(np.median(lat)), 3), "min_ms": round(min(lat), 3)}))


if __name__ == "__main__":
    main()
