"""Stage times of lone steps-organisation calls of 4,096 ... 16,384 sets (128-set requests) with
the level products both ways (LB_LEVEL=1 / 0) and the accumulation's lane split (LB_STEP_SPLIT),
p50 of 5 calls each.  Usage (GPU box): python tools/level_probe.py"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import workloads as W
    from lodestar_amd.native import Device, pack_blobs
    sizes = (4096, 6144, 8192, 16384)
    dev = Device(0)
    keys = W.make_keys(dev, max(sizes))
    msgs = [hashlib.sha256(b"lvl" + i.to_bytes(4, "little")).digest() for i in range(max(sizes))]
    sigs = W.sign_many(dev, keys.sks[:max(sizes)], msgs)
    dev.close()
    seed = hashlib.sha256(b"lvl-seed").digest()
    pk_all = np.frombuffer(b"".join(keys.pks[:max(sizes)]), np.uint8)
    mg_all = np.frombuffer(b"".join(msgs), np.uint8)
    out = {}
    for name, env in (("level1", {}), ("level0", {"LB_LEVEL": "0"}), ("level1_split1", {"LB_STEP_SPLIT": "1"}),
                      ("level1_split2", {"LB_STEP_SPLIT": "2"}), ("level1_split4", {"LB_STEP_SPLIT": "4"})):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            d = Device(0)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        res = {}
        for n in sizes:
            ro = np.arange(0, n + 1, 128, dtype=np.uint32)
            bl, of = pack_blobs(sigs[:n])
            ts, st = [], []
            for rep in range(6):
                t1 = time.perf_counter()
                r = d.verify_requests(ro, pk_all[:96 * n], None, mg_all[:32 * n], bl, of, seed)
                dt = (time.perf_counter() - t1) * 1e3
                assert r.valid.all(), (name, n)
                if rep:
                    ts.append(dt)
                    st.append(dict(d.last_stage_times()))
            keys_ = ("step_acc", "level_prod", "level_wc", "mtail", "lines", "hash_finish", "decode_sigs")
            res["n%d" % n] = {"p50_ms": round(float(np.median(ts)), 3),
                              "stage_ms": {k: round(float(np.median([s.get(k, 0.0) for s in st])), 3) for k in keys_}}
        d.close()
        out[name] = res
        print(name, json.dumps({k: v["p50_ms"] for k, v in res.items()}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
