"""Which verification organisation a mid-size call should take.

The library picks the Miller organisation by call size (bls_host.hip run_pipeline):
the latency path up to lp_max_sets, one wave per pair up to wave_max_sets, one pair per
lane (k_miller_sets + the one-lane merged tail) below lines_min_sets, the stored lines +
step-major accumulation + the merged-check round program (mtail) from there.  Round 6's
probe (profiles/r06/orgs_probe_r06f.json, then defaults 8192 / 4096) moved both thresholds
to 1025 ("lines_msm_from_1k"), so "default" now equals that configuration.  This probe
times lone synchronous calls of the C5 epoch (valid, and with its 1e-3 injection) and of
uniform 128-set-request calls of 1.5k ... 8k sets in contexts built with different
thresholds (LB_LINES_MIN, LB_MSM_MIN) and LB_MTAIL, checking every verdict.

Usage (GPU box): python tools/orgs_probe.py > gpurun_out/orgs.json
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CONFIGS = {
    "default": {},
    "level_prod_one_lane": {"LB_LEVEL": "0"},
    "default_mtail_off": {"LB_MTAIL": "0"},
    "round5_thresholds": {"LB_LINES_MIN": "8192", "LB_MSM_MIN": "4096"},
}
SIZES = (1536, 2048, 3072, 4096, 6144, 8192)
# (ORGS_CONFIGS: a JSON object replacing CONFIGS; ORGS_SIZES: comma-separated call sizes)
if os.environ.get("ORGS_CONFIGS"):
    CONFIGS = json.loads(os.environ["ORGS_CONFIGS"])
if os.environ.get("ORGS_SIZES"):
    SIZES = tuple(int(x) for x in os.environ["ORGS_SIZES"].split(","))


def p50(fn, reps):
    ts = []
    for _ in range(reps):
        t1 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t1) * 1e3)
    return float(np.median(ts))


def main():
    import workloads as W
    from lodestar_amd.native import Device, pack_blobs
    reps = int(os.environ.get("ORGS_REPS", "5"))
    dev = Device(0)
    keys = W.make_keys(dev, 65536)
    c5 = W.c5_epoch(dev, keys)
    msgs = [hashlib.sha256(b"orgs" + i.to_bytes(4, "little")).digest() for i in range(max(SIZES))]
    sigs = W.sign_many(dev, keys.sks[:max(SIZES)], msgs)
    dev.close()
    seed = hashlib.sha256(b"orgs-seed").digest()
    b5, o5 = c5.blobs()
    m5 = c5.msg_array()
    bv, ov = pack_blobs(c5.clean_sigs)
    mv = np.frombuffer(b"".join(c5.clean_msgs), np.uint8)
    want5 = [k not in c5.expect_invalid_requests for k in range(c5.n_req)]
    pk_all = np.frombuffer(b"".join(keys.pks[:max(SIZES)]), np.uint8)
    mg_all = np.frombuffer(b"".join(msgs), np.uint8)
    out = {"reps": reps, "configs": {}}
    for name, env in CONFIGS.items():
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            d = Device(0)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        d.pubkey_table_append(keys.pks)
        res = {"env": env}

        def c5_call(valid):
            r = (d.verify_requests(c5.req_off, None, c5.pk_off, mv, bv, ov, seed, pk_indices=c5.idx) if valid else
                 d.verify_requests(c5.req_off, None, c5.pk_off, m5, b5, o5, seed, pk_indices=c5.idx))
            assert [bool(v) for v in r.valid] == ([True] * c5.n_req if valid else want5), (name, valid)
        for valid in (True, False):
            c5_call(valid)
            ms = p50(lambda: c5_call(valid), reps)
            res["c5_valid" if valid else "c5_injected"] = {"p50_ms": round(ms, 3), "stage_ms": {
                k: round(v, 3) for k, v in d.last_stage_times()}}
        for n in SIZES:
            ro = np.arange(0, n + 1, 128, dtype=np.uint32)
            bl, of = pack_blobs(sigs[:n])

            def call():
                r = d.verify_requests(ro, pk_all[:96 * n], None, mg_all[:32 * n], bl, of, seed)
                assert r.valid.all(), (name, n)
            call()
            ms = p50(call, reps)
            res["n%d" % n] = {"p50_ms": round(ms, 3), "stage_ms": {
                k: round(v, 3) for k, v in d.last_stage_times()}}
        d.close()
        out["configs"][name] = res
        print(name, json.dumps({k: (v["p50_ms"] if isinstance(v, dict) and "p50_ms" in v else None)
                                for k, v in res.items()}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
